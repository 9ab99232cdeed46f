"""Probe: are hipMemsetAsync / hipMemcpyAsync nodes of a captured HIP graph ordered before the kernels
that consume them on replay?  Pure data checks (no data-dependent addressing, cannot fault).

graph body:  memset(buf, 0) -> buf += 1 (kernel) -> bad1 += (buf != 1).sum()
             tag += 1 (kernel) -> src = tag (kernel) -> memcpy(dst <- src) -> bad2 += (dst != tag).sum()
Run for 501 int32 (the 2004-byte counter clear fr_embedding_bwd captured before it switched to a
clearing kernel), 64 KiB and 64 MiB; prints mismatch counts for eager and graph-replayed execution.
"""
import ctypes
import sys

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemsetAsync.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t, ctypes.c_void_p]
hip.hipMemsetAsync.restype = ctypes.c_int
hip.hipMemcpyAsync.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p]
hip.hipMemcpyAsync.restype = ctypes.c_int
D2D = 3
dev = torch.device("cuda")


def probe(N, reps):
    buf = torch.ones(N, dtype=torch.int32, device=dev) * 7
    src = torch.zeros(N, dtype=torch.int32, device=dev)
    dst = torch.zeros(N, dtype=torch.int32, device=dev)
    tag = torch.zeros((), dtype=torch.int32, device=dev)
    bad1 = torch.zeros((), dtype=torch.int64, device=dev)
    bad2 = torch.zeros((), dtype=torch.int64, device=dev)

    def body():
        st = torch.cuda.current_stream().cuda_stream
        assert hip.hipMemsetAsync(buf.data_ptr(), 0, N * 4, st) == 0
        buf.add_(1)
        bad1.add_((buf != 1).sum())
        tag.add_(1)
        src.copy_(tag.expand(N))
        assert hip.hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), N * 4, D2D, st) == 0
        bad2.add_((dst != tag).sum())

    for _ in range(50):
        body()
    torch.cuda.synchronize()
    print(f"N={N:>9} eager : 50 reps, memset-order mismatches {int(bad1)}, memcpy-order mismatches {int(bad2)}",
          flush=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        body()
    torch.cuda.current_stream().wait_stream(s)
    bad1.zero_()
    bad2.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        body()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    print(f"N={N:>9} graph : {reps} replays, memset-order mismatches {int(bad1)}, memcpy-order mismatches "
          f"{int(bad2)} (elements; tag={int(tag)})", flush=True)


if __name__ == "__main__":
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
    for n in (501, 1 << 14, 1 << 24):
        probe(n, reps)
