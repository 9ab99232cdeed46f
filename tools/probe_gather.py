"""Probe: time of gathering 1,024 random 8-KB rows from HealthRec's 45,630 x 2,048 image table (374 MB)
against the same gather from a 1,024-row table (no page spread), and with the ids sorted -- whether the
projection kernels' ~14 us are the row gather's address translation rather than bandwidth."""
import json
import torch

dev = torch.device("cuda:0")
torch.manual_seed(0)
R, K, n = 45630, 2048, 1024
big = torch.randn(R, K, device=dev)
small = torch.randn(n, K, device=dev)
ids = torch.randint(0, R, (n,), device=dev)
ids_sorted = ids.sort().values
seq = torch.arange(n, device=dev)


def t(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1000.0


out = torch.empty(n, K, device=dev)
res = {
    "big_random_us": t(lambda: torch.index_select(big, 0, ids, out=out)),
    "big_sorted_us": t(lambda: torch.index_select(big, 0, ids_sorted, out=out)),
    "big_first_rows_us": t(lambda: torch.index_select(big, 0, seq, out=out)),
    "small_us": t(lambda: torch.index_select(small, 0, seq, out=out)),
    "copy_8MB_us": t(lambda: out.copy_(small)),
}
res["bytes"] = n * K * 4
print(json.dumps(res))

# the engine's projection kernels on the same rows (warm caches, back to back)
import ctypes  # noqa: E402
import sys  # noqa: E402
sys.path.insert(0, "multi-modal-food-recommendation_amd")
from FoodRec.engine import native  # noqa: E402

lib = native.lib()
text = torch.randn(R, 512, device=dev)
W1, W2 = torch.randn(64, K, device=dev), torch.randn(64, 512, device=dev)
b1, b2 = torch.randn(64, device=dev), torch.randn(64, device=dev)
Y = torch.empty(n, 128, device=dev)
s = native.stream_of(big)


def proj(idx):
    native.check(lib.fr_gather_linear_fwd_multi(
        idx.data_ptr(), n, 2, (ctypes.c_void_p * 2)(big.data_ptr(), text.data_ptr()), (ctypes.c_int64 * 2)(K, 512),
        (ctypes.c_int * 2)(K, 512), (ctypes.c_void_p * 2)(W1.data_ptr(), W2.data_ptr()),
        (ctypes.c_void_p * 2)(b1.data_ptr(), b2.data_ptr()), Y.data_ptr(), 128, s), "proj")


dW1, dW2, db1, db2 = torch.empty_like(W1), torch.empty_like(W2), torch.empty_like(b1), torch.empty_like(b2)
Ks = (ctypes.c_int * 2)(K, 512)
ws = torch.empty(lib.fr_linear_wgrad_gather_multi_workspace(n, 64, 2, Ks) // 4 + 64, device=dev)
dY = torch.randn(n, 128, device=dev)


def wgrad(idx):
    native.check(lib.fr_linear_wgrad_gather_multi(
        dY.data_ptr(), 128, idx.data_ptr(), n, 64, 2, (ctypes.c_void_p * 2)(big.data_ptr(), text.data_ptr()),
        (ctypes.c_int64 * 2)(K, 512), Ks, (ctypes.c_void_p * 2)(dW1.data_ptr(), dW2.data_ptr()),
        (ctypes.c_int64 * 2)(K, 512), (ctypes.c_void_p * 2)(db1.data_ptr(), db2.data_ptr()), ws.data_ptr(),
        ws.numel() * 4, s), "wgrad")


flush = torch.empty(512 * 1024 * 1024 // 4, device=dev)  # 512 MB: evicts the 256 MB MALL


def cold(fn):
    tot = 0.0
    for _ in range(10):
        flush.add_(1.0)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        tot += a.elapsed_time(b) * 1000.0
    return tot / 10


res2 = {"proj_warm_us": t(lambda: proj(ids)), "proj_warm_sorted_us": t(lambda: proj(ids_sorted)),
        "proj_cold_us": cold(lambda: proj(ids)), "wgrad_warm_us": t(lambda: wgrad(ids)),
        "wgrad_cold_us": cold(lambda: wgrad(ids)), "index_select_cold_us": cold(lambda: torch.index_select(big, 0, ids, out=out))}
print(json.dumps(res2))
