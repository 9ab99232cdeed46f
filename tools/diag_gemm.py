"""Time the fp32 projection GEMM shapes of the HealthRec step under each torch BLAS backend."""
import torch, time
dev = torch.device("cuda")
M, K, N = 1024, 2048, 64
X = torch.randn(M, K, device=dev); W = torch.randn(N, K, device=dev); b = torch.randn(N, device=dev)
G = torch.randn(M, N, device=dev)
def t(f, n=50):
    f(); torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): f()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3
for lib in ["cublaslt", "cublas"]:
    try:
        torch.backends.cuda.preferred_blas_library(lib)
    except Exception as ex:
        print(lib, "unavailable", ex); continue
    fwd = t(lambda: torch.nn.functional.linear(X, W, b))
    dW = t(lambda: G.t() @ X)
    dX = t(lambda: G @ W)
    fwd512 = t(lambda: torch.nn.functional.linear(X[:, :512].contiguous(), W[:, :512].contiguous(), b))
    print(f"{lib}: fwd {fwd:.1f}us  dW {dW:.1f}us  dX {dX:.1f}us  fwd(K=512) {fwd512:.1f}us")
