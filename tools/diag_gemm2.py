import torch
dev = torch.device("cuda")
shapes = [(256, 20480, 64), (192, 20480, 64), (64, 20480, 256), (64, 20480, 64), (20480, 64, 256), (20480, 256, 64), (20480, 64, 192)]
def t(f, n=50):
    f(); torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True); e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n): f()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3
for lib in ["cublaslt", "cublas"]:
    torch.backends.cuda.preferred_blas_library(lib)
    out = []
    for (m, k, n) in shapes:
        A = torch.randn(k, m, device=dev).t()  # transposed operand like autograd's grad.t() @ x
        B = torch.randn(k, n, device=dev)
        out.append(f"{m}x{k}x{n}: {t(lambda: A @ B):.1f}")
    print(lib, " | ".join(out))
