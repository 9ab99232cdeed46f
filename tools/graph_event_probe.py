"""Probe: timing events recorded inside a captured HIP graph (event record nodes): does
elapsed_time between them give the kernel's time on replay?  (round-5 measurement experiment)"""
import torch

x = torch.randn(1 << 24, device="cuda")
y = torch.empty_like(x)
side = torch.cuda.Stream()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for _ in range(3):
    torch.mul(x, 2.0, out=y)
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(10):
    torch.mul(x, 2.0, out=y)
b.record()
torch.cuda.synchronize()
print("eager per launch ms", a.elapsed_time(b) / 10)
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    torch.mul(x, 2.0, out=y)
torch.cuda.current_stream().wait_stream(s)
with torch.cuda.graph(g):
    torch.mul(x, 3.0, out=y)
    e0.record()
    torch.mul(x, 2.0, out=y)
    e1.record()
    torch.mul(x, 4.0, out=y)
for k in range(3):
    g.replay()
    torch.cuda.synchronize()
    try:
        print("replay", k, "in-graph event ms", e0.elapsed_time(e1))
    except Exception as ex:  # noqa: BLE001
        print("replay", k, "elapsed_time failed:", ex)
