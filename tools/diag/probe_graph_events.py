import torch, time
dev = torch.device("cuda", 0)
x = torch.randn(4096, 4096, device=dev)
y = torch.empty_like(x)
s = torch.cuda.Stream()
e0 = torch.cuda.Event(enable_timing=True)
e1 = torch.cuda.Event(enable_timing=True)
torch.cuda.synchronize()
with torch.cuda.stream(s):
    for _ in range(3):
        torch.mm(x, x, out=y)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
try:
    with torch.cuda.graph(g, stream=s):
        torch.mm(x, x, out=y)
        e0.record()
        torch.mm(x, x, out=y)
        e1.record()
        torch.mm(x, x, out=y)
    for _ in range(5):
        g.replay()
    torch.cuda.synchronize()
    print("graph events ms", e0.elapsed_time(e1))
except Exception as ex:
    print("capture failed:", repr(ex))
a = torch.cuda.Event(enable_timing=True); b = torch.cuda.Event(enable_timing=True)
a.record(); torch.mm(x, x, out=y); b.record(); torch.cuda.synchronize(); print("eager events ms", a.elapsed_time(b))
