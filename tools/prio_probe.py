"""Probe: do kernels captured from prioritised streams carry a per-node priority, and does a graph
instantiated with hipGraphInstantiateFlagUseNodePriority launch?  (round-5 scheduling experiment)"""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
lo, hi = ctypes.c_int(), ctypes.c_int()
hip.hipDeviceGetStreamPriorityRange(ctypes.byref(lo), ctypes.byref(hi))
print("priority range least / greatest", lo.value, hi.value)
x = torch.zeros(1 << 20, device="cuda")
y = torch.zeros_like(x)
s_hi = torch.cuda.Stream(priority=hi.value)
s_lo = torch.cuda.Stream(priority=lo.value)
print("stream priorities", s_hi.priority, s_lo.priority)
g = torch.cuda.CUDAGraph(keep_graph=True)
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    x.add_(1)
    y.add_(2)
torch.cuda.current_stream().wait_stream(side)
with torch.cuda.graph(g):
    main = torch.cuda.current_stream()
    s_hi.wait_stream(main)
    s_lo.wait_stream(main)
    with torch.cuda.stream(s_hi):
        x.add_(1)
    with torch.cuda.stream(s_lo):
        y.add_(2)
    main.wait_stream(s_hi)
    main.wait_stream(s_lo)
raw = g.raw_cuda_graph()
print("raw graph", type(raw), raw)
n = ctypes.c_size_t(0)
hip.hipGraphGetNodes(ctypes.c_void_p(raw), None, ctypes.byref(n))
nodes = (ctypes.c_void_p * n.value)()
hip.hipGraphGetNodes(ctypes.c_void_p(raw), nodes, ctypes.byref(n))
for nd in nodes:
    t = ctypes.c_int()
    hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
    if t.value == 0:
        val = (ctypes.c_char * 64)()
        rc = hip.hipGraphKernelNodeGetAttribute(ctypes.c_void_p(nd), 8, ctypes.byref(val))
        print("kernel node: rc", rc, "priority", int.from_bytes(bytes(val[:4]), "little", signed=True))
k = 0
for nd in nodes:
    t = ctypes.c_int()
    hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
    if t.value == 0:
        val = (ctypes.c_char * 64)()
        ctypes.memmove(val, ctypes.byref(ctypes.c_int(-1 if k == 0 else 1)), 4)
        rc = hip.hipGraphKernelNodeSetAttribute(ctypes.c_void_p(nd), 8, ctypes.byref(val))
        got = (ctypes.c_char * 64)()
        hip.hipGraphKernelNodeGetAttribute(ctypes.c_void_p(nd), 8, ctypes.byref(got))
        print("set node priority rc", rc, "now", int.from_bytes(bytes(got[:4]), "little", signed=True))
        k += 1
ex = ctypes.c_void_p()
rc = hip.hipGraphInstantiateWithFlags(ctypes.byref(ex), ctypes.c_void_p(raw), ctypes.c_ulonglong(8))
print("instantiate UseNodePriority rc", rc)
x.zero_()
y.zero_()
rc = hip.hipGraphLaunch(ex, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
print("launch rc", rc, x[0].item(), y[0].item())
