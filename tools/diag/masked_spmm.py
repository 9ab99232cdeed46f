"""Masked UI-backward SpMM of the HealthRec step in isolation: A1 gate on/off, the upstream buffer
zero-filled or left uninitialised outside the batch rows."""
import os
import sys
R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path[:0] = [os.path.join(R, "multi-modal-food-recommendation_amd"), R]
import torch
import bench
from FoodRec.engine import ops

dev = torch.device("cuda:0")
cfg, data, model = bench.build(dev, 512)
adj = model.norm_adj_matrix
U, I = model.n_users, model.n_items
torch.manual_seed(0)
u = torch.randint(0, U, (512,), device=dev)
p = torch.randint(0, I, (512,), device=dev)
n = torch.randint(0, I, (512,), device=dev)
rows = [(u, 0), (p, U), (n, U)]
mask = torch.zeros(U + I, dtype=torch.uint8, device=dev)
ops.rows_mark(mask, rows, 1)
d_user = torch.empty(U, 64, device=dev)
G_ri = torch.zeros(I + 20000, 64, device=dev)
for init in ("zeros", "garbage", "nan"):
    G = torch.zeros(U + I, 64, device=dev) if init == "zeros" else \
        torch.full((U + I, 64), float("nan") if init == "nan" else 1e-39, device=dev)
    G[u] = torch.randn(512, 64, device=dev)
    G[U + p] = torch.randn(512, 64, device=dev)
    G[U + n] = torch.randn(512, 64, device=dev)
    for gate in (False, True):
        if init != "zeros" and not gate:
            continue
        f = lambda: ops.spmm_ex(adj, G, Y2=d_user, Y2_hi=G_ri, split=U, alpha=0.5, A1=G, beta1=0.5, col_mask=mask,
                                a1_gate=mask if gate else None, nbytes=0)
        for _ in range(5):
            f()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            f()
        e.record()
        torch.cuda.synchronize()
        print(f"init={init:8s} gate={gate}: {s.elapsed_time(e) / 50 * 1e3:.1f} us   nan_out={bool(torch.isnan(d_user).any())}")
