"""SpMM at BASELINE config-4 scale (10M users x 1M items x ~200M edges, d=64 fp32): per-launch
time of fr_spmm_csr and algorithmic GB/s (SURVEY 8(d) byte model) vs the 8 TB/s HBM peak."""
import argparse, json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT, os.path.join(ROOT, "tools")]
import torch
from FoodRec.engine import ops
from FoodRec.engine.graph import Adjacency, bipartite_norm_csr_torch
from FoodRec.utils.interaction_graph import synth_bipartite

ap = argparse.ArgumentParser()
ap.add_argument("--users", type=int, default=10_000_000)
ap.add_argument("--items", type=int, default=1_000_000)
ap.add_argument("--deg", type=float, default=20.0)
ap.add_argument("--chunk", type=int, nargs="+", default=[256])
ap.add_argument("--iters", type=int, default=10)
ap.add_argument("--d", type=int, default=64)
a = ap.parse_args()
dev = torch.device("cuda")
t0 = time.time()
u, i = synth_bipartite(a.users, a.items, a.deg, device=dev)
rp, col, val = bipartite_norm_csr_torch(a.users, a.items, u, i)
del u, i
torch.cuda.synchronize()
N = a.users + a.items
print(f"graph built in {time.time()-t0:.1f}s: N={N} nnz={col.numel()} max_row={int((rp[1:]-rp[:-1]).max())}", flush=True)
X = torch.randn(N, a.d, device=dev)
Y = torch.empty_like(X)
res = []
for ch in a.chunk:
    adj = Adjacency(rp, col, val, (N, N), chunk=ch, device=dev)
    ops.spmm_launch(adj, X, Y1=Y)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(a.iters):
        ops.spmm_launch(adj, X, Y1=Y)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / a.iters
    b = ops.spmm_bytes(adj, a.d, 1)
    r = {"chunk": ch, "n_units": adj.n_units, "n_split": adj.n_split, "avg_ms": round(ms, 3),
         "bytes": b, "gbps": round(b / ms / 1e6, 1), "frac": round(b / ms / 1e6 / 8000, 4)}
    res.append(r)
    print(json.dumps(r), flush=True)
# spot-check correctness on a few rows against a float64 gather
rows = torch.randint(0, N, (64,), device=dev)
ok = True
for r_ in rows.tolist():
    s_, e_ = int(rp[r_]), int(rp[r_ + 1])
    ref = (val[s_:e_].double()[:, None] * X[col[s_:e_].long()].double()).sum(0)
    ok &= bool(torch.allclose(Y[r_].double(), ref, rtol=1e-4, atol=1e-5))
print("spot-check", ok)
