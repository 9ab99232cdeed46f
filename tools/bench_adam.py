"""The dense fused Adam launch alone at HealthRec's shape (user 68,768 / item 45,630 / ingredient
19,988 rows x 64 plus ~0.4M small parameters: 8.9M parameters, 28 B each = 249 MB per launch):
average launch time over back-to-back launches and the HBM rate it implies.  FR_ENGINE_LIB selects
another build of the library (A/B of kernel versions)."""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]
import torch  # noqa: E402

from FoodRec.engine import native  # noqa: E402

dev = torch.device("cuda:0")
torch.manual_seed(0)
shapes = [(68768, 64), (45630, 64), (19988, 64), (192, 64), (192,), (64, 64), (64,), (256, 64), (256,), (64, 256),
          (64,), (64, 2048), (64,), (64, 512), (64,)] + [(64,)] * 20
P = [torch.randn(*s, device=dev) * 0.1 for s in shapes]
G = [torch.randn(*s, device=dev) * 1e-3 for s in shapes]
M = [torch.zeros(*s, device=dev) for s in shapes]
V = [torch.zeros(*s, device=dev) for s in shapes]
S = [torch.zeros((), dtype=torch.int64, device=dev) for _ in shapes]
n = len(shapes)
arr = lambda ts: (ctypes.c_void_p * n)(*[t.data_ptr() for t in ts])  # noqa: E731
N = (ctypes.c_int64 * n)(*[t.numel() for t in P])
lr = torch.full((), 1e-3, dtype=torch.float64, device=dev)
ticket = torch.zeros(32, dtype=torch.int32, device=dev)
lib = native.lib()
stream = native.stream_of(P[0])


def step():
    native.check(lib.fr_adam_step_dev(arr(P), arr(G), arr(M), arr(V), arr(S), N, n, lr.data_ptr(), 1e-3, 0.9, 0.999,
                                      1e-8, 0.0, None, ticket.data_ptr(), stream), "fr_adam_step_dev")


for _ in range(5):
    step()
torch.cuda.synchronize()
reps = 100
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(reps):
    step()
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) / reps * 1e3
numel = sum(t.numel() for t in P)
print(json.dumps({"lib": os.environ.get("FR_ENGINE_LIB", "head"), "params": numel, "bytes": 28 * numel,
                  "us_per_launch": round(us, 2), "tb_per_s": round(28 * numel / us / 1e6, 3)}))
