"""The epoch's host sampling pieces on the Allrecipes shape (TripleSampler): the permutation, the
stream-exact negatives drawn through it into a pinned buffer, the host-to-device copies."""
import sys, time
sys.path[:0]=["multi-modal-food-recommendation_amd", "."]
import numpy as np, torch
from FoodRec.utils.dataset import FoodData
from FoodRec.utils.synthetic import make_synthetic
from FoodRec.engine.sampler import TripleSampler
data = FoodData.from_synthetic(make_synthetic("allrecipes", 0, negatives=False))
s = TripleSampler(data, 512, torch.device("cuda"), replay_python_random=False)
buf = torch.empty(s.n, dtype=torch.int64, pin_memory=True)
for rep in range(4):
    t0=time.perf_counter(); perm = s.epoch_order().numpy(); t1=time.perf_counter()
    s._negatives(s.users, perm=perm, out=buf.numpy()); t2=time.perf_counter()
    d = buf.to("cuda", non_blocking=True); pd = torch.from_numpy(perm).to("cuda", non_blocking=True); torch.cuda.synchronize(); t3=time.perf_counter()
    print(f"perm {1e3*(t1-t0):.2f} ms  negatives {1e3*(t2-t1):.2f} ms  h2d {1e3*(t3-t2):.2f} ms", flush=True)
