"""Where the HealthRec graphed step's wall time goes: (a) the bench loop (sampler + replay),
(b) graph replays alone (static inputs), (c) the host sampler alone, (d) host time of one
replay call.  Usage: python tools/diag_host.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from FoodRec.common.trainer import Trainer  # noqa: E402
from FoodRec.engine.sampler import TripleSampler  # noqa: E402

dev = torch.device("cuda", 0)
cfg, data, model = bench.build(dev, 512)
tr = Trainer(cfg, model)
np.random.seed(1000)
sampler = TripleSampler(data, 512, dev, replay_python_random=False)
g = tr.graphed_step(512, warmup=3)
state = g.state
feed = g.attach_feed(sampler) if os.environ.get("FR_NO_FEED") is None else None


def batches():
    while True:
        for t in sampler.epoch(out=g.inputs, feed=feed):
            yield t


it = batches()
for i in range(8):
    g(*next(it), i, state)
torch.cuda.synchronize()
K = 50
t0 = time.perf_counter()
for i in range(K):
    g(*next(it), i, state)
torch.cuda.synchronize()
a = (time.perf_counter() - t0) / K * 1e3
t0 = time.perf_counter()
for i in range(K):
    g.graph.replay()
torch.cuda.synchronize()
b = (time.perf_counter() - t0) / K * 1e3
t0 = time.perf_counter()
for i in range(K):
    g.graph.replay()
th = (time.perf_counter() - t0) / K * 1e3
torch.cuda.synchronize()
t0 = time.perf_counter()
for i in range(K):
    next(it)
torch.cuda.synchronize()
c = (time.perf_counter() - t0) / K * 1e3
print(f"bench loop {a:.3f} ms/step | replays only {b:.3f} ms | host time per replay call {th:.3f} ms | "
      f"sampler only {c:.3f} ms", flush=True)
