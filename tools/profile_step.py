"""torch.profiler breakdown of the HealthRec training step (op-level GPU time with shapes)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]
import numpy as np, torch
import bench
from FoodRec.common.trainer import Trainer
from FoodRec.engine.sampler import TripleSampler
dev = torch.device("cuda")
cfg, data, model = bench.build(dev, 512)
tr = Trainer(cfg, model)
sampler = TripleSampler(data, 512, dev, replay_python_random=False)
feats = tr._features(); st = tr.new_step_state(); model.train()
it = sampler.epoch()
for i in range(5):
    u, p, n = next(it); tr.train_step(feats.batch(u, p, n), i, st)
torch.cuda.synchronize()
from torch.profiler import profile, ProfilerActivity
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True) as prof:
    for i in range(5):
        u, p, n = next(it); tr.train_step(feats.batch(u, p, n), i, st)
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=40, max_name_column_width=60, max_shapes_column_width=70))
