"""Where the small PyTorch kernels of the eager config-3 step (CLUSSL, dCor SSL) come from: every ATen
op with device time, grouped by (op, call site) -- the model's Python frame for forward ops, the
autograd node for backward ops -- with calls and device microseconds per step."""
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from FoodRec.common.trainer import Trainer  # noqa: E402
from FoodRec.engine.sampler import TripleSampler  # noqa: E402
from FoodRec.utils.configurator import Config  # noqa: E402
from FoodRec.utils.dataset import FoodData  # noqa: E402
from FoodRec.utils.synthetic import make_synthetic  # noqa: E402
from FoodRec.utils.utils import get_model, init_seed  # noqa: E402

STEPS = 5
B = 512
dev = torch.device("cuda")
mode = sys.argv[1] if len(sys.argv) > 1 else "dcor"
data = FoodData.from_synthetic(make_synthetic("foodcom", 0, negatives=False))
cfg = Config("PRICAI_ModelX", "Foodcom", {"use_gpu": True, "seed": 999, "cuda_graph": False, "train_batch_size": B,
                                          "ssl_mode": mode, "n_cluster": 2000, "log_root": "/tmp/frlog/",
                                          "ckp_root": "/tmp/frckp/"})
cfg["device"] = dev
init_seed(999)
model = get_model("PRICAI_ModelX")(cfg, data).to(dev)
tr = Trainer(cfg, model)
np.random.seed(2000)
sampler = TripleSampler(data, B, dev, replay_python_random=False)
feats = tr._features()
st = tr.new_step_state()
model.train()
it = sampler.epoch()
for i in range(5):
    u, p, n = next(it)
    tr.train_step(feats.batch(u, p, n), i, st)
torch.cuda.synchronize()
from torch.profiler import ProfilerActivity, profile  # noqa: E402

with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
    for i in range(STEPS):
        u, p, n = next(it)
        tr.train_step(feats.batch(u, p, n), i, st)
    torch.cuda.synchronize()


def site(ev):
    p = ev
    while p is not None:
        if p.name.startswith("autograd::engine::evaluate_function"):
            return p.name.split(": ", 1)[-1]
        p = p.cpu_parent
    for fr in ev.stack or []:
        if "FoodRec" in fr and "profiler" not in fr:
            return fr.split("multi-modal-food-recommendation_amd/")[-1]
    return "?"


agg = defaultdict(lambda: [0, 0.0])
for ev in prof.events():
    if not ev.name.startswith("aten::"):
        continue
    t = ev.self_device_time_total if hasattr(ev, "self_device_time_total") else ev.self_cuda_time_total
    if t <= 0:
        continue
    k = (ev.name, site(ev))
    agg[k][0] += 1
    agg[k][1] += t
rows = sorted(agg.items(), key=lambda kv: -kv[1][1])
tot = sum(v[1] for _, v in rows) / STEPS
print(f"ATen ops with device time: {tot:.1f} us/step")
for (name, where), (c, t) in rows[:70]:
    print(f"{c / STEPS:5.1f}/step {t / STEPS:8.1f} us/step  {name:32s} {where}")
