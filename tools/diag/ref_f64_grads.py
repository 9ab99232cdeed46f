"""Diagnose (build container only; reads /root/reference): the reference's HealthRec step-0
gradients at the Allrecipes width in float64, vs its float32 golden (tests/golden) and the GPU's
(gpurun_out/wide_grads_gpu_CIKM_Model.npz from tools/diag/wide_grads.py)."""
import os
import sys
import tempfile

import numpy as np

R = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(R, "oracle"))
import gen_golden as G  # noqa: E402

make_synthetic, write_reference_format = G._setup_reference()
import torch  # noqa: E402
from FoodRec.utils.configurator import Config  # noqa: E402
from FoodRec.utils.dataset import FoodData  # noqa: E402
from FoodRec.utils.utils import init_seed, get_model  # noqa: E402
from FoodRec.utils.dataloader import TrainDataLoader  # noqa: E402
from torch.utils.data import RandomSampler, DataLoader  # noqa: E402

torch.set_num_threads(8)
name = "CIKM_Model"
shape, dsname, steps, extra = G.WIDE[name]
ds = make_synthetic(shape, 0, negatives=False)
ds.valid_neg = np.zeros((len(ds.valid_users), 1), np.int64)
ds.test_neg = np.zeros((ds.n_users, 1), np.int64)
root = tempfile.mkdtemp(prefix="frdiag_")
write_reference_format(ds, root + "/", dsname)
cd = {"data_path": root + "/", "log_root": root + "/log/", "ckp_root": root + "/ckp/", "use_gpu": False,
      "seed": 999, "n_cluster": ds.n_cluster, **extra}
cfg = Config(name, dsname, cd)
pp = root + f"/{dsname}/processed_dataset/"
cfg["interaction_data_path"], cfg["graph_data_path"], cfg["ingre_data_path"] = pp, pp + "graph_edge/", pp
data = FoodData(cfg)
init_seed(999)
model = get_model(name)(cfg, data)
pre = TrainDataLoader(cfg, data, use_neg_list=False)
TrainDataLoader(cfg, data, use_neg_list=True)
batch = next(iter(DataLoader(pre, sampler=RandomSampler(pre), batch_size=cfg["train_batch_size"])))
g = np.load(os.path.join(R, "tests/golden/wide_CIKM_Model_allrecipes.npz"))
assert np.array_equal(batch["u_id"].numpy(), g["step0/u_id"])
model = model.double()
for k, v in list(vars(model).items()):
    if torch.is_tensor(v) and v.is_floating_point():
        setattr(model, k, v.double())
batch = {k: (v.double() if v.is_floating_point() else v) for k, v in batch.items()}
model.train()
losses = model.calculate_loss(batch)
print("f64 loss", [float(x) for x in losses], "f32 golden", g["step0/loss"].tolist())
sum(losses).backward()
gpu = np.load(os.path.join(R, "gpurun_out/wide_grads_gpu_CIKM_Model.npz"))
for k, p in model.named_parameters():
    if p.grad is None or "grad0/" + k not in g.files:
        continue
    gr = p.grad
    if "rows/" + k in g.files:
        gr = gr[torch.from_numpy(g["rows/" + k])]
    f64 = gr.numpy()
    ref32, ours = g["grad0/" + k].astype(np.float64), gpu[k].astype(np.float64)
    n = np.linalg.norm(f64) + 1e-300
    print(f"{k:55s} cpu32-vs-f64 {np.linalg.norm(ref32 - f64) / n:.2e}  gpu-vs-f64 {np.linalg.norm(ours - f64) / n:.2e}")
