"""Diagnose: step-0 gradient errors vs the reference at Allrecipes width (per parameter)."""
import os
import sys
R = os.path.join(os.path.dirname(__file__), "..", "..")
sys.path[:0] = [os.path.join(R, "tests"), os.path.join(R, "multi-modal-food-recommendation_amd"), R]
import numpy as np
import torch
import test_wide_gpu as W

cuda = torch.device("cuda:0")
for name in sys.argv[1:] or ("CIKM_Model", "PRICAI_ModelX"):
    g, cfg, model, tr, sampler = W._setup(cuda, name, graph=False)
    feats = tr._features()
    model.train()
    u, p, n = next(sampler.epoch())
    batch = feats.batch(u, p, n)
    tr.optimizer.zero_grad()
    losses = model.calculate_loss(batch)
    print(name, "loss", [float(x) for x in losses], g["step0/loss"].tolist())
    sum(losses).backward()
    tr.optimizer.materialize_row_grads()
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(f"gpurun_out/wide_grads_gpu_{name}.npz", **{
        k: W._rows(g, k, prm.grad).cpu().numpy() for k, prm in model.named_parameters() if prm.grad is not None})
    for pre in ("grad0/", "grad0_f64/"):
        print(" vs", pre)
        for k, prm in model.named_parameters():
            if pre + k not in g.files:
                continue
            ref = g[pre + k].astype(np.float64)
            got = W._rows(g, k, prm.grad).cpu().numpy().astype(np.float64)
            d = np.abs(got - ref)
            i = np.unravel_index(np.argmax(d), d.shape)
            print(f"  {k:55s} max_err/max={d.max() / max(np.abs(ref).max(), 1e-30):.2e} "
                  f"norm_rel={np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-30):.2e} at {i} ref={ref[i]:.4e}")
