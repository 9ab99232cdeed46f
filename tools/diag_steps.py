"""Diagnostic: tiny HealthRec (the training-parity test's model), parameters after each of the
first training steps, saved to an npz for comparing two engine builds (FR_ENGINE_LIB)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT, os.path.join(ROOT, "tests")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from helpers import tiny_config, tiny_data  # noqa: E402


def main(out_path, n_steps=3):
    from FoodRec.common.trainer import Trainer
    from FoodRec.utils.utils import get_model, init_seed
    cfg = tiny_config("CIKM_Model", True)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("CIKM_Model")(cfg, data).to(torch.device("cuda:0"))
    tr = Trainer(cfg, model)
    snaps = {}
    real_step = tr.optimizer.step
    k = [0]

    def step(*a, **kw):
        if k[0] == 0:
            for name, p in model.named_parameters():
                if p.grad is not None:
                    snaps[f"g0/{name}"] = p.grad.detach().float().cpu().numpy()
        r = real_step(*a, **kw)
        if k[0] < n_steps:
            if hasattr(tr.optimizer, "flush_rows"):
                pass
            for name, p in model.named_parameters():
                snaps[f"s{k[0]}/{name}"] = p.detach().float().cpu().numpy()
        k[0] += 1
        return r
    tr.optimizer.step = step
    cfg["epochs"] = 1
    tr.fit(data, hyper_tuple=(999,), saved=False, verbose=False)
    np.savez(out_path, **snaps)
    print("steps", k[0], "saved", len(snaps))


if __name__ == "__main__":
    main(sys.argv[1])
