"""SpMM work-unit size (chunk) sweep on the Allrecipes-shape graphs HealthRec propagates over
(UI: 114k nodes / 1.35M nnz, RI: 65.6k nodes / 0.79M nnz), d=64 fp32: per-launch HIP-event time
of fr_spmm_csr for each chunk, one JSON line."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multi-modal-food-recommendation_amd"))

import torch  # noqa: E402


def main():
    from FoodRec.engine import ops
    from FoodRec.models._graphs import side_adjacency, ui_adjacency
    from FoodRec.utils.dataset import FoodData
    from FoodRec.utils.synthetic import make_synthetic
    dev = torch.device("cuda:0")
    data = FoodData.from_synthetic(make_synthetic("allrecipes", 0, negatives=False))
    out = {}
    for name, make in (("ui", lambda c: ui_adjacency(data, data.n_users, data.n_items, dev, chunk=c)),
                       ("ri", lambda c: side_adjacency(data.rIngre_triples, data.n_items, data.num_ingredients, dev,
                                                      chunk=c))):
        res = {}
        for chunk in (16, 32, 64, 128, 256, 1024):
            adj = make(chunk)
            X = torch.randn(adj.shape[0], 64, device=dev)
            Y = torch.empty_like(X)
            for _ in range(3):
                ops.spmm_launch(adj, X, Y1=Y)
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            s.record()
            for _ in range(20):
                ops.spmm_launch(adj, X, Y1=Y)
            e.record()
            torch.cuda.synchronize()
            res[chunk] = round(s.elapsed_time(e) / 20 * 1e3, 1)
        out[name] = {"nnz": adj.nnz, "max_row_nnz": adj.max_row_nnz, "us_per_launch_by_chunk": res}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
