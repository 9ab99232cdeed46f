"""Config-4 step alone (for rocprofv3 --kernel-trace --stats): the single-GPU LightGCN_ID step or the
row-sharded step at P = 1 (engine/sharded.py), on the 10M x 1M x 200M synthetic graph.

  python tools/profile_c4.py --mode single|sharded --batch 8192 --steps 3

Prints one JSON line with the per-step wall time (after --warmup untimed steps)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["single", "sharded"], default="sharded")
    ap.add_argument("--batch", type=int, default=8192)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    from FoodRec.common.trainer import Trainer
    from FoodRec.utils.configurator import Config
    dev = torch.device("cuda:0")
    U, I, d = 10_000_000, 1_000_000, 64
    cfg = Config("LightGCN_ID", "Synthetic10M", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                                 "ckp_root": "/tmp/frckp/"})
    cfg["device"] = dev
    if args.mode == "single":
        from FoodRec.models.lightgcn_id import LightGCN_ID
        from FoodRec.utils.interaction_graph import InteractionGraph
        g = InteractionGraph(U, I, 20.0, seed=0, device=dev)
        torch.manual_seed(999)
        model = LightGCN_ID(cfg, g)

        def batch(k):
            u, p, n = g.triples(args.batch)
            return {"u_id": u, "pos_i_id": p, "neg_i_id": n}
    else:
        from FoodRec.engine.sharded import ShardedGraph, ShardedLightGCN
        from FoodRec.utils.interaction_graph import synth_bipartite
        u, i = synth_bipartite(U, I, 20.0, seed=0, device=dev)
        g = ShardedGraph(U, I, u, i, 0, 1, dev)
        del u, i
        model = ShardedLightGCN(g, d, 2, 0.1, group=None, seed=999)

        def batch(k):
            uu, pp, nn_ = g.triples(args.batch, 999, k)
            return {"u_id": uu, "pos_i_id": pp, "neg_i_id": nn_}
    tr = Trainer(cfg, model)
    state = tr.new_step_state()
    for k in range(args.warmup):
        tr.train_step(batch(k), k, state)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        tr.train_step(batch(args.warmup + k), args.warmup + k, state)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    print(json.dumps({"mode": args.mode, "batch": args.batch, "ms_per_step": round(dt * 1e3, 3)}), flush=True)


if __name__ == "__main__":
    main()
