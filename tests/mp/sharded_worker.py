"""Rank worker of tests/test_multirank_gpu.py: the row-sharded config-4 step (engine/sharded.py) with
world_size ranks on ONE GPU (gloo over device tensors; RCCL refuses two ranks on one device, the
8-GPU RCCL run is the driver's).  Launched by the test as

  python -m torch.distributed.run --nnodes=1 --nproc-per-node {2,4} --master-addr 127.0.0.1 \
      --master-port P tests/mp/sharded_worker.py

The step must run the rows form (_ShardedRowsStep: item-flag all-reduce, the |S| layer-1 rows,
the 2B batch item rows, the item-row blocks of the last backward layer) -- counted below.

Every rank compares, on a 20k-user graph:
  * the sharded step (P ranks) with the same step unsharded (P=1, no collectives) and with the
    single-GPU LightGCN_ID model on the same tables/batch: losses rel 1e-5, gradients 1e-4 * max;
  * after 3 FusedAdam steps, the replicated item tables bit-identical across ranks.
Exit status 0 = pass.
"""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import sharded
    from FoodRec.engine.sharded import ShardedGraph, ShardedLightGCN
    rows_calls = [0]
    _apply = sharded._ShardedRowsStep.apply

    def counted(*a):
        rows_calls[0] += 1
        return _apply(*a)

    sharded._ShardedRowsStep.apply = staticmethod(counted)
    from FoodRec.models.lightgcn_id import LightGCN_ID
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.interaction_graph import InteractionGraph, synth_bipartite
    U, I, d, B = 20000, 3000, 64, 512
    u, i = synth_bipartite(U, I, 10.0, seed=3, device=dev)
    gP = ShardedGraph(U, I, u, i, rank, world, dev, chunk=64)
    g1 = ShardedGraph(U, I, u, i, 0, 1, dev, chunk=64)
    mP = ShardedLightGCN(gP, d, 2, 0.1, group=dist.group.WORLD, seed=7)
    m1 = ShardedLightGCN(g1, d, 2, 0.1, group=None, seed=7)
    uu, pp, nn_ = gP.triples(B, 5, 0)
    batch = {"u_id": uu, "pos_i_id": pp, "neg_i_id": nn_}
    fails = []

    def close(name, a, b, rel):
        err = (a - b).abs().max().item()
        ref = b.abs().max().item()
        if not err <= rel * ref + 1e-7:
            fails.append(f"{name}: max err {err:.3e} vs {rel:.0e} * {ref:.3e}")

    mfP, regP = mP.calculate_loss(batch)
    (mfP + regP.sum()).backward()
    mf1, reg1 = m1.calculate_loss(batch)
    (mf1 + reg1.sum()).backward()
    close("mf P vs 1", mfP.detach(), mf1.detach(), 1e-5)
    close("reg P vs 1", regP.detach(), reg1.detach(), 1e-5)
    close("item grad P vs 1", mP.ego_i.grad, m1.ego_i.grad, 1e-4)
    close("user grad P vs 1", mP.ego_u.grad, m1.ego_u.grad[gP.lo:gP.hi], 1e-4)
    # the single-GPU model on the same tables and batch
    g = InteractionGraph(U, I, pairs=(u, i), device=dev, chunk=64)
    cfg = Config("LightGCN_ID", "Synthetic", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                              "ckp_root": "/tmp/frckp/"})
    cfg["device"] = dev
    ms = LightGCN_ID(cfg, g)
    with torch.no_grad():
        ms.ego.copy_(torch.cat([m1.ego_u, m1.ego_i]))
    mfS, regS = ms.calculate_loss(batch)
    (mfS + regS.sum()).backward()
    close("mf single-GPU model vs P=1", mf1.detach(), mfS.detach(), 1e-5)
    close("reg single-GPU model vs P=1", reg1.detach().reshape(-1), regS.detach().reshape(-1), 1e-5)
    close("grad single-GPU model vs P=1", torch.cat([m1.ego_u.grad, m1.ego_i.grad]), ms.ego.grad, 1e-4)
    # optimiser steps keep the replicated item tables identical
    mP.zero_grad(set_to_none=True)
    trainer = Trainer(cfg, mP)
    state = trainer.new_step_state()
    for k in range(3):
        a, b, c = gP.triples(B, 5, 1 + k)
        trainer.train_step({"u_id": a, "pos_i_id": b, "neg_i_id": c}, k, state)
    items = [torch.empty_like(mP.ego_i) for _ in range(world)]
    dist.all_gather(items, mP.ego_i.detach().contiguous())
    if not all(torch.equal(items[0], x) for x in items):
        fails.append("replicated item tables diverged across ranks after 3 Adam steps")
    if rows_calls[0] < 4:  # 1 loss + 3 training steps of the sharded model
        fails.append(f"rows form ran {rows_calls[0]} times (expected >= 4)")
    if len(gP.iu_blocks) < 2:
        fails.append("transpose slice not cut into item-row blocks")
    torch.cuda.synchronize()
    print(f"[rank {rank}/{world}] users [{gP.lo},{gP.hi}) nnz {gP.local_nnz}: "
          + ("PASS" if not fails else "FAIL " + "; ".join(fails)), flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
