"""Rank worker of tests/test_multirank_gpu.py: HealthRec data parallelism with the row-exchanged
feature-table gradients (ops._EmbeddingExchanged + engine.dist.GradAllReduce) and the graphed
data-parallel step (engine.dist.GraphedDPStep), world_size ranks on ONE GPU (gloo over device
tensors).  Launched by the test as

  python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port P tests/mp/dp_worker.py

Each rank trains its own batch.  Reference: the same step with every gradient all-reduced densely
and averaged.  Checks: exchanged image/text table gradients equal the dense mean (|err| <= 1e-6 *
max) and are bit-identical across ranks; all other gradients equal the reference bit for bit.
"""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(ROOT, "multi-modal-food-recommendation_amd"), ROOT]


def build(dev):
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.dataset import FoodData
    from FoodRec.utils.synthetic import make_synthetic
    from FoodRec.utils.utils import get_model, init_seed
    data = FoodData.from_synthetic(make_synthetic("tiny", 0))
    cfg = Config("CIKM_Model", "Tiny", {"use_gpu": True, "seed": 999, "attention_probs_dropout_prob": 0.0,
                                        "log_root": "/tmp/frlog/", "ckp_root": "/tmp/frckp/"})
    cfg["device"] = dev
    data.args_config = cfg
    init_seed(999)
    return cfg, data, get_model("CIKM_Model")(cfg, data).to(dev)


def main():
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine.dist import GradAllReduce
    from FoodRec.engine.sampler import TripleSampler
    cfg, data, mx = build(dev)
    _, _, mr = build(dev)
    np.random.seed(1000 + rank)
    sampler = TripleSampler(data, 256, dev, replay_python_random=False)
    u, p, n = next(iter(sampler.epoch()))
    fails = []
    # exchanged
    tx = Trainer(cfg, mx)
    hook = GradAllReduce(mx, world)
    batch = tx._features().batch(u, p, n)
    sum(mx.calculate_loss(batch)).backward()
    hook(mx)
    # dense reference
    tr = Trainer(cfg, mr)
    sum(mr.calculate_loss(tr._features().batch(u, p, n))).backward()
    tr.optimizer.materialize_row_grads()  # dense .grad of the row-gathered tables
    for prm in mr.parameters():
        if prm.grad is not None:
            dist.all_reduce(prm.grad)
            prm.grad.mul_(1.0 / world)
    sparse = {id(t) for t in mx.row_sparse_tables()}
    for (name, a), (_, b) in zip(mx.named_parameters(), mr.named_parameters()):
        if a.grad is None or b.grad is None:
            if (a.grad is None) != (b.grad is None):
                fails.append(f"{name}: gradient presence differs")
            continue
        if id(a) in sparse:
            err = (a.grad - b.grad).abs().max().item()
            if err > 1e-6 * b.grad.abs().max().item() + 1e-9:
                fails.append(f"{name}: exchanged gradient err {err:.3e}")
            allg = [torch.empty_like(a.grad) for _ in range(world)]
            dist.all_gather(allg, a.grad.contiguous())
            if not all(torch.equal(allg[0], x) for x in allg):
                fails.append(f"{name}: exchanged gradient differs across ranks")
        elif not torch.equal(a.grad, b.grad):
            err = (a.grad - b.grad).abs().max().item()
            if err > 1e-6 * b.grad.abs().max().item() + 1e-9:
                fails.append(f"{name}: dense gradient err {err:.3e}")
    # graphed data-parallel steps (GraphedDPStep) == eager data-parallel steps
    _, _, mg = build(dev)
    _, _, me = build(dev)
    tg, te = Trainer(cfg, mg), Trainer(cfg, me)
    tg.grad_hook, te.grad_hook = GradAllReduce(mg, world), GradAllReduce(me, world)
    graphed = tg.graphed_step(256, warmup=2)
    from FoodRec.common.trainer import GraphedDPStep
    if not isinstance(graphed, GraphedDPStep):
        fails.append(f"graphed_step returned {type(graphed).__name__}, not GraphedDPStep")
    sg, se = tg.new_step_state(), te.new_step_state()
    def cycle():
        while True:
            yield from sampler.epoch()

    it = cycle()
    # per step, at identical parameters: losses and every gradient agree (fp32 reduction order).
    # Parameters are re-synchronised before each step because Adam turns the ~1e-9 gradient noise
    # of zero-gradient parameters (the key part of in_proj_bias) into +-lr updates in any mode.
    for k in range(5):
        bu, bp, bn = next(it)
        tg.flush_optimizer()  # lazy row Adam: every deferred row step applied before comparing/copying
        te.flush_optimizer()
        with torch.no_grad():  # same parameters in both modes (graphs read parameter memory)
            for a, b in zip(mg.parameters(), me.parameters()):
                a.copy_(b)
        before_g, before_e = sg["acc"].clone() if sg["acc"] is not None else 0, \
            se["acc"].clone() if se["acc"] is not None else 0
        graphed(bu, bp, bn, k, sg)
        te.train_step(te._features().batch(bu, bp, bn), k, se)
        dl_g, dl_e = sg["acc"] - before_g, se["acc"] - before_e
        if not torch.allclose(dl_g, dl_e, rtol=1e-4, atol=1e-7):
            fails.append(f"step {k}: losses {dl_g.tolist()} vs {dl_e.tolist()}")
        for (name, a), (_, b) in zip(mg.named_parameters(), me.named_parameters()):
            if (a.grad is None) != (b.grad is None):
                fails.append(f"step {k}: {name} gradient presence differs")
            elif a.grad is not None:
                err = (a.grad - b.grad).abs().max().item()
                if err > 1e-3 * b.grad.abs().max().item() + 1e-6:
                    fails.append(f"step {k}: graphed vs eager gradient {name} err {err:.3e}")
    torch.cuda.synchronize()
    print(f"[rank {rank}/{world}] exchanged tables {len(sparse)}, flat all-reduce params "
          f"{sum(x.numel() for x in hook.params)}: " + ("PASS" if not fails else "FAIL " + "; ".join(fails)),
          flush=True)
    dist.barrier()
    dist.destroy_process_group()
    sys.exit(1 if fails else 0)


if __name__ == "__main__":
    main()
