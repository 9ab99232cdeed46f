"""Row-sharded config-4 step (engine/sharded.py) on CPU: gloo, world_size 1 and 2,
engine ops through the oracle CPU backend.  Checks against the oracle's single-process LightGCN
arithmetic (models/lightgcn.py:134-177, common/loss.py) on the same graph, batch and initial tables:

* every rank reports the same BPR and EmbLoss values as the oracle (rel 1e-5);
* the replicated item-table gradient is bit-identical on all ranks and matches the oracle's;
* rank r's user-row gradient matches the oracle's rows [lo_r, hi_r);
* the partition covers all users with nnz-balanced contiguous blocks.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

U, I, D, L, B, SEED = 300, 120, 16, 2, 64, 5


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    rng = np.random.default_rng(0)
    deg = rng.poisson(6, U) + 1
    u = np.repeat(np.arange(U), deg)
    i = (rng.zipf(1.6, u.size) - 1) % I
    batch = rng.integers(0, u.size, B)
    bu, bp = u[batch], i[batch]
    bn = rng.integers(0, I, B)
    return u, i, bu, bp, bn


def _worker(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import cpu_backend
    from FoodRec.engine.sharded import ShardedGraph, ShardedLightGCN
    u, i, bu, bp, bn = _data()
    with cpu_backend.installed():
        g = ShardedGraph(U, I, u, i, rank, world, "cpu", chunk=8)
        m = ShardedLightGCN(g, d=D, n_layers=L, reg_weight=0.1, group=dist.group.WORLD, seed=SEED)
        batch = {"u_id": torch.as_tensor(bu), "pos_i_id": torch.as_tensor(bp), "neg_i_id": torch.as_tensor(bn)}
        mf, reg = m.calculate_loss(batch)
        (mf + reg.sum()).backward()
    torch.save({"mf": mf.detach(), "reg": reg.detach(), "gu": m.ego_u.grad, "gi": m.ego_i.grad,
                "lo": g.lo, "hi": g.hi, "bounds": g.bounds, "nnz": g.local_nnz},
               os.path.join(out_dir, f"r{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def _oracle():
    import math
    from oracle import ops as O
    u, i, bu, bp, bn = _data()
    gen = torch.Generator().manual_seed(SEED)
    full_u = torch.empty(U, D).uniform_(-math.sqrt(6.0 / (U + D)), math.sqrt(6.0 / (U + D)), generator=gen)
    ego_i = torch.empty(I, D).uniform_(-math.sqrt(6.0 / (I + D)), math.sqrt(6.0 / (I + D)), generator=gen)
    r, c, v = O.norm_adj_coo(U + I, u, i + U)
    A = O.coo_to_torch(U + I, r, c, v)
    E = torch.cat([full_u, ego_i]).requires_grad_(True)
    out = O.propagate_mean(A, E, L)
    bu, bp, bn = (torch.as_tensor(x) for x in (bu, bp, bn))
    mf = O.bpr_loss((out[bu] * out[bp + U]).sum(1), (out[bu] * out[bn + U]).sum(1))
    reg = 0.1 * O.emb_loss(E[bu], E[bp + U], E[bn + U])
    (mf + reg.sum()).backward()
    return mf.detach(), reg.detach(), E.grad


@pytest.mark.parametrize("world", [1, 2])
def test_sharded_step_matches_oracle_gloo(tmp_path, world):
    mp.start_processes(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    mf_r, reg_r, grad_r = _oracle()
    res = [torch.load(tmp_path / f"r{r}.pt", weights_only=True) for r in range(world)]
    assert res[0]["bounds"][0] == 0 and res[0]["bounds"][-1] == U
    u, i, *_ = _data()
    assert sum(x["nnz"] for x in res) == np.unique(u * I + i).size  # every interaction on exactly one rank
    for x in res:
        torch.testing.assert_close(x["mf"], mf_r, rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(x["reg"].reshape(-1), reg_r.reshape(-1), rtol=1e-5, atol=1e-7)
        torch.testing.assert_close(x["gu"], grad_r[x["lo"]:x["hi"]], rtol=1e-4, atol=1e-6)
        torch.testing.assert_close(x["gi"], grad_r[U:], rtol=1e-4, atol=1e-6)
        assert torch.equal(x["gi"], res[0]["gi"]), "replicated item gradient must agree bit for bit"
    if world > 1:
        nnz = [x["nnz"] for x in res]
        assert min(nnz) > 0.5 * max(nnz), f"partition not nnz-balanced: {nnz}"


def _worker_train(rank, world, port, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import cpu_backend
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine.sharded import ShardedGraph, ShardedLightGCN
    from FoodRec.utils.configurator import Config
    u, i, *_ = _data()
    with cpu_backend.installed():
        g = ShardedGraph(U, I, u, i, rank, world, "cpu", chunk=8)
        cfg = Config("LightGCN_ID", "Synthetic", {"use_gpu": False, "seed": 999, "log_root": str(out_dir) + "/",
                                                  "ckp_root": str(out_dir) + "/"})
        cfg["device"] = torch.device("cpu")
        m = ShardedLightGCN(g, d=D, n_layers=L, reg_weight=0.1, group=dist.group.WORLD, seed=SEED)
        trainer = Trainer(cfg, m)
        state = trainer.new_step_state()
        trip = []
        for k in range(3):
            bu, bp, bn = g.triples(B, 11, k)
            trip.append(torch.stack([bu, bp, bn]))
            trainer.train_step({"u_id": bu, "pos_i_id": bp, "neg_i_id": bn}, k, state)
    torch.save({"trip": torch.stack(trip), "ego_i": m.ego_i.detach(), "acc": state["acc"],
                "keys": g.keys}, os.path.join(out_dir, f"t{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_sampler_and_trainer_steps_gloo(tmp_path):
    world = 2
    mp.start_processes(_worker_train, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    res = [torch.load(tmp_path / f"t{r}.pt", weights_only=True) for r in range(world)]
    assert torch.equal(res[0]["trip"], res[1]["trip"]), "every rank must draw the same global batch"
    keys = set(res[0]["keys"].tolist())
    for step in res[0]["trip"]:
        bu, bp, bn = step.tolist()
        assert all(a * I + b in keys for a, b in zip(bu, bp))
        assert not any(a * I + c in keys for a, c in zip(bu, bn))
    assert torch.equal(res[0]["ego_i"], res[1]["ego_i"]), "replicated item tables must stay identical"
    assert torch.equal(res[0]["acc"], res[1]["acc"]) and torch.isfinite(res[0]["acc"]).all()
