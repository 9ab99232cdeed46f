"""BASELINE config 4 at its full size on the MI355X: the synthetic 10M users x 1M items x ~200M
interactions graph (nnz = 400M in the symmetric adjacency), d = 64, fp32.

Too large for the oracle to redo whole, so size-independent properties are checked:
  * fr_spmm_csr over the full adjacency on 10,000 rows (the 10 densest item rows, up to ~4e5
    neighbours each, plus 9,990 uniformly drawn rows) against a float64 host restatement of those
    rows: |err| <= 1e-5 * sum_j |a_ij| |x_j| + 1e-7 per element;
  * the row-sharded step (engine/sharded.py, P = 1, every collective forced through RCCL) equals
    the single-GPU LightGCN_ID step on the same tables and global batch: BPR and EmbLoss rel 1e-5,
    gradients 1e-4 * max over all 11M x 64 rows; after one fused-Adam step each, every parameter
    differs by at most 2 lr (Adam's first step is lr * sign(g)) and by more than 1e-6 on at most
    1e-4 of the elements.
"""
import os
import tempfile

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

U, I, D = 10_000_000, 1_000_000, 64


@pytest.fixture(scope="module")
def big(cuda):
    from FoodRec.utils.interaction_graph import InteractionGraph, synth_bipartite
    u, i = synth_bipartite(U, I, 20.0, seed=0, device=cuda)
    g = InteractionGraph(U, I, pairs=(u, i), device=cuda)
    yield u, i, g
    del g
    torch.cuda.empty_cache()


def test_spmm_full_graph_sampled_rows_vs_float64(cuda, big):
    from FoodRec.engine import ops
    _, _, g = big
    adj = g.adj
    assert adj.nnz > 3.9e8 and adj.shape == (U + I, U + I)
    gen = torch.Generator(device=cuda).manual_seed(11)
    X = torch.randn(U + I, D, device=cuda, generator=gen)
    Y = torch.empty_like(X)
    ops.spmm_launch(adj, X, Y1=Y)
    deg = adj.rowptr[1:] - adj.rowptr[:-1]
    heavy = torch.topk(deg, 10).indices
    rnd = torch.randint(0, U + I, (9990,), device=cuda, generator=gen)
    rows = torch.unique(torch.cat([heavy, rnd]))
    starts, ends = adj.rowptr[rows], adj.rowptr[rows + 1]
    lens = (ends - starts).cpu().numpy()
    seg = torch.repeat_interleave(torch.arange(rows.numel(), device=cuda), ends - starts)
    offs = torch.arange(int(lens.sum()), device=cuda) - torch.repeat_interleave(
        torch.cumsum(ends - starts, 0) - (ends - starts), ends - starts)
    pos = torch.repeat_interleave(starts, ends - starts) + offs
    cols = adj.col[pos].long()
    vals = adj.val[pos].double().cpu().numpy()
    xr = X[cols].double().cpu().numpy()
    seg_np = seg.cpu().numpy()
    ref = np.zeros((rows.numel(), D))
    np.add.at(ref, seg_np, vals[:, None] * xr)
    mag = np.zeros((rows.numel(), D))
    np.add.at(mag, seg_np, np.abs(vals)[:, None] * np.abs(xr))
    got = Y[rows].double().cpu().numpy()
    assert int(lens.max()) > 100_000  # the heavy item rows are in the sample
    err = np.abs(got - ref)
    assert np.all(err <= 1e-5 * mag + 1e-7), float((err / (mag + 1e-30)).max())


def test_sharded_p1_equals_single_gpu_step_full_size(cuda, big):
    import torch.distributed as dist
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import sharded
    from FoodRec.engine.sharded import ShardedGraph, ShardedLightGCN
    from FoodRec.models.lightgcn_id import LightGCN_ID
    from FoodRec.utils.configurator import Config
    u, i, g = big
    own_pg = not dist.is_initialized()
    if own_pg:
        store = dist.FileStore(os.path.join(tempfile.mkdtemp(prefix="frpg_"), "store"), 1)
        dist.init_process_group("nccl", store=store, rank=0, world_size=1, device_id=cuda)
    try:
        gs = ShardedGraph(U, I, u, i, 0, 1, cuda)
        assert gs.local_nnz == g.n_edges
        cfg = Config("LightGCN_ID", "Synthetic10M", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                                     "ckp_root": "/tmp/frckp/"})
        cfg["device"] = cuda
        B = 512
        with sharded.collectives_at_world_one():
            mS = ShardedLightGCN(gs, D, 2, 0.1, group=dist.group.WORLD, seed=7)
            ms = LightGCN_ID(cfg, g)
            with torch.no_grad():
                ms.ego.copy_(torch.cat([mS.ego_u, mS.ego_i]))
            a, b, c = gs.triples(B, 5, 0)
            batch = {"u_id": a, "pos_i_id": b, "neg_i_id": c}
            mf1, reg1 = mS.calculate_loss(batch)
            (mf1 + reg1.sum()).backward()
            mf2, reg2 = ms.calculate_loss(batch)
            (mf2 + reg2.sum()).backward()
            for x, y in ((mf1, mf2), (reg1.reshape(-1), reg2.reshape(-1))):
                assert abs(float(x.sum()) - float(y.sum())) <= 1e-5 * abs(float(y.sum())) + 1e-8
            gS = torch.cat([mS.ego_u.grad, mS.ego_i.grad])
            err = (gS - ms.ego.grad).abs().max().item()
            assert err <= 1e-4 * ms.ego.grad.abs().max().item(), err
            del gS
            trS, trs = Trainer(cfg, mS), Trainer(cfg, ms)
            trS.optimizer.step()
            trs.optimizer.step()
            torch.cuda.synchronize()
            lr = float(cfg["learning_rate"])
            diff = (torch.cat([mS.ego_u.detach(), mS.ego_i.detach()]) - ms.ego.detach()).abs()
            assert diff.max().item() <= 2 * lr + 1e-6
            assert (diff > 1e-6).sum().item() <= 1e-4 * diff.numel()
    finally:
        if own_pg:
            dist.destroy_process_group()
