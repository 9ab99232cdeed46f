"""BASELINE config 5 at its full size on the GPU: the synthetic 10M users x 1M items x ~200M
interactions graph with d = 256 bf16 tables (the bench's config5 leg), checked by properties a
float64 host restatement can afford at this size.

* bf16 SpMM (fr_spmm_csr_bf16) on 10,000 sampled rows (8,000 uniform, 2,000 item rows: Zipf-heavy,
  split into chunks) vs the float64 sum of their edges on the host: the small-graph tolerance of
  tests/test_config5_gpu.py (one bf16 output rounding + fp32 accumulation order);
* one bf16 training step (LightGCN_ID, BPR + EmbLoss, mixed-precision Adam): finite losses, no NaN
  flag, the batch users' rows moved (lightgcn.py:134-177 + common/loss.py + torch.optim.Adam);
* full_sort_topk for 64 users over all 1,000,000 items (training items masked) vs a float64 host
  recompute of those users' scores: the check of test_config5_gpu._check_topk (returned scores
  within 1e-5 * max sum|u_k i_k| of float64, the k-th score too, every item clearing it returned,
  no training item returned).  The reference contract: common/abstract_recommender.py:39-50.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

U, I, D = 10_000_000, 1_000_000, 256


@pytest.fixture(scope="module")
def graph(cuda):
    from FoodRec.utils.interaction_graph import InteractionGraph
    g = InteractionGraph(U, I, 20.0, seed=0, device=cuda)
    yield g
    del g
    torch.cuda.empty_cache()


def _edges(adj, rows):
    rp = adj.rowptr
    s, e = rp[rows], rp[rows + 1]
    lens = e - s
    total = int(lens.sum().item())
    first = torch.cumsum(lens, 0) - lens
    pos = torch.repeat_interleave(s - first, lens) + torch.arange(total, device=rows.device)
    return lens, adj.col[pos].long(), adj.val[pos]


def test_spmm_bf16_sampled_rows_vs_float64(cuda, graph):
    from FoodRec.engine import ops
    adj = graph.adj
    gen = torch.Generator(device=cuda).manual_seed(3)
    X = torch.randn(U + I, D, device=cuda, generator=gen).to(torch.bfloat16)
    Y = ops.spmm(adj, X)
    assert Y.dtype == torch.bfloat16
    rows = torch.randint(0, U + I, (10_000,), device=cuda, generator=gen)
    rows[:2000] = U + torch.randint(0, I, (2000,), device=cuda, generator=gen)
    got = Y[rows].double().cpu().numpy()
    lens, cols, vals = _edges(adj, rows)
    seg = np.concatenate([[0], np.cumsum(lens.cpu().numpy())])
    ref = np.zeros((rows.numel(), D))
    scale = np.zeros((rows.numel(), D))
    vals_h = vals.double().cpu().numpy()
    for r0 in range(0, rows.numel(), 500):  # 500 rows (their edges are contiguous) per host chunk
        r1 = min(r0 + 500, rows.numel())
        a, b = seg[r0], seg[r1]
        xs = X[cols[a:b]].double().cpu().numpy()
        w = vals_h[a:b, None]
        starts = seg[r0:r1] - a
        nz = np.diff(seg[r0:r1 + 1]) > 0  # reduceat of an empty segment returns the next element
        ref[r0:r1][nz] = np.add.reduceat(w * xs, starts[nz], axis=0)
        scale[r0:r1][nz] = np.add.reduceat(np.abs(w) * np.abs(xs), starts[nz], axis=0)
    assert int(lens.max()) > 1024  # heavy item rows (split into chunks) are among the samples
    assert np.all(np.abs(got - ref) <= 2.0 ** -8 * np.abs(ref) + 2e-5 * scale + 1e-6)


def test_bf16_step_and_full_sort_topk(cuda, graph):
    from test_config5_gpu import _check_topk

    from FoodRec.common.trainer import Trainer
    from FoodRec.models.lightgcn_id import LightGCN_ID
    from FoodRec.utils.configurator import Config
    cfg = Config("LightGCN_ID", "Synthetic10M", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                                 "ckp_root": "/tmp/frckp/", "embedding_size": D,
                                                 "embedding_dtype": "bf16"})
    cfg["device"] = cuda
    torch.manual_seed(999)
    model = LightGCN_ID(cfg, graph)
    assert model.ego.dtype == torch.bfloat16 and model.ego.shape == (U + I, D)
    tr = Trainer(cfg, model)
    st = tr.new_step_state()
    u, p, n = graph.triples(512)
    before = model.ego.detach()[u].clone()
    loss = tr.train_step({"u_id": u, "pos_i_id": p, "neg_i_id": n}, 0, st)
    torch.cuda.synchronize()
    assert not int(st["nan"].item())
    assert torch.isfinite(st["acc"]).all() and (loss is None or torch.isfinite(loss).all())
    moved = (model.ego.detach()[u] != before).any(dim=1)
    assert bool(moved.all())
    # full-sort top-k of 64 users over all items, training items masked
    with torch.no_grad():
        tables = model.forward()
        users = torch.randint(0, U, (64,), device=cuda, generator=torch.Generator(device=cuda).manual_seed(11))
        s, i, _ = model.full_sort_topk(users, 20, tables=tables)
    Uh = tables[0][users].float().cpu().numpy()
    Ih = tables[1].float().cpu().numpy()
    rp = graph.adj.rowptr.cpu().numpy()
    col = graph.adj.col
    excl = []
    for uu in users.cpu().numpy().tolist():
        c = col[rp[uu]:rp[uu + 1]].cpu().numpy().astype(np.int64)
        excl.append((c[c >= U] - U).tolist())
    assert sum(len(x) for x in excl) > 0
    _check_topk(s.float().cpu().numpy(), i.cpu().numpy(), Uh, Ih, 20, excl, 1e-5)
