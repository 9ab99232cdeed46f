"""fr_rank_metrics (the evaluation ranking on the device) vs the reference's per-user numpy loop
(metrics_by_user / get_auc_fast over np.argsort(pred)[::-1], /root/reference/FoodRec/common/
trainer.py:49-69, 231-282).

Bar: bit-equal metrics.  The kernel's hit masks and AUC counts are exact for users whose 21 largest
scores are strictly decreasing; users with ties there (numpy's introsort tie order decides their
ranking) or with a NaN are flagged and re-ranked by the host path, so every user's metrics equal the
reference's: on the reference's own metrics golden (tests/golden/metrics.npz), on random lists with
injected ties and long lists (> 2,048 candidates, host path), and through Trainer._valid_by_user_epoch
at Allrecipes' test-user count (68,768 users x ~500 candidates).
"""
import time

import numpy as np
import pytest
import torch

from helpers import golden

pytestmark = pytest.mark.gpu


def _ref(scores, npos, neg_num=500):
    from FoodRec.common.trainer import rank_user_host
    return np.stack([rank_user_host(pr.copy(), int(n), neg_num) for pr, n in zip(scores, npos)])


def _device(cuda, scores, npos, neg_num=500):
    from FoodRec.common.trainer import metrics_from_hits, rank_user_host
    from FoodRec.engine import ops
    lens = np.array([len(x) for x in scores], np.int64)
    flat = torch.from_numpy(np.concatenate(scores).astype(np.float32)).to(cuda)
    hits, auc, flags = ops.rank_metrics(flat, lens, npos, 20)
    res = metrics_from_hits(hits, lens, npos, auc, neg_num)
    for k in np.nonzero(flags)[0].tolist():
        res[k] = rank_user_host(scores[k].copy(), int(npos[k]), neg_num)
    return res, hits, auc, flags


def test_rank_metrics_on_reference_golden(cuda):
    g = golden("metrics.npz")
    n = len([k for k in g.files if k.endswith("/pred")])
    scores = [g[f"u{u}/pred"].astype(np.float32) for u in range(n)]
    npos = np.array([int(g[f"u{u}/npos"]) for u in range(n)])
    res, _, _, flags = _device(cuda, scores, npos, neg_num=30)  # the golden's get_auc_fast(..., 30)
    for u in range(n):
        np.testing.assert_array_equal(res[u, 0], g[f"u{u}/recall"])
        np.testing.assert_array_equal(res[u, 1], g[f"u{u}/ndcg"])
        assert res[u, 2, 0] == float(g[f"u{u}/auc"])


def test_rank_metrics_random_ties_long_lists(cuda):
    rng = np.random.default_rng(5)
    U = 3000
    lens = rng.integers(1, 700, U)
    lens[:5] = [1, 2, 20, 21, 2049]  # tiny lists and one beyond the register capacity (host path)
    npos = np.minimum(rng.integers(1, 12, U), lens)
    scores = [rng.standard_normal(n).astype(np.float32) for n in lens]
    tie_users = rng.choice(np.arange(5, U), 200, replace=False)
    for u in tie_users:  # duplicate the max into another candidate (a tie at rank 0/1)
        pr = scores[u]
        if len(pr) > 1:
            pr[rng.integers(0, len(pr))] = pr.max()
    coarse = rng.choice(np.arange(5, U), 200, replace=False)
    for u in coarse:  # coarse scores: ties below the top 21 only matter for AUC (exact anyway)
        scores[u] = np.round(scores[u] * 2) / 2
    scores[7][3] = np.nan
    res, hits, auc, flags = _device(cuda, scores, npos)
    ref = _ref(scores, npos)
    bad = [u for u in range(U) if not np.array_equal(res[u], ref[u], equal_nan=True)]
    assert not bad, [(u, int(flags[u]), int(lens[u]), int(npos[u]), hex(int(hits[u])), int(auc[u]),
                      res[u].tolist(), ref[u].tolist()) for u in bad[:4]]
    assert flags[4] == 2 and flags[7] == 1
    # exact users: the kernel's own masks and counts equal numpy's
    for u in np.nonzero(flags == 0)[0][:500].tolist():
        order = np.argsort(scores[u])[::-1][:20]
        assert hits[u] == sum(1 << t for t, d in enumerate(order) if d < npos[u])
        assert auc[u] == sum(int(np.sum(scores[u][npos[u]:] < scores[u][p])) for p in range(npos[u]))
    assert (flags == 1).sum() >= 150  # the injected max ties are caught


def test_rank_metrics_allrecipes_scale_timing(cuda):
    """68,768 users x (3 positives + 500 negatives): device ranking vs the reference-style host loop on
    the same scores (equal metrics); the timings are printed for DESIGN.md."""
    from FoodRec.common.trainer import metrics_from_hits
    from FoodRec.engine import ops
    rng = np.random.default_rng(0)
    U = 68_768
    npos = rng.integers(1, 6, U)
    lens = npos + 500
    flat = rng.standard_normal(int(lens.sum())).astype(np.float32)
    off = np.concatenate([[0], np.cumsum(lens)])
    dev = torch.from_numpy(flat).to(cuda)
    ops.rank_metrics(dev, lens, npos, 20)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    hits, auc, flags = ops.rank_metrics(dev, lens, npos, 20)
    res = metrics_from_hits(hits, lens, npos, auc, 500)
    t_dev = time.perf_counter() - t0
    sample = 4000  # the host loop on a sample (its per-user cost is flat), scaled to all users
    t0 = time.perf_counter()
    ref = _ref([flat[off[u]:off[u + 1]] for u in range(sample)], npos[:sample])
    t_host = (time.perf_counter() - t0) * U / sample
    ok = np.nonzero(flags[:sample] == 0)[0]
    assert np.array_equal(res[:sample][ok], ref[ok])
    print(f"\nrank {U} users: device {t_dev * 1e3:.1f} ms (incl. host metric assembly), "
          f"reference-style host loop ~{t_host:.1f} s (from {sample} users)")


@pytest.mark.parametrize("U,I,stride_pad", [(68_768, 45_630, 0), (300, 50, 8), (1, 7, 0)])
def test_score_segments_matches_gather_dot(cuda, U, I, stride_pad):
    """fr_score_segments (the evaluation's fused gather-dot, one wave per user segment) vs torch's
    mul(user[u], item[i]).sum(1) (the models' inference_fast) on the same fp32 tables: rel 1e-6 of
    the score scale (fp32 summation order only), including row strides wider than 64 (table views)."""
    from FoodRec.engine import ops
    g = torch.Generator().manual_seed(U + I)
    Ut = torch.randn(U, 64 + stride_pad, generator=g).to(cuda)[:, :64]
    It = torch.randn(I, 64 + stride_pad, generator=g).to(cuda)[:, :64]
    n_seg = min(U, 4096)
    lens = torch.randint(1, 600, (n_seg,), generator=g)
    off = torch.zeros(n_seg + 1, dtype=torch.int64)
    torch.cumsum(lens, 0, out=off[1:])
    uid = torch.randint(0, U, (n_seg,), generator=g)
    items = torch.randint(0, I, (int(off[-1]),), generator=g)
    got = ops.score_segments(Ut, It, uid.to(cuda), off.to(cuda), items.to(cuda))
    users = torch.repeat_interleave(uid, lens).to(cuda)
    ref = torch.mul(Ut[users], It[items.to(cuda)]).sum(1)
    torch.testing.assert_close(got, ref, rtol=0, atol=1e-6 * float(ref.abs().max()) + 1e-7)


def test_fused_scoring_evaluation_matches_torch_path(cuda):
    """Trainer._valid_by_user_epoch with fused scoring (cached device lists + fr_score_segments) vs the
    same trainer with the model's torch inference_fast path, on the tiny HealthRec fixture: equal
    metrics (the scores differ only in fp32 summation order, far below any ranking gap here)."""
    from helpers import tiny_config, tiny_data
    from FoodRec.common.trainer import Trainer
    from FoodRec.utils.utils import get_model, init_seed
    cfg = tiny_config("CIKM_Model", True, cuda_graph=False)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("CIKM_Model")(cfg, data).to(cfg["device"])
    tr = Trainer(cfg, model)
    model.eval()
    assert tr._fused_scoring()
    fused = [tr._valid_by_user_epoch(is_test=t)[1] for t in (False, True, True)]
    type(model).fused_scores = False
    try:
        plain = [tr._valid_by_user_epoch(is_test=t)[1] for t in (False, True)]
    finally:
        type(model).fused_scores = True
    for a, b in zip(fused, plain + [plain[1]]):
        assert a.keys() == b.keys()
        for k in a:
            assert abs(a[k] - b[k]) <= 1e-9, (k, a[k], b[k])


@pytest.mark.parametrize("emb", [32, 128])
def test_fused_scoring_falls_back_for_other_widths(cuda, emb):
    """a model declaring ``fused_scores`` whose forward() tables are not fp32 [*, 64]
    (here LightGCN at embedding_size 32 / 128) is evaluated through inference_fast instead of
    fr_score_segments, with the same metrics as the non-fused path."""
    from helpers import tiny_config, tiny_data
    from FoodRec.common.trainer import Trainer
    from FoodRec.utils.utils import get_model, init_seed
    cfg = tiny_config("LightGCN", True, embedding_size=emb, graph_inference_fast=True)
    data = tiny_data(cfg)
    init_seed(999)
    model = get_model("LightGCN")(cfg, data).to(cfg["device"])
    tr = Trainer(cfg, model)
    assert tr._fused_scoring()
    score, metrics = tr._valid_by_user_epoch(is_test=True)
    cls = type(model)
    saved = cls.__dict__.get("fused_scores", None)
    cls.fused_scores = False
    try:
        score2, metrics2 = tr._valid_by_user_epoch(is_test=True)
    finally:
        if saved is None:
            del cls.fused_scores
        else:
            cls.fused_scores = saved
    assert metrics == metrics2
