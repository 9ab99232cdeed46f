"""Device-ranking bookkeeping on the host (no GPU): metrics_from_hits turns per-user hit masks and
AUC counts into exactly the float64 values the reference's per-user loop computes
(metrics_by_user / get_auc_fast, /root/reference/FoodRec/common/trainer.py:49-69, 231-282).  The
masks here are derived from numpy's own argsort order on tie-free random scores, i.e. what
fr_rank_metrics reports; the GPU test compares the kernel with that."""
import numpy as np

from FoodRec.common.trainer import metrics_from_hits, rank_user_host


def _case(seed, U=300):
    rng = np.random.default_rng(seed)
    lens = rng.integers(1, 60, U)
    npos = np.minimum(rng.integers(1, 8, U), lens)
    scores = [rng.standard_normal(n).astype(np.float32) for n in lens]
    return lens, npos, scores


def _hits_from_numpy(scores, npos, K=20):
    hits, auc = [], []
    for pr, npo in zip(scores, npos):
        order = np.argsort(pr)[::-1][:K]
        hits.append(sum(1 << t for t, d in enumerate(order) if d < npo))
        auc.append(int(sum(np.sum(pr[npo:] < pr[p]) for p in range(npo))))
    return np.array(hits, np.uint32), np.array(auc, np.int64)


def test_metrics_from_hits_bit_equal_host_loop():
    for seed in range(3):
        lens, npos, scores = _case(seed)
        hits, auc = _hits_from_numpy(scores, npos)
        got = metrics_from_hits(hits, lens, npos, auc, 500)
        ref = np.stack([rank_user_host(pr, int(npo), 500) for pr, npo in zip(scores, npos)])
        assert np.array_equal(got, ref)  # bit for bit, per user
        assert np.array_equal(got.mean(axis=0), ref.mean(axis=0))
