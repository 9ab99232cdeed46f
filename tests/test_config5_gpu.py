"""BASELINE config 5 kernels on the GPU: bf16 tables (SpMM, BPR + EmbLoss, mixed-precision Adam) and
the fused full-sort top-k on the matrix cores, each against the oracle.

Tolerances (inputs are exactly-representable bf16 values; references in fp64 on those values):
  bf16 SpMM       : |err| <= 2^-8 |ref| (one output rounding to bf16) + 2e-5 * (|A||X| row scale) + 1e-6
  bf16 BPR values : rel 1e-5 (fp32 arithmetic on exact bf16 inputs);  gradients: 2^-8 rel + 1e-6
  bf16 Adam       : master / exp_avg / exp_avg_sq follow torch.optim.Adam on the fp32 master
                    (m, v bit-identical; master within 4 ulp of p or of the ~lr update);
                    param == master rounded to bf16
  full-sort top-k : returned scores within 1e-5 * sum|u_k i_k| of fp64 scores of the returned items;
                    the k-th score within that tolerance of the fp64 k-th score; every item whose fp64
                    score clears the k-th by more than the tolerance is returned; excluded (training)
                    items never returned; hit flags exact.
"""
import numpy as np
import pytest
import torch

from oracle import ops as O

pytestmark = pytest.mark.gpu


def _graph(n_rows, n_cols, avg_deg, heavy=(), seed=0):
    rng = np.random.default_rng(seed)
    deg = rng.poisson(avg_deg, n_rows)
    for r, d in heavy:
        deg[r] = d
    deg[rng.integers(n_rows)] = 0
    rows = np.repeat(np.arange(n_rows), deg)
    cols = rng.integers(0, n_cols, rows.shape[0])
    key = np.unique(rows * n_cols + cols)
    return key // n_cols, key % n_cols


def _adj(n, rows, cols, cuda, chunk=64):
    from FoodRec.engine.graph import Adjacency
    return Adjacency.sym_normalized(n, rows, cols, device=cuda, chunk=chunk)


def _bf(x):
    return torch.as_tensor(x).to(torch.bfloat16)


@pytest.mark.parametrize("d", [256, 64, 128, 8, 32])
def test_spmm_bf16_matches_fp64(cuda, d):
    from FoodRec.engine import ops
    n = 600
    r, c = _graph(n, n, 6, heavy=[(3, 400), (10, 129)], seed=d)
    adj = _adj(n, r, c, cuda, chunk=64)
    assert adj.n_split >= 2
    row, col, val = O.norm_adj_coo(n, r, c)
    X = _bf(torch.randn(n, d))
    ref = O.spmm_f64(row, col, val, n, X.float().numpy())
    Y = ops.spmm(adj, X.to(cuda))
    assert Y.dtype == torch.bfloat16
    Y = Y.float().cpu().numpy()
    scale = O.spmm_f64(row, col, np.abs(val), n, np.abs(X.float().numpy()))
    assert np.all(np.abs(Y - ref) <= 2.0 ** -8 * np.abs(ref) + 2e-5 * scale + 1e-6)


def test_spmm_bf16_epilogue_and_ld(cuda):
    from FoodRec.engine import ops
    n, d = 300, 256
    r, c = _graph(n, n, 5, heavy=[(7, 300)], seed=3)
    adj = _adj(n, r, c, cuda, chunk=32)
    row, col, val = O.norm_adj_coo(n, r, c)
    big = _bf(torch.randn(n, 320)).to(cuda)
    X = big[:, 32:288]  # strided view, ld = 320
    A1 = _bf(torch.randn(n, d)).to(cuda)
    A2 = _bf(torch.randn(n, d)).to(cuda)
    Y1 = torch.empty(n, d, dtype=torch.bfloat16, device=cuda)
    Y2 = torch.empty(n, d, dtype=torch.bfloat16, device=cuda)
    ops.spmm_launch(adj, X, Y1=Y1, Y2=Y2, alpha=0.25, A1=A1, beta1=0.5, A2=A2, beta2=-2.0)
    acc = O.spmm_f64(row, col, val, n, X.float().cpu().numpy())
    tol = 2.0 ** -8
    np.testing.assert_allclose(Y1.float().cpu().numpy(), acc, rtol=tol, atol=1e-5)
    want = 0.25 * acc + 0.5 * A1.float().cpu().numpy() - 2.0 * A2.float().cpu().numpy()
    np.testing.assert_allclose(Y2.float().cpu().numpy(), want, rtol=tol, atol=1e-4)
    with pytest.raises(Exception):
        ops.spmm_launch(adj, X, Y1=torch.empty(n, d, device=cuda))  # mixed dtypes are refused


def test_spmm_bf16_deterministic(cuda):
    from FoodRec.engine import ops
    n = 2000
    r, c = _graph(n, n, 20, heavy=[(1, 1900), (5, 1500)], seed=11)
    adj = _adj(n, r, c, cuda, chunk=128)
    X = torch.randn(n, 256, device=cuda).to(torch.bfloat16)
    assert torch.equal(ops.spmm(adj, X), ops.spmm(adj, X))


def test_bpr_bf16_matches_fp64(cuda):
    from FoodRec.engine import ops
    torch.manual_seed(0)
    nU, nI, d, B = 50, 70, 256, 96
    U = _bf(torch.randn(nU, d) * 0.1)
    I = _bf(torch.randn(nI, d) * 0.1)
    Ue = _bf(torch.randn(nU, d) * 0.1)
    Ie = _bf(torch.randn(nI, d) * 0.1)
    u = torch.randint(0, nU, (B,))
    p = torch.randint(0, nI, (B,))
    n = torch.randint(0, nI, (B,))
    tabs = [t.to(cuda).requires_grad_(True) for t in (U, I, Ue, Ie)]
    mf, emb = ops.bpr_emb_loss(*tabs, u.to(cuda), p.to(cuda), n.to(cuda))
    (mf + 0.1 * emb.sum()).backward()
    ref = [t.double().requires_grad_(True) for t in (U, I, Ue, Ie)]
    rmf, rreg = O.bpr_step_reference(ref[0], ref[1], ref[2], ref[3], u, p, n, 0.1)
    (rmf + rreg.sum()).backward()
    assert abs(mf.item() - rmf.item()) <= 1e-5 * abs(rmf.item())
    assert abs(0.1 * emb.item() - rreg.item()) <= 1e-5 * abs(rreg.item())
    for g, r_ in zip(tabs, ref):
        assert g.grad.dtype == torch.bfloat16
        got, want = g.grad.float().cpu().double(), r_.grad
        assert torch.all((got - want).abs() <= 2.0 ** -8 * want.abs() + 1e-6), (got - want).abs().max()


def test_adam_bf16_master(cuda):
    from FoodRec.engine.optim import FusedAdam
    torch.manual_seed(1)
    w0 = _bf(torch.randn(4096, 256))
    p = torch.nn.Parameter(w0.clone().to(cuda))
    opt = FusedAdam([p], lr=1e-2)
    ref = torch.nn.Parameter(w0.float().clone())
    ropt = torch.optim.Adam([ref], lr=1e-2)
    for _ in range(3):
        g = _bf(torch.randn(4096, 256))
        p.grad = g.to(cuda)
        ref.grad = g.float()
        opt.step()
        ropt.step()
    st, rst = opt.state[p], ropt.state[ref]
    assert torch.equal(st["exp_avg"].cpu(), rst["exp_avg"])
    assert torch.equal(st["exp_avg_sq"].cpu(), rst["exp_avg_sq"])
    m = st["master"].cpu()
    a, b = m.numpy(), ref.detach().numpy()
    # as the fp32 test: a few ulp of p, or of the update (~lr) for parameters near zero
    assert np.all(np.abs(a - b) <= 4 * np.spacing(np.abs(b)) + 4 * np.spacing(np.float32(2e-2)))
    assert torch.equal(p.detach().cpu(), m.to(torch.bfloat16))


def _excl_csr(lists, base, device):
    rp = np.zeros(len(lists) + 1, np.int64)
    rp[1:] = np.cumsum([len(x) for x in lists])
    col = np.concatenate([np.sort(np.asarray(x, np.int64)) + base for x in lists]).astype(np.int32) \
        if rp[-1] else np.zeros(1, np.int32)
    return torch.from_numpy(rp).to(device), torch.from_numpy(col).to(device), base


def _check_topk(got_s, got_i, U, I, k, exclude, tol_scale):
    S = U.astype(np.float64) @ I.astype(np.float64).T
    ref_s, ref_i, _ = O.full_sort_topk(U, I, k, exclude)
    absS = np.abs(U.astype(np.float64)) @ np.abs(I.astype(np.float64)).T
    for u in range(U.shape[0]):
        tol = tol_scale * absS[u].max() + 1e-6
        gi = got_i[u]
        assert len(set(gi.tolist())) == k
        assert not set(gi.tolist()) & set(exclude[u] if exclude is not None else [])
        np.testing.assert_allclose(got_s[u], S[u, gi], atol=tol, rtol=0)
        assert np.all(np.diff(got_s[u]) <= 0)
        assert abs(got_s[u, -1] - ref_s[u, -1]) <= tol
        sure = ref_i[u][ref_s[u] > ref_s[u, -1] + 2 * tol]
        assert set(sure.tolist()) <= set(gi.tolist())


@pytest.mark.parametrize("dtype,d,n_users,n_items,k", [
    (torch.bfloat16, 256, 300, 5000, 20),
    (torch.bfloat16, 64, 40, 777, 10),
    (torch.bfloat16, 128, 513, 3001, 32),
    (torch.float32, 64, 260, 4099, 20),
    (torch.float32, 128, 33, 1000, 5),
])
def test_full_sort_topk_matches_oracle(cuda, dtype, d, n_users, n_items, k):
    from FoodRec.engine import ops
    rng = np.random.default_rng(d + n_users)
    U = rng.standard_normal((n_users, d)).astype(np.float32)
    I = rng.standard_normal((n_items, d)).astype(np.float32)
    I[7] = I[5]  # exact ties (ordered by item id)
    if dtype == torch.bfloat16:
        U, I = O.bf16_round(U), O.bf16_round(I)
    excl = [rng.choice(n_items, size=rng.integers(0, 40), replace=False).tolist() for _ in range(n_users)]
    held = [rng.choice(n_items, size=rng.integers(1, 30), replace=False).tolist() for _ in range(n_users)]
    uid = torch.arange(n_users, dtype=torch.int64)
    ex = _excl_csr(excl, 3, cuda)
    ho = _excl_csr(held, 0, cuda)
    s, i, h = ops.full_sort_topk(torch.from_numpy(U).to(dtype).to(cuda), torch.from_numpy(I).to(dtype).to(cuda), k,
                                 user_ids=uid, exclude=ex, held_out=ho)
    s, i, h = s.cpu().numpy(), i.cpu().numpy(), h.cpu().numpy().astype(bool)
    _check_topk(s, i, U, I, k, excl, 1e-5 if dtype == torch.bfloat16 else 2e-6)
    want_h = np.array([[x in set(held[u]) for x in i[u]] for u in range(n_users)])
    assert np.array_equal(h, want_h)


@pytest.mark.parametrize("dtype,d,n_users,n_items,k", [
    (torch.bfloat16, 256, 600, 40000, 20),
    (torch.bfloat16, 64, 1100, 33001, 10),
    (torch.float32, 64, 300, 40000, 32),
])
def test_full_sort_topk_sampled_path(cuda, dtype, d, n_users, n_items, k):
    """n_items >= 32768: the sampled path (LIST on a strided sub-sample, APPEND + MERGE over the sample
    -> thresholds, APPEND over all items, MERGE) against the oracle's exact top-k (the small cases
    above take one LIST pass)."""
    from FoodRec.engine import ops
    rng = np.random.default_rng(d + n_users + k)
    U = rng.standard_normal((n_users, d)).astype(np.float32)
    I = rng.standard_normal((n_items, d)).astype(np.float32)
    I[7] = I[5]
    if dtype == torch.bfloat16:
        U, I = O.bf16_round(U), O.bf16_round(I)
    excl = [rng.choice(n_items, size=rng.integers(0, 40), replace=False).tolist() for _ in range(n_users)]
    ex = _excl_csr(excl, 0, cuda)
    s, i, _ = ops.full_sort_topk(torch.from_numpy(U).to(dtype).to(cuda), torch.from_numpy(I).to(dtype).to(cuda), k,
                                 exclude=ex)
    _check_topk(s.cpu().numpy(), i.cpu().numpy(), U, I, k, excl, 1e-5 if dtype == torch.bfloat16 else 2e-6)


def test_full_sort_topk_overflow_paths(cuda):
    """Adversarial score order for the sampled path: the sub-sample (multiples of 32) scores lowest,
    the rest of the sample (even items) in the middle, odd items highest -- with the two-level
    thresholds the sample pass's regions overflow (the user keeps the sub-sample's looser threshold);
    with the position-group maxima the threshold sits at the sample's (middle) level; either way the
    all-items pass overflows and the user is recomputed by the exact LIST pass.  Result = the exact
    top-k."""
    from FoodRec.engine import ops
    rng = np.random.default_rng(77)
    n_users, n_items, d, k = 64, 140000, 64, 20
    U = (rng.standard_normal((n_users, d)) + 3.0).astype(np.float32)
    tier = np.where(np.arange(n_items) % 2 == 1, 1.0, np.where(np.arange(n_items) % 32 == 0, -1.0, 0.0))
    I = (tier[:, None] / d + 0.01 * rng.standard_normal((n_items, d))).astype(np.float32)
    excl = [rng.choice(n_items, size=rng.integers(0, 40), replace=False).tolist() for _ in range(n_users)]
    ex = _excl_csr(excl, 0, cuda)
    s, i, _ = ops.full_sort_topk(torch.from_numpy(U).to(cuda), torch.from_numpy(I).to(cuda), k, exclude=ex)
    _check_topk(s.cpu().numpy(), i.cpu().numpy(), U, I, k, excl, 2e-6)
    assert (i.cpu().numpy() % 2 == 1).all()


def test_full_sort_topk_many_users_two_level(cuda):
    """>= 128k users: one split per user tile, too few position-group maxima per user for the
    threshold -- the two-level (sub-sample LIST, sample APPEND + merge) thresholds run instead.
    Checked on a subset of users against the oracle."""
    from FoodRec.engine import ops
    rng = np.random.default_rng(31)
    n_users, n_items, d, k = 140000, 33000, 64, 20
    U = rng.standard_normal((n_users, d)).astype(np.float32)
    I = rng.standard_normal((n_items, d)).astype(np.float32)
    excl = [rng.choice(n_items, size=rng.integers(0, 30), replace=False).tolist() for _ in range(n_users)]
    ex = _excl_csr(excl, 0, cuda)
    s, i, _ = ops.full_sort_topk(torch.from_numpy(U).to(cuda), torch.from_numpy(I).to(cuda), k, exclude=ex)
    sel = rng.choice(n_users, size=48, replace=False)
    _check_topk(s.cpu().numpy()[sel], i.cpu().numpy()[sel], U[sel], I, k, [excl[x] for x in sel], 2e-6)


def test_full_sort_topk_no_mask_and_permuted_ids(cuda):
    from FoodRec.engine import ops
    rng = np.random.default_rng(5)
    U = O.bf16_round(rng.standard_normal((64, 256)))
    I = O.bf16_round(rng.standard_normal((2000, 256)))
    s, i, h = ops.full_sort_topk(torch.from_numpy(U).to(torch.bfloat16).to(cuda),
                                 torch.from_numpy(I).to(torch.bfloat16).to(cuda), 20)
    assert h is None
    _check_topk(s.cpu().numpy(), i.cpu().numpy(), U, I, 20, None, 1e-5)
    # exclusion rows are looked up by user id, not by row
    ids = torch.tensor(rng.permutation(64), dtype=torch.int64)
    excl = [[int(x)] for x in range(64)]  # user id x excludes item x
    ex = _excl_csr(excl, 0, cuda)
    s2, i2, _ = ops.full_sort_topk(torch.from_numpy(U).to(torch.bfloat16).to(cuda),
                                   torch.from_numpy(I).to(torch.bfloat16).to(cuda), 20, user_ids=ids, exclude=ex)
    i2 = i2.cpu().numpy()
    for r in range(64):
        assert int(ids[r]) not in set(i2[r].tolist())


def test_lightgcn_id_bf16_step(cuda):
    """Config-5 training step (d=256, bf16 tables) against the same step in fp32 on the same
    bf16-rounded weights: losses agree to bf16 precision, parameters move, nothing is NaN."""
    from FoodRec.common.trainer import Trainer
    from FoodRec.models.lightgcn_id import LightGCN_ID
    from FoodRec.utils.configurator import Config
    from FoodRec.utils.interaction_graph import InteractionGraph
    g = InteractionGraph(3000, 800, 12.0, seed=1, device=cuda)

    def make(dtype):
        cfg = Config("LightGCN_ID", "Synthetic10M", {"use_gpu": True, "seed": 999, "log_root": "/tmp/frlog/",
                                                     "ckp_root": "/tmp/frckp/", "embedding_size": 256,
                                                     "embedding_dtype": dtype})
        cfg["device"] = cuda
        torch.manual_seed(999)
        return cfg, LightGCN_ID(cfg, g)

    cfg16, m16 = make("bf16")
    cfg32, m32 = make("fp32")
    with torch.no_grad():
        m32.ego.copy_(m16.ego.float())
    assert m16.ego.dtype == torch.bfloat16
    u, p, n = g.triples(512)
    batch = {"u_id": u, "pos_i_id": p, "neg_i_id": n}
    l16 = [x.item() for x in m16.calculate_loss(batch)]
    l32 = [x.item() for x in m32.calculate_loss(batch)]
    assert abs(l16[0] - l32[0]) <= 2e-3 * abs(l32[0])
    assert abs(l16[1] - l32[1]) <= 2e-3 * abs(l32[1])
    tr = Trainer(cfg16, m16)
    st = tr.new_step_state()
    before = m16.ego.detach().clone()
    for k in range(3):
        uu, pp, nn_ = g.triples(512)
        tr.train_step({"u_id": uu, "pos_i_id": pp, "neg_i_id": nn_}, k, st)
    torch.cuda.synchronize()
    assert not int(st["nan"].item())
    assert not torch.equal(before, m16.ego.detach())
    s, i, _ = m16.full_sort_topk(torch.arange(64, device=cuda), 20)
    assert torch.isfinite(s).all() and int(i.min()) >= 0
