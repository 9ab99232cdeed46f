"""GPU parity of the HIP kernels against the oracle (torch-CPU / fp64 restatements).

Tolerances (fp32 kernels vs fp64 or torch-CPU fp32 references):
  SpMM / propagation   : |err| <= 2e-5 * (|A||X| row scale) + 1e-6   (fp32 accumulate, reordered sum)
  BPR / EmbLoss values : rel 1e-5;  gradients rel 1e-4 (atomic scatter order)
  dCor                 : value and gradients no further from float64 than the reference's own fp32
                         arithmetic is (the same restatement run in fp32), or within 1e-5 / 1e-4 * max
  InfoNCE              : rel 1e-5 value, 1e-4 gradients
  Adam                 : exp_avg/exp_avg_sq bit-identical to torch.optim.Adam (CPU); params
                         within 4 ulp after 3 steps (torch-CPU addcdiv rounding on ~0.1% of elements)
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
    deg[rng.integers(n_rows)] = 0  # an empty row
    rows = np.repeat(np.arange(n_rows), deg)
    cols = rng.integers(0, n_cols, rows.shape[0])
    key = np.unique(rows * n_cols + cols)
    return key // n_cols, key % n_cols


def _adj(n, rows, cols, cuda, chunk=64):
    from FoodRec.engine.graph import Adjacency
    return Adjacency.sym_normalized(n, rows, cols, device=cuda, chunk=chunk)


@pytest.mark.parametrize("d", [64, 16, 32, 128, 256])
def test_spmm_matches_fp64(cuda, d):
    from FoodRec.engine import ops
    n = 700
    r, c = _graph(n, n, 6, heavy=[(3, 400), (10, 129)], seed=d)
    adj = _adj(n, r, c, cuda, chunk=64)
    assert adj.n_split >= 2
    row, col, val = O.norm_adj_coo(n, r, c)
    X = torch.randn(n, d, dtype=torch.float32)
    ref = O.spmm_f64(row, col, val, n, X.numpy())
    Y = ops.spmm(adj, X.to(cuda)).cpu().numpy()
    scale = O.spmm_f64(row, col, np.abs(val), n, np.abs(X.numpy()))
    assert np.all(np.abs(Y - ref) <= 2e-5 * scale + 1e-6)


def test_spmm_epilogue_and_ld(cuda):
    from FoodRec.engine import ops
    n, d = 300, 64
    r, c = _graph(n, n, 5, heavy=[(7, 300)], seed=3)
    adj = _adj(n, r, c, cuda, chunk=32)
    row, col, val = O.norm_adj_coo(n, r, c)
    big = torch.randn(n, 96, device=cuda)
    X = big[:, 16:80]  # strided view, ld = 96
    A1 = torch.randn(n, d, device=cuda)
    A2 = torch.randn(n, d, device=cuda)
    Y1 = torch.empty(n, d, device=cuda)
    Y2 = torch.empty(n, d, device=cuda)
    ops.spmm_launch(adj, X, Y1=Y1, Y2=Y2, alpha=0.25, A1=A1, beta1=0.5, A2=A2, beta2=-2.0)
    acc = O.spmm_f64(row, col, val, n, X.cpu().numpy())
    np.testing.assert_allclose(Y1.cpu().numpy(), acc, rtol=1e-5, atol=1e-5)
    want = 0.25 * acc + 0.5 * A1.cpu().numpy() - 2.0 * A2.cpu().numpy()
    np.testing.assert_allclose(Y2.cpu().numpy(), want, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n,max_deg,ldx", [(65617, 45, 64), (37, 33, 96), (5000, 16, 64)])
def test_spmm_plain_rows_pipelined(cuda, n, max_deg, ldx):
    """Every row a plain unit (the RI propagation's shape): the pipelined row walk
    (spmm_plain16_kernel) vs float64, with the full epilogue (Y1, Y2 = alpha acc + beta1 A1 +
    beta2 A2), empty rows, rows of exactly 16 / 32 edges, a strided X; rows of <= 16 edges are
    bit-identical to the general unit kernel (the same adjacency planned with chunk 16, which
    splits the longer rows and so takes the general path)."""
    from FoodRec.engine import ops
    from FoodRec.engine.graph import Adjacency
    rng = np.random.default_rng(n)
    deg = rng.integers(0, max_deg + 1, n)
    deg[: min(n, 3)] = [0, 16, min(32, max_deg)][: min(n, 3)]
    rowptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    col = rng.integers(0, n, rowptr[-1]).astype(np.int32)
    val = rng.standard_normal(rowptr[-1]).astype(np.float32)
    a = Adjacency(rowptr, col, val, (n, n), chunk=64, symmetric=False, device=cuda)
    b = Adjacency(rowptr, col, val, (n, n), chunk=16, symmetric=False, device=cuda)
    assert a.n_units == n and a.n_split == 0 and (max_deg <= 16 or b.n_split > 0)
    big = torch.randn(n, ldx, device=cuda)
    X = big[:, :64]
    A1, A2 = torch.randn(n, 64, device=cuda), torch.randn(n, 64, device=cuda)
    out = {}
    for name, adj in (("a", a), ("b", b)):
        Y1, Y2 = torch.empty(n, 64, device=cuda), torch.empty(n, 64, device=cuda)
        ops.spmm_launch(adj, X, Y1=Y1, Y2=Y2, alpha=0.5, A1=A1, beta1=0.25, A2=A2, beta2=-1.5)
        out[name] = (Y1.cpu(), Y2.cpu())
    rows = np.repeat(np.arange(n), deg)
    acc = np.zeros((n, 64))
    np.add.at(acc, rows, val[:, None].astype(np.float64) * X.double().cpu().numpy()[col])
    scale = np.zeros((n, 64))
    np.add.at(scale, rows, np.abs(val[:, None]).astype(np.float64) * np.abs(X.double().cpu().numpy()[col]))
    Y1, Y2 = out["a"]
    assert np.all(np.abs(Y1.numpy() - acc) <= 2e-6 * scale + 1e-6)
    want = 0.5 * acc + 0.25 * A1.double().cpu().numpy() - 1.5 * A2.double().cpu().numpy()
    assert np.all(np.abs(Y2.numpy() - want) <= 2e-6 * scale + 2e-6 * np.abs(want) + 1e-6)
    short = torch.as_tensor(deg <= 16)
    assert torch.equal(Y1[short], out["b"][0][short]) and torch.equal(Y2[short], out["b"][1][short])


def test_bipartite_half_graph_propagation(cuda):
    """HealthRec's RI propagation on a bipartite adjacency (models/_graphs.side_adjacency marks it):
    the last forward layer over the item rows only (fr_spmm_csr_range) equals the full launch's
    item rows bit for bit; the two-layer backward of an item-only upstream gradient in two
    half-graph launches (ops._prop_bwd_bipartite2) equals the full form within fp32 rounding, and
    its item rows bit for bit."""
    from FoodRec.engine import ops
    from FoodRec.models._graphs import side_adjacency
    rng = np.random.default_rng(5)
    I, NI = 3000, 700
    triples = np.stack([rng.integers(0, I, 20000), rng.integers(0, NI, 20000)], 1)
    adj = side_adjacency(triples, I, NI, cuda)
    assert adj.bipartite_split == I
    item = torch.randn(I, 64, device=cuda)
    ingre = torch.randn(NI + 1, 64, device=cuda)
    full = ops._prop_fwd_split(adj, item, ingre, I, 2)
    half = ops._prop_fwd_split(adj, item, ingre, I, 2, lo_rows_only=True)
    assert torch.equal(full[:I], half[:I])
    G = torch.zeros(I + NI, 64, device=cuda)
    G[:I] = torch.randn(I, 64, device=cuda)
    outs = []
    for fast in (False, True):
        d_item, d_ingre = torch.empty(I, 64, device=cuda), torch.full((NI + 1, 64), 7.0, device=cuda)
        if fast:
            ops._prop_bwd_bipartite2(adj, G[:I], d_item, d_ingre, I)
        else:
            ops._prop_bwd_split(adj, G, 2, d_item, d_ingre, I)
        outs.append((d_item.cpu(), d_ingre.cpu()))
    (a_item, a_ing), (b_item, b_ing) = outs
    assert torch.equal(a_item, b_item)
    torch.testing.assert_close(b_ing[:NI], a_ing[:NI], rtol=2e-6, atol=1e-7)
    assert torch.all(b_ing[NI:] == 7.0)  # the padding row is not written


@pytest.mark.parametrize("L", [1, 2, 3])
def test_propagate_lo_matches_full(cuda, L):
    """ops.propagate_lo (CLUSSL's modality views: item rows of the propagation over a bipartite
    item-side graph, no concatenation or split) vs split(propagate_mean(cat(item, side)))[0]:
    values and both tables' gradients (side rows beyond the graph: zero gradient)."""
    from FoodRec.engine import ops
    from FoodRec.models._graphs import side_adjacency
    rng = np.random.default_rng(L)
    I, NS = 2500, 400
    triples = np.stack([rng.integers(0, I, 9000), rng.integers(0, NS, 9000)], 1)
    adj = side_adjacency(triples, I, NS, cuda)
    lo0, hi0 = torch.randn(I, 64, device=cuda), torch.randn(NS + 1, 64, device=cuda)
    g = torch.randn(I, 64, device=cuda)
    res = []
    for fast in (False, True):
        lo, hi = lo0.clone().requires_grad_(True), hi0.clone().requires_grad_(True)
        if fast:
            out = ops.propagate_lo(adj, lo, hi, L)
        else:
            out = ops.propagate_mean(adj, torch.cat([lo, hi[:NS]]), L)[:I]
        (out * g).sum().backward()
        res.append((out.detach(), lo.grad, hi.grad))
    (a, ga_lo, ga_hi), (b, gb_lo, gb_hi) = res
    assert torch.equal(a, b)
    torch.testing.assert_close(gb_lo, ga_lo, rtol=2e-6, atol=1e-7)
    torch.testing.assert_close(gb_hi, ga_hi, rtol=2e-6, atol=1e-7)
    assert torch.all(gb_hi[NS:] == 0)


@pytest.mark.parametrize("V", [1, 3, 4])
def test_views_sum_gather(cuda, V):
    """ops.views_sum_gather (fr_views_sum_gather: CLUSSL's view sum in torch's add order and the
    views at the batch items, one launch) vs torch: bit-identical sum and gathers (duplicate ids
    included); backward vs autograd through the torch form."""
    from FoodRec.engine import ops
    g = torch.Generator().manual_seed(V)
    n, m = 29943, 1024
    views0 = [torch.randn(n, 64, generator=g).to(cuda) for _ in range(V)]
    ids = torch.randint(0, n, (m,), generator=g).to(cuda)
    ids[:8] = ids[8]  # duplicates
    res = []
    for fused in (False, True):
        views = [v.clone().requires_grad_(True) for v in views0]
        if fused:
            total, gathered = ops.views_sum_gather(views, ids)
        else:
            total = views[0] if V == 1 else torch.add(views[0], views[1])
            for v in views[2:]:
                total = total + v
            gathered = [v.index_select(0, ids) for v in views]
        gs = torch.randn(n, 64, generator=g).to(cuda)
        loss = (total * gs).sum() + sum((x * (k + 1)).sum() for k, x in enumerate(gathered))
        loss.backward()
        res.append((total.detach(), [x.detach() for x in gathered], [v.grad for v in views]))
        g = torch.Generator().manual_seed(V)  # same upstream for both runs
        [torch.randn(n, 64, generator=g) for _ in range(V)]
        torch.randint(0, n, (m,), generator=g)
    (ta, ga, da), (tb, gb, db) = res
    assert torch.equal(ta, tb)
    for a, b in zip(ga, gb):
        assert torch.equal(a, b)
    for a, b in zip(da, db):
        torch.testing.assert_close(b, a, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("L", [1, 2])
def test_propagate_lo_views_matches_per_view(cuda, L):
    """ops.propagate_lo_views (CLUSSL's three views as one node, the item-row gradients summed in the
    SpMM epilogue) vs one propagate_lo per view: equal values; the item table's gradient to fp32
    round-off of the different summation order; each side table's gradient (padding row included)."""
    from FoodRec.engine import ops
    from FoodRec.models._graphs import side_adjacency
    rng = np.random.default_rng(10 + L)
    I, sides = 2500, (400, 150, 150)
    adjs = [side_adjacency(np.stack([rng.integers(0, I, 9000), rng.integers(0, ns, 9000)], 1), I, ns, cuda)
            for ns in sides]
    lo0 = torch.randn(I, 64, device=cuda)
    his0 = [torch.randn(ns + (1 if k == 0 else 0), 64, device=cuda) for k, ns in enumerate(sides)]
    gs = [torch.randn(I, 64, device=cuda) for _ in sides]
    res = []
    for fused in (False, True):
        lo = lo0.clone().requires_grad_(True)
        his = [h.clone().requires_grad_(True) for h in his0]
        if fused:
            outs = ops.propagate_lo_views(adjs, lo, his, L)
        else:
            outs = [ops.propagate_lo(a, lo, h, L) for a, h in zip(adjs, his)]
        sum((o * g).sum() for o, g in zip(outs, gs)).backward()
        res.append(([o.detach() for o in outs], lo.grad, [h.grad for h in his]))
    (oa, la, ha), (ob, lb, hb) = res
    for a, b in zip(oa, ob):
        assert torch.equal(a, b)
    torch.testing.assert_close(lb, la, rtol=1e-5, atol=1e-6)
    for a, b in zip(ha, hb):
        torch.testing.assert_close(b, a, rtol=2e-6, atol=1e-7)
    assert torch.all(hb[0][sides[0]:] == 0)


@pytest.mark.parametrize("N,L,bip", [(3000, 2, False), (300_000, 2, False), (300_000, 1, False), (5000, 3, False),
                                     (6000, 2, True), (300_000, 2, True)])
def test_propagate_rows_matches_full(cuda, N, L, bip):
    """ops.propagate_rows (LightGCN_ID's loss rows: last layer at the batch rows, backward from the
    sparse upstream gradient) vs propagate_mean: the listed rows' values and the ego gradient of a
    loss on those rows (duplicate ids included).  N > 262,144 exercises the sparse launch with its
    bitmask in L2 instead of LDS."""
    from FoodRec.engine import ops
    rng = np.random.default_rng(N + L)
    U = N // 2
    if bip:  # users [0, U) <-> items [U, N) (config 4's graph): layer 1's item block at the needed rows only
        from FoodRec.utils.interaction_graph import InteractionGraph
        uu = rng.integers(0, U, 4 * N)
        uu[:3000] = 5  # a heavy user row
        g = InteractionGraph(U, N - U, pairs=(torch.as_tensor(uu), torch.as_tensor(rng.integers(0, N - U, 4 * N))),
                             device=cuda, chunk=256)
        adj = g.adj
        assert adj.bipartite_split == U
    else:
        r, c = _graph(N, N, 4, heavy=[(5, 3000)], seed=N)
        adj = _adj(N, r, c, cuda, chunk=256)
    ego0 = torch.randn(N, 64, device=cuda)
    u = torch.as_tensor(rng.integers(0, U, 200), device=cuda)
    p = torch.as_tensor(rng.integers(0, N - U, 200), device=cuda)
    n = torch.as_tensor(rng.integers(0, N - U, 200), device=cuda)
    u[:3] = 5  # the heavy row
    u[:10] = u[10]  # duplicates
    idx = torch.cat([u, p + U, n + U])
    w = torch.randn(idx.numel(), 64, device=cuda)
    res = []
    for fast in (False, True):
        ego = ego0.clone().requires_grad_(True)
        out = (ops.propagate_rows(adj, ego, L, [(u, 0), (p, U), (n, U)]) if fast
               else ops.propagate_mean(adj, ego, L))
        rows = out[idx]
        (rows * w).sum().backward()
        res.append((rows.detach(), ego.grad))
    (a, ga), (b, gb) = res
    torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(gb, ga, rtol=1e-5, atol=1e-6 * float(ga.abs().max()))


def test_spmm_deterministic(cuda):
    from FoodRec.engine import ops
    n = 2000
    r, c = _graph(n, n, 20, heavy=[(1, 1900), (5, 1500)], seed=11)
    adj = _adj(n, r, c, cuda, chunk=128)
    X = torch.randn(n, 64, device=cuda)
    a = ops.spmm(adj, X)
    b = ops.spmm(adj, X)
    assert torch.equal(a, b)


@pytest.mark.parametrize("L", [1, 2, 3])
def test_propagate_mean_fwd_bwd(cuda, L):
    from FoodRec.engine import ops
    n, d = 400, 64
    r, c = _graph(n, n, 4, heavy=[(2, 200)], seed=L)
    adj = _adj(n, r, c, cuda, chunk=64)
    row, col, val = O.norm_adj_coo(n, r, c)
    A = O.coo_to_torch(n, row, col, val).double()
    ego = torch.randn(n, d, dtype=torch.float64, requires_grad=True)
    G = torch.randn(n, d, dtype=torch.float64)
    ref = O.propagate_mean(A, ego, L)
    (ref * G).sum().backward()
    e2 = ego.detach().float().to(cuda).requires_grad_(True)
    out = ops.propagate_mean(adj, e2, L)
    (out * G.float().to(cuda)).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref.detach().numpy(), rtol=1e-5, atol=2e-6)
    np.testing.assert_allclose(e2.grad.cpu().numpy(), ego.grad.numpy(), rtol=1e-5, atol=2e-6)


@pytest.mark.parametrize("det", [False, True])
def test_bpr_emb_fwd_bwd(cuda, det):
    from FoodRec.engine import ops
    U_n, I_n, d, B = 50, 40, 64, 300  # small tables -> many duplicate rows in the batch
    g = torch.Generator().manual_seed(5)
    U = torch.randn(U_n, d, generator=g, dtype=torch.float64, requires_grad=True)
    I = torch.randn(I_n, d, generator=g, dtype=torch.float64, requires_grad=True)
    Ue = torch.randn(U_n, d, generator=g, dtype=torch.float64, requires_grad=True)
    Ie = torch.randn(I_n, d, generator=g, dtype=torch.float64, requires_grad=True)
    u = torch.randint(0, U_n, (B,), generator=g)
    p = torch.randint(0, I_n, (B,), generator=g)
    n = torch.randint(0, I_n, (B,), generator=g)
    mf, reg = O.bpr_step_reference(U, I, Ue, Ie, u, p, n, reg_weight=0.3)
    (2.0 * mf + reg.sum()).backward()
    dev = [t.detach().float().to(cuda).requires_grad_(True) for t in (U, I, Ue, Ie)]
    mf2, emb2 = ops.bpr_emb_loss(*dev, u.to(cuda), p.to(cuda), n.to(cuda), deterministic=det)
    (2.0 * mf2 + 0.3 * emb2.sum()).backward()
    assert abs(mf2.item() - mf.item()) <= 1e-5 * abs(mf.item())
    assert abs(0.3 * emb2.item() - reg.item()) <= 1e-5 * abs(reg.item())
    for ref_t, got in zip((U, I, Ue, Ie), dev):
        np.testing.assert_allclose(got.grad.cpu().numpy(), ref_t.grad.numpy(), rtol=1e-4, atol=1e-6)


def test_bpr_shared_tables(cuda):
    """BPRMF case: the ego tables are the propagated tables (same tensors)."""
    from FoodRec.engine import ops
    U_n, I_n, d, B = 30, 20, 64, 64
    g = torch.Generator().manual_seed(9)
    U = torch.randn(U_n, d, generator=g, dtype=torch.float64, requires_grad=True)
    I = torch.randn(I_n, d, generator=g, dtype=torch.float64, requires_grad=True)
    u, p, n = (torch.randint(0, m, (B,), generator=g) for m in (U_n, I_n, I_n))
    mf, reg = O.bpr_step_reference(U, I, U, I, u, p, n, reg_weight=0.1)
    (mf + reg.sum()).backward()
    Ud, Id = (t.detach().float().to(cuda).requires_grad_(True) for t in (U, I))
    mf2, emb2 = ops.bpr_emb_loss(Ud, Id, Ud, Id, u.to(cuda), p.to(cuda), n.to(cuda))
    (mf2 + 0.1 * emb2.sum()).backward()
    np.testing.assert_allclose(Ud.grad.cpu().numpy(), U.grad.numpy(), rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(Id.grad.cpu().numpy(), I.grad.numpy(), rtol=1e-4, atol=1e-6)


@pytest.fixture(params=["mfma", "valu"])
def ssl_kernels(request, cuda):
    """Both Gram-tile forms of the SSL kernels (fr_ssl_kernels): the MFMA default and the VALU tiles."""
    from FoodRec.engine import native
    lib = native.lib()
    prev = lib.fr_ssl_kernels(1 if request.param == "mfma" else 0)
    yield request.param
    lib.fr_ssl_kernels(prev)


@pytest.mark.parametrize("n", [1024, 200])
def test_dcor_three_views(cuda, n, ssl_kernels):
    from FoodRec.engine import ops
    d = 64
    g = torch.Generator().manual_seed(n)
    views = [torch.randn(n, d, generator=g, dtype=torch.float64, requires_grad=True) for _ in range(3)]
    pairs = [(0, 1), (0, 2), (2, 1)]  # (image,text), (image,ingre), (ingre,text) as pricai_modelx.py:263
    ref = sum(O.correlation_distance(views[a], views[b]) for a, b in pairs)
    (1.7 * ref.sum()).backward()
    # the reference's own precision: the same restatement in fp32 (pricai_modelx.py:409-437 runs in
    # fp32 on the CPU), measured against float64
    v32 = [v.detach().float().requires_grad_(True) for v in views]
    ref32 = sum(O.correlation_distance(v32[a], v32[b]) for a, b in pairs)
    (1.7 * ref32.sum()).backward()
    dv = [v.detach().float().to(cuda).requires_grad_(True) for v in views]
    got = ops.dcor_loss(dv, pairs)
    (1.7 * got.sum()).backward()
    err_val, err32_val = abs(got.item() - ref.item()), abs(ref32.item() - ref.item())
    # value: no further from float64 than the fp32 reference, or within 1e-5 relative
    assert err_val <= max(err32_val, 1e-5 * abs(ref.item())), (err_val, err32_val)
    for v, v3, w in zip(views, v32, dv):
        gr, g3, gg = v.grad.numpy(), v3.grad.numpy(), w.grad.cpu().numpy()
        err, err32 = np.abs(gg - gr).max(), np.abs(g3 - gr).max()
        # gradients: no further from float64 than the fp32 reference is, or within 1e-4 * max
        assert err <= max(err32, 1e-4 * np.abs(gr).max()) + 1e-9, (err, err32, np.abs(gr).max())


@pytest.mark.parametrize("n,nv,nograd", [(1500, 3, 1), (1500, 2, -1), (700, 4, 2), (130, 2, 0)])
def test_dcor_views_splits_and_no_grad(cuda, n, nv, nograd, ssl_kernels):
    """View counts 2..4 (the all-views-staged backward for <= 3, the per-view one for 4), more
    than 16 row tiles (workgroups of the backward loop over several j tiles), and a view that needs
    no gradient (the kernels skip its dX)."""
    from FoodRec.engine import ops
    d = 64
    g = torch.Generator().manual_seed(n + nv)
    views = [torch.randn(n, d, generator=g, dtype=torch.float64, requires_grad=True) for _ in range(nv)]
    pairs = {1: [(0, 0)], 2: [(0, 1)], 3: [(0, 1), (0, 2), (2, 1)], 4: [(0, 1), (2, 3), (1, 3)]}[nv]
    ref = sum(O.correlation_distance(views[a], views[b]) for a, b in pairs)
    (0.9 * ref.sum()).backward()
    v32 = [v.detach().float().requires_grad_(True) for v in views]
    ref32 = sum(O.correlation_distance(v32[a], v32[b]) for a, b in pairs)
    (0.9 * ref32.sum()).backward()
    dv = [v.detach().float().to(cuda).requires_grad_(k != nograd) for k, v in enumerate(views)]
    got = ops.dcor_loss(dv, pairs)
    (0.9 * got.sum()).backward()
    err_val, err32_val = abs(got.item() - ref.item()), abs(ref32.item() - ref.item())
    assert err_val <= max(err32_val, 1e-5 * abs(ref.item())), (err_val, err32_val)
    for k, (v, v3, w) in enumerate(zip(views, v32, dv)):
        if k == nograd:
            assert w.grad is None
            continue
        gr, g3, gg = v.grad.numpy(), v3.grad.numpy(), w.grad.cpu().numpy()
        err, err32 = np.abs(gg - gr).max(), np.abs(g3 - gr).max()
        assert err <= max(err32, 1e-4 * np.abs(gr).max()) + 1e-9, (k, err, err32, np.abs(gr).max())


@pytest.mark.parametrize("d", [16, 32, 64, 128])
@pytest.mark.parametrize("b", [512, 37])
def test_infonce(cuda, b, d, ssl_kernels):
    from FoodRec.engine import ops
    g = torch.Generator().manual_seed(b)
    H = torch.randn(2 * b, d, generator=g, dtype=torch.float64, requires_grad=True)
    ref = O.cl_loss(H, 0.5)
    (3.0 * ref).backward()
    Hd = H.detach().float().to(cuda).requires_grad_(True)
    got = ops.infonce_loss(Hd, 0.5)
    (3.0 * got).backward()
    assert abs(got.item() - ref.item()) <= 1e-5 * abs(ref.item())
    np.testing.assert_allclose(Hd.grad.cpu().numpy(), H.grad.numpy(), rtol=1e-4,
                               atol=1e-4 * float(H.grad.abs().max()))


@pytest.mark.parametrize("d", [16, 32, 64, 128])
@pytest.mark.parametrize("b", [1024, 512, 37])
def test_infonce_pairs(cuda, b, d, ssl_kernels):
    """ops.infonce_pairs (all pairs in the same launches, views normalised once, no concatenation)
    against the float64 oracle sum of CL_loss(cat([views[a], views[b]])) over CLUSSL's three pairs:
    value rel 1e-5, gradients rel 1e-4; the value is bit-identical to summing the single-pair op in
    pair order (the same per-pair arithmetic, the same fp32 sum).  Every d the kernels accept: each
    has its own row staging (1 / 2 / 4 / 8 lanes per row) and normalisation layout."""
    from FoodRec.engine import ops
    pairs = ((0, 1), (0, 2), (2, 1))
    g = torch.Generator().manual_seed(100 + b + d)
    V = [torch.randn(b, d, generator=g, dtype=torch.float64, requires_grad=True) for _ in range(3)]
    ref = sum(O.cl_loss(torch.cat([V[a], V[c]]), 0.5) for a, c in pairs)
    (2.5 * ref).backward()
    Vd = [v.detach().float().to(cuda).requires_grad_(True) for v in V]
    got = ops.infonce_pairs(Vd, pairs, 0.5)
    (2.5 * got).backward()
    assert got.dim() == 0
    assert abs(got.item() - ref.item()) <= 1e-5 * abs(ref.item())
    for v, w in zip(V, Vd):
        np.testing.assert_allclose(w.grad.cpu().numpy(), v.grad.numpy(), rtol=1e-4,
                                   atol=1e-4 * float(v.grad.abs().max()))
    with torch.no_grad():
        single = sum(ops.infonce_loss(torch.cat([Vd[a], Vd[c]]), 0.5) for a, c in pairs)
    assert torch.equal(single, got.detach())


def test_infonce_pairs_unpaired_view(cuda, ssl_kernels):
    """A view that no pair holds: the launches fall back to the separate normalize pass (the
    round-5 log-sum-exp kernel normalises only the rows of paired views while staging them); the
    loss matches the float64 oracle and the unpaired view's gradient is exactly zero."""
    from FoodRec.engine import ops
    b, d, pairs = 200, 64, ((0, 2),)
    g = torch.Generator().manual_seed(7)
    V = [torch.randn(b, d, generator=g, dtype=torch.float64, requires_grad=True) for _ in range(3)]
    ref = sum(O.cl_loss(torch.cat([V[a], V[c]]), 0.5) for a, c in pairs)
    ref.backward()
    Vd = [v.detach().float().to(cuda).requires_grad_(True) for v in V]
    got = ops.infonce_pairs(Vd, pairs, 0.5)
    got.backward()
    assert abs(got.item() - ref.item()) <= 1e-5 * abs(ref.item())
    for k in (0, 2):
        np.testing.assert_allclose(Vd[k].grad.cpu().numpy(), V[k].grad.numpy(), rtol=1e-4,
                                   atol=1e-4 * float(V[k].grad.abs().max()))
    assert Vd[1].grad is None or not Vd[1].grad.any()


@pytest.mark.parametrize("d", [16, 32, 64, 128])
def test_infonce_fused_norm_matches_normalize_pass(cuda, d, ssl_kernels):
    """The views normalised inside the log-sum-exp staging (every view in a pair) and by the separate
    normalize pass (a view in no pair) share one arithmetic (nce_row_sumsq, Hn = x / max(|x|, 1e-12)):
    the same pair gives a bit-identical loss and bit-identical gradients either way."""
    from FoodRec.engine import ops
    b = 300
    g = torch.Generator().manual_seed(d)
    V = [torch.randn(b, d, generator=g).to(cuda) for _ in range(3)]
    a = [V[0].clone().requires_grad_(True), V[2].clone().requires_grad_(True)]
    fused = ops.infonce_pairs(a, ((0, 1),), 0.5)          # every view paired: fused normalisation
    fused.backward()
    c = [v.clone().requires_grad_(True) for v in V]
    sep = ops.infonce_pairs(c, ((0, 2),), 0.5)           # view 1 unpaired: the normalize pass
    sep.backward()
    assert torch.equal(fused.detach(), sep.detach())
    assert torch.equal(a[0].grad, c[0].grad) and torch.equal(a[1].grad, c[2].grad)


def test_fused_adam_matches_torch(cuda):
    from FoodRec.engine.optim import FusedAdam
    g = torch.Generator().manual_seed(1)
    shapes = [(37, 64), (1000,), (3,), (128, 5)]
    ref_p = [torch.randn(s, generator=g) for s in shapes]
    dev_p = [p.clone().to(cuda).requires_grad_(True) for p in ref_p]
    ref_p = [p.clone().requires_grad_(True) for p in ref_p]
    o_ref = torch.optim.Adam(ref_p, lr=2e-3, foreach=False)
    o_dev = FusedAdam(dev_p, lr=2e-3)
    for step in range(3):
        grads = [torch.randn(s, generator=g) for s in shapes]
        for p, q, gr in zip(ref_p, dev_p, grads):
            p.grad = gr.clone()
            q.grad = gr.clone().to(cuda)
        dev_p[2].grad = None if step == 1 else dev_p[2].grad  # skipped param, as torch does
        if step == 1:
            ref_p[2].grad = None
        o_ref.step()
        o_dev.step()
    for p, q in zip(ref_p, dev_p):
        a, b = q.detach().cpu().numpy(), p.detach().numpy()
        # torch-CPU addcdiv rounds differently on ~0.1% of elements: <= a few ulp of p, or of
        # the update lr*m/denom (~lr) for parameters near zero
        err = np.abs(a - b)
        assert np.all(err <= 4 * np.spacing(np.abs(b)) + 4 * np.spacing(np.float32(2e-3))), err.max()
        assert np.mean(a == b) > 0.99
    for p, q in zip(ref_p, dev_p):
        st_r, st_d = o_ref.state[p], o_dev.state[q]
        np.testing.assert_array_equal(st_d["exp_avg"].cpu().numpy(), st_r["exp_avg"].numpy())
        np.testing.assert_array_equal(st_d["exp_avg_sq"].cpu().numpy(), st_r["exp_avg_sq"].numpy())
    sd = o_dev.state_dict()
    assert set(sd["state"][0]) == {"step", "exp_avg", "exp_avg_sq"}


def test_fused_adam_two_optimisers_two_streams(cuda):
    """Two FusedAdam instances stepping at the same time on two streams (many-block launches: the
    device step counters are bumped by each launch's last workgroup through per-optimiser ticket
    words): both step counters advance by one per step and both match torch.optim.Adam."""
    from FoodRec.engine.optim import FusedAdam
    g = torch.Generator().manual_seed(3)
    shapes = [(4096, 64), (300_000,)]  # > 8 chunks per launch: many workgroups arrive
    refs, devs, opts, orefs = [], [], [], []
    for _ in range(2):
        rp = [torch.randn(s, generator=g) for s in shapes]
        dp = [p.clone().to(cuda).requires_grad_(True) for p in rp]
        rp = [p.clone().requires_grad_(True) for p in rp]
        refs.append(rp)
        devs.append(dp)
        opts.append(FusedAdam(dp, lr=1e-3))
        orefs.append(torch.optim.Adam(rp, lr=1e-3, foreach=False))
    streams = [torch.cuda.Stream(cuda), torch.cuda.Stream(cuda)]
    for step in range(5):
        for k in range(2):
            grads = [torch.randn(s, generator=g) for s in shapes]
            for p, q, gr in zip(refs[k], devs[k], grads):
                p.grad = gr.clone()
                q.grad = gr.to(cuda)
            orefs[k].step()
        torch.cuda.synchronize()
        for k in range(2):
            streams[k].wait_stream(torch.cuda.current_stream(cuda))
            with torch.cuda.stream(streams[k]):
                opts[k].step()
        torch.cuda.synchronize()
    for k in range(2):
        for p, q in zip(refs[k], devs[k]):
            assert int(opts[k].state[q]["step"].item()) == 5
            np.testing.assert_array_equal(opts[k].state[q]["exp_avg"].cpu().numpy(),
                                          orefs[k].state[p]["exp_avg"].numpy())
            a, b = q.detach().cpu().numpy(), p.detach().numpy()
            assert np.all(np.abs(a - b) <= 4 * np.spacing(np.abs(b)) + 4 * np.spacing(np.float32(1e-3)))


def test_adam_skip_flag(cuda):
    from FoodRec.engine.optim import FusedAdam
    p = torch.randn(100, device=cuda, requires_grad=True)
    p.grad = torch.randn(100, device=cuda)
    before = p.detach().clone()
    opt = FusedAdam([p], lr=0.1)
    opt.step(skip_flag=torch.ones((), dtype=torch.int32, device=cuda))
    assert torch.equal(p.detach(), before)


def test_cpu_tensor_is_an_error():
    """No silent CPU fallback: engine ops refuse host tensors."""
    from FoodRec.engine import native
    from FoodRec.engine import ops
    with pytest.raises(native.EngineError):
        ops.infonce_loss(torch.randn(8, 64), 0.5)


# ----------------------------------------------------------------------------- embedding backward
def _emb_case(kind, seed=0):
    """(idx, n_rows, d, padding_idx) for the edge cases of the reference's row gathers."""
    rng = np.random.default_rng(seed)
    if kind == "ingredients":      # HealthRec: 1024 items x 20 codes, ~half padding (the hot row)
        R, d = 20001, 64
        ids = rng.integers(0, R - 1, (1024, 20))
        ids[rng.random((1024, 20)) < 0.5] = R - 1
        return ids, R, d, None
    if kind == "ingredients_pad":  # same ids through ingre_embedding(padding_idx=n_ingredients)
        ids, R, d, _ = _emb_case("ingredients", seed)
        return ids, R, d, R - 1
    if kind == "one_row":          # every position hits one row: one big bucket over all chunks
        return np.full(5000, 7), 50, 64, None
    if kind == "one_row_small":    # owner pass: one owner sums all 4000 positions
        return np.full(4000, 7), 50, 64, None
    if kind == "wide":             # image/text feature tables: 2B ids, d = 2048 (32 column slices)
        return rng.integers(0, 3000, 1024), 3000, 2048, None
    if kind == "ragged":           # d not a multiple of 64, n not a multiple of the chunk
        return rng.integers(0, 40, 777), 40, 20, 3
    if kind == "few_dups":         # buckets of 2..32 (register sort) and 33+ (bitmap sort)
        base = np.repeat(np.arange(60), rng.integers(1, 70, 60))
        return rng.permutation(base), 64, 32, None
    if kind == "few_dups_large":   # the same bucket mix through the counting-sort chain (n > 4096)
        base = np.repeat(np.arange(200), rng.integers(1, 70, 200))
        return rng.permutation(base), 256, 32, None
    if kind == "empty":
        return np.zeros(0, np.int64), 10, 16, None
    raise KeyError(kind)


@pytest.mark.parametrize("kind", ["ingredients", "ingredients_pad", "one_row", "one_row_small", "wide",
                                  "ragged", "few_dups", "few_dups_large", "empty"])
def test_embedding_bwd_matches_fp64(cuda, kind):
    """fr_embedding_bwd vs the fp64 restatement; tolerance: |err| <= 1e-5 * sum|G| per element
    (fp32 chunked summation of up to n terms) + 1e-6; rows with no contribution exactly zero."""
    from FoodRec.engine import ops
    ids, R, d, pad = _emb_case(kind)
    g = torch.Generator().manual_seed(1)
    W = torch.randn(R, d, generator=g).to(cuda).requires_grad_(True)
    idx = torch.as_tensor(ids, dtype=torch.int64, device=cuda)
    G = torch.randn(*ids.shape, d, generator=g)
    ops._EMB_STATUS = []
    try:
        out = ops.embedding(idx, W, padding_idx=pad)
        ref_fwd = W.detach()[idx]
        assert torch.equal(out.detach(), ref_fwd)
        out.backward(G.to(cuda))
        assert [int(t) for t in ops._EMB_STATUS] == [0]
    finally:
        ops._EMB_STATUS = None
    got = W.grad.double().cpu().numpy()
    ref = O.embedding_bwd_f64(ids, G.numpy(), R, pad)
    scale = O.embedding_bwd_f64(ids, np.abs(G.numpy()), R, pad)
    assert np.all(np.abs(got - ref) <= 1e-5 * scale + 1e-6)
    untouched = scale.sum(1) == 0
    assert np.all(got[untouched] == 0.0)


def test_embedding_bwd_deterministic_and_matches_torch(cuda):
    """Two launches are bit-identical; torch's own embedding backward agrees to fp32 rounding."""
    from FoodRec.engine import ops
    ids, R, d, pad = _emb_case("ingredients_pad", seed=3)
    idx = torch.as_tensor(ids, device=cuda)
    G = torch.randn(*ids.shape, d, device=cuda)
    grads = []
    for _ in range(2):
        W = torch.zeros(R, d, device=cuda, requires_grad=True)
        ops.embedding(idx, W, padding_idx=pad).backward(G)
        grads.append(W.grad.clone())
    assert torch.equal(grads[0], grads[1])
    Wt = torch.zeros(R, d, device=cuda, requires_grad=True)
    torch.nn.functional.embedding(idx, Wt, padding_idx=pad).backward(G)
    torch.testing.assert_close(grads[0], Wt.grad, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("n", [3000, 6000])  # owner pass (n <= 4096) and the counting-sort chain
def test_embedding_bwd_in_graph(cuda, n):
    """fr_embedding_bwd captures into a HIP graph and replays with new ids."""
    from FoodRec.engine import ops
    R, d = 500, 64
    idx = torch.zeros(n, dtype=torch.int64, device=cuda)
    G = torch.randn(n, d, device=cuda)
    W = torch.zeros(R, d, device=cuda, requires_grad=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.embedding(idx, W).backward(G)  # warm-up (allocator, library load)
    torch.cuda.current_stream().wait_stream(s)
    W.grad = None
    graph = torch.cuda.CUDAGraph()
    ops._EMB_STATUS = []
    try:
        with torch.cuda.graph(graph):
            ops.embedding(idx, W).backward(G)
        (status,) = ops._EMB_STATUS
    finally:
        ops._EMB_STATUS = None
    rng = np.random.default_rng(5)
    for trial in range(3):
        ids = rng.integers(0, R if trial else 3, n)  # trial 0: three hot rows
        idx.copy_(torch.as_tensor(ids))
        graph.replay()
        torch.cuda.synchronize()
        assert int(status) == 0, f"replay {trial}: fr_embedding_bwd status {int(status)}"
        ref = O.embedding_bwd_f64(ids, G.cpu().numpy(), R)
        scale = O.embedding_bwd_f64(ids, np.abs(G.cpu().numpy()), R)
        assert np.all(np.abs(W.grad.double().cpu().numpy() - ref) <= 1e-5 * scale + 1e-6)


# ----------------------------------------------------------------------------- Linear weight grad
@pytest.mark.parametrize("M,N,K", [(20480, 192, 64), (20480, 64, 64), (20480, 256, 64), (20480, 64, 256),
                                   (1024, 64, 2048), (1000, 12, 20), (77, 4, 8)])
def test_linear_wgrad_matches_fp64(cuda, M, N, K):
    """fr_linear_wgrad vs fp64: |err| <= 1e-5 * sum_m |dY||X| + 1e-6 (fp32 slab sums); bit-identical
    on a second launch (fixed slab order)."""
    from FoodRec.engine import native
    g = torch.Generator().manual_seed(M + N + K)
    dY = torch.randn(M, N, generator=g)
    X = torch.randn(M, K, generator=g)
    lib = native.lib()
    ws = native.workspace(lib.fr_linear_wgrad_workspace(M, N, K), cuda)
    dYg, Xg = dY.to(cuda), X.to(cuda)
    outs = []
    for _ in range(2):
        dW = torch.full((N, K), float("nan"), device=cuda)
        db = torch.full((N,), float("nan"), device=cuda)
        native.check(lib.fr_linear_wgrad(dYg.data_ptr(), N, Xg.data_ptr(), K, M, N, K, dW.data_ptr(), K,
                                         db.data_ptr(), ws.data_ptr(), ws.numel(),
                                         torch.cuda.current_stream().cuda_stream), "fr_linear_wgrad")
        outs.append((dW.cpu(), db.cpu()))
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref = dY.double().t() @ X.double()
    scale = dY.double().abs().t() @ X.double().abs()
    assert torch.all((outs[0][0].double() - ref).abs() <= 1e-5 * scale + 1e-6)
    refb = dY.double().sum(0)
    assert torch.all((outs[0][1].double() - refb).abs() <= 1e-5 * dY.double().abs().sum(0) + 1e-6)


def test_engine_encoder_layer_gpu(cuda):
    """The engine TransformerEncoderLayer at HealthRec's shape (20 x 1024 tokens, d=64) vs torch's
    module with the same weights: outputs rel 1e-5, every gradient within 1e-4 * max|grad|."""
    import torch.nn as nn
    from FoodRec.engine import layers
    torch.manual_seed(0)
    ref = nn.TransformerEncoder(nn.TransformerEncoderLayer(64, 2, 256, dropout=0.0, activation="gelu"),
                                num_layers=2, enable_nested_tensor=False).to(cuda)
    torch.manual_seed(0)
    eng = nn.TransformerEncoder(layers.TransformerEncoderLayer(64, 2, 256, dropout=0.0, activation="gelu"),
                                num_layers=2, enable_nested_tensor=False).to(cuda)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(20, 1024, 64, generator=g).to(cuda)
    mask = (torch.rand(1024, 20, generator=g) < 0.5).to(cuda)
    mask[:, 0] = False
    xr, xe = x.clone().requires_grad_(True), x.clone().requires_grad_(True)
    yr = ref(xr, src_key_padding_mask=mask)
    ye = eng(xe, src_key_padding_mask=mask)
    torch.testing.assert_close(ye, yr, rtol=1e-5, atol=1e-5)
    w = torch.randn(yr.shape, generator=g).to(cuda)
    (yr * w).sum().backward()
    (ye * w).sum().backward()
    pairs = [("x", xr.grad, xe.grad)] + [(n, pr.grad, pe.grad) for (n, pr), (_, pe) in
                                         zip(ref.named_parameters(), eng.named_parameters())]
    for name, a, b in pairs:
        assert (a - b).abs().max() <= 1e-4 * a.abs().max() + 1e-6, name


# ----------------------------------------------------------------------------- LayerNorm
@pytest.mark.parametrize("rows,d,eps,affine", [(20480, 64, 1e-5, True), (40960, 32, 1e-12, True),
                                              (4096, 32, 1e-12, True), (777, 256, 1e-5, True),
                                              (1000, 16, 1e-5, False), (0, 64, 1e-5, True)])
def test_layernorm_matches_fp64(cuda, rows, d, eps, affine):
    """ops.layer_norm (fr_layernorm_fwd/_bwd) vs float64 F.layer_norm: y and dx within 2e-5 * max,
    dgamma/dbeta within 1e-5 * sum|terms|; deterministic (second backward bit-identical)."""
    from FoodRec.engine import ops
    g = torch.Generator().manual_seed(rows + d)
    x = torch.randn(rows, d, generator=g) * 3 + 1
    w = torch.randn(d, generator=g) if affine else None
    b = torch.randn(d, generator=g) if affine else None
    gy = torch.randn(rows, d, generator=g)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True) if affine else None
    br = b.double().requires_grad_(True) if affine else None
    yr = torch.nn.functional.layer_norm(xr, (d,), wr, br, eps)
    yr.backward(gy.double())
    grads = []
    for _ in range(2):
        xg = x.to(cuda).requires_grad_(True)
        wg = w.to(cuda).requires_grad_(True) if affine else None
        bg = b.to(cuda).requires_grad_(True) if affine else None
        y = ops.layer_norm(xg, (d,), wg, bg, eps)
        y.backward(gy.to(cuda))
        grads.append((y.detach().cpu(), xg.grad.cpu(), None if wg is None else wg.grad.cpu(),
                      None if bg is None else bg.grad.cpu()))
    for a, c in zip(grads[0], grads[1]):
        assert (a is None and c is None) or torch.equal(a, c)
    y, dx, dw, db = grads[0]
    if rows == 0:
        return
    assert (y.double() - yr.detach()).abs().max() <= 2e-5 * yr.detach().abs().max()
    assert (dx.double() - xr.grad).abs().max() <= 2e-5 * xr.grad.abs().max()
    if affine:
        xhat = torch.nn.functional.layer_norm(x.double(), (d,), None, None, eps)
        sw = (gy.double().abs() * xhat.abs()).sum(0)
        assert torch.all((dw.double() - wr.grad).abs() <= 1e-5 * sw + 1e-6)
        assert torch.all((db.double() - br.grad).abs() <= 1e-5 * gy.double().abs().sum(0) + 1e-6)


def test_spmm_ex_split_rows_mask_bitwise(cuda):
    """fr_spmm_csr_ex against fr_spmm_csr on the concatenated tables: split X / A1 / Y2 ([lo ; hi]
    at a row) and a column mask over an X that is zero outside the mask bit for bit; the row-list
    mode (listed rows only, duplicates allowed, heavy rows spread over the workgroup) to fp32
    rounding and run-to-run identical."""
    from FoodRec.engine import ops
    n, d, split = 1500, 64, 600
    r, c = _graph(n, n, 8, heavy=[(3, 1400), (700, 900), (11, 129)], seed=21)
    adj = _adj(n, r, c, cuda, chunk=128)
    assert adj.n_split >= 2
    lo = torch.randn(split, d, device=cuda)
    hi = torch.randn(n - split + 37, d, device=cuda)   # longer than needed: only rows < n - split are read
    X = torch.cat([lo, hi[:n - split]])
    full = torch.empty(n, d, device=cuda)
    ops.spmm_launch(adj, X, Y2=full, alpha=0.5, A1=X, beta1=0.5)
    y = torch.empty(n, d, device=cuda)
    ops.spmm_ex(adj, lo, hi, split, Y2=y, alpha=0.5, A1=lo, A1_hi=hi, beta1=0.5)
    assert torch.equal(y, full)
    # split output
    out_lo, out_hi = torch.empty(split, d, device=cuda), torch.empty(n - split, d, device=cuda)
    ops.spmm_ex(adj, X, Y2=out_lo, Y2_hi=out_hi, split=split, alpha=0.5, A1=X, beta1=0.5)
    assert torch.equal(torch.cat([out_lo, out_hi]), full)
    # row list: three segments with offsets and duplicates, heavy rows included
    a = torch.tensor([3, 5, 3, 0], device=cuda)
    b = torch.tensor([100, 200, 1], device=cuda)
    e = torch.tensor([899, 11], device=cuda)
    ry = torch.full((n, d), float("nan"), device=cuda)
    ops.spmm_ex(adj, lo, hi, split, Y2=ry, alpha=0.5, A1=lo, A1_hi=hi, beta1=0.5,
                rows=[(a, 0), (b, split), (e, 1)], region="spmm_rows")
    listed = torch.unique(torch.cat([a, b + split, e + 1]))
    # row-list rows: deterministic, summed in another order than the full launch (fp32 rounding)
    torch.testing.assert_close(ry[listed], full[listed], rtol=1e-5, atol=1e-6)
    ry2 = torch.full((n, d), float("nan"), device=cuda)
    ops.spmm_ex(adj, lo, hi, split, Y2=ry2, alpha=0.5, A1=lo, A1_hi=hi, beta1=0.5,
                rows=[(a, 0), (b, split), (e, 1)], region="spmm_rows")
    assert torch.equal(ry2[listed], ry[listed])
    others = torch.ones(n, dtype=torch.bool, device=cuda)
    others[listed] = False
    assert torch.isnan(ry[others]).all()
    # column mask: X zero outside the marked rows
    mask = torch.zeros(n, dtype=torch.uint8, device=cuda)
    ops.rows_mark(mask, [(a, 0), (b, split)], 1)
    assert int(mask.sum()) == len(set([3, 5, 0] + [100 + split, 200 + split, 1 + split]))
    Xs = X * mask.unsqueeze(1).float()
    ref = torch.empty(n, d, device=cuda)
    ops.spmm_launch(adj, Xs, Y2=ref, alpha=0.5, A1=Xs, beta1=0.5)
    got = torch.empty(n, d, device=cuda)
    ops.spmm_ex(adj, Xs, Y2=got, alpha=0.5, A1=Xs, beta1=0.5, col_mask=mask)
    assert torch.equal(got, ref)
    ops.rows_mark(mask, [(a, 0), (b, split)], 0)
    assert int(mask.sum()) == 0


@pytest.mark.parametrize("planned", [False, True])
@pytest.mark.parametrize("frac", [0.01, 0.6])
def test_spmm_sparse_upstream(cuda, frac, planned, monkeypatch):
    """fr_spmm_sparse_upstream against fr_spmm_csr over the zero-filled upstream: X is garbage (NaN)
    outside the marked rows and never read there; heavy rows span several 1024-edge scan rounds;
    split output; bitmask set and cleared by fr_rows_mark_zero.  ``planned``: the edge-balanced
    block plan (fr_spmm_sparse_upstream_blocks) with a 256-edge budget, so the heavy rows (1400 and
    900 edges) run as chunks added atomically onto their initialised rows.  Float-atomic order:
    fp32 rounding."""
    from FoodRec.engine import ops
    if planned:
        monkeypatch.setattr(ops, "SPARSE_PLAN_TRIGGER", 0)
        monkeypatch.setattr(ops, "SPARSE_BLOCK_EDGES", 256)
    n, d, split = 1500, 64, 600
    r, c = _graph(n, n, 8, heavy=[(3, 1400), (700, 900), (11, 129)], seed=23)
    adj = _adj(n, r, c, cuda, chunk=128)
    g = torch.Generator().manual_seed(int(frac * 100))
    marked = torch.unique(torch.randint(0, n, (max(1, int(frac * n)),), generator=g)).to(cuda)
    marked = torch.cat([marked, torch.tensor([3, 700, n - 1], device=cuda)])
    mask = torch.zeros(n, dtype=torch.uint8, device=cuda)
    bits = torch.zeros((n + 31) // 32, dtype=torch.int32, device=cuda)
    X = torch.full((n, d), float("nan"), device=cuda)
    ops.rows_mark(mask, [(marked, 0)], 1, zero=X, bits=bits)
    keep = mask.bool()
    X[keep] = torch.randn(int(keep.sum()), d, device=cuda)
    want = torch.tensor([sum(1 << b for b in range(32) if w * 32 + b < n and bool(keep[w * 32 + b]))
                         for w in range(bits.numel())], dtype=torch.int64)
    assert torch.equal(bits.cpu().to(torch.int64) & 0xFFFFFFFF, want)
    Xz = torch.where(keep.unsqueeze(1), X, torch.zeros_like(X))
    ref = torch.empty(n, d, device=cuda)
    ops.spmm_launch(adj, Xz, Y2=ref, alpha=0.5, A1=Xz, beta1=0.5)
    lo, hi = torch.full((split, d), 7.0, device=cuda), torch.full((n - split, d), 7.0, device=cuda)
    side = torch.full((777, 64), 3.0, device=cuda)  # the launch's side job zeroes it (no memset node)
    ops.spmm_sparse_upstream(adj, bits, X, lo, hi, split, alpha=0.5, beta1=0.5, zero=side)
    assert not side.any()
    got = torch.cat([lo, hi])
    assert torch.isfinite(got).all()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    assert (ops._sparse_plan(adj) is not None) == planned
    ops.rows_mark(mask, [(marked, 0)], 0, bits=bits)
    assert int(mask.sum()) == 0 and int(bits.abs().sum()) == 0


@pytest.mark.parametrize("planned", [False, True])
def test_spmm_sparse_rect(cuda, planned, monkeypatch):
    """fr_spmm_sparse_upstream_rect (a rectangular [rows x cols] slice, X marked by column, A1 read
    at every row) against fr_spmm_csr over the zero-filled X, uniform 64-row blocks and the
    edge-balanced plan with heavy rows chunked (fr_spmm_sparse_upstream_blocks, ungated).  The
    row-sharded config-4 step's first backward layer (engine/sharded.py)."""
    from FoodRec.engine import ops
    from FoodRec.engine.graph import Adjacency
    if planned:
        monkeypatch.setattr(ops, "SPARSE_PLAN_TRIGGER", 0)
        monkeypatch.setattr(ops, "SPARSE_BLOCK_EDGES", 200)
    R, C, d = 900, 1300, 64
    g = torch.Generator().manual_seed(41)
    deg = torch.randint(0, 12, (R,), generator=g)
    deg[[5, 400, 899]] = torch.tensor([1100, 700, 450])
    rp = torch.zeros(R + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(deg, 0)
    col = torch.cat([torch.sort(torch.randperm(C, generator=g)[:int(k)]).values for k in deg]).to(torch.int32)
    val = torch.rand(int(rp[-1]), generator=g)
    adj = Adjacency(rp.to(cuda), col.to(cuda), val.to(cuda), (R, C), device=cuda, symmetric=False)
    marked = torch.unique(torch.randint(0, C, (200,), generator=g)).to(cuda)
    bits = torch.zeros((C + 31) // 32, dtype=torch.int32, device=cuda)
    cmask = torch.zeros(C, dtype=torch.uint8, device=cuda)
    ops.rows_mark(cmask, [(marked, 0)], 1, bits=bits)
    X = torch.full((C, d), float("nan"), device=cuda)
    X[marked] = torch.randn(marked.numel(), d, device=cuda)
    Xz = torch.where(cmask.bool().unsqueeze(1), X, torch.zeros_like(X))
    A1 = torch.randn(R, d, device=cuda)
    ref = torch.empty(R, d, device=cuda)
    ops.spmm_launch(adj, Xz, Y2=ref, alpha=0.5, A1=A1, beta1=0.25)
    got = torch.full((R, d), 7.0, device=cuda)
    ops.spmm_sparse_rect(adj, bits, X, got, alpha=0.5, A1=A1, beta1=0.25)
    assert torch.isfinite(got).all()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-5)
    assert (ops._sparse_plan(adj) is not None) == planned


@pytest.mark.parametrize("bad", ["rows65", "edges"])
def test_spmm_sparse_plan_guard(cuda, bad):
    """A hand-made block plan the sparse-upstream kernel cannot run -- a 65-row block (its LDS row
    accumulator holds fr_spmm_sparse_block_rows() = 64), or a block whose edge range leaves its rows --
    is refused by the kernel: the block computes nothing (its rows keep their sentinel), the valid
    blocks are exact, and fr_spmm_plan_status reports it (then reads 0 once cleared).  The host plan
    builder refuses the same plan before it reaches the device."""
    from FoodRec.engine import native, ops
    lib = native.lib()
    limit = ops.sparse_block_rows()
    assert limit == 64
    lib.fr_spmm_plan_status(1)
    R, C, d = 300, 200, 64
    g = torch.Generator().manual_seed(5)
    deg = torch.randint(1, 6, (R,), generator=g)
    rp = torch.zeros(R + 1, dtype=torch.int64)
    rp[1:] = torch.cumsum(deg, 0)
    col = torch.cat([torch.sort(torch.randperm(C, generator=g)[:int(k)]).values for k in deg]).to(torch.int32)
    val = torch.rand(int(rp[-1]), generator=g)
    from FoodRec.engine.graph import Adjacency
    adj = Adjacency(rp.to(cuda), col.to(cuda), val.to(cuda), (R, C), device=cuda, symmetric=False)
    bits = torch.zeros((C + 31) // 32, dtype=torch.int32, device=cuda)
    cmask = torch.zeros(C, dtype=torch.uint8, device=cuda)
    ops.rows_mark(cmask, [(torch.arange(C, device=cuda), 0)], 1, bits=bits)
    X = torch.randn(C, d, device=cuda)
    ref = torch.empty(R, d, device=cuda)
    ops.spmm_launch(adj, X, Y2=ref, alpha=1.0)
    rpn = rp.numpy()
    cuts = [0, 64, 128 + (bad == "rows65"), 192, 256, R]  # (rows65: the second block has 65 rows)
    blocks = [(a, b, rpn[a], rpn[b]) for a, b in zip(cuts[:-1], cuts[1:])]
    if bad == "edges":
        blocks[1] = (64, 128, rpn[64], rpn[130])
    bad_rows = slice(64, cuts[2])
    plan_np = np.asarray(blocks, dtype=np.int64)
    with pytest.raises(native.EngineError):
        ops.check_sparse_plan(plan_np, rpn, limit)
    plan = (torch.from_numpy(plan_np).to(cuda), torch.zeros(0, dtype=torch.int64, device=cuda))
    got = torch.full((R, d), 7.0, device=cuda)
    ops._sparse_blocks(adj, True, bits, X, got, None, 0, 1.0, None, 0.0, plan)
    torch.cuda.synchronize()
    status = lib.fr_spmm_plan_status(1)
    assert status == (1 if bad == "rows65" else 2)
    assert lib.fr_spmm_plan_status(0) == 0
    keep = torch.ones(R, dtype=torch.bool)
    keep[bad_rows] = False
    assert bool((got[~keep.to(cuda)] == 7.0).all())
    torch.testing.assert_close(got[keep.to(cuda)], ref[keep.to(cuda)], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("frac", [0.02, 0.3])
def test_spmm_scatter_upstream(cuda, frac):
    """fr_spmm_scatter_upstream (scatter from the listed rows' own CSR rows, symmetric A) against
    fr_spmm_csr over the zero-filled upstream: listed rows with duplicates across three segments and
    a negative id (no row), X garbage (NaN) outside them, heavy rows, split output; the listed rows'
    bits are clear afterwards.  Float-atomic order: fp32 rounding."""
    from FoodRec.engine import ops
    n, d, split = 1500, 64, 600
    r, c = _graph(n, n, 8, heavy=[(3, 1400), (700, 900), (11, 129)], seed=29)
    adj = _adj(n, r, c, cuda, chunk=128)
    assert adj.symmetric
    g = torch.Generator().manual_seed(int(frac * 100) + 1)
    a = torch.randint(0, split, (max(1, int(frac * n)),), generator=g).to(cuda)
    b = torch.randint(0, n - split, (max(1, int(frac * n)),), generator=g).to(cuda)
    # third segment: duplicates of the second, a negative id (no row) and the heavy row 700
    rows = [(a, 0), (b, split), (torch.cat([b[:5], torch.tensor([-1, 700 - split], device=cuda)]), split)]
    mask = torch.zeros(n, dtype=torch.uint8, device=cuda)
    bits = torch.zeros((n + 31) // 32, dtype=torch.int32, device=cuda)
    X = torch.full((n, d), float("nan"), device=cuda)
    ops.rows_mark(mask, rows, 1, zero=X, bits=bits)
    keep = mask.bool()
    X[keep] = torch.randn(int(keep.sum()), d, device=cuda)
    Xz = torch.where(keep.unsqueeze(1), X, torch.zeros_like(X))
    ref = torch.empty(n, d, device=cuda)
    ops.spmm_launch(adj, Xz, Y2=ref, alpha=0.5, A1=Xz, beta1=0.5)
    lo, hi = torch.full((split, d), 7.0, device=cuda), torch.full((n - split, d), 7.0, device=cuda)
    ops.spmm_scatter_upstream(adj, mask, bits, rows, X, lo, hi, split, alpha=0.5, beta1=0.5)
    got = torch.cat([lo, hi])
    assert torch.isfinite(got).all()
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)
    assert int(bits.abs().sum()) == 0  # claimed rows cleared their bits
    ops.rows_mark(mask, rows, 0, bits=bits)
    assert int(mask.sum()) == 0


@pytest.mark.parametrize("front", [(True, True), (True, False), (False, False)])
def test_healthrec_graph_bpr_matches_unfused(cuda, front, monkeypatch):
    """ops.graph_bpr (split-table propagation, UI rows of the batch only, masked UI backward,
    gradients written into the parameters' buffers) against the concatenated full propagation +
    fused BPR op it replaces: losses rel 1e-6, every gradient 1e-5 of its max.  ``front``: the RI
    forward at the frontier item rows only / the RI backward's ingredient rows scattered from them."""
    from helpers import golden, tiny_config, tiny_data
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import ops
    from FoodRec.models import healthrec
    from FoodRec.utils.utils import get_model, init_seed
    monkeypatch.setattr(ops, "RI_FRONTIER", front[0])
    monkeypatch.setattr(ops, "RI_FRONTIER_BWD", front[1])
    g = golden("model_CIKM_Model.npz")
    batch = {k[len("batch/"):]: torch.from_numpy(g[k]).to(cuda) for k in g.files if k.startswith("batch/")}
    runs = []
    for fused in (True, False):
        healthrec.FUSED_GRAPH = fused
        try:
            cfg = tiny_config("CIKM_Model", True)
            data = tiny_data(cfg)
            init_seed(999)
            model = get_model("CIKM_Model")(cfg, data).to(cuda)
            tr = Trainer(cfg, model)
            tr.optimizer.zero_grad()
            losses = model.calculate_loss(batch)
            sum(losses).backward()
            tr.optimizer.materialize_row_grads()
            runs.append(([float(x.detach().reshape(-1)[0]) for x in losses],
                         {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}))
        finally:
            healthrec.FUSED_GRAPH = True
    (la, ga), (lb, gb) = runs
    np.testing.assert_allclose(la, lb, rtol=1e-6)
    assert ga.keys() == gb.keys()
    for k in ga:
        err = (ga[k] - gb[k]).abs().max().item()
        assert err <= 1e-5 * gb[k].abs().max().item() + 1e-9, (k, err)


@pytest.mark.parametrize("det", [False, True])
def test_views_sum_gather_bwd_heavy_duplicates(cuda, det, monkeypatch):
    """fr_views_sum_gather_bwd with ids drawn from 40 rows (every row hit ~25 times): vs a float64
    scatter reference; deterministic mode bit-identical across runs (sorted, ordered adds)."""
    from FoodRec.engine import ops
    monkeypatch.setattr(ops, "_DETERMINISTIC", det)
    g = torch.Generator().manual_seed(5)
    n, m, V = 3001, 1000, 3
    views = [torch.randn(n, 64, generator=g).to(cuda).requires_grad_(True) for _ in range(V)]
    ids = torch.randint(0, 40, (m,), generator=g).to(cuda)
    gs = torch.randn(n, 64, generator=g)
    gr = [torch.randn(m, 64, generator=g) for _ in range(V)]
    runs = []
    for _ in range(2):
        for v in views:
            v.grad = None
        total, gathered = ops.views_sum_gather(views, ids)
        torch.autograd.backward([total] + gathered, [gs.to(cuda)] + [x.to(cuda) for x in gr])
        runs.append([v.grad.clone() for v in views])
    if det:
        for a, b in zip(*runs):
            assert torch.equal(a, b)
    ic = ids.cpu()
    for k in range(V):
        ref = gs.double().clone().index_add_(0, ic, gr[k].double())
        torch.testing.assert_close(runs[0][k].cpu().double(), ref, rtol=0, atol=2e-5)


def test_ssl_and_bpr_weights_in_kernel(cuda):
    """dcor_loss / infonce_pairs (weight) and bpr_emb_loss (w_emb): the weighted loss equals the fp32
    product w * (unweighted loss) bit for bit, and the gradients equal those of the multiply form
    (the same products in the same order: bit-identical; the BPR scatter in its deterministic mode)."""
    from FoodRec.engine import ops
    from FoodRec.models.clussl import _DCOR_PAIRS
    g = torch.Generator().manual_seed(3)
    w = 0.037
    views0 = [torch.randn(1024, 64, generator=g).to(cuda) for _ in range(3)]
    for fn in (lambda vs, wt: ops.dcor_loss(vs, _DCOR_PAIRS, weight=wt),
               lambda vs, wt: ops.infonce_pairs(vs, _DCOR_PAIRS, 0.5, weight=wt)):
        va = [v.clone().requires_grad_(True) for v in views0]
        vb = [v.clone().requires_grad_(True) for v in views0]
        la = fn(va, w)
        lb = w * fn(vb, 1.0)
        assert torch.equal(la.detach(), lb.detach())
        la.sum().backward()
        lb.sum().backward()
        for a, b in zip(va, vb):
            assert torch.equal(a.grad, b.grad)
    U = torch.randn(500, 64, generator=g).to(cuda)
    E = [torch.randn(300, 64, generator=g).to(cuda) for _ in range(2)]
    u = torch.randint(0, 200, (256,), generator=g).to(cuda)
    p, n = (torch.randint(0, 300, (256,), generator=g).to(cuda) for _ in range(2))
    res = []
    for weighted in (True, False):
        Ug = U.clone().requires_grad_(True)
        Eg = [e.clone().requires_grad_(True) for e in E]
        if weighted:
            mf, reg = ops.bpr_emb_loss(Ug, None, Eg[0], Eg[1], u, p, n, item_offset=200, w_emb=w, deterministic=True)
        else:
            mf, reg = ops.bpr_emb_loss(Ug, None, Eg[0], Eg[1], u, p, n, item_offset=200, deterministic=True)
            reg = w * reg
        (mf + reg.sum()).backward()
        res.append((mf.detach(), reg.detach(), Ug.grad, Eg[0].grad, Eg[1].grad))
    for a, b in zip(*res):
        assert torch.equal(a, b)


def test_propagate_mean_split_matches_cat(cuda):
    """ops.propagate_mean_split(adj, lo, hi) vs propagate_mean(adj, cat([lo, hi])): bit-identical
    output and gradients (the same SpMM launches, split addressing)."""
    from FoodRec.engine import ops
    from FoodRec.engine.graph import Adjacency
    g = torch.Generator().manual_seed(11)
    nu, ni, e = 700, 900, 9000
    r = torch.randint(0, nu, (e,), generator=g)
    c = torch.randint(0, ni, (e,), generator=g) + nu
    rows, cols = torch.cat([r, c]), torch.cat([c, r])
    deg = torch.bincount(rows, minlength=nu + ni).clamp(min=1).float()
    vals = deg[rows].rsqrt() * deg[cols].rsqrt()
    adj = Adjacency.from_coo(rows, cols, vals, (nu + ni, nu + ni), device=cuda)
    lo0, hi0 = torch.randn(nu, 64, generator=g).to(cuda), torch.randn(ni, 64, generator=g).to(cuda)
    G = torch.randn(nu + ni, 64, generator=g).to(cuda)
    for L in (1, 2, 3):
        la, ha = lo0.clone().requires_grad_(True), hi0.clone().requires_grad_(True)
        lb, hb = lo0.clone().requires_grad_(True), hi0.clone().requires_grad_(True)
        ya = ops.propagate_mean_split(adj, la, ha, L)
        yb = ops.propagate_mean(adj, torch.cat([lb, hb]), L)
        assert torch.equal(ya, yb), L
        (ya * G).sum().backward()
        (yb * G).sum().backward()
        assert torch.equal(la.grad, lb.grad) and torch.equal(ha.grad, hb.grad), L


def test_ui_bpr_matches_unfused(cuda):
    """ops.ui_bpr (UI layer at the batch rows + BPR + EmbLoss, sparse-upstream backward) vs
    propagate_mean_split + bpr_emb_loss on the same inputs: losses rel 1e-6, every gradient within
    1e-5 of its max (float-atomic summation orders differ)."""
    from FoodRec.engine import ops
    from FoodRec.engine.graph import Adjacency
    g = torch.Generator().manual_seed(21)
    U, I, e = 600, 900, 8000
    r = torch.randint(0, U, (e,), generator=g)
    c = torch.randint(0, I, (e,), generator=g) + U
    rows, cols = torch.cat([r, c]), torch.cat([c, r])
    deg = torch.bincount(rows, minlength=U + I).clamp(min=1).float()
    adj = Adjacency.from_coo(rows, cols, deg[rows].rsqrt() * deg[cols].rsqrt(), (U + I, U + I), device=cuda)
    t0 = [torch.randn(U, 64, generator=g), torch.randn(I, 64, generator=g), torch.randn(I, 64, generator=g)]
    u = torch.randint(0, U, (256,), generator=g).to(cuda)
    p, n = (torch.randint(0, I, (256,), generator=g).to(cuda) for _ in range(2))
    res = []
    for fused in (True, False):
        uw, hi, iw = (x.clone().to(cuda).requires_grad_(True) for x in t0)
        if fused:
            mf, reg = ops.ui_bpr(adj, uw, hi, iw, u, p, n, w_emb=0.01)
        else:
            ui = ops.propagate_mean_split(adj, uw, hi, 1)
            mf, reg = ops.bpr_emb_loss(ui, None, uw, iw, u, p, n, item_offset=U, w_emb=0.01)
        (mf + reg.sum()).backward()
        res.append((mf.detach(), reg.detach(), uw.grad, hi.grad, iw.grad))
    (ma, ra, *ga), (mb, rb, *gb) = res
    torch.testing.assert_close(ma, mb, rtol=1e-6, atol=0)
    torch.testing.assert_close(ra, rb, rtol=1e-6, atol=0)
    for a, b in zip(ga, gb):
        assert (a - b).abs().max() <= 1e-5 * b.abs().max() + 1e-9


def test_emb_rows_into_views_matches_dense(cuda, monkeypatch):
    """CLUSSL's step shape: item views (propagate_lo_views, one side table with a padding row) summed
    into ui_bpr's item input.  The EmbLoss item rows parked by ui_bpr and added by the views' backward
    (one launch that also zeroes the padding row) vs ui_bpr's dense zero-filled item gradient summed
    by autograd: every gradient within 1e-5 of its max, the padding row exactly zero."""
    from FoodRec.engine import ops
    from FoodRec.engine.graph import Adjacency
    g = torch.Generator().manual_seed(23)
    U, I, S, e = 500, 700, 90, 6000
    r = torch.randint(0, U, (e,), generator=g)
    c = torch.randint(0, I, (e,), generator=g) + U
    rows, cols = torch.cat([r, c]), torch.cat([c, r])
    deg = torch.bincount(rows, minlength=U + I).clamp(min=1).float()
    ui = Adjacency.from_coo(rows, cols, deg[rows].rsqrt() * deg[cols].rsqrt(), (U + I, U + I), device=cuda)
    ui.mark_bipartite(U)
    sides = []
    for seed in (1, 2):
        ri, si = _graph(I, S, 3.0, seed=seed)
        a = _adj(I + S, ri, si + I, cuda)
        a.mark_bipartite(I)
        sides.append(a)
    t0 = [torch.randn(U, 64, generator=g), torch.randn(I, 64, generator=g), torch.randn(S + 1, 64, generator=g),
          torch.randn(S, 64, generator=g)]
    u = torch.randint(0, U, (256,), generator=g).to(cuda)
    p, n = (torch.randint(0, I, (256,), generator=g).to(cuda) for _ in range(2))
    res = []
    for into_views in (True, False):
        monkeypatch.setattr(ops, "EMB_ROWS_INTO_VIEWS", into_views)
        uw, iw, s1, s2 = (x.clone().to(cuda).requires_grad_(True) for x in t0)
        v1, v2 = ops.propagate_lo_views(sides, iw, [s1, s2], 2)
        mf, reg = ops.ui_bpr(ui, uw, v1 + v2, iw, u, p, n, w_emb=0.01)
        (mf + reg.sum()).backward()
        res.append((uw.grad, iw.grad, s1.grad, s2.grad))
    for a, b in zip(*res):
        assert (a - b).abs().max() <= 1e-5 * b.abs().max() + 1e-9
    assert torch.equal(res[0][2][S:], torch.zeros(1, 64, device=cuda))


@pytest.mark.parametrize("n_items", [2051, 4096])
def test_rows_frontier_and_list_scatter(cuda, n_items):
    """fr_rows_frontier: the list holds exactly the batch users' item columns and the batch items
    (each once), the mark buffer is left zero, for item counts off and on the compaction's
    4-item / 1024-item granules.  fr_spmm_list_scatter over that list on a bipartite RI graph:
    (alpha A X)[split:] for an X zero outside the list, vs float64, with Y's garbage zeroed first."""
    from FoodRec.engine import native
    lib = native.lib()
    s = native.stream_of(torch.empty(0, device=cuda))
    U, I, B = 300, n_items, 128
    r, c = _graph(U, I, 6.0, seed=11)
    ui = _adj(U + I, r, c + U, cuda)
    g = torch.Generator().manual_seed(2)
    u = torch.randint(0, U, (B,), generator=g)
    p, n = (torch.randint(0, I, (B,), generator=g) for _ in range(2))
    mark = torch.zeros(I, dtype=torch.uint8, device=cuda)
    lst = torch.full((I,), -7, dtype=torch.int32, device=cuda)
    cnt = torch.full((1,), 99, dtype=torch.int32, device=cuda)
    ud, pd, nd = (x.to(cuda) for x in (u, p, n))
    for _ in range(2):  # the second call starts from the mark buffer the first left behind
        native.check(lib.fr_rows_frontier(ui.rowptr.data_ptr(), ui.col.data_ptr(), U, I, ud.data_ptr(), pd.data_ptr(),
                                          nd.data_ptr(), B, mark.data_ptr(), lst.data_ptr(), cnt.data_ptr(), s),
                     "fr_rows_frontier")
        torch.cuda.synchronize()
        k = int(cnt.item())
        rp, col = ui.rowptr.cpu(), ui.col.cpu()
        want = set(p.tolist()) | set(n.tolist())
        for x in u.tolist():
            want |= {int(cc) - U for cc in col[int(rp[x]):int(rp[x + 1])].tolist() if cc >= U}
        got = lst[:k].cpu().tolist()
        assert len(got) == len(set(got)) and set(got) == want
        assert int(mark.sum()) == 0
    NI = 700
    r2, c2 = _graph(I, NI, 5.0, seed=12)
    ri = _adj(I + NI, r2, c2 + I, cuda)
    X = torch.zeros(I, 64)
    X[torch.tensor(got, dtype=torch.int64)] = torch.randn(len(got), 64, generator=g)
    Y = torch.full((NI + 1, 64), 3.5, device=cuda)
    alpha = 1.0 / 3.0
    Xd = X.to(cuda)
    native.check(lib.fr_spmm_list_scatter(ri.rowptr.data_ptr(), ri.col.data_ptr(), ri.val.data_ptr(), I + NI, I,
                                          lst.data_ptr(), cnt.data_ptr(), I, Xd.data_ptr(), 64, Y.data_ptr(), 64,
                                          alpha, 1, s), "fr_spmm_list_scatter")
    torch.cuda.synchronize()
    A = torch.sparse_csr_tensor(ri.rowptr.cpu(), ri.col.cpu().long(), ri.val.cpu().double(),
                                (I + NI, I + NI)).to_dense()
    ref = alpha * (A @ torch.cat([X.double(), torch.zeros(NI, 64, dtype=torch.float64)]))[I:]
    torch.testing.assert_close(Y[:NI].cpu().double(), ref, rtol=0, atol=2e-6)
    assert torch.equal(Y[NI:].cpu(), torch.full((1, 64), 3.5))  # rows past n_rows - split untouched
