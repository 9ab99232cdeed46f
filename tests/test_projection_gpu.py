"""Modal projections over gathered rows (fr_gather_linear_fwd, fr_linear_wgrad_gather, fr_rows_matmul)
vs float64 torch references of HealthRec's image_trs / text_trs over embImage / embText rows
(cikm_model.py:240-243).

Tolerances (fp32 MFMA / FMA vs float64):
  Y                        : |err| <= 1e-5 * max|ref| + 1e-6
  dW, db, table gradients  : |err| <= 1e-5 * max|ref| + 1e-7
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(n, Ks, R, seed, cuda):
    g = torch.Generator().manual_seed(seed)
    ids = torch.randint(0, R, (n,), generator=g)
    ids[: n // 4] = ids[n // 4: n // 2]  # duplicates: several positions per table row
    tabs = [torch.randn(R, K, generator=g) for K in Ks]
    lins = []
    for K in Ks:
        lin = torch.nn.Linear(K, 64)
        with torch.no_grad():
            lin.weight.copy_(torch.randn(64, K, generator=g) / K ** 0.5)
            lin.bias.copy_(torch.randn(64, generator=g))
        lins.append(lin.to(cuda))
    gy = torch.randn(n, len(Ks), 64, generator=g)
    return ids, tabs, lins, gy


def _ref(ids, tabs, lins, gy):
    outs, grads = [], []
    for t, (X, lin) in enumerate(zip(tabs, lins)):
        Xd = X.double().requires_grad_(True)
        W = lin.weight.detach().cpu().double().requires_grad_(True)
        b = lin.bias.detach().cpu().double().requires_grad_(True)
        Y = torch.nn.functional.linear(Xd[ids], W, b)
        (Y * gy[:, t].double()).sum().backward()
        outs.append(Y.detach())
        grads.append((Xd.grad, W.grad, b.grad))
    return torch.stack(outs, 1), grads


def _close(got, ref, rel, what):
    err = (got.double().cpu() - ref).abs().max().item()
    bound = rel * ref.abs().max().item() + 1e-7
    assert err <= bound, f"{what}: {err:.3e} > {bound:.3e}"


@pytest.mark.parametrize("n,Ks,R", [(1024, (2048, 512), 5000), (37, (512, 48), 90), (1, (16, 64), 3)])
def test_modal_projection_dense_matches_float64(cuda, n, Ks, R):
    from FoodRec.engine import ops
    ids, tabs, lins, gy = _setup(n, Ks, R, n, cuda)
    Y_ref, g_ref = _ref(ids, tabs, lins, gy)
    tg = [t.to(cuda).requires_grad_(True) for t in tabs]
    Y = ops.modal_projection(ids.to(cuda), list(zip(tg, lins)))
    (Y * gy.to(cuda)).sum().backward()
    _close(Y.detach(), Y_ref, 1e-5, "Y")
    for t in range(len(Ks)):
        _close(tg[t].grad, g_ref[t][0], 1e-5, f"table {t}")
        _close(lins[t].weight.grad, g_ref[t][1], 1e-5, f"dW {t}")
        _close(lins[t].bias.grad, g_ref[t][2], 1e-5, f"db {t}")
    # deterministic: the same launch twice is bitwise equal (tickets re-zeroed)
    Y2 = ops.modal_projection(ids.to(cuda), list(zip(tg, lins)))
    assert torch.equal(Y.detach(), Y2.detach())


def test_factored_row_gradients_match_dense(cuda):
    """FusedAdam's factored path: rmap + compact rows = per-id sum of dY times W (one row pass over
    both modalities' adjacent dY columns, fr_rows_matmul per table) equal the dense table gradient."""
    from FoodRec.engine import ops
    from FoodRec.engine.optim import FusedAdam
    from FoodRec.engine import native
    n, Ks, R = 1024, (2048, 512), 4000
    ids, tabs, lins, gy = _setup(n, Ks, R, 3, cuda)
    _, g_ref = _ref(ids, tabs, lins, gy)
    tg = [torch.nn.Parameter(t.to(cuda)) for t in tabs]
    opt = FusedAdam(tg + [p for lin in lins for p in lin.parameters()], lr=1e-3)
    Y = ops.modal_projection(ids.to(cuda), list(zip(tg, lins)), exchange=opt.row_grads)
    (Y * gy.to(cuda)).sum().backward()
    assert all(p.grad is None for p in tg) and len(opt.row_grads.factored) == 2
    prepared = opt._prepare_factored(native.lib())
    for t, p in enumerate(tg):
        tag, rmap, crow = prepared[id(p)][:3]
        rmap, crow = rmap.cpu().long(), crow.cpu().double()
        dense = torch.zeros(R, Ks[t], dtype=torch.float64)
        has = rmap >= 0
        dense[has] = crow[rmap[has]]
        assert set(torch.nonzero(has).flatten().tolist()) == set(ids.tolist())
        _close(dense, g_ref[t][0], 1e-5, f"factored table {t}")


@pytest.mark.parametrize("B,L,R", [(512, 20, 5000), (3, 7, 40)])
def test_embedding_norms_matches_float64(cuda, B, L, R):
    """ops.embedding_norms (fr_gather_norms_fwd / fr_norms_bwd_coef): E = W[ids] and the two halves'
    Frobenius norms (cikm_model.py:230, 270-279); gradient G + (gn_h / ||E_h||) E on non-padding
    positions, scattered per row -- vs float64 autograd of the same expression."""
    from FoodRec.engine import ops
    g = torch.Generator().manual_seed(B)
    pad = R - 1
    ids = torch.randint(0, R, (2 * B, L), generator=g)
    ids[:, L - 2:] = pad  # padded tails
    W = torch.randn(R, 64, generator=g)
    gE = torch.randn(2 * B, L, 64, generator=g)
    for gn in (torch.randn(2, generator=g), torch.full((2,), 0.7)):
        Wd = W.double().requires_grad_(True)
        Ed = Wd[ids]
        keep = (ids != pad).unsqueeze(-1).double()
        Ek = Ed * keep + (Ed * (1 - keep)).detach()  # padding positions: value counted, no gradient
        nrm_d = torch.stack([Ek[:B].reshape(-1).norm(), Ek[B:].reshape(-1).norm()])
        ((Ed * gE.double()).sum() + (nrm_d * gn.double()).sum()).backward()
        Wg = W.to(cuda).requires_grad_(True)
        E, nrm = ops.embedding_norms(ids.to(cuda), Wg, pad, B)
        gn_c = gn.to(cuda) if gn[0] != gn[1] else torch.tensor(0.7, device=cuda).expand(2)
        ((E * gE.to(cuda)).sum() + (nrm * gn_c).sum()).backward()
        _close(E.detach(), Ed.detach(), 1e-6, "E")
        _close(nrm.detach(), nrm_d.detach(), 1e-5, "norms")
        _close(Wg.grad, Wd.grad, 1e-5, "dW")
