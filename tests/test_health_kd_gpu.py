"""Fused HealthRec loss head (fr_health_kd_fwd / _bwd) vs the oracle.

Replaces health_mlp + sigmoid + BCELoss-sum and 1 - cosine_similarity(...).mean() through norm_loss,
both weighted (cikm_model.py:249-264, 304-308).  Oracle: oracle.ops.health_kd_f64 (the reference's
formula in float64 torch-CPU, gradients by autograd).

Tolerances (fp32 wave sums vs float64):
  loss terms           : |err| <= 2e-5 * |ref| + 1e-6
  gradients            : |err| <= 1e-4 * max|ref grad| + 1e-7
"""
import pytest
import torch

from oracle import ops as O

pytestmark = pytest.mark.gpu


def _inputs(n, H, seed):
    g = torch.Generator().manual_seed(seed)
    f = lambda *s, sc=1.0: torch.randn(*s, generator=g, dtype=torch.float64) * sc
    hin, know, rows = f(n, 64, sc=0.5), f(n, 64), f(n, 64)
    rows[:, :8] += know[:, :8]  # some correlation: mean cosine away from 0
    labels = (torch.rand(n, H, generator=g, dtype=torch.float64) < 0.35).to(torch.float64)
    w1, b1 = f(64, 64, sc=0.125), f(64, sc=0.1)
    w2, b2 = f(H, 64, sc=0.125), f(H, sc=0.1)
    return [hin, know, rows, labels, w1, b1, w2, b2]


def _oracle(x, thr, wh, wk, gh, gk):
    x = [t.clone().requires_grad_(i != 3) for i, t in enumerate(x)]
    h, k = O.health_kd_f64(*x, thr, wh, wk)
    (h * gh + k * gk).backward()
    return h.detach(), k.detach(), [None if i == 3 else t.grad for i, t in enumerate(x)]


def _engine(x, thr, wh, wk, gh, gk, cuda):
    from FoodRec.engine import ops
    xs = [t.to(cuda, torch.float32).requires_grad_(i != 3) for i, t in enumerate(x)]
    mlp = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.ReLU(), torch.nn.Linear(64, x[3].shape[1])).to(cuda)
    with torch.no_grad():
        mlp[0].weight.copy_(xs[4]); mlp[0].bias.copy_(xs[5]); mlp[2].weight.copy_(xs[6]); mlp[2].bias.copy_(xs[7])
    h, k = ops.health_kd_loss(xs[0], xs[1], xs[2], xs[3], mlp, thr, wh, wk)
    (h * gh + k * gk).backward()
    grads = [xs[0].grad, xs[1].grad, xs[2].grad, None, mlp[0].weight.grad, mlp[0].bias.grad, mlp[2].weight.grad,
             mlp[2].bias.grad]
    return h.detach().cpu().double(), k.detach().cpu().double(), [None if t is None else t.cpu().double()
                                                                   for t in grads]


def _close(got, ref, rel, what):
    err = (got - ref).abs().max().item()
    bound = rel * max(ref.abs().max().item(), 1e-30) + (1e-6 if ref.dim() == 0 else 1e-7)
    assert err <= bound, f"{what}: max err {err:.3e} > {bound:.3e}"


@pytest.mark.parametrize("n,H,thr", [(1024, 7, 0.4), (1024, 7, 5.0), (37, 6, 0.1), (1, 16, -1.0), (300, 1, 0.2)])
def test_health_kd_matches_oracle(cuda, n, H, thr):
    x = _inputs(n, H, seed=n + H)
    wh, wk, gh, gk = 0.1, 0.05, 1.3, 0.7
    rh, rk, rg = _oracle(x, thr, wh, wk, gh, gk)
    eh, ek, eg = _engine(x, thr, wh, wk, gh, gk, cuda)
    _close(eh, rh, 2e-5, "health term")
    _close(ek, rk, 2e-5, "kd term")
    names = ["d_hin", "d_know", "d_rows", None, "dW1", "db1", "dW2", "db2"]
    for name, g, r in zip(names, eg, rg):
        if name is not None:
            _close(g, r, 1e-4, name)
    if thr >= 5.0:  # gate closed: no KD gradient at all
        assert eg[1].abs().max() == 0 and eg[2].abs().max() == 0 and ek.item() == 0


def test_health_kd_tie_halves_kd_gradient(cuda):
    """maximum(0, x) at x == 0 passes half the gradient (ATen's maximum backward): the threshold is
    set to the kernel's own fp32 kd value so the tie is exact."""
    from FoodRec.engine import ops
    x = _inputs(256, 7, seed=3)
    _, _, g_open = _engine(x, -10.0, 0.1, 0.05, 1.0, 1.0, cuda)
    xs = [t.to(cuda, torch.float32) for t in x]
    mlp = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.ReLU(), torch.nn.Linear(64, 7)).to(cuda)
    with torch.no_grad():
        mlp[0].weight.copy_(xs[4]); mlp[0].bias.copy_(xs[5]); mlp[2].weight.copy_(xs[6]); mlp[2].bias.copy_(xs[7])
    _, k = ops.health_kd_loss(xs[0], xs[1], xs[2], xs[3], mlp, 0.0, 0.1, 0.05)
    kd32 = k._base[2].item()  # the saved gate kd - 0: the kernel's fp32 kd
    _, k_tie, g_tie = _engine(x, kd32, 0.1, 0.05, 1.0, 1.0, cuda)
    if k_tie.item() != 0.0:
        pytest.skip("fp32 kd did not round-trip through the threshold exactly")
    for a, b in ((g_tie[1], g_open[1]), (g_tie[2], g_open[2])):
        torch.testing.assert_close(a, 0.5 * b, rtol=1e-6, atol=1e-9)


def test_health_kd_deterministic_and_reusable(cuda):
    """Bitwise-identical outputs and gradients over repeated launches (block-order sums; the
    forward's ticket word is re-zeroed by the kernel)."""
    x = _inputs(1024, 7, seed=11)
    first = _engine(x, 0.4, 0.1, 0.05, 1.0, 1.0, cuda)
    for _ in range(3):
        again = _engine(x, 0.4, 0.1, 0.05, 1.0, 1.0, cuda)
        assert torch.equal(first[0], again[0]) and torch.equal(first[1], again[1])
        for a, b in zip(first[2], again[2]):
            if a is not None:
                assert torch.equal(a, b)
