"""Fused HealthRec loss head (fr_modal_head_fwd / _bwd: target attentions + normalize heads + health
MLP / BCE + KD cosine as one node) vs the oracle and vs the two separate engine ops.

Replaces cikm_model.py:245-264 (+ 304-308, 311-369) after the ingredient encoder.  Oracle:
oracle.ops.modal_fusion_f64 feeding oracle.ops.health_kd_f64 (float64 torch-CPU, autograd).

Tolerances (fp32 wave sums / softmax vs float64):
  loss terms                    : |err| <= 2e-5 * |ref| + 1e-6
  every gradient                : |err| <= 1e-4 * max|ref grad| + 1e-7
  vs the separate engine ops    : losses rel 1e-6, gradients 1e-5 * max (the same per-item
                                  arithmetic; only block-partial summation orders differ)
"""
import pytest
import torch

from oracle import ops as O

pytestmark = pytest.mark.gpu


class _LN:
    def __init__(self, w, b, eps=1e-12):
        self.weight, self.bias, self.eps = w, b, eps


def _inputs(n, L, H, pad_id, seed):
    g = torch.Generator().manual_seed(seed)
    f = lambda *s, sc=1.0: torch.randn(*s, generator=g, dtype=torch.float64) * sc  # noqa: E731
    enc, query = f(n, L, 64), f(n, 2, 64)
    num = torch.randint(1, L + 1, (n,), generator=g)
    ids = torch.randint(0, pad_id, (n, L), generator=g)
    ids[torch.arange(L).view(1, L) >= num.view(n, 1)] = pad_id
    ln = [1.0 + 0.2 * f(32), 0.1 * f(32), 1.0 + 0.2 * f(32), 0.1 * f(32)]
    rows = f(n, 64)
    labels = (torch.rand(n, H, generator=g, dtype=torch.float64) < 0.35).to(torch.float64)
    mlp = [f(64, 64, sc=0.125), f(64, sc=0.1), f(H, 64, sc=0.125), f(H, sc=0.1)]
    return enc, query, ids, num, ln, rows, labels, mlp


def _oracle(x, pad_id, thr, wh, wk, gh, gk):
    enc, query, ids, num, ln, rows, labels, mlp = x
    er, qr, rr = (t.clone().requires_grad_(True) for t in (enc, query, rows))
    lr_ = [p.clone().requires_grad_(True) for p in ln]
    mr = [p.clone().requires_grad_(True) for p in mlp]
    know, hin = O.modal_fusion_f64(er, qr, ids, num, pad_id, lr_[:2], lr_[2:])
    h, k = O.health_kd_f64(hin, know, rr, labels, *mr, thr, wh, wk)
    (h * gh + k * gk).backward()
    return h.detach(), k.detach(), [er.grad, qr.grad, rr.grad] + [p.grad for p in lr_] + [p.grad for p in mr]


def _engine(x, pad_id, thr, wh, wk, gh, gk, cuda, fused=True):
    from FoodRec.engine import ops
    enc, query, ids, num, ln, rows, labels, mlp = x
    H = labels.shape[1]
    eg, qg, rg = (t.float().to(cuda).requires_grad_(True) for t in (enc, query, rows))
    lg = [p.float().to(cuda).requires_grad_(True) for p in ln]
    net = torch.nn.Sequential(torch.nn.Linear(64, 64), torch.nn.ReLU(), torch.nn.Linear(64, H)).to(cuda)
    with torch.no_grad():
        for p, v in zip((net[0].weight, net[0].bias, net[2].weight, net[2].bias), mlp):
            p.copy_(v)
    la, lb = _LN(lg[0], lg[1]), _LN(lg[2], lg[3])
    ig, ng, yg = ids.to(cuda), num.to(cuda), labels.float().to(cuda)
    if fused:
        h, k = ops.modal_head(eg, qg, ig, ng, pad_id, rg, yg, la, lb, net, thr, wh, wk)
    else:
        know, hin = ops.modal_fusion(eg, qg, ig, ng, pad_id, la, lb)
        h, k = ops.health_kd_loss(hin, know, rg, yg, net, thr, wh, wk)
    (h * gh + k * gk).backward()
    grads = [eg.grad, qg.grad, rg.grad] + [p.grad for p in lg] + [net[0].weight.grad, net[0].bias.grad,
                                                                    net[2].weight.grad, net[2].bias.grad]
    return h.detach().cpu().double(), k.detach().cpu().double(), [t.cpu().double() for t in grads]


NAMES = ["d_enc", "d_query", "d_rows", "d_ln_a.w", "d_ln_a.b", "d_ln_b.w", "d_ln_b.b", "dW1", "db1", "dW2", "db2"]


def _close(got, ref, rel, what, atol=1e-7):
    err = (got - ref).abs().max().item()
    bound = rel * max(ref.abs().max().item(), 1e-30) + atol
    assert err <= bound, f"{what}: max err {err:.3e} > {bound:.3e}"


@pytest.mark.parametrize("n,L,H,thr", [(1024, 20, 7, 0.4), (1024, 20, 7, 5.0), (37, 16, 16, 0.1), (5, 4, 1, -1.0),
                                       (1023, 20, 7, 0.2)])
def test_modal_head_matches_oracle(cuda, n, L, H, thr):
    pad_id = 500
    x = _inputs(n, L, H, pad_id, n + L + H)
    wh, wk, gh, gk = 0.1, 0.05, 1.3, 0.7
    rh, rk, rg = _oracle(x, pad_id, thr, wh, wk, gh, gk)
    eh, ek, eg = _engine(x, pad_id, thr, wh, wk, gh, gk, cuda)
    _close(eh, rh, 2e-5, "health term", 1e-6)
    _close(ek, rk, 2e-5, "kd term", 1e-6)
    for name, g, r in zip(NAMES, eg, rg):
        _close(g, r, 1e-4, name)
    if thr >= 5.0:  # gate closed: no KD gradient reaches the rows
        assert eg[2].abs().max() == 0 and ek.item() == 0


def test_modal_head_equals_separate_ops(cuda):
    """The fused node against ops.modal_fusion + ops.health_kd_loss (the path it replaces) on the
    same fp32 inputs: same per-item arithmetic, so only the partial summation order differs."""
    pad_id = 300
    x = _inputs(1024, 20, 7, pad_id, 5)
    a = _engine(x, pad_id, 0.3, 0.1, 0.05, 1.0, 1.0, cuda, fused=True)
    b = _engine(x, pad_id, 0.3, 0.1, 0.05, 1.0, 1.0, cuda, fused=False)
    _close(a[0], b[0], 1e-6, "health term", 0)
    _close(a[1], b[1], 1e-6, "kd term", 0)
    for name, ga, gb in zip(NAMES, a[2], b[2]):
        _close(ga, gb, 1e-5, name, 0)


@pytest.mark.parametrize("ticket", [False, True])
def test_modal_head_finalize_forms_equal(cuda, ticket, monkeypatch):
    """The finalize as its own launch or run by the forward's last-arriving block (FR_HEAD_TICKET):
    the same fixed-order sums, bit-identical losses; repeated launches (the ticket resets itself)."""
    from FoodRec.engine import ops
    pad_id = 211
    x = _inputs(1021, 20, 7, pad_id, 3)
    monkeypatch.setattr(ops, "HEAD_TICKET", False)
    ref = _engine(x, pad_id, 0.25, 0.1, 0.05, 1.0, 1.0, cuda)
    monkeypatch.setattr(ops, "HEAD_TICKET", ticket)
    for _ in range(3):
        got = _engine(x, pad_id, 0.25, 0.1, 0.05, 1.0, 1.0, cuda)
        assert torch.equal(got[0], ref[0]) and torch.equal(got[1], ref[1])


def test_modal_head_deterministic(cuda):
    pad_id = 77
    x = _inputs(300, 20, 5, pad_id, 9)
    first = _engine(x, pad_id, 0.2, 0.1, 0.05, 1.0, 1.0, cuda)
    again = _engine(x, pad_id, 0.2, 0.1, 0.05, 1.0, 1.0, cuda)
    assert torch.equal(first[0], again[0]) and torch.equal(first[1], again[1])
    for ga, gb in zip(first[2], again[2]):
        assert torch.equal(ga, gb)


def test_healthrec_loss_finalize_step_equals_separate_launches(cuda, monkeypatch):
    """A booked HealthRec trainer step with the loss terms finalized by one fr_healthrec_loss_finalize
    launch (head finalize + ingredient norms + EmbLoss assembly + the step's bookkeeping) vs the
    separate launches (FR_LOSS_FINALIZE=0: head finalize, reg_combine, fr_step_book): the same
    arithmetic, so in deterministic mode the booked loss sums, the returned loss and every parameter
    after three steps are bit-identical."""
    import numpy as np
    from helpers import tiny_config, tiny_data
    from FoodRec.common.trainer import Trainer
    from FoodRec.engine import ops
    from FoodRec.engine.sampler import TripleSampler
    from FoodRec.utils.utils import get_model, init_seed
    det0 = torch.are_deterministic_algorithms_enabled()
    runs = []
    try:
        torch.use_deterministic_algorithms(True, warn_only=True)
        for fused in (True, False):
            monkeypatch.setattr(ops, "LOSS_FINALIZE", fused)
            cfg = tiny_config("CIKM_Model", True, train_batch_size=32, cuda_graph=False, deterministic=True)
            data = tiny_data(cfg)
            init_seed(999)
            model = get_model("CIKM_Model")(cfg, data).to(cuda)
            tr = Trainer(cfg, model)
            np.random.seed(7)
            sampler = TripleSampler(data, 32, cuda)
            feats = tr._features()
            state = tr.new_step_state()
            model.train()
            losses = []
            for k, (u, p, n) in enumerate(sampler.epoch()):
                if k == 3:
                    break
                losses.append(float(tr.train_step(feats.batch(u, p, n), k, state)))
            tr.flush_optimizer()
            runs.append((state["acc"].cpu().numpy().copy(), losses,
                         {k: v.detach().clone() for k, v in model.state_dict().items()}))
            assert not ops._PENDING_HEAD and not ops._PENDING_NORMS
    finally:
        torch.use_deterministic_algorithms(det0)
    (aa, la, sa), (ab, lb, sb) = runs
    np.testing.assert_array_equal(aa, ab)
    assert la == lb
    for k in sa:
        assert torch.equal(sa[k], sb[k]), k
