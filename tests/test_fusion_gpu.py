"""Fused modal fusion (fr_modal_fusion_fwd / _bwd) vs the oracle.

Replaces HealthRec's two target attentions and the F.normalize heads (cikm_model.py:245-249,
311-369).  Oracle: oracle.ops.modal_fusion_f64, the reference's target_attention_layer restated in
float64 (torch-CPU).  The model-level goldens (test_models_gpu, CIKM_Model) also run through this op.

Tolerances (fp32 shuffle reductions / softmax vs float64):
  know, hin             : |err| <= 2e-5 * max|ref| + 1e-6
  d_enc, d_query, d_ln  : |err| <= 1e-4 * max|ref grad| + 1e-7
"""
import pytest
import torch

from oracle import ops as O

pytestmark = pytest.mark.gpu


def _inputs(n, L, pad_id, seed, scale=1.0):
    g = torch.Generator().manual_seed(seed)
    enc = torch.randn(n, L, 64, generator=g, dtype=torch.float64) * scale
    query = torch.randn(n, 2, 64, generator=g, dtype=torch.float64) * scale
    num = torch.randint(1, L + 1, (n,), generator=g)
    ids = torch.randint(0, pad_id, (n, L), generator=g)
    ids[torch.arange(L).view(1, L) >= num.view(n, 1)] = pad_id   # padded tails, as the dataset writes them
    ids[0] = pad_id  # an all-padded row: uniform attention, no NaN (as in the reference)
    ln = [1.0 + 0.2 * torch.randn(32, generator=g, dtype=torch.float64), 0.1 * torch.randn(32, generator=g,
                                                                                            dtype=torch.float64),
          1.0 + 0.2 * torch.randn(32, generator=g, dtype=torch.float64), 0.1 * torch.randn(32, generator=g,
                                                                                            dtype=torch.float64)]
    gk = torch.randn(n, 64, generator=g, dtype=torch.float64)
    gh = torch.randn(n, 64, generator=g, dtype=torch.float64)
    return enc, query, ids, num, ln, gk, gh


class _LN:
    def __init__(self, w, b, eps=1e-12):
        self.weight, self.bias, self.eps = w, b, eps


@pytest.mark.parametrize("n,L", [(1024, 20), (1023, 20), (37, 16), (9, 8), (5, 4)])
def test_modal_fusion_matches_f64(cuda, n, L):
    from FoodRec.engine import ops
    pad_id = 500
    enc, query, ids, num, ln, gk, gh = _inputs(n, L, pad_id, n + L)
    # reference (float64, autograd)
    er, qr = enc.clone().requires_grad_(True), query.clone().requires_grad_(True)
    lr_ = [p.clone().requires_grad_(True) for p in ln]
    kr, hr = O.modal_fusion_f64(er, qr, ids, num, pad_id, lr_[:2], lr_[2:])
    ((kr * gk).sum() + (hr * gh).sum()).backward()
    # fused (fp32 on the GPU)
    eg, qg = enc.float().to(cuda).requires_grad_(True), query.float().to(cuda).requires_grad_(True)
    lg = [p.float().to(cuda).requires_grad_(True) for p in ln]
    kg, hg = ops.modal_fusion(eg, qg, ids.to(cuda), num.to(cuda), pad_id, _LN(lg[0], lg[1]), _LN(lg[2], lg[3]))
    ((kg * gk.float().to(cuda)).sum() + (hg * gh.float().to(cuda)).sum()).backward()
    for name, a, b in (("know", kg, kr), ("hin", hg, hr)):
        a, b = a.detach().double().cpu(), b.detach()
        assert (a - b).abs().max() <= 2e-5 * b.abs().max() + 1e-6, name
    for name, a, b in [("d_enc", eg, er), ("d_query", qg, qr)] + [(f"d_ln{k}", lg[k], lr_[k]) for k in range(4)]:
        ga, gb = a.grad.double().cpu(), b.grad
        assert (ga - gb).abs().max() <= 1e-4 * gb.abs().max() + 1e-7, name


def test_modal_fusion_deterministic(cuda):
    from FoodRec.engine import ops
    enc, query, ids, num, ln, gk, gh = _inputs(300, 20, 77, 5)
    outs = []
    for _ in range(2):
        eg = enc.float().to(cuda).requires_grad_(True)
        lg = [p.float().to(cuda).requires_grad_(True) for p in ln]
        k, h = ops.modal_fusion(eg, query.float().to(cuda), ids.to(cuda), num.to(cuda), 77, _LN(lg[0], lg[1]),
                                _LN(lg[2], lg[3]))
        (k.sum() + 2 * h.sum()).backward()
        outs.append([k.detach(), h.detach(), eg.grad] + [p.grad for p in lg])
    for a, b in zip(*outs):
        assert torch.equal(a, b)
