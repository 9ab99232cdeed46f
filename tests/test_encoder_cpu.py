"""CPU pins of the fused encoder's oracle (oracle.ops.encoder_layer_f64 / encoder_keep_masks).

With all-ones masks the restatement must equal torch's own nn.TransformerEncoderLayer (the module
the reference builds at cikm_model.py:33-35) in float64 -- forward and gradients -- so the GPU
tests in test_encoder_gpu.py compare the HIP kernels against torch's semantics.
"""
import numpy as np
import torch
import torch.nn as nn

from oracle import ops as O


def _torch_params(layer):
    m = layer.self_attn
    return [m.in_proj_weight, m.in_proj_bias, m.out_proj.weight, m.out_proj.bias, layer.norm1.weight,
            layer.norm1.bias, layer.linear1.weight, layer.linear1.bias, layer.linear2.weight, layer.linear2.bias,
            layer.norm2.weight, layer.norm2.bias]


def test_restatement_equals_torch_module():
    torch.manual_seed(0)
    layer = nn.TransformerEncoderLayer(64, 2, 256, dropout=0.0, activation="gelu").double()
    NS, L = 6, 20
    x = torch.randn(NS, L, 64, dtype=torch.float64)
    pad = torch.rand(NS, L) < 0.4
    pad[:, 0] = False
    ref = layer(x.transpose(0, 1), src_key_padding_mask=pad).transpose(0, 1)
    masks = O.encoder_keep_masks(1, 0, NS, L, (0.0,) * 4)
    fmask = torch.zeros(NS, L, dtype=torch.float64).masked_fill(pad, float("-inf"))
    out = O.encoder_layer_f64(x, fmask, _torch_params(layer), masks, (0.0,) * 4)
    torch.testing.assert_close(out, ref, rtol=1e-12, atol=1e-12)
    g = torch.randn_like(ref)
    gr = torch.autograd.grad((ref * g).sum(), _torch_params(layer))
    go = torch.autograd.grad((out * g).sum(), _torch_params(layer))
    for a, b in zip(go, gr):
        torch.testing.assert_close(a, b, rtol=1e-10, atol=1e-12)


def test_keep_masks_rate_and_independence():
    m = O.encoder_keep_masks(42, 3, 256, 20, (0.5, 0.25, 0.1, 0.0))
    assert abs(m[0].mean() - 0.5) < 0.01 and abs(m[1].mean() - 0.75) < 0.01
    assert abs(m[2].mean() - 0.9) < 0.01 and m[3].min() == 1.0
    m2 = O.encoder_keep_masks(43, 3, 256, 20, (0.5, 0.25, 0.1, 0.0))
    assert 0.45 < (m[0] != m2[0]).mean() < 0.55
    assert np.array_equal(O.encoder_keep_masks(42, 3, 256, 20, (0.5,) * 4)[0], m[0])
