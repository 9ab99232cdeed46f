"""Engine versions of torch.nn layers on the hot path, parameter-for-parameter identical.

``TransformerEncoderLayer`` is ``torch.nn.TransformerEncoderLayer`` (same constructor, parameters,
names, seeded initialisation, state_dict) whose training forward is the module's own post-norm path
-- ``norm1(x + dropout1(self_attn(x)))``, ``norm2(x + dropout2(linear2(dropout(act(linear1(x))))))``
with ``F.multi_head_attention_forward``'s self-attention steps (packed in-projection and its
[3, E] layout, key-padding mask merged per head, SDPA, out-projection) -- restated so the four
Linear layers go through ``ops.linear``: over the ingredient tokens (2B x 20 = 20480 rows at B=512)
their weight gradients are the split-K HIP kernel ``fr_linear_wgrad`` instead of ~100 us library
GEMMs.  The reference builds this layer at cikm_model.py:33-35 (d=64, nhead 2, FF 4d, post-norm,
sequence-first).  Configurations outside that path (norm_first, attn_mask, causal, batch_first,
eval / no-grad) run the torch module unchanged.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops

# HealthRec's shape (d=64, 2 heads, FF 256, L ingredient tokens) runs the fused HIP layer
# (ops.encoder_layer); FR_FUSED_ENCODER=0 keeps the unfused engine path for A/B comparisons.
FUSED_ENCODER = os.environ.get("FR_FUSED_ENCODER", "1") != "0"
_LAYER_ORDINAL = 0


class TransformerEncoderLayer(nn.TransformerEncoderLayer):
    def _engine_path(self, src, src_mask, is_causal) -> bool:
        mha = self.self_attn
        return (self.training and torch.is_grad_enabled() and src.is_cuda and src.dim() == 3
                and src.dtype == torch.float32 and not self.norm_first and src_mask is None
                and not is_causal and not mha.batch_first and mha._qkv_same_embed_dim
                and mha.in_proj_bias is not None and mha.bias_k is None and not mha.add_zero_attn)

    def forward(self, src, src_mask=None, src_key_padding_mask=None, is_causal=False):
        if not self._engine_path(src, src_mask, is_causal):
            return super().forward(src, src_mask=src_mask, src_key_padding_mask=src_key_padding_mask,
                                   is_causal=is_causal)
        kpm = F._canonical_mask(mask=src_key_padding_mask, mask_name="src_key_padding_mask",
                                other_type=None, other_name="", target_type=src.dtype)
        if self._fused_ok(src, kpm):
            # one fused HIP launch per direction (fr_encoder_fwd/_bwd); batch-first in memory, so the
            # model's permute(1, 0, 2) views cost no copies
            out = ops.encoder_layer(src.transpose(0, 1), kpm, self._fused_cfg(src.device), self._fused_params())
            return out.transpose(0, 1)
        x = src
        n1, n2 = self.norm1, self.norm2
        x = ops.layer_norm(x + self._engine_sa_block(x, kpm), n1.normalized_shape, n1.weight, n1.bias, n1.eps)
        x = ops.layer_norm(x + self._engine_ff_block(x), n2.normalized_shape, n2.weight, n2.bias, n2.eps)
        return x

    def _fused_params(self):
        mha = self.self_attn
        return (mha.in_proj_weight, mha.in_proj_bias, mha.out_proj.weight, mha.out_proj.bias,
                self.norm1.weight, self.norm1.bias, self.linear1.weight, self.linear1.bias,
                self.linear2.weight, self.linear2.bias, self.norm2.weight, self.norm2.bias)

    def _fused_ok(self, src, kpm) -> bool:
        L, NS, E = src.shape
        mha = self.self_attn
        return (FUSED_ENCODER and src.is_cuda and E == 64 and mha.num_heads == 2 and self.linear1.out_features == 256
                and L in ops.ENCODER_LENGTHS and getattr(self, "activation_relu_or_gelu", 0) in (1, 2)
                and mha.out_proj.bias is not None and self.linear1.bias is not None
                and self.linear2.bias is not None and self.norm1.bias is not None and self.norm2.bias is not None
                and (kpm is None or tuple(kpm.shape) == (NS, L))
                and all(p.dtype == torch.float32 and p.is_contiguous() for p in self._fused_params()))

    def _fused_cfg(self, device):
        cfg = self.__dict__.get("_fr_encoder_cfg")
        if cfg is None or cfg.counter.device != device:
            salt = self.__dict__.get("_fr_salt")  # the layer's index in its model (set by the model)
            if salt is None:
                global _LAYER_ORDINAL
                _LAYER_ORDINAL += 1
                salt = 1000 + _LAYER_ORDINAL
            # hash seed from the seeded torch state without consuming it (init parity), distinct per layer
            seed = (torch.initial_seed() * 0x9E3779B97F4A7C15 + salt + 1) & (2 ** 64 - 1)
            cfg = ops.EncoderConfig((self.norm1.eps, self.norm2.eps),
                                    (self.self_attn.dropout, self.dropout1.p, self.dropout.p, self.dropout2.p),
                                    self.activation_relu_or_gelu == 2, seed, device)
            self.__dict__["_fr_encoder_cfg"] = cfg
        return cfg

    def _engine_sa_block(self, x, kpm):
        mha = self.self_attn
        L, B, E = x.shape
        h = mha.num_heads
        hd = E // h
        proj = ops.linear(x, mha.in_proj_weight, mha.in_proj_bias)
        proj = proj.unflatten(-1, (3, E)).unsqueeze(0).transpose(0, -2).squeeze(-2).contiguous()
        q, k, v = proj[0], proj[1], proj[2]
        q = q.view(L, B * h, hd).transpose(0, 1)
        k = k.view(L, B * h, hd).transpose(0, 1)
        v = v.view(L, B * h, hd).transpose(0, 1)
        attn_mask = None
        if kpm is not None:
            attn_mask = kpm.view(B, 1, 1, L).expand(-1, h, -1, -1).reshape(B * h, 1, L)
            if attn_mask.size(0) == 1:
                attn_mask = attn_mask.unsqueeze(0)
            else:
                attn_mask = attn_mask.view(B, h, -1, L)
        q = q.view(B, h, L, hd)
        k = k.view(B, h, L, hd)
        v = v.view(B, h, L, hd)
        out = F.scaled_dot_product_attention(q, k, v, attn_mask, mha.dropout, False)
        out = out.permute(2, 0, 1, 3).contiguous().view(B * L, E)
        out = ops.linear(out, mha.out_proj.weight, mha.out_proj.bias).view(L, B, E)
        return self.dropout1(out)

    def _engine_ff_block(self, x):
        y = ops.linear(self.dropout(self.activation(ops.linear(x, self.linear1.weight, self.linear1.bias))),
                       self.linear2.weight, self.linear2.bias)
        return self.dropout2(y)


def run_encoder(encoder: nn.TransformerEncoder, src, src_key_padding_mask=None):
    """``encoder(src, src_key_padding_mask=...)`` for an nn.TransformerEncoder of engine layers
    (cikm_model.py:232): when every layer takes the fused path, the whole stack is ONE autograd node
    (ops.encoder_stack: each layer's weight-gradient reduction folded into the next backward launch);
    otherwise the module runs as is."""
    layers_ = list(encoder.layers)
    if (encoder.norm is None and layers_ and all(isinstance(m, TransformerEncoderLayer) for m in layers_)
            and all(m._engine_path(src, None, False) for m in layers_)):
        kpm = F._canonical_mask(mask=src_key_padding_mask, mask_name="src_key_padding_mask", other_type=None,
                                other_name="", target_type=src.dtype)
        if all(m._fused_ok(src, kpm) for m in layers_):
            out = ops.encoder_stack(src.transpose(0, 1), kpm, [m._fused_cfg(src.device) for m in layers_],
                                    [m._fused_params() for m in layers_])
            return out.transpose(0, 1)
    return encoder(src, src_key_padding_mask=src_key_padding_mask)
