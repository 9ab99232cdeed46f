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

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops


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
        x = src
        n1, n2 = self.norm1, self.norm2
        x = ops.layer_norm(x + self._engine_sa_block(x, kpm), n1.normalized_shape, n1.weight, n1.bias, n1.eps)
        x = ops.layer_norm(x + self._engine_ff_block(x), n2.normalized_shape, n2.weight, n2.bias, n2.eps)
        return x

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
