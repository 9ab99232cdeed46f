"""BERT-style Transformer blocks of the reference's common/module.py (SCHGN's ingredient encoder).

Same classes, constructor signatures, sub-module names and parameters (so ``state_dict`` keys and
the seeded initialisation order match: ``layer.<k>.attention.{query,key,value,dense,LayerNorm}``,
``layer.<k>.intermediate.{dense_1,dense_2,LayerNorm}``), same arithmetic:

  SelfAttention   (module.py:43-111)  scores = q k^T / sqrt(head) + mask; softmax; dropout; @ v;
                                      dense; dropout; LayerNorm(. + input)
  Intermediate    (:114-136)          dense_2(act(dense_1(x))); dropout; LayerNorm(. + input)
  Layer / Encoder (:139-199)          attention then intermediate, stacked; returns the list of
                                      every layer's output (or only the last)
  LayerNorm       (:32-40)            TF-style, epsilon inside the square root
  MLPLayers       (:202-263)          [Dropout, Linear, ReLU]* (optionally BatchNorm1d)

Used only by SCHGN (models/schgn.py:11,57-64); not on the HealthRec hot path.
"""
from __future__ import annotations

import copy
import math

import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.init import normal_


def gelu(x):
    """erf GELU, x * Phi(x)."""
    return 0.5 * x * (1.0 + torch.erf(x / math.sqrt(2.0)))


def swish(x):
    return x * torch.sigmoid(x)


ACT2FN = {"gelu": gelu, "relu": F.relu, "swish": swish}


class LayerNorm(nn.Module):
    """Layer normalisation with the epsilon inside the square root (TF style)."""

    def __init__(self, hidden_size, eps=1e-12):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(hidden_size), requires_grad=True)
        self.bias = nn.Parameter(torch.zeros(hidden_size), requires_grad=True)
        self.variance_epsilon = eps

    def forward(self, x):
        mean = x.mean(-1, keepdim=True)
        var = (x - mean).pow(2).mean(-1, keepdim=True)
        return self.weight * ((x - mean) / torch.sqrt(var + self.variance_epsilon)) + self.bias


class SelfAttention(nn.Module):
    def __init__(self, n_heads, hidden_size, hidden_dropout_prob, attn_dropout_prob, layer_norm_eps):
        super().__init__()
        if hidden_size % n_heads != 0:
            raise ValueError("The hidden size (%d) is not a multiple of the number of attention heads (%d)"
                             % (hidden_size, n_heads))
        self.num_attention_heads = n_heads
        self.attention_head_size = hidden_size // n_heads
        self.all_head_size = n_heads * self.attention_head_size
        self.sqrt_attention_head_size = math.sqrt(self.attention_head_size)
        # construction order fixes the seeded initialisation (query, key, value, dense, LayerNorm)
        self.query = nn.Linear(hidden_size, self.all_head_size)
        self.key = nn.Linear(hidden_size, self.all_head_size)
        self.value = nn.Linear(hidden_size, self.all_head_size)
        self.softmax = nn.Softmax(dim=-1)
        self.attn_dropout = nn.Dropout(attn_dropout_prob)
        self.dense = nn.Linear(hidden_size, hidden_size)
        self.LayerNorm = nn.LayerNorm(hidden_size, eps=layer_norm_eps)
        self.out_dropout = nn.Dropout(hidden_dropout_prob)

    def transpose_for_scores(self, x):
        """[B, L, H*D] -> [B, H, L, D]"""
        return x.view(*x.shape[:-1], self.num_attention_heads, self.attention_head_size).permute(0, 2, 1, 3)

    def forward(self, input_tensor, attention_mask):
        q = self.transpose_for_scores(self.query(input_tensor))
        k = self.transpose_for_scores(self.key(input_tensor))
        v = self.transpose_for_scores(self.value(input_tensor))
        scores = torch.matmul(q, k.transpose(-1, -2)) / math.sqrt(self.attention_head_size)
        probs = self.attn_dropout(self.softmax(scores + attention_mask))
        ctx = torch.matmul(probs, v).permute(0, 2, 1, 3).contiguous()
        ctx = ctx.view(*ctx.shape[:-2], self.all_head_size)
        return self.LayerNorm(self.out_dropout(self.dense(ctx)) + input_tensor)


class Intermediate(nn.Module):
    def __init__(self, hidden_size, inner_size, hidden_dropout_prob, hidden_act, layer_norm_eps):
        super().__init__()
        self.dense_1 = nn.Linear(hidden_size, inner_size)
        self.intermediate_act_fn = ACT2FN[hidden_act] if isinstance(hidden_act, str) else hidden_act
        self.dense_2 = nn.Linear(inner_size, hidden_size)
        self.LayerNorm = nn.LayerNorm(hidden_size, eps=layer_norm_eps)
        self.dropout = nn.Dropout(hidden_dropout_prob)

    def forward(self, input_tensor):
        h = self.dense_2(self.intermediate_act_fn(self.dense_1(input_tensor)))
        return self.LayerNorm(self.dropout(h) + input_tensor)


class Layer(nn.Module):
    def __init__(self, n_heads, hidden_size, intermediate_size, hidden_dropout_prob, attn_dropout_prob, hidden_act,
                 layer_norm_eps):
        super().__init__()
        self.attention = SelfAttention(n_heads, hidden_size, hidden_dropout_prob, attn_dropout_prob, layer_norm_eps)
        self.intermediate = Intermediate(hidden_size, intermediate_size, hidden_dropout_prob, hidden_act,
                                         layer_norm_eps)

    def forward(self, hidden_states, attention_mask):
        return self.intermediate(self.attention(hidden_states, attention_mask))


class Encoder(nn.Module):
    """``n_layers`` deep copies of one Layer (all copies start from the same initial weights, as
    in the reference)."""

    def __init__(self, n_layers=2, n_heads=2, hidden_size=64, inner_size=256, hidden_dropout_prob=0.5,
                 attn_dropout_prob=0.5, hidden_act="gelu", layer_norm_eps=1e-12):
        super().__init__()
        proto = Layer(n_heads, hidden_size, inner_size, hidden_dropout_prob, attn_dropout_prob, hidden_act,
                      layer_norm_eps)
        self.layer = nn.ModuleList([copy.deepcopy(proto) for _ in range(n_layers)])

    def forward(self, hidden_states, attention_mask, output_all_encoded_layers=True):
        outs = []
        for layer_module in self.layer:
            hidden_states = layer_module(hidden_states, attention_mask)
            if output_all_encoded_layers:
                outs.append(hidden_states)
        if not output_all_encoded_layers:
            outs.append(hidden_states)
        return outs


class MLPLayers(nn.Module):
    """[Dropout(p), Linear(in, out), (BatchNorm1d), ReLU] per consecutive pair of ``layers``; the
    last ReLU is dropped when ``last_activation`` is False and ``activation`` is not None.
    ``init_method='norm'`` draws Linear weights from N(0, 0.01) and zeroes the biases."""

    def __init__(self, layers, dropout=0.0, activation="relu", bn=False, init_method=None, last_activation=True):
        super().__init__()
        self.layers = layers
        self.dropout = dropout
        self.activation = activation
        self.use_bn = bn
        self.init_method = init_method
        mods = []
        for fan_in, fan_out in zip(layers[:-1], layers[1:]):
            mods.append(nn.Dropout(p=dropout))
            mods.append(nn.Linear(fan_in, fan_out))
            if bn:
                mods.append(nn.BatchNorm1d(num_features=fan_out))
            mods.append(nn.ReLU())  # the reference appends ReLU whatever `activation` names
        if activation is not None and not last_activation:
            mods.pop()
        self.mlp_layers = nn.Sequential(*mods)
        if init_method is not None:
            self.apply(self.init_weights)

    def init_weights(self, module):
        if isinstance(module, nn.Linear):
            if self.init_method == "norm":
                normal_(module.weight.data, 0, 0.01)
            if module.bias is not None:
                module.bias.data.fill_(0.0)

    def forward(self, input_feature):
        return self.mlp_layers(input_feature)
