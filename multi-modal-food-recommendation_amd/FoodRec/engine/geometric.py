"""``torch_geometric.nn.GCNConv`` provider on the HIP SpMM (SCHGN's graph layer).

SCHGN (models/schgn.py:6,29-41) does ``import torch_geometric as geometric`` and builds
``geometric.nn.GCNConv(64, 64)``; torch_geometric is absent from this image.  When it is not
importable, :func:`install` registers a minimal ``torch_geometric`` / ``torch_geometric.nn`` exposing
this GCNConv, so the reference model file imports unchanged; an installed torch_geometric always
wins.  Restated from PyG's documented GCNConv (parity unpinned: no PyG here to compare against):

  * parameters: ``lin.weight`` [out, in] (PyG ``Linear(bias=False, weight_initializer='glorot')``:
    U(-a, a), a = sqrt(6 / (in + out))) and ``bias`` [out] (zeros).  As in PyG, the weight is drawn
    twice at construction (Linear's own reset, then GCNConv.reset_parameters), which fixes the
    seeded RNG consumption.
  * forward(x, edge_index, edge_weight=None), flow source_to_target, aggr 'add':
      add_remaining_self_loops (fill 1, or 2 if improved; an existing loop keeps its weight),
      deg[i] = sum of the weights of edges into i, w_e = deg^-1/2[src] * w_e * deg^-1/2[dst]
      (inf -> 0), out[i] = sum_e w_e * (x W^T)[src_e] + bias.
    The normalised graph is a CSR over targets (rows) resident in HBM; the aggregation is one
    ``fr_spmm_csr`` launch (ops.spmm, backward = transposed CSR), deterministic in edge order.
  * the normalised graph is cached per module: reused without a check when ``cached=True`` (PyG's
    contract), otherwise reused while the next call's edge_index has the same values.
"""
from __future__ import annotations

import importlib.util
import math
import sys
import types

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import ops
from .graph import Adjacency


def glorot_(w: torch.Tensor) -> None:
    """torch_geometric.nn.inits.glorot."""
    a = math.sqrt(6.0 / (w.size(-2) + w.size(-1)))
    with torch.no_grad():
        w.uniform_(-a, a)


class Linear(nn.Module):
    """torch_geometric.nn.Linear as GCNConv uses it: weight [out, in], glorot init, optional bias
    (zeros).  Not an nn.Linear subclass, as in PyG (models' ``isinstance(m, nn.Linear)`` init hooks
    skip it)."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = True, weight_initializer: str = "glorot"):
        super().__init__()
        if weight_initializer != "glorot":
            raise NotImplementedError("only weight_initializer='glorot' is provided")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.weight = nn.Parameter(torch.empty(out_channels, in_channels))
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        glorot_(self.weight)
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)


def gcn_norm(edge_index: torch.Tensor, edge_weight, num_nodes: int, improved: bool = False,
             add_self_loops: bool = True, flow: str = "source_to_target", dtype=torch.float32):
    """torch_geometric.nn.conv.gcn_conv.gcn_norm for a [2, E] edge_index -> (edge_index, weight)."""
    fill = 2.0 if improved else 1.0
    dev = edge_index.device
    if edge_weight is None:
        edge_weight = torch.ones(edge_index.size(1), dtype=dtype, device=dev)
    if add_self_loops:
        keep = edge_index[0] != edge_index[1]
        loop_w = torch.full((num_nodes,), fill, dtype=edge_weight.dtype, device=dev)
        loops = ~keep
        if bool(loops.any()):
            loop_w[edge_index[0][loops]] = edge_weight[loops]
        ar = torch.arange(num_nodes, device=dev)
        edge_index = torch.cat([edge_index[:, keep], torch.stack([ar, ar])], dim=1)
        edge_weight = torch.cat([edge_weight[keep], loop_w])
    row, col = edge_index[0], edge_index[1]
    idx = col if flow == "source_to_target" else row
    deg = torch.zeros(num_nodes, dtype=edge_weight.dtype, device=dev).scatter_add_(0, idx, edge_weight)
    dinv = deg.pow(-0.5)
    dinv.masked_fill_(dinv == float("inf"), 0.0)
    return edge_index, dinv[row] * edge_weight * dinv[col]


class GCNConv(nn.Module):
    def __init__(self, in_channels: int, out_channels: int, improved: bool = False, cached: bool = False,
                 add_self_loops=None, normalize: bool = True, bias: bool = True, **kwargs):
        super().__init__()
        aggr = kwargs.pop("aggr", "add")
        self.flow = kwargs.pop("flow", "source_to_target")
        kwargs.pop("node_dim", None)
        if aggr != "add" or self.flow not in ("source_to_target", "target_to_source") or kwargs:
            raise NotImplementedError(f"GCNConv options not provided by the engine: aggr={aggr}, "
                                      f"flow={self.flow}, {sorted(kwargs)}")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.improved, self.cached, self.normalize = improved, cached, normalize
        self.add_self_loops = normalize if add_self_loops is None else add_self_loops
        self.lin = Linear(in_channels, out_channels, bias=False, weight_initializer="glorot")
        if bias:
            self.bias = nn.Parameter(torch.empty(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        self.lin.reset_parameters()
        if self.bias is not None:
            with torch.no_grad():
                self.bias.zero_()
        self.__dict__["_fr_graph"] = None

    def _graph(self, edge_index, edge_weight, num_nodes: int) -> Adjacency:
        hit = self.__dict__.get("_fr_graph")
        if hit is not None:
            ei, ew, n, adj = hit
            if self.cached or (n == num_nodes and ei.shape == edge_index.shape and ei.device == edge_index.device
                               and torch.equal(ei, edge_index)
                               and ((ew is None and edge_weight is None)
                                    or (ew is not None and edge_weight is not None and torch.equal(ew, edge_weight)))):
                return adj
        if self.normalize:
            ei_n, w = gcn_norm(edge_index, edge_weight, num_nodes, self.improved, self.add_self_loops, self.flow)
        else:
            ei_n = edge_index
            w = edge_weight if edge_weight is not None else torch.ones(edge_index.size(1), device=edge_index.device)
        # messages flow src -> dst: a CSR over dst rows with src columns
        src, dst = (ei_n[0], ei_n[1]) if self.flow == "source_to_target" else (ei_n[1], ei_n[0])
        adj = Adjacency.from_coo(dst, src, w.to(torch.float32), (num_nodes, num_nodes), symmetric=False,
                                 device=edge_index.device)
        self.__dict__["_fr_graph"] = (edge_index.detach().clone(),
                                      None if edge_weight is None else edge_weight.detach().clone(), num_nodes, adj)
        return adj

    def forward(self, x, edge_index, edge_weight=None):
        if not torch.is_tensor(edge_index) or edge_index.dim() != 2 or edge_index.size(0) != 2:
            raise NotImplementedError("GCNConv: a [2, E] edge_index tensor is required (no SparseTensor)")
        adj = self._graph(edge_index, edge_weight, x.size(0))
        out = ops.spmm(adj, self.lin(x))
        if self.bias is not None:
            out = out + self.bias
        return out

    def __repr__(self):
        return f"GCNConv({self.in_channels}, {self.out_channels})"


def install() -> bool:
    """Register this provider as ``torch_geometric`` when the real package is not importable.
    Returns True if the engine provider is (now) the one bound to ``torch_geometric``."""
    mod = sys.modules.get("torch_geometric")
    if mod is not None:
        return bool(getattr(mod, "__fr_engine__", False))
    if importlib.util.find_spec("torch_geometric") is not None:
        return False
    pkg = types.ModuleType("torch_geometric")
    pkg.__doc__ = "FoodRec MI355X engine provider of torch_geometric.nn.GCNConv (torch_geometric not installed)"
    pkg.__fr_engine__ = True
    nn_mod = types.ModuleType("torch_geometric.nn")
    nn_mod.GCNConv = GCNConv
    nn_mod.Linear = Linear
    pkg.nn = nn_mod
    sys.modules["torch_geometric"] = pkg
    sys.modules["torch_geometric.nn"] = nn_mod
    return True
