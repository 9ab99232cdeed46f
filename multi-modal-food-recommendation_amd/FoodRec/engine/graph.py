"""Normalised adjacency in CSR + the torch.sparse.mm interception.

Builders restate the reference's dok/scipy construction vectorised (and on the GPU for large
graphs), value for value:

* ``get_norm_adj_mat`` (models/lightgcn.py:76-120 == cikm_model.py:136-180 == pricai_modelx.py:133-177):
  (U+I)^2 bipartite graph, user u -> column i+U plus the transpose, duplicates collapse to 1.
* ``get_norm_adj_recipe_ing`` / ``_infor`` (cikm_model.py:91-134, pricai_modelx.py:88-131):
  item <-> ingredient (or cluster) graph, node ids [0,I) items, [I, I+NI) ingredients.

deg_r = #nonzeros of row r + 1e-7 (float64);  val = fp32(deg_r^-1/2 * deg_c^-1/2)  (scipy D*A*D in
float64, then torch.FloatTensor).  Rows sorted, columns sorted within a row (the coo order of
the reference's ``sp.coo_matrix(L)``).

HBM layout: rowptr int64 [N+1], col int32 [nnz], val fp32 [nnz]; the work plan is
int32 {row, chunk} pairs (nnz-balanced units) + {row, first_partial, n_chunks} split-row triples.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import native

DEFAULT_CHUNK = None  # None: auto_chunk(nnz), widened by plain_chunk(rowptr)
# widest chunk plain_chunk() widens to: rows up to this degree are walked whole by one 16-lane group
PLAIN_MAX_DEGREE = 256 if os.environ.get("FR_PLAIN_CHUNK", "1") != "0" else 0


def auto_chunk(nnz: int) -> int:
    """Edges per SpMM work unit: the smallest power of two >= nnz / 16384, in [32, 1024].  A unit
    is gathered serially by one 16-lane group, so the heaviest unit bounds a small graph's launch
    (Allrecipes UI graph, 1.35M nnz, item rows up to ~3k edges: 135 us at 1024, 69 us at 128 on
    MI355X, tools/bench_spmm_small.py) while large graphs keep 1024-edge units (config 4)."""
    c = 32
    while c < 1024 and c * 16384 < nnz:
        c *= 2
    return c


def plain_chunk(chunk: int, max_degree: int) -> int:
    """Widen an auto chunk so that every row is one plain unit when no row is heavier than
    PLAIN_MAX_DEGREE edges.  A graph with no split rows runs the pipelined row walk
    (spmm_plain16_kernel) in one launch instead of the unit kernel plus the split-row fixup: the
    CLUSSL item-cluster and recipe-ingredient graphs (Foodcom shape, rows up to ~125 edges) had
    2,000-2,200 split rows at the auto chunk of 32/64.  Graphs with heavier rows keep the auto
    chunk (a heavy row in one unit would bound the launch, auto_chunk's note)."""
    if max_degree <= chunk or max_degree > PLAIN_MAX_DEGREE:
        return chunk
    c = chunk
    while c < max_degree:
        c *= 2
    return c


def _sym_keys_np(n_nodes: int, rows: np.ndarray, cols: np.ndarray) -> np.ndarray:
    rows = rows.astype(np.int64, copy=False)
    cols = cols.astype(np.int64, copy=False)
    n = np.int64(n_nodes)
    return np.unique(np.concatenate([rows * n + cols, cols * n + rows]))


def sym_norm_csr_np(n_nodes: int, rows, cols):
    """Symmetric D^-1/2 A D^-1/2 of the binary graph {(r,c)} U {(c,r)} -> CSR numpy arrays."""
    keys = _sym_keys_np(n_nodes, np.asarray(rows), np.asarray(cols))
    r = keys // n_nodes
    c = keys % n_nodes
    deg = np.bincount(r, minlength=n_nodes).astype(np.float64)
    dinv = np.power(deg + 1e-7, -0.5)
    val = (dinv[r] * dinv[c]).astype(np.float32)
    rowptr = np.zeros(n_nodes + 1, np.int64)
    np.cumsum(np.bincount(r, minlength=n_nodes), out=rowptr[1:])
    return rowptr, c.astype(np.int32), val


def sym_norm_csr_torch(n_nodes: int, rows: torch.Tensor, cols: torch.Tensor):
    """Same as :func:`sym_norm_csr_np` with torch ops (runs on the GPU for 10^8-edge graphs)."""
    n = int(n_nodes)
    rows = rows.to(torch.int64)
    cols = cols.to(torch.int64)
    keys = torch.cat([rows * n + cols, cols * n + rows])
    keys = torch.unique(keys, sorted=True)
    r = torch.div(keys, n, rounding_mode="floor")
    c = keys - r * n
    del keys
    cnt = torch.bincount(r, minlength=n)
    dinv = torch.pow(cnt.to(torch.float64) + 1e-7, -0.5)
    val = (dinv[r] * dinv[c]).to(torch.float32)
    rowptr = torch.zeros(n + 1, dtype=torch.int64, device=r.device)
    torch.cumsum(cnt, 0, out=rowptr[1:])
    return rowptr, c.to(torch.int32), val


def bipartite_norm_csr_torch(n_users: int, n_items: int, u: torch.Tensor, i: torch.Tensor):
    """Symmetric-normalised (U+I)^2 adjacency of a bipartite edge list, built on the device
    without symmetrising through a 2E-key sort: the user block comes from the (u,i)-sorted
    unique keys, the item block from one (i,u) sort.  Same values as sym_norm_csr_torch on
    (u, i+U): deg counts distinct neighbours, val = fp32(deg_r^-1/2 deg_c^-1/2) in float64."""
    U, I = int(n_users), int(n_items)
    key = torch.unique(u.to(torch.int64) * I + i.to(torch.int64), sorted=True)
    uu = torch.div(key, I, rounding_mode="floor")
    ii = key - uu * I
    del key
    deg_u = torch.bincount(uu, minlength=U)
    deg_i = torch.bincount(ii, minlength=I)
    dinv = torch.pow(torch.cat([deg_u, deg_i]).to(torch.float64) + 1e-7, -0.5)
    order = torch.argsort(ii * U + uu)
    iu_u = uu[order]
    del order
    col = torch.cat([(ii + U).to(torch.int32), iu_u.to(torch.int32)])
    row_u = uu
    val_u = (dinv[row_u] * dinv[ii + U]).to(torch.float32)
    del row_u
    ii_sorted = torch.repeat_interleave(torch.arange(I, device=u.device), deg_i)
    val_i = (dinv[ii_sorted + U] * dinv[iu_u]).to(torch.float32)
    val = torch.cat([val_u, val_i])
    rowptr = torch.zeros(U + I + 1, dtype=torch.int64, device=u.device)
    torch.cumsum(torch.cat([deg_u, deg_i]), 0, out=rowptr[1:])
    return rowptr, col, val


def ui_edges(inter_rows, inter_cols, n_users):
    """user-item interactions -> (row, col) of the upper block of the (U+I)^2 adjacency."""
    return inter_rows, inter_cols + n_users


def side_edges(triples, n_items):
    """(item, side-node) triples -> (side+I, item) as the reference's load_graph builds them."""
    t = np.asarray(triples)
    return t[:, 1].astype(np.int64) + n_items, t[:, 0].astype(np.int64)


class Adjacency:
    """A CSR normalised adjacency resident in HBM with its SpMM work plan.

    Stands in for the reference's ``torch.sparse.FloatTensor`` attributes: any
    ``torch.sparse.mm(adj, X)`` with an Adjacency first argument is routed to the HIP SpMM
    (``__torch_function__``), with autograd (backward = adj^T @ grad).
    """

    def __init__(self, rowptr, col, val, shape, chunk: int = DEFAULT_CHUNK, symmetric: bool = True,
                 device=None):
        device = torch.device(device) if device is not None else (
            rowptr.device if torch.is_tensor(rowptr) else torch.device("cpu"))
        self.shape = (int(shape[0]), int(shape[1]))
        self.symmetric = bool(symmetric)
        rp = torch.as_tensor(rowptr, dtype=torch.int64)
        self.rowptr = rp.to(device)
        self.col = torch.as_tensor(col, dtype=torch.int32).to(device)
        self.val = torch.as_tensor(val, dtype=torch.float32).to(device)
        self.nnz = int(self.col.numel())
        if chunk is None:
            max_deg = int((rp[1:] - rp[:-1]).max().item()) if rp.numel() > 1 else 0
            self.chunk = plain_chunk(auto_chunk(self.nnz), max_deg)
        else:
            self.chunk = int(chunk)
        self._build_plan(rp.cpu())
        self._t = None
        self.bipartite_split = None  # see mark_bipartite
        self.nnz_below_split = 0

    def mark_bipartite(self, split: int):
        """Declare that rows [0, split) have columns in [split, n) only and vice versa (a
        [[0, R], [R^T, 0]] graph such as the recipe-ingredient adjacency): the propagation then
        skips the output rows a layer is known not to need or to be zero at (ops.graph_bpr)."""
        split = int(split)
        if not 0 < split < self.shape[0] or self.shape[0] != self.shape[1]:
            raise ValueError("mark_bipartite: split must lie inside a square adjacency")
        self.bipartite_split = split
        self.nnz_below_split = int(self.rowptr[split].item())

    # ------------------------------------------------------------------ construction helpers
    @classmethod
    def from_coo(cls, rows, cols, vals, shape, **kw):
        rows = torch.as_tensor(rows, dtype=torch.int64)
        cols = torch.as_tensor(cols, dtype=torch.int64)
        vals = torch.as_tensor(vals, dtype=torch.float32)
        n = int(shape[1])
        key = rows.to(torch.int64) * n + cols
        order = torch.argsort(key, stable=True)
        rows, cols, vals = rows[order], cols[order], vals[order]
        # duplicates are summed (torch.sparse.mm on an uncoalesced tensor sums them)
        key = rows * n + cols
        uniq, inv = torch.unique_consecutive(key, return_inverse=True)
        if uniq.numel() != key.numel():
            v2 = torch.zeros(uniq.numel(), dtype=torch.float32, device=vals.device)
            v2.index_add_(0, inv, vals)
            rows = torch.div(uniq, n, rounding_mode="floor")
            cols = uniq - rows * n
            vals = v2
        cnt = torch.bincount(rows, minlength=int(shape[0]))
        rowptr = torch.zeros(int(shape[0]) + 1, dtype=torch.int64, device=rows.device)
        torch.cumsum(cnt, 0, out=rowptr[1:])
        sym = kw.pop("symmetric", None)
        if sym is None:
            sym = cls._is_symmetric(rows, cols, vals, shape)
        return cls(rowptr, cols.to(torch.int32), vals, shape, symmetric=sym, **kw)

    @classmethod
    def from_torch_sparse(cls, sp: torch.Tensor, **kw):
        """Convert a reference-style torch sparse COO matrix (e.g. model.norm_adj_matrix)."""
        sp = sp.coalesce()
        idx = sp.indices()
        return cls.from_coo(idx[0].cpu(), idx[1].cpu(), sp.values().float().cpu(), sp.shape,
                            device=kw.pop("device", sp.device), **kw)

    @classmethod
    def sym_normalized(cls, n_nodes, rows, cols, device=None, **kw):
        if torch.is_tensor(rows) and rows.is_cuda:
            rp, c, v = sym_norm_csr_torch(n_nodes, rows, cols)
        else:
            rp, c, v = sym_norm_csr_np(n_nodes, np.asarray(rows), np.asarray(cols))
        return cls(rp, c, v, (n_nodes, n_nodes), symmetric=True, device=device, **kw)

    @staticmethod
    def _is_symmetric(rows, cols, vals, shape) -> bool:
        if shape[0] != shape[1]:
            return False
        n = int(shape[1])
        k1 = rows * n + cols
        k2 = cols * n + rows
        o2 = torch.argsort(k2)
        return bool(torch.equal(k1, k2[o2]) and torch.equal(vals, vals[o2]))

    def _build_plan(self, rowptr_cpu: torch.Tensor):
        n = self.shape[0]
        lib = native.lib()
        rp = np.ascontiguousarray(rowptr_cpu.numpy(), dtype=np.int64)
        cap_units = n + (self.nnz // self.chunk) + 2
        units = np.empty((cap_units, 2), np.int32)
        splits = np.empty((max(n, 1), 3), np.int32)
        nu, npl, ns = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        native.check(lib.fr_spmm_plan_host(rp.ctypes.data, n, self.chunk, units.ctypes.data,
                                           ctypes.byref(nu), ctypes.byref(npl), splits.ctypes.data,
                                           ctypes.byref(ns)), "fr_spmm_plan_host")
        dev = self.rowptr.device
        self.units = torch.from_numpy(units[: nu.value].copy()).to(dev)
        self.split_rows = torch.from_numpy(splits[: ns.value].copy()).to(dev)
        self.n_units, self.n_plain, self.n_split = nu.value, npl.value, ns.value
        self.max_row_nnz = int((rp[1:] - rp[:-1]).max()) if n else 0

    def plan(self) -> native.FrSpmmPlan:
        return native.FrSpmmPlan(self.units.data_ptr(), self.split_rows.data_ptr(), self.n_units,
                                 self.n_plain, self.n_split, self.chunk)

    # ------------------------------------------------------------------ tensor-like surface
    @property
    def device(self):
        return self.rowptr.device

    def to(self, device, *args, **kwargs):
        device = torch.device(device)
        if device == self.device:
            return self
        out = Adjacency.__new__(Adjacency)
        out.__dict__.update(self.__dict__)
        for k in ("rowptr", "col", "val", "units", "split_rows"):
            setattr(out, k, getattr(self, k).to(device))
        out._t = None
        return out

    def transpose_csr(self) -> "Adjacency":
        if self.symmetric:
            return self
        if self._t is None:
            rows = torch.repeat_interleave(torch.arange(self.shape[0], device=self.device),
                                           self.rowptr[1:] - self.rowptr[:-1])
            self._t = Adjacency.from_coo(self.col.long(), rows, self.val,
                                         (self.shape[1], self.shape[0]), symmetric=False,
                                         device=self.device)
        return self._t

    def to_dense(self) -> torch.Tensor:
        rows = torch.repeat_interleave(torch.arange(self.shape[0], device=self.device),
                                       self.rowptr[1:] - self.rowptr[:-1])
        out = torch.zeros(self.shape, dtype=torch.float32, device=self.device)
        out[rows, self.col.long()] = self.val
        return out

    def __repr__(self):
        return (f"Adjacency(shape={self.shape}, nnz={self.nnz}, units={self.n_units}, "
                f"split_rows={self.n_split}, device={self.device})")

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in (torch.sparse.mm, torch.mm, torch.spmm, torch.matmul) and len(args) == 2 \
                and isinstance(args[0], Adjacency) and torch.is_tensor(args[1]):
            from .ops import spmm
            return spmm(args[0], args[1])
        return NotImplemented

    def __matmul__(self, other):
        from .ops import spmm
        return spmm(self, other)


def swap_sparse_attributes(module: torch.nn.Module, chunk: int = DEFAULT_CHUNK) -> list:
    """Replace every torch sparse COO tensor held as a plain attribute of ``module`` (or its
    submodules) by an :class:`Adjacency`, so unchanged reference model code
    (``torch.sparse.mm(self.norm_adj_matrix, x)``) runs the HIP SpMM.  Returns swapped names."""
    swapped = []
    for mname, mod in module.named_modules():
        for k, v in list(vars(mod).items()):
            if torch.is_tensor(v) and v.layout == torch.sparse_coo:
                setattr(mod, k, Adjacency.from_torch_sparse(v, chunk=chunk))
                swapped.append(f"{mname}.{k}" if mname else k)
    return swapped
