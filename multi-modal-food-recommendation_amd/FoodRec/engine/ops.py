"""Autograd ops over the HIP kernels (C-ABI in include/fr_engine.h).

Every op here runs on the GPU through ``libfr_engine.so``; a CPU tensor raises EngineError.
Upstream gradients are consumed on the device (``d_gscale``), so no op forces a host sync.

Op                       reference call site it replaces
-----------------------  ------------------------------------------------------------------
spmm(adj, X)             torch.sparse.mm(adj, X)          lightgcn.py:139, cikm_model.py:187,199
propagate_mean(adj,e,L)  L x sparse.mm + stack().mean(1)  lightgcn.py:134-144, cikm_model.py:182-208
bpr_emb_loss(...)        gather/mul/sum + BPRLoss + EmbLoss  lightgcn.py:158-177, loss.py:32-50
dcor_loss(views, pairs)  sum of correlation_distance       pricai_modelx.py:263,409-437
infonce_loss(H, tau)     CL_loss                           pricai_modelx.py:354-378
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch

from . import native, profiling
from .graph import Adjacency

_f = ctypes.c_float


def _rowmajor(t: torch.Tensor, f32_only: bool = False) -> torch.Tensor:
    """Row-major table with 16-B aligned rows: fp32 (ld % 4 == 0) or bf16 storage (ld % 8 == 0,
    the config-5 tables; arithmetic stays fp32 inside the kernels)."""
    if t.dtype != torch.float32 and (f32_only or t.dtype != torch.bfloat16):
        raise native.EngineError(f"engine tables are fp32 or bf16 (got {t.dtype})")
    if t.dim() != 2:
        raise native.EngineError(f"expected a 2-D table, got shape {tuple(t.shape)}")
    per16 = 16 // t.element_size()
    if t.stride(1) != 1 or t.stride(0) % per16 or t.data_ptr() % 16:
        t = t.contiguous()
    return t


def _same_dtype(*ts) -> torch.dtype:
    dts = {t.dtype for t in ts if t is not None}
    if len(dts) != 1:
        raise native.EngineError(f"mixed table dtypes {sorted(map(str, dts))}")
    return dts.pop()


def _grad_like(t: torch.Tensor) -> torch.Tensor:
    """Zero gradient buffer with exactly ``t``'s strides (kernels write grads with the input's ld)."""
    if t.stride(0) == t.shape[1] or t.shape[0] <= 1:
        return torch.zeros(t.shape, dtype=t.dtype, device=t.device)
    n = (t.shape[0] - 1) * t.stride(0) + t.shape[1]
    return torch.zeros(n, dtype=t.dtype, device=t.device).as_strided(t.shape, t.stride())


def _ws_for(adj: Adjacency, d: int, device) -> torch.Tensor:
    cache = adj.__dict__.setdefault("_ws_cache", {})
    key = (d, str(device))
    if key not in cache:
        plan = adj.plan()
        cache[key] = native.workspace(native.lib().fr_spmm_workspace(ctypes.byref(plan), d), device)
    return cache[key]


def spmm_launch(adj: Adjacency, X: torch.Tensor, Y1=None, Y2=None, alpha=1.0, A1=None, beta1=0.0,
                A2=None, beta2=0.0, stream=None) -> None:
    """Raw launch: Y1 = adj@X;  Y2 = alpha*(adj@X) + beta1*A1 + beta2*A2 (each optional)."""
    native.require_device(X)
    if X.shape[0] != adj.shape[1]:
        raise native.EngineError(f"spmm: adjacency {adj.shape} vs X {tuple(X.shape)}")
    d = X.shape[1]
    plan = adj.plan()
    ws = _ws_for(adj, d, X.device)
    s = stream if stream is not None else native.stream_of(X)
    dt = _same_dtype(X, Y1, Y2, A1, A2)

    def ld(t):
        return t.stride(0) if t is not None else 0

    with profiling.region("spmm", spmm_bytes(adj, d, sum(x is not None for x in (Y1, Y2, A1, A2)),
                                             X.element_size())):
        call = _spmm_call_bf16 if dt == torch.bfloat16 else _spmm_call
        call(adj, X, d, plan, ws, s, Y1, Y2, alpha, A1, beta1, A2, beta2, ld)


def spmm_bytes(adj: Adjacency, d: int, n_rowio: int = 1, elem: int = 4) -> int:
    """Algorithmic HBM bytes of one SpMM launch (no-reuse gather model):
    rowptr 8(N+1) + col/val 8 nnz + gathered rows s d nnz + s d N per output written / addend read
    (s = 4 fp32, 2 bf16)."""
    n = adj.shape[0]
    return 8 * (n + 1) + 8 * adj.nnz + elem * d * adj.nnz + elem * d * n * n_rowio


def mean_degree(adj: Adjacency, row: int = 0) -> float:
    """Mean edges per row of the side of ``row`` (a bipartite adjacency's two sides differ: users vs
    items, items vs ingredients), else of the whole adjacency."""
    n, split = adj.shape[0], adj.bipartite_split
    if split is None or not 0 < split < n:
        return adj.nnz / max(n, 1)
    if row < split:
        return adj.nnz_below_split / split
    return (adj.nnz - adj.nnz_below_split) / (n - split)


def rows_bytes(adj: Adjacency, rows, d: int = 64, n_rowio: int = 1, elem: int = 4) -> int:
    """Expected HBM bytes of a row-list SpMM (only the listed rows computed): per listed row its rowptr
    pair (16), its edges' col/val (8) and gathered rows (elem d) at the mean degree of its side
    (the degrees of the listed rows are on the device), and elem d per output written / addend read.
    ``rows``: [(ids, offset), ...] or a row count (at side 0)."""
    if isinstance(rows, int):
        segs = [(rows, 0)]
    else:
        segs = [(int(ids.numel()), int(off)) for ids, off in rows]
    tot = 0.0
    for n, off in segs:
        deg = mean_degree(adj, off)
        tot += n * (16 + deg * (8 + elem * d) + elem * d * n_rowio)
    return int(tot)


def frontier_rows(ui_adj: Adjacency, B: int, n_items: int) -> int:
    """Expected size of the RI frontier (fr_rows_frontier: the items adjacent to B batch users plus the
    2B batch items; the count is on the device): min(I, B * mean user degree + 2B)."""
    return int(min(n_items, B * mean_degree(ui_adj, 0) + 2 * B))


def sparse_upstream_bytes(adj: Adjacency, d: int = 64, elem: int = 4) -> int:
    """Scan + write bytes of a sparse-upstream SpMM (spmm_sparse_upstream / _rect / _blocks): rowptr,
    every edge's col/val, every output row written.  The gathers at marked columns (hits) are left
    out: their count is on the device (a lower bound)."""
    n = adj.shape[0]
    return 8 * (n + 1) + 8 * adj.nnz + elem * d * n


def scatter_upstream_bytes(adj: Adjacency, rows, d: int = 64, elem: int = 4) -> int:
    """fr_spmm_scatter_upstream: per listed row its X row read, per edge col/val (8) and an atomic
    read-modify-write of the target row (2 elem d), at the listed side's mean degree."""
    tot = 0.0
    for ids, off in rows:
        n = int(ids.numel())
        tot += n * (16 + elem * d + mean_degree(adj, int(off)) * (8 + 2 * elem * d))
    return int(tot)


def bpr_bwd_bytes(B: int, d: int = 64, elem: int = 4) -> int:
    """fr_bpr_bwd(_ex): per triple row (3B: u, p, n) its id (8), the propagated and the ego rows read
    (2 elem d) and the gradient row's read-modify-write (2 elem d)."""
    return 3 * B * (8 + 4 * elem * d)


def bpr_finish_bytes(B: int, d: int = 64, elem: int = 4) -> int:
    """fr_graph_bpr_finish: per triple row its id and mask byte (9), the ego row read (elem d) and the
    gradient row's read-modify-write (2 elem d)."""
    return 3 * B * (9 + 3 * elem * d)


def _spmm_call_bf16(adj, X, d, plan, ws, s, Y1, Y2, alpha, A1, beta1, A2, beta2, ld):
    rc = native.lib().fr_spmm_csr_bf16(
        adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.val.data_ptr(), adj.shape[0], ctypes.byref(plan),
        X.data_ptr(), ld(X), d,
        native.ptr(Y1), ld(Y1),
        native.ptr(Y2), ld(Y2), _f(alpha),
        native.ptr(A1), ld(A1), _f(beta1),
        native.ptr(A2), ld(A2), _f(beta2),
        ws.data_ptr(), ws.numel(), s)
    native.check(rc, "fr_spmm_csr_bf16")


def _spmm_call(adj, X, d, plan, ws, s, Y1, Y2, alpha, A1, beta1, A2, beta2, ld):
    rc = native.lib().fr_spmm_csr(
        adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.val.data_ptr(), adj.shape[0], ctypes.byref(plan),
        X.data_ptr(), ld(X), d,
        native.ptr(Y1), ld(Y1),
        native.ptr(Y2), ld(Y2), _f(alpha),
        native.ptr(A1), ld(A1), _f(beta1),
        native.ptr(A2), ld(A2), _f(beta2),
        ws.data_ptr(), ws.numel(), s)
    native.check(rc, "fr_spmm_csr")


class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, adj, X):
        X = _rowmajor(X)
        Y = torch.empty((adj.shape[0], X.shape[1]), dtype=X.dtype, device=X.device)
        spmm_launch(adj, X, Y1=Y)
        ctx.adj = adj
        return Y

    @staticmethod
    def backward(ctx, G):
        G = _rowmajor(G)
        at = ctx.adj.transpose_csr()
        dX = torch.empty((at.shape[0], G.shape[1]), dtype=G.dtype, device=G.device)
        spmm_launch(at, G, Y1=dX)
        return None, dX


def spmm(adj: Adjacency, X: torch.Tensor) -> torch.Tensor:
    return _SpMM.apply(adj, X)


def _propagate_mean_fwd(adj: Adjacency, ego: torch.Tensor, L: int) -> torch.Tensor:
    N, d = ego.shape
    out = torch.empty_like(ego)
    if L == 1:
        spmm_launch(adj, ego, Y2=out, alpha=0.5, A1=ego, beta1=0.5)
        return out
    inv = 1.0 / (L + 1)
    E1 = torch.empty_like(ego)
    if L == 2:
        spmm_launch(adj, ego, Y1=E1)
        spmm_launch(adj, E1, Y2=out, alpha=inv, A1=ego, beta1=inv, A2=E1, beta2=inv)
        return out
    S = torch.empty_like(ego)
    spmm_launch(adj, ego, Y1=E1, Y2=S, alpha=1.0, A1=ego, beta1=1.0)
    prev, nxt = E1, torch.empty_like(ego)
    for _ in range(2, L):
        spmm_launch(adj, prev, Y1=nxt, Y2=S, alpha=1.0, A1=S, beta1=1.0)
        prev, nxt = nxt, prev
    spmm_launch(adj, prev, Y2=out, alpha=inv, A1=S, beta1=inv)
    return out


def _prop_bwd_bipartite2(adj, g, out_lo, out_hi, split, acc=None):
    """_prop_bwd_split for L = 2 on a bipartite adjacency split at ``split`` (adj.mark_bipartite)
    for an upstream gradient G = [g ; 0], zero at rows [split, n) (HealthRec's RI graph and CLUSSL's
    modality graphs: the side rows of the propagation are discarded).  ``g``: the rows [0, split)
    of G.  With A = [[0, R], [R^T, 0]]:
      H   = (A G + G) / 3     = [g / 3 ; R^T g / 3]
      out = A H + G / 3       = [R (R^T g / 3) + g / 3 ; R^T g / 3]
    so the side rows of the result equal those of H: one launch over rows [split, n) writes them
    (into out_hi) and the item rows read them there -- two half-graph launches instead of two full
    ones.  The item rows are the full form's sums in the same order (the skipped products are exact
    zeros); the side rows apply the 1/3 after the sum instead of to each term (a rounding-level
    difference).  ``acc``: item-row gradients of other views added into out_lo in the same epilogue."""
    inv = 1.0 / 3.0
    N = adj.shape[0]
    # side rows gather item columns only: X = [g ; (never read)]
    pad = _persistent(adj, ("bwd_pad", str(g.device)), lambda: torch.zeros(N - split, g.shape[1], device=g.device))
    spmm_range(adj, g, split, N, X_hi=pad, split=split, Y2=out_lo, Y2_hi=out_hi, alpha=inv)
    # item rows gather side columns only: X = [(never read) ; out_hi]
    spmm_range(adj, g, 0, split, X_hi=out_hi, split=split, Y2=out_lo, alpha=1.0, A1=g, beta1=inv,
               A2=acc, beta2=0.0 if acc is None else 1.0)


class _PropagateLo(torch.autograd.Function):
    """split(mean_k A^k [lo ; hi], [split, n - split])[0] on a bipartite adjacency split at
    ``split = lo.shape[0]``: the reference's propagate-then-keep-the-item-rows
    (pricai_modelx.py:183-226, cikm_model.py:185-208) without the concatenation, the split or the
    side rows the result does not contain (_prop_fwd_split(lo_rows_only), _prop_bwd_bipartite2)."""

    @staticmethod
    def forward(ctx, adj, lo, hi, L):
        native.require_device(lo, hi)
        split = lo.shape[0]
        ctx.adj, ctx.L, ctx.split, ctx.hi_rows = adj, L, split, hi.shape[0]
        return _prop_fwd_split(adj, lo, hi, split, L, lo_rows_only=True)[:split]

    @staticmethod
    def backward(ctx, g):
        adj, L, split = ctx.adj, ctx.L, ctx.split
        g = _rowmajor(g)
        N, d = adj.shape[0], g.shape[1]
        d_lo = torch.empty(split, d, dtype=g.dtype, device=g.device)
        d_hi = torch.empty(ctx.hi_rows, d, dtype=g.dtype, device=g.device)
        if ctx.hi_rows > N - split:
            d_hi[N - split:].zero_()  # rows past the graph (e.g. a padding row) get no gradient
        if L == 2:
            _prop_bwd_bipartite2(adj, g, d_lo, d_hi, split)
        else:
            G = torch.zeros(N, d, dtype=g.dtype, device=g.device)
            G[:split] = g
            _prop_bwd_split(adj, G, L, d_lo, d_hi, split)
        return None, d_lo, d_hi, None


class _PropagateRows(torch.autograd.Function):
    """mean_k A^k ego where the caller reads the result at the listed rows only (a BPR loss reads
    the propagated table at its batch's users and items, lightgcn.py:134-147 + :149-168): the last
    layer is evaluated there only (row-list launch), and the backward of an upstream gradient that is
    non-zero only at those rows starts with the sparse-upstream launch (edges scanned against a
    bitmask of the rows, X gathered only there).  The result is valid at the listed rows only.
    Float-atomic summation in the sparse launch: not for the deterministic mode."""

    @staticmethod
    def forward(ctx, adj, ego, L, rows):
        ego = _rowmajor(ego)
        native.require_device(ego)
        out = torch.empty_like(ego)  # valid at the listed rows
        inv = 1.0 / (L + 1)
        if L == 1:
            spmm_ex(adj, ego, Y2=out, alpha=0.5, A1=ego, beta1=0.5, rows=rows, region="spmm_rows")
        elif L == 2:
            E1 = torch.empty_like(ego)
            s = adj.bipartite_split
            if s is not None:
                # layer 1 is read at the loss rows R and their neighbours: the [0, s) block in full (the
                # neighbours of R's high rows span it) and the [s, n) block only at R's high rows and
                # the neighbours of its low rows (fewer rows than the block)
                S = _bipartite_layer1_rows(adj, rows, s)
                spmm_range(adj, ego, 0, s, Y1=E1)
                if S.numel():
                    spmm_ex(adj, ego, Y1=E1, rows=[(S, 0)], region="spmm_rows")
            else:
                spmm_launch(adj, ego, Y1=E1)
            spmm_ex(adj, E1, Y2=out, alpha=inv, A1=ego, beta1=inv, A2=E1, beta2=inv, rows=rows, region="spmm_rows")
        else:
            S, E1 = torch.empty_like(ego), torch.empty_like(ego)
            spmm_launch(adj, ego, Y1=E1, Y2=S, alpha=1.0, A1=ego, beta1=1.0)
            prev, nxt = E1, torch.empty_like(ego)
            for _ in range(2, L):
                spmm_launch(adj, prev, Y1=nxt, Y2=S, alpha=1.0, A1=S, beta1=1.0)
                prev, nxt = nxt, prev
            spmm_ex(adj, prev, Y2=out, alpha=inv, A1=S, beta1=inv, rows=rows, region="spmm_rows")
        ctx.adj, ctx.L, ctx.rows = adj, L, rows
        return out

    @staticmethod
    def backward(ctx, G):
        adj, L, rows = ctx.adj, ctx.L, ctx.rows
        G = _rowmajor(G)
        at = adj.transpose_csr()
        N, dev = at.shape[0], G.device
        bits = _persistent(at, ("rows_bits", str(dev)), lambda: torch.zeros((N + 31) // 32, dtype=torch.int32, device=dev))
        mask = _persistent(at, ("rows_mask", str(dev)), lambda: torch.zeros(N, dtype=torch.uint8, device=dev))
        rows_mark(mask, rows, 1, bits=bits)
        inv = 1.0 / (L + 1)
        H = torch.empty_like(G)
        # H_L = (A^T G + G) / (L + 1): G is zero outside the rows -> gathered only there
        spmm_sparse_upstream(at, bits, G, H, alpha=0.5 if L == 1 else inv, beta1=0.5 if L == 1 else inv)
        rows_mark(mask, rows, 0, bits=bits)
        if L == 1:
            return None, H, None, None
        H2 = torch.empty_like(G)
        for _ in range(1, L):
            spmm_launch(at, H, Y2=H2, alpha=1.0, A1=G, beta1=inv)
            H, H2 = H2, H
        return None, H, None, None


def _bipartite_layer1_rows(adj: Adjacency, rows, s: int) -> torch.Tensor:
    """Rows >= s of a bipartite adjacency (split s) that a row-list layer 2 at ``rows`` reads layer 1
    at: the listed rows >= s and the columns of the listed rows < s (sorted, unique)."""
    ids = torch.cat([ids + off for ids, off in rows])
    lo = ids[ids < s]
    hi = ids[ids >= s]
    rp = adj.rowptr
    starts = rp[lo]
    lens = rp[lo + 1] - starts
    total = int(lens.sum().item())
    if total:
        first = torch.cumsum(lens, 0) - lens
        pos = torch.repeat_interleave(starts - first, lens) + torch.arange(total, device=ids.device)
        hi = torch.cat([hi, adj.col[pos].to(torch.int64)])
    return torch.unique(hi)


def propagate_rows(adj: Adjacency, ego: torch.Tensor, n_layers: int, rows) -> torch.Tensor:
    """mean([ego, A ego, ..., A^L ego]) evaluated at the listed rows only ([(ids, offset), ...], up
    to three segments) -- the table is valid there and nowhere else; the gradient flowing back must
    be zero outside those rows (a BPR / EmbLoss on them).  fp32, d = 64 on the GPU, non-deterministic
    mode; otherwise the full propagate_mean.  The row set is built with host reads (its size sets
    the launch shapes), so inside a HIP-graph capture the full propagation runs instead (its
    results agree at the listed rows)."""
    if (n_layers >= 1 and ego.is_cuda and ego.dtype == torch.float32 and ego.shape[1] == 64 and not _DETERMINISTIC
            and adj.shape[0] == adj.shape[1] and 1 <= len(rows) <= 3
            and not torch.cuda.is_current_stream_capturing()):
        rows = [(ids.reshape(-1).to(torch.int64).contiguous(), int(off)) for ids, off in rows]
        return _PropagateRows.apply(adj, ego, int(n_layers), rows)
    return propagate_mean(adj, ego, n_layers)


class _EmbRowsSink:
    """EmbLoss ego-row gradients of an item table that a later backward node adds into its own
    gradient of that table (CLUSSL: ui_bpr's item rows, added by the item views' node into its
    d item): no dense zero-filled buffer for the rows and no autograd sum of the two gradients.
    Opened by _PropagateLoViews.forward on the table, filled by _UiBpr.backward (which autograd runs
    first: the views' backward needs its gradient), drained and closed by _PropagateLoViews.backward."""
    __slots__ = ("open", "entries")

    def __init__(self):
        self.open, self.entries = True, []


# FR_EMB_ROWS_INTO_VIEWS=0: ui_bpr returns its EmbLoss item rows as a dense zero-filled gradient
EMB_ROWS_INTO_VIEWS = os.environ.get("FR_EMB_ROWS_INTO_VIEWS", "1") != "0"


class _PropagateLoViews(torch.autograd.Function):
    """_PropagateLo over several bipartite graphs sharing the item table ``lo`` (CLUSSL's ingredient,
    image-cluster and text-cluster views, pricai_modelx.py:183-226): one node, so the backward
    chains the views' item-row gradients through the SpMM epilogue (A2 = the previous views' sum)
    instead of leaving autograd a zero-initialised buffer and an add per view; the EmbLoss ego rows a
    ui_bpr node parked in the table's _EmbRowsSink are added into that gradient by one launch, which
    also zeroes a side table's padding row."""

    @staticmethod
    def forward(ctx, adjs, L, lo, *his):
        native.require_device(lo, *his)
        split = lo.shape[0]
        ctx.adjs, ctx.L, ctx.split, ctx.hi_rows = adjs, L, split, [h.shape[0] for h in his]
        ctx.sink = None
        if EMB_ROWS_INTO_VIEWS and lo.requires_grad and not _DETERMINISTIC:
            ctx.sink = lo.__dict__["_fr_emb_rows"] = _EmbRowsSink()
        return tuple(_prop_fwd_split(adj, lo, hi, split, L, lo_rows_only=True)[:split] for adj, hi in zip(adjs, his))

    @staticmethod
    def backward(ctx, *gs):
        split, L = ctx.split, ctx.L
        d_lo, d_his = None, []
        sink = ctx.sink
        rows = []
        if sink is not None:
            sink.open = False
            rows, sink.entries = sink.entries, []
        pad = None  # (the first padding block, zeroed by the EmbLoss rows' launch when there is one)
        for adj, g, hi_rows in zip(ctx.adjs, gs, ctx.hi_rows):
            N = adj.shape[0]
            if g is None:  # a view nothing read
                d_his.append(None)
                continue
            g = _rowmajor(g)
            d = g.shape[1]
            out = torch.empty(split, d, dtype=g.dtype, device=g.device)
            d_hi = torch.empty(hi_rows, d, dtype=g.dtype, device=g.device)
            if hi_rows > N - split:  # rows past the graph (e.g. a padding row) get no gradient
                if rows and pad is None:
                    pad = d_hi[N - split:]
                else:
                    d_hi[N - split:].zero_()
            if L == 2:
                _prop_bwd_bipartite2(adj, g, out, d_hi, split, acc=d_lo)
            else:
                G = torch.zeros(N, d, dtype=g.dtype, device=g.device)
                G[:split] = g
                _prop_bwd_split(adj, G, L, out, d_hi, split)
                if d_lo is not None:
                    out.add_(d_lo)
            d_lo = out
            d_his.append(d_hi)
        for k, (user_w, item_w, u, p, n, ws, w_emb, ge) in enumerate(rows):
            if d_lo is None:
                d_lo = torch.zeros_like(item_w)  # (no view carried a gradient: the rows alone)
            z = pad if k == 0 else None
            with profiling.region("bpr_bwd", bpr_finish_bytes(int(u.numel()))):
                native.check(native.lib().fr_graph_bpr_finish(
                    None, 0, user_w.data_ptr(), 64, item_w.data_ptr(), 64, u.data_ptr(), p.data_ptr(), n.data_ptr(),
                    int(u.numel()), 64, _f(w_emb), native.ptr(ge), None, d_lo.data_ptr(), native.ptr(z),
                    0 if z is None else z.numel(), None, ws.data_ptr(), ws.numel(), native.stream_of(d_lo)),
                    "fr_graph_bpr_finish")
        return (None, None, d_lo) + tuple(d_his)


def propagate_lo_views(adjs, lo: torch.Tensor, his, n_layers: int):
    """[propagate_lo(adj, lo, hi, n_layers) for adj, hi in zip(adjs, his)] as one autograd node
    (_PropagateLoViews) when every view takes the bipartite path."""
    his = list(his)
    ok = (n_layers >= 1 and lo.is_cuda and lo.dtype == torch.float32 and lo.shape[1] == 64 and len(adjs) == len(his)
          and all(getattr(a, "bipartite_split", None) == lo.shape[0] and h.dtype == torch.float32
                  and h.shape[1] == 64 and h.shape[0] >= a.shape[0] - lo.shape[0] for a, h in zip(adjs, his)))
    if not ok:
        return [propagate_lo(a, lo, h, n_layers) for a, h in zip(adjs, his)]
    return list(_PropagateLoViews.apply(tuple(adjs), int(n_layers), lo, *his))


def propagate_lo(adj: Adjacency, lo: torch.Tensor, hi: torch.Tensor, n_layers: int) -> torch.Tensor:
    """Rows [0, len(lo)) of mean([E, A E, ..., A^L E]), E = [lo ; hi], for an adjacency marked
    bipartite at len(lo) (fp32, d = 64 on the GPU); otherwise the full propagation, split."""
    split = lo.shape[0]
    if (n_layers >= 1 and lo.is_cuda and getattr(adj, "bipartite_split", None) == split
            and lo.dtype == torch.float32 and hi.dtype == torch.float32 and lo.shape[1] == 64 == hi.shape[1]
            and hi.shape[0] >= adj.shape[0] - split):
        return _PropagateLo.apply(adj, lo, hi, int(n_layers))
    out = propagate_mean(adj, torch.cat([lo, hi[:adj.shape[0] - split]], dim=0), n_layers)
    return out[:split]


def _propagate_mean_bwd(adj: Adjacency, G: torch.Tensor, L: int) -> torch.Tensor:
    # d/d ego of mean_k A^k ego:  H_L = G/(L+1);  H_k = A^T H_{k+1} + G/(L+1);  grad = H_0
    at = adj.transpose_csr()
    inv = 1.0 / (L + 1)
    H = torch.empty_like(G)
    spmm_launch(at, G, Y2=H, alpha=inv, A1=G, beta1=inv)
    if L == 1:
        return H
    H2 = torch.empty_like(G)
    for _ in range(1, L):
        spmm_launch(at, H, Y2=H2, alpha=1.0, A1=G, beta1=inv)
        H, H2 = H2, H
    return H


class _PropagateMean(torch.autograd.Function):
    @staticmethod
    def forward(ctx, adj, ego, L):
        ego = _rowmajor(ego)
        native.require_device(ego)
        ctx.adj, ctx.L = adj, L
        return _propagate_mean_fwd(adj, ego, L)

    @staticmethod
    def backward(ctx, G):
        return None, _propagate_mean_bwd(ctx.adj, _rowmajor(G), ctx.L), None


def propagate_mean(adj: Adjacency, ego: torch.Tensor, n_layers: int) -> torch.Tensor:
    """mean([ego, A ego, ..., A^L ego]) — LightGCN propagation with the layer mean fused."""
    if n_layers == 0:
        return ego
    return _PropagateMean.apply(adj, ego, int(n_layers))


class _PropagateMeanSplit(torch.autograd.Function):
    """propagate_mean(adj, cat([lo, hi])) with the concatenation folded into the SpMM addressing
    (split tables): no [N, d] copy forward, and the two gradients are written straight into their
    own buffers backward (no split of a concatenated gradient)."""

    @staticmethod
    def forward(ctx, adj, lo, hi, L):
        lo, hi = _rowmajor(lo), _rowmajor(hi)
        native.require_device(lo, hi)
        ctx.adj, ctx.L, ctx.split = adj, L, lo.shape[0]
        ctx.shapes = (lo.shape, hi.shape)
        return _prop_fwd_split(adj, lo, hi, lo.shape[0], L)

    @staticmethod
    def backward(ctx, G):
        G = _rowmajor(G)
        d_lo = torch.empty(ctx.shapes[0], dtype=G.dtype, device=G.device)
        d_hi = torch.empty(ctx.shapes[1], dtype=G.dtype, device=G.device)
        _prop_bwd_split(ctx.adj, G, ctx.L, d_lo, d_hi, ctx.split)
        return None, d_lo, d_hi, None


def propagate_mean_split(adj: Adjacency, lo: torch.Tensor, hi: torch.Tensor, n_layers: int) -> torch.Tensor:
    """propagate_mean(adj, torch.cat([lo, hi]), n_layers) without the concatenation (fp32, d = 64
    on the GPU, a symmetric adjacency of len(lo) + len(hi) rows); otherwise exactly that."""
    if (n_layers >= 1 and getattr(adj, "symmetric", False) and lo.is_cuda and lo.dtype == torch.float32 == hi.dtype and lo.shape[1] == 64 == hi.shape[1]
            and lo.shape[0] + hi.shape[0] == adj.shape[0]):
        return _PropagateMeanSplit.apply(adj, lo, hi, int(n_layers))
    return propagate_mean(adj, torch.cat([lo, hi], dim=0), n_layers)


# ----------------------------------------------------------------------------- BPR + EmbLoss
class _BprEmb(torch.autograd.Function):
    @staticmethod
    def forward(ctx, U, I, Ue, Ie, u, p, n, gamma, deterministic, item_rows=False, item_offset=None, w_emb=1.0):
        # item_offset: items are rows [item_offset:] of U (one propagated table, one gradient buffer,
        # item ids unchanged); the kernels just see the offset base pointers
        ctx.ioff = None if item_offset is None else int(item_offset)
        if ctx.ioff is not None:
            I = U[ctx.ioff:]
        # one table for users and items (item ids offset past the users): one gradient buffer
        alias_ui, alias_e = I is U, Ie is not None and Ie is Ue
        U = _rowmajor(U)
        I = U if alias_ui else _rowmajor(I)
        Ue = _rowmajor(Ue) if Ue is not None else None
        Ie = Ue if alias_e else (_rowmajor(Ie) if Ie is not None else None)
        native.require_device(U, I, Ue, Ie, u, p, n)
        u, p, n = (x.to(torch.int64).contiguous() for x in (u, p, n))
        B, d = int(u.numel()), U.shape[1]
        bf16 = _same_dtype(U, I, Ue, Ie) == torch.bfloat16
        lib = native.lib()
        ws = native.workspace(lib.fr_bpr_workspace(B), U.device)
        out = torch.empty(5, dtype=torch.float32, device=U.device)
        ld = lambda t: t.stride(0) if t is not None else 0  # noqa: E731
        rows = None
        if bf16:
            if w_emb != 1.0:
                raise native.EngineError("bpr_emb_loss: w_emb needs fp32 tables")
            native.check(lib.fr_bpr_fwd_bf16(U.data_ptr(), ld(U), I.data_ptr(), ld(I), native.ptr(Ue), ld(Ue),
                                             native.ptr(Ie), ld(Ie), u.data_ptr(), p.data_ptr(), n.data_ptr(),
                                             B, d, _f(gamma), out.data_ptr(), ws.data_ptr(), ws.numel(),
                                             native.stream_of(U)), "fr_bpr_fwd_bf16")
        else:
            # out[4] = w_emb * EmbLoss in the kernel (no multiply launch); [I[pos]; I[neg]] written by the
            # same launch when asked for
            if item_rows:
                rows = torch.empty(2 * B, d, dtype=I.dtype, device=I.device)
            native.check(lib.fr_bpr_fwd_ex(U.data_ptr(), ld(U), I.data_ptr(), ld(I), native.ptr(Ue), ld(Ue),
                                           native.ptr(Ie), ld(Ie), u.data_ptr(), p.data_ptr(), n.data_ptr(),
                                           B, d, _f(gamma), _f(w_emb), out.data_ptr(), native.ptr(rows),
                                           d if rows is not None else 0, ws.data_ptr(), ws.numel(),
                                           native.stream_of(U)), "fr_bpr_fwd_ex")
        ctx.save_for_backward(U, I, Ue, Ie, u, p, n)
        ctx.ws, ctx.gamma, ctx.det, ctx.w_emb = ws, gamma, int(deterministic), float(w_emb)
        ctx.same_u, ctx.same_i = Ue is U, Ie is I
        ctx.alias_ui, ctx.alias_e = alias_ui, alias_e
        ctx.item_rows = bool(item_rows) and not deterministic and I.dtype == torch.float32
        if not item_rows:
            return out[0], out[4:5]
        # [I[pos]; I[neg]] for another consumer; its gradient joins the backward's own scatter
        if rows is None:
            rows = torch.index_select(I, 0, torch.cat([p, n]))
        return out[0], out[4:5], rows

    @staticmethod
    def backward(ctx, g_mf, g_emb, g_rows=None):
        U, I, Ue, Ie, u, p, n = ctx.saved_tensors
        dev = U.device
        if _is_unit(g_mf) and _is_unit(g_emb):
            gscale = None  # both upstream gradients are the trainer's ones seeds: no device scale needed
        else:
            g_mf = g_mf if g_mf is not None else torch.zeros((), device=dev)
            g_emb = g_emb if g_emb is not None else torch.zeros(1, device=dev)
            gscale = torch.cat([g_mf.reshape(1), g_emb.reshape(1)]).float().contiguous()
        g_reg = _f(ctx.w_emb)
        need = ctx.needs_input_grad
        if ctx.ioff is not None:
            dU = _grad_like(U) if need[0] else None
            dI = dU[ctx.ioff:] if dU is not None else None
        else:
            dU = _grad_like(U) if (need[0] or (ctx.alias_ui and need[1])) else None
            dI = dU if ctx.alias_ui else (_grad_like(I) if need[1] else None)
        dUe = dIe = None
        if Ue is not None:
            dUe = dU if (ctx.same_u and dU is not None) else (
                _grad_like(Ue) if (need[2] or (ctx.alias_e and need[3])) else None)
            dIe = dUe if ctx.alias_e else (dI if (ctx.same_i and dI is not None) else
                                           (_grad_like(Ie) if need[3] else None))
        B, d = int(u.numel()), U.shape[1]
        ld = lambda t: t.stride(0) if t is not None else 0  # noqa: E731
        if U.dtype == torch.bfloat16:
            native.check(native.lib().fr_bpr_bwd_bf16(
                U.data_ptr(), ld(U), I.data_ptr(), ld(I), native.ptr(Ue), ld(Ue), native.ptr(Ie), ld(Ie),
                u.data_ptr(), p.data_ptr(), n.data_ptr(), B, d, _f(ctx.gamma), _f(1.0), g_reg,
                native.ptr(gscale), native.ptr(dU), native.ptr(dI), native.ptr(dUe), native.ptr(dIe),
                ctx.ws.data_ptr(), ctx.ws.numel(), native.stream_of(U)), "fr_bpr_bwd_bf16")
        elif g_rows is not None and dI is not None and ctx.item_rows:
            g_rows = g_rows.contiguous()
            native.check(native.lib().fr_bpr_bwd_ex(
                U.data_ptr(), ld(U), I.data_ptr(), ld(I), native.ptr(Ue), ld(Ue), native.ptr(Ie), ld(Ie),
                u.data_ptr(), p.data_ptr(), n.data_ptr(), B, d, _f(ctx.gamma), _f(1.0), g_reg,
                native.ptr(gscale), native.ptr(dU), native.ptr(dI), native.ptr(dUe), native.ptr(dIe),
                g_rows.data_ptr(), g_rows.stride(0), ctx.ws.data_ptr(), ctx.ws.numel(), native.stream_of(U)),
                "fr_bpr_bwd_ex")
            g_rows = None
        else:
            native.check(native.lib().fr_bpr_bwd(
                U.data_ptr(), ld(U), I.data_ptr(), ld(I), native.ptr(Ue), ld(Ue), native.ptr(Ie), ld(Ie),
                u.data_ptr(), p.data_ptr(), n.data_ptr(), B, d, _f(ctx.gamma), _f(1.0), g_reg,
                native.ptr(gscale), native.ptr(dU), native.ptr(dI), native.ptr(dUe), native.ptr(dIe),
                ctx.det, ctx.ws.data_ptr(), ctx.ws.numel(), native.stream_of(U)), "fr_bpr_bwd")
        if ctx.same_u:
            dUe = None
        if ctx.same_i or ctx.alias_e:
            dIe = None
        if g_rows is not None and dI is not None:  # not folded into the kernel (bf16 / deterministic)
            dI.index_add_(0, torch.cat([p, n]), g_rows.to(dI.dtype))
        if ctx.alias_ui or ctx.ioff is not None:
            dI = None
        return dU, dI, dUe, dIe, None, None, None, None, None, None, None, None


def _is_unit(g) -> bool:
    """An upstream gradient known to be exactly one: the trainer's cached backward seeds
    (Trainer._ones_like marks them ``_fr_unit``; they are never written)."""
    return g is not None and getattr(g, "_fr_unit", False)


_DETERMINISTIC = False

# device step counters whose per-step increment is deferred to the step's fr_step_book launch
# (Trainer._book_fused).  A counter still pending when it is about to be read again is advanced on
# the spot, so a forward run outside a booked training step keeps the one-per-use semantics.
_PENDING_COUNTERS = []
_DEFER = [False]


def defer_counters(on: bool) -> None:
    """Inside a training step that ends in fr_step_book (Trainer) counter increments are deferred
    to that launch; outside one they happen immediately (``defer_increment`` falls back to add_)."""
    _DEFER[0] = bool(on)
    if not on:
        settle_all_counters()


def defer_increment(counter: torch.Tensor) -> None:
    """Advance ``counter`` (a device int64 scalar) by one at the end of this training step (or now,
    outside a deferring step)."""
    if not _DEFER[0]:
        counter.add_(1)
        return
    for k, c in enumerate(_PENDING_COUNTERS):
        if c is counter:
            del _PENDING_COUNTERS[k]
            counter.add_(1)
            break
    _PENDING_COUNTERS.append(counter)


def settle_counter(counter: torch.Tensor) -> None:
    """Apply a pending deferred increment of ``counter`` now (before it is read again)."""
    for k, c in enumerate(_PENDING_COUNTERS):
        if c is counter:
            del _PENDING_COUNTERS[k]
            counter.add_(1)
            return


def drop_pending(counter: torch.Tensor) -> None:
    """Forget a pending increment (the counter is being reset)."""
    _PENDING_COUNTERS[:] = [c for c in _PENDING_COUNTERS if c is not counter]


def take_pending_counters(limit: int = 8) -> list:
    """The deferred counters for fr_step_book (at most ``limit``; the rest are advanced now)."""
    out = _PENDING_COUNTERS[:limit]
    for c in _PENDING_COUNTERS[limit:]:
        c.add_(1)
    _PENDING_COUNTERS.clear()
    return out


def settle_all_counters() -> None:
    for c in _PENDING_COUNTERS:
        c.add_(1)
    _PENDING_COUNTERS.clear()


def set_deterministic(on: bool) -> None:
    """Engine-wide run-to-run reproducible scatters (config key ``deterministic``, set by the
    Trainer): the BPR backward scatters by owner slots instead of float atomics.  Combine with
    ``torch.use_deterministic_algorithms(True)`` for PyTorch's own index_add_ / index_put_."""
    global _DETERMINISTIC
    _DETERMINISTIC = bool(on)


def bpr_emb_loss(U, I, Ue, Ie, user, pos, neg, gamma: float = 1e-10, deterministic: bool = False,
                 item_rows: bool = False, item_offset: int | None = None, w_emb: float = 1.0):
    """Returns (BPRLoss, EmbLoss-unweighted [1]) with gathers, dots and norms fused; with
    ``item_rows`` also the gathered [I[pos]; I[neg]] rows, whose gradient is added inside the fused
    backward's scatter (no separate gather backward).  ``item_offset`` (with I None): the item table
    is U[item_offset:] -- one [users + items] gradient buffer instead of two plus a concatenation.
    ``w_emb``: the EmbLoss output is w_emb * EmbLoss (the models' reg_weight), applied in the kernels."""
    return _BprEmb.apply(U, I, Ue, Ie, user, pos, neg, gamma, deterministic or _DETERMINISTIC, item_rows,
                         item_offset, float(w_emb))


# ----------------------------------------------------------------------------- split-table SpMM
def _tab(lo, hi=None):
    if lo is None:
        return native.FrTab(None, 0, None, 0)
    return native.FrTab(lo.data_ptr(), lo.stride(0), hi.data_ptr() if hi is not None else None,
                        hi.stride(0) if hi is not None else 0)


def _rowlist(segs):
    """[(int64 ids, offset), ...] (at most 3) -> fr_rowlist."""
    rl = native.FrRowList()
    for k, (ids, off) in enumerate(segs):
        rl.ids[k] = ids.data_ptr()
        rl.n[k] = ids.numel()
        rl.off[k] = int(off)
    return rl


def _check_tab(name, lo, hi, split, n, d):
    if lo is None:
        return
    for t in (lo, hi):
        if t is not None and (t.dtype != torch.float32 or t.dim() != 2 or t.shape[1] != d or t.stride(1) != 1
                              or t.stride(0) % 4 or t.data_ptr() % 16):
            raise native.EngineError(f"spmm_ex: {name} must be fp32 [rows, {d}] with 16-B aligned rows")
    if hi is None and lo.shape[0] < n:
        raise native.EngineError(f"spmm_ex: {name} has {lo.shape[0]} rows, needs {n}")
    if hi is not None and (lo.shape[0] < split or hi.shape[0] < n - split):
        raise native.EngineError(f"spmm_ex: {name} split at {split} does not cover {n} rows")


def spmm_ex(adj: Adjacency, X, X_hi=None, split=0, Y1=None, Y1_hi=None, Y2=None, Y2_hi=None, alpha=1.0,
            A1=None, A1_hi=None, beta1=0.0, A2=None, A2_hi=None, beta2=0.0, col_mask=None, rows=None,
            a1_gate=None, region="spmm", nbytes=None):
    """fr_spmm_csr_ex: the fr_spmm_csr epilogue over split tables ([lo ; hi] at row ``split``), an
    optional column mask (uint8 per X row, skipped where 0), an optional row list
    ([(ids, offset), ...]: only those rows of Y are computed and written) and an optional A1 row
    gate (uint8 per output row: A1 read only where set, zero elsewhere)."""
    native.require_device(X)
    N, d = adj.shape[0], X.shape[1]
    _check_tab("X", X, X_hi, split, adj.shape[1], d)
    for name, lo, hi in (("Y1", Y1, Y1_hi), ("Y2", Y2, Y2_hi), ("A1", A1, A1_hi), ("A2", A2, A2_hi)):
        _check_tab(name, lo, hi, split, N, d)
    if col_mask is not None and (col_mask.dtype != torch.uint8 or col_mask.numel() < adj.shape[1]):
        raise native.EngineError("spmm_ex: col_mask must be uint8 with one entry per X row")
    if a1_gate is not None and (a1_gate.dtype != torch.uint8 or a1_gate.numel() < N):
        raise native.EngineError("spmm_ex: a1_gate must be uint8 with one entry per output row")
    plan = adj.plan()
    ws = _ws_for(adj, d, X.device)
    rl = _rowlist(rows) if rows is not None else None
    if nbytes is None:
        nio = sum(x is not None for x in (Y1, Y2, A1, A2))
        nbytes = spmm_bytes(adj, d, nio) if rows is None else rows_bytes(adj, rows, d, nio)
    with profiling.region(region, nbytes):
        native.check(native.lib().fr_spmm_csr_ex(
            adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.val.data_ptr(), N, ctypes.byref(plan), int(split),
            ctypes.byref(_tab(X, X_hi)), d, ctypes.byref(_tab(Y1, Y1_hi)), ctypes.byref(_tab(Y2, Y2_hi)), _f(alpha),
            ctypes.byref(_tab(A1, A1_hi)), _f(beta1), ctypes.byref(_tab(A2, A2_hi)), _f(beta2),
            native.ptr(col_mask), ctypes.byref(rl) if rl is not None else None, native.ptr(a1_gate), ws.data_ptr(),
            ws.numel(), native.stream_of(X)), "fr_spmm_csr_ex")


def spmm_range(adj: Adjacency, X, row_lo: int, row_hi: int, X_hi=None, split=0, Y1=None, Y1_hi=None, Y2=None,
               Y2_hi=None, alpha=1.0, A1=None, A1_hi=None, beta1=0.0, A2=None, A2_hi=None, beta2=0.0,
               region="spmm", nbytes=None):
    """fr_spmm_csr_range: spmm_ex (no mask, no row list) over output rows [row_lo, row_hi) only."""
    native.require_device(X)
    N, d = adj.shape[0], X.shape[1]
    _check_tab("X", X, X_hi, split, adj.shape[1], d)
    if not 0 <= row_lo <= row_hi <= N:
        raise native.EngineError(f"spmm_range: rows [{row_lo}, {row_hi}) outside [0, {N})")
    for name, lo, hi in (("Y1", Y1, Y1_hi), ("Y2", Y2, Y2_hi), ("A1", A1, A1_hi), ("A2", A2, A2_hi)):
        _check_tab(name, lo, hi, split, row_hi if hi is None else N, d)  # rows are addressed absolutely
    plan = adj.plan()
    ws = _ws_for(adj, d, X.device)
    if nbytes is None:
        nnz = adj.nnz
        if adj.bipartite_split is not None and (row_lo, row_hi) == (0, adj.bipartite_split):
            nnz = adj.nnz_below_split
        elif adj.bipartite_split is not None and (row_lo, row_hi) == (adj.bipartite_split, N):
            nnz = adj.nnz - adj.nnz_below_split
        rows = row_hi - row_lo
        nio = sum(x is not None for x in (Y1, Y2, A1, A2))
        nbytes = 8 * (rows + 1) + 8 * nnz + 4 * d * nnz + 4 * d * rows * nio
    with profiling.region(region, nbytes):
        native.check(native.lib().fr_spmm_csr_range(
            adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.val.data_ptr(), N, ctypes.byref(plan), int(split),
            ctypes.byref(_tab(X, X_hi)), d, ctypes.byref(_tab(Y1, Y1_hi)), ctypes.byref(_tab(Y2, Y2_hi)), _f(alpha),
            ctypes.byref(_tab(A1, A1_hi)), _f(beta1), ctypes.byref(_tab(A2, A2_hi)), _f(beta2), int(row_lo),
            int(row_hi), ws.data_ptr(), ws.numel(), native.stream_of(X)), "fr_spmm_csr_range")


def rows_mark(mask: torch.Tensor, rows, value: int, zero: torch.Tensor | None = None,
              bits: torch.Tensor | None = None) -> None:
    """mask[row] = value at the listed rows; with ``zero`` ([*, d] fp32), those rows of it set to 0;
    with ``bits`` (int32 words, bit row & 31 of word row >> 5), those bits set / cleared."""
    if zero is None and bits is None:
        native.check(native.lib().fr_rows_mark(mask.data_ptr(), ctypes.byref(_rowlist(rows)), int(value),
                                               native.stream_of(mask)), "fr_rows_mark")
        return
    native.check(native.lib().fr_rows_mark_zero(mask.data_ptr(), ctypes.byref(_rowlist(rows)), int(value),
                                                native.ptr(zero), zero.stride(0) if zero is not None else 0,
                                                zero.shape[1] if zero is not None else 0, native.ptr(bits),
                                                native.stream_of(mask)), "fr_rows_mark_zero")


SPARSE_UPSTREAM_MAX_ROWS = 262144  # HealthRec's UI backward in the sparse-upstream form up to here


def spmm_sparse_upstream(adj: Adjacency, bits: torch.Tensor, X: torch.Tensor, Y2, Y2_hi=None, split=0,
                         alpha=1.0, beta1=0.0, region="spmm_masked", zero=None):
    """fr_spmm_sparse_upstream: Y2 = alpha A X + beta1 gate(X) for an X that is non-zero only at the
    rows set in ``bits`` (int32 words); X is read only there.  d = 64; float-atomic summation order
    (non-deterministic mode only).  ``zero``: a contiguous fp32 tensor the same launch zeroes (a side
    job, fr_spmm_sparse_upstream_zero: the next kernel's accumulation target, no memset node)."""
    native.require_device(X, bits)
    N = adj.shape[0]
    if adj.shape[1] != N or X.shape[1] != 64 or X.shape[0] < N:
        raise native.EngineError("spmm_sparse_upstream: square adjacency, X [rows, 64]")
    if zero is not None and (zero.dtype != torch.float32 or not zero.is_contiguous() or zero.numel() % 4
                             or zero.data_ptr() % 16 or zero.device != X.device):
        raise native.EngineError("spmm_sparse_upstream: zero must be a contiguous 16-B aligned fp32 tensor "
                                 "(a multiple of 4 floats) on X's device")
    zp, zn = (zero.data_ptr(), zero.numel()) if zero is not None else (None, 0)
    if bits.dtype != torch.int32 or bits.numel() < (N + 31) // 32:
        raise native.EngineError("spmm_sparse_upstream: bits must be int32 with ceil(rows / 32) words")
    _check_tab("Y2", Y2, Y2_hi, split, N, 64)
    plan = _sparse_plan(adj)
    with profiling.region(region, sparse_upstream_bytes(adj)):
        if plan is not None:  # heavy rows (config 4's Zipf items): edge-balanced blocks
            _sparse_blocks(adj, False, bits, X, Y2, Y2_hi, split, alpha, X, beta1, plan, zero=zero)
            return
        native.check(native.lib().fr_spmm_sparse_upstream_zero(
            adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.val.data_ptr(), N, bits.data_ptr(), X.data_ptr(),
            X.stride(0), int(split), ctypes.byref(_tab(Y2, Y2_hi)), _f(alpha), ctypes.byref(_tab(X)), _f(beta1),
            zp, zn, native.stream_of(X)), "fr_spmm_sparse_upstream_zero")


def sparse_block_rows() -> int:
    """Rows per block of the sparse-upstream kernel: its LDS row accumulator (kSpRows), as the
    library exports it (fr_spmm_sparse_block_rows) -- never restated by hand."""
    return int(native.lib().fr_spmm_sparse_block_rows())


SPARSE_BLOCK_EDGES = 2048     # edge budget of a plan block (two 1024-edge scan rounds)
SPARSE_PLAN_TRIGGER = 8192    # use a plan when some uniform 64-row block would scan more edges


def check_sparse_plan(blocks: np.ndarray, rowptr: np.ndarray, max_rows: int) -> None:
    """Refuse a sparse-upstream block plan the kernel cannot run: a block of more than ``max_rows``
    rows (its LDS accumulator), rows outside the adjacency, or an edge range outside the block's rows
    (a multi-row block must cover its rows' edges exactly; a chunk is one row's sub-range)."""
    b = np.asarray(blocks, dtype=np.int64).reshape(-1, 4)
    rp = np.asarray(rowptr, dtype=np.int64)
    n = rp.shape[0] - 1
    lo, hi, e0, e1 = b[:, 0], b[:, 1], b[:, 2], b[:, 3]
    bad = (lo < 0) | (hi < lo) | (hi - lo > max_rows) | (hi > n)
    if bad.any():
        k = int(np.nonzero(bad)[0][0])
        raise native.EngineError(f"sparse block plan: block {k} rows [{lo[k]}, {hi[k]}) exceed the kernel's "
                                 f"{max_rows}-row accumulator or the adjacency's {n} rows")
    lo_c, hi_c = np.clip(lo, 0, n), np.clip(hi, 0, n)
    inside = (e0 >= rp[lo_c]) & (e1 <= rp[hi_c]) & (e0 <= e1)
    chunk = (e0 != rp[lo_c]) | (e1 != rp[hi_c])
    bad = ~inside | (chunk & (hi - lo != 1))
    if bad.any():
        k = int(np.nonzero(bad)[0][0])
        raise native.EngineError(f"sparse block plan: block {k} edges [{e0[k]}, {e1[k]}) leave rows "
                                 f"[{lo[k]}, {hi[k]})")


def sparse_block_plan(rowptr: np.ndarray, rows_per_block=None, edges=SPARSE_BLOCK_EDGES):
    """Edge-balanced row blocks for the sparse-upstream kernel: (blocks [n, 4] = (row_lo, row_hi,
    edge_lo, edge_hi), split_rows).  Cuts fall every ``rows_per_block`` rows, wherever the running
    edge count crosses a multiple of ``edges``, and around every row of more than ``edges`` edges;
    such a heavy row becomes ceil(deg / edges) chunks (listed in split_rows).  A block of light rows
    scans at most 2 * edges edges.  ``rows_per_block`` defaults to the kernel's exported limit and may
    not exceed it (check_sparse_plan)."""
    limit = sparse_block_rows()
    if rows_per_block is None:
        rows_per_block = limit
    if not 0 < rows_per_block <= limit:
        raise native.EngineError(f"sparse_block_plan: rows_per_block {rows_per_block} exceeds the kernel's "
                                 f"{limit}-row accumulator")
    rp = np.asarray(rowptr, dtype=np.int64)
    n = rp.shape[0] - 1
    if n <= 0:
        return np.zeros((0, 4), np.int64), np.zeros(0, np.int64)
    deg = np.diff(rp)
    heavy = np.nonzero(deg > edges)[0]
    band = rp // edges
    cuts = np.concatenate([np.arange(0, n + 1, rows_per_block), np.nonzero(band[1:] != band[:-1])[0] + 1,
                           heavy, heavy + 1, [0, n]])
    cuts = np.unique(cuts[(cuts >= 0) & (cuts <= n)])
    lo, hi = cuts[:-1], cuts[1:]
    single_heavy = (hi - lo == 1) & (deg[lo] > edges)
    light = np.stack([lo, hi, rp[lo], rp[hi]], 1)[~single_heavy]
    hr = lo[single_heavy]
    nch = (deg[hr] + edges - 1) // edges
    rows = np.repeat(hr, nch)
    k = np.arange(rows.shape[0]) - np.repeat(np.cumsum(nch) - nch, nch)
    e_lo = rp[rows] + k * edges
    e_hi = np.minimum(e_lo + edges, rp[rows + 1])
    chunks = np.stack([rows, rows + 1, e_lo, e_hi], 1)
    blocks = np.concatenate([light, chunks])
    blocks = blocks[np.argsort(blocks[:, 2], kind="stable")]
    check_sparse_plan(blocks, rp, limit)
    return blocks, hr.astype(np.int64)


def _sparse_plan(adj: Adjacency):
    """The adjacency's sparse-upstream block plan on its device, or None when uniform 64-row blocks
    are balanced enough (no block over SPARSE_PLAN_TRIGGER edges).  Built once per adjacency."""
    def make():
        rp = adj.rowptr.cpu().numpy()
        nb = sparse_block_rows()
        ends = rp[np.minimum(np.arange(nb, rp.shape[0] - 1 + nb, nb), rp.shape[0] - 1)]
        starts = rp[np.arange(0, rp.shape[0] - 1, nb)]
        if ends.shape[0] == 0 or int((ends - starts).max()) <= SPARSE_PLAN_TRIGGER:
            return False
        blocks, split_rows = sparse_block_plan(rp, nb, SPARSE_BLOCK_EDGES)
        dev = adj.rowptr.device
        return (torch.from_numpy(np.ascontiguousarray(blocks)).to(dev), torch.from_numpy(split_rows).to(dev))
    plan = _persistent(adj, "sparse_plan", make)
    return plan if plan is not False else None


def _sparse_blocks(adj, ungated, bits, X, Y2, Y2_hi, split, alpha, A1, beta1, plan, zero=None):
    blocks, split_rows = plan
    R, C = adj.shape
    zp, zn = (zero.data_ptr(), zero.numel()) if zero is not None else (None, 0)
    native.check(native.lib().fr_spmm_sparse_upstream_blocks_zero(
        adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.val.data_ptr(), R, C, int(ungated), bits.data_ptr(),
        X.data_ptr(), X.stride(0), int(split), ctypes.byref(_tab(Y2, Y2_hi)), _f(alpha), ctypes.byref(_tab(A1)),
        _f(beta1), blocks.data_ptr(), blocks.shape[0], split_rows.data_ptr(), split_rows.numel(), zp, zn,
        native.stream_of(X)), "fr_spmm_sparse_upstream_blocks_zero")


def spmm_scatter_upstream(adj: Adjacency, mask: torch.Tensor, bits: torch.Tensor, rows, X: torch.Tensor, Y2,
                          Y2_hi=None, split=0, alpha=1.0, beta1=0.0, region="spmm_masked"):
    """fr_spmm_scatter_upstream: spmm_sparse_upstream's Y2 = alpha A X + beta1 gate(X) for a symmetric
    adjacency, scattered from the listed rows' own CSR rows (work proportional to their degrees, not
    to the edge count); ``mask`` / ``bits`` mark the listed rows (rows_mark) and the listed rows' bits
    are clear on return.  d = 64; float-atomic summation order (non-deterministic mode only)."""
    native.require_device(X, bits, mask)
    N = adj.shape[0]
    if adj.shape[1] != N or not adj.symmetric or X.shape[1] != 64 or X.shape[0] < N:
        raise native.EngineError("spmm_scatter_upstream: symmetric square adjacency, X [rows, 64]")
    if bits.dtype != torch.int32 or bits.numel() < (N + 31) // 32 or mask.numel() < N:
        raise native.EngineError("spmm_scatter_upstream: uint8 mask and int32 bits over the rows")
    _check_tab("Y2", Y2, Y2_hi, split, N, 64)
    with profiling.region(region, scatter_upstream_bytes(adj, rows)):
        native.check(native.lib().fr_spmm_scatter_upstream(
            adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.val.data_ptr(), N, mask.data_ptr(), bits.data_ptr(),
            ctypes.byref(_rowlist(rows)), X.data_ptr(), X.stride(0), int(split), ctypes.byref(_tab(Y2, Y2_hi)),
            _f(alpha), _f(beta1), native.stream_of(X)), "fr_spmm_scatter_upstream")


def spmm_sparse_rect(adj: Adjacency, bits: torch.Tensor, X: torch.Tensor, Y2, alpha=1.0, A1=None, beta1=0.0,
                     region="spmm_masked"):
    """fr_spmm_sparse_upstream_rect: Y2 = alpha A X + beta1 A1 over a rectangular [rows x cols]
    slice, X non-zero only at the rows of X marked in ``bits`` (int32 words over cols) and read only
    there; A1 (optional) read at every row.  d = 64; float-atomic summation order."""
    native.require_device(X, bits)
    R, C = adj.shape
    if X.shape[1] != 64 or X.shape[0] < C or bits.dtype != torch.int32 or bits.numel() < (C + 31) // 32:
        raise native.EngineError("spmm_sparse_rect: X [cols, 64] and int32 bits over the columns required")
    _check_tab("Y2", Y2, None, 0, R, 64)
    _check_tab("A1", A1, None, 0, R, 64)
    plan = _sparse_plan(adj)
    with profiling.region(region, sparse_upstream_bytes(adj) + (256 * R if A1 is not None else 0)):
        if plan is not None:  # heavy rows (the transpose slice's Zipf items): edge-balanced blocks
            _sparse_blocks(adj, True, bits, X, Y2, None, 0, alpha, A1, beta1, plan)
            return
        native.check(native.lib().fr_spmm_sparse_upstream_rect(
            adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.val.data_ptr(), R, C, bits.data_ptr(), X.data_ptr(),
            X.stride(0), ctypes.byref(_tab(Y2)), _f(alpha), ctypes.byref(_tab(A1)), _f(beta1),
            native.stream_of(X)), "fr_spmm_sparse_upstream_rect")


def _adjacent_rows(lo, hi, rows):
    """[lo ; hi] as one [rows, d] view when hi's rows follow lo's in memory (same storage, contiguous
    row-major: a model placed them so, e.g. HealthRec.engine_layout), else None."""
    if not (lo.is_contiguous() and hi.is_contiguous() and lo.dim() == 2 and hi.dim() == 2
            and lo.shape[1] == hi.shape[1] and lo.dtype == hi.dtype
            and lo.untyped_storage().data_ptr() == hi.untyped_storage().data_ptr()
            and hi.data_ptr() == lo.data_ptr() + lo.numel() * lo.element_size()
            and lo.shape[0] + hi.shape[0] >= rows):
        return None
    return lo.as_strided((rows, lo.shape[1]), (lo.shape[1], 1))


def _prop_fwd_split(adj, lo, hi, split, L, lo_rows_only=False):
    """mean([E, A E, ..., A^L E]) for E = [lo ; hi] split at ``split`` (no concatenated copy).
    ``lo_rows_only`` (a bipartite adjacency split at ``split``, adj.mark_bipartite): only rows
    [0, split) of the mean are wanted -- the last layer is evaluated there only (half its edges);
    the other rows of the result are left unwritten."""
    N, d = adj.shape[0], lo.shape[1]
    if split == lo.shape[0]:
        one = _adjacent_rows(lo, hi, adj.shape[1])
        if one is not None:  # the tables are one buffer already: plain gathers
            lo, hi = one, None
    out = torch.empty(N, d, dtype=lo.dtype, device=lo.device)
    last = (0, split) if lo_rows_only and adj.bipartite_split == split else None
    if L == 1:
        if last is not None:
            spmm_range(adj, lo, *last, X_hi=hi, split=split, Y2=out, alpha=0.5, A1=lo, A1_hi=hi, beta1=0.5)
        else:
            spmm_ex(adj, lo, hi, split, Y2=out, alpha=0.5, A1=lo, A1_hi=hi, beta1=0.5)
        return out
    inv = 1.0 / (L + 1)
    E1 = torch.empty_like(out)
    if L == 2:
        spmm_ex(adj, lo, hi, split, Y1=E1)
        if last is not None:
            spmm_range(adj, E1, *last, Y2=out, alpha=inv, A1=lo, A1_hi=hi, beta1=inv, A2=E1, beta2=inv, split=split)
        else:
            spmm_ex(adj, E1, Y2=out, alpha=inv, A1=lo, A1_hi=hi, beta1=inv, A2=E1, beta2=inv, split=split)
        return out
    S = torch.empty_like(out)
    spmm_ex(adj, lo, hi, split, Y1=E1, Y2=S, alpha=1.0, A1=lo, A1_hi=hi, beta1=1.0)
    prev, nxt = E1, torch.empty_like(out)
    for _ in range(2, L):
        spmm_launch(adj, prev, Y1=nxt, Y2=S, alpha=1.0, A1=S, beta1=1.0)
        prev, nxt = nxt, prev
    if last is not None:
        spmm_range(adj, prev, *last, Y2=out, alpha=inv, A1=S, beta1=inv)
    else:
        spmm_launch(adj, prev, Y2=out, alpha=inv, A1=S, beta1=inv)
    return out


def _prop_bwd_split(adj, G, L, out_lo, out_hi, split, col_mask=None, gate=False):
    """d/dE of mean_k A^k E (A symmetric) for upstream G, written into [out_lo ; out_hi] split at
    ``split``.  ``col_mask``: rows where G is known to be zero (first layer only); ``gate`` (L = 1):
    G is only valid at those rows (not zero-filled elsewhere), so its residual read is gated too."""
    inv = 1.0 / (L + 1)
    # a masked launch skips most gathers: not a full-gather (roofline) launch, timed under its own name
    reg = "spmm_masked" if col_mask is not None else "spmm"
    nb = 0 if col_mask is not None else None
    if L == 1:
        spmm_ex(adj, G, Y2=out_lo, Y2_hi=out_hi, split=split, alpha=inv, A1=G, beta1=inv, col_mask=col_mask,
                a1_gate=col_mask if gate else None, region=reg, nbytes=nb)
        return
    H = torch.empty_like(G)
    spmm_ex(adj, G, Y2=H, alpha=inv, A1=G, beta1=inv, col_mask=col_mask, region=reg, nbytes=nb)
    H2 = torch.empty_like(G) if L > 2 else None
    for _ in range(1, L - 1):
        spmm_launch(adj, H, Y2=H2, alpha=1.0, A1=G, beta1=inv)
        H, H2 = H2, H
    spmm_ex(adj, H, Y2=out_lo, Y2_hi=out_hi, split=split, alpha=1.0, A1=G, beta1=inv)


def _prop_bwd_ri(adj, G, L, out_lo, out_hi, split, front=None, zeroed=False):
    """The RI backward of graph_bpr (G zero at the ingredient rows): the half-graph form on a
    bipartite adjacency with two layers, _prop_bwd_split otherwise.  ``front``: the forward's
    frontier list (lst, cnt) when G's item rows are zero outside it (the fast UI backward writes
    them from the batch rows only) -- the ingredient rows R^T g / 3 are then the listed rows'
    scatter (fr_spmm_list_scatter, which zeroes them first) instead of a gather over every
    ingredient row.  (Zeroing d ingre at the backward's start instead, ahead of the UI backward,
    measured ~5 us/step slower.)"""
    if L == 2 and adj.bipartite_split == split and not _RI_FULL_GRAPH:
        if front is not None and adj.symmetric:
            inv = 1.0 / 3.0
            g = G[:split]
            lst, cnt = front[0], front[1]
            # the frontier's item rows (expected count: front[2], the count itself is on the device)
            # scattered into the ingredient rows: X row read, per edge col/val + an atomic row update
            nf = front[2] if len(front) > 2 else int(lst.numel())
            with profiling.region("spmm_rows", int(nf * (16 + 256 + mean_degree(adj, 0) * (8 + 512)))):
                native.check(native.lib().fr_spmm_list_scatter(
                    adj.rowptr.data_ptr(), adj.col.data_ptr(), adj.val.data_ptr(), adj.shape[0], split,
                    lst.data_ptr(), cnt.data_ptr(), split, g.data_ptr(), g.stride(0), out_hi.data_ptr(),
                    out_hi.stride(0), _f(inv), 0 if zeroed else 1, native.stream_of(g)), "fr_spmm_list_scatter")
            spmm_range(adj, g, 0, split, X_hi=out_hi, split=split, Y2=out_lo, alpha=1.0, A1=g, beta1=inv)
            return
        _prop_bwd_bipartite2(adj, G[:split], out_lo, out_hi, split)
    else:
        _prop_bwd_split(adj, G, L, out_lo, out_hi, split)


_RI_FULL_GRAPH = False  # test hook: True runs the full-graph RI launches


def _persistent(adj, key, make):
    cache = adj.__dict__.setdefault("_persist", {})
    t = cache.get(key)
    if t is None:
        t = make()
        cache[key] = t
    return t


def grad_buffer(w: torch.Tensor) -> torch.Tensor:
    """Where a backward writes parameter ``w``'s full gradient: the slot a data-parallel gradient
    hook keeps for it in its flat all-reduce buffer (engine.dist.GradAllReduce sets
    ``w._fr_grad_dest``; autograd adopts the returned view as ``w.grad``, so the hook's pack has
    nothing to copy), else a new tensor."""
    dest = w.__dict__.get("_fr_grad_dest")
    if dest is not None:
        v = dest()
        if v is not None and v.shape == w.shape and v.dtype == w.dtype and v.device == w.device:
            return v
    return torch.empty_like(w)


# FR_RI_FRONTIER=0: HealthRec's RI forward at every item row (full layer 1, item rows of layer 2)
RI_FRONTIER = os.environ.get("FR_RI_FRONTIER", "1") != "0"
# FR_RI_FRONTIER_BWD=0: the RI backward's ingredient rows gathered over every ingredient row instead
# of scattered from the frontier rows (the only item rows of its upstream gradient that are non-zero)
RI_FRONTIER_BWD = os.environ.get("FR_RI_FRONTIER_BWD", "1") != "0"


def _ri_fwd_frontier(ri_adj, ui_adj, item_w, ingre_w, U, I, u, p, n):
    """mean(E, A E, A^2 E) of the bipartite RI graph at the item rows the batch's UI layer reads:
    layer 1 over every ingredient row (layer 2 reads them all) and at the listed item rows, layer 2
    at the listed item rows.  Rows outside the list are left unwritten (nothing reads them).
    Returns (rows, (list, count)); the list (this forward's own buffers) also serves the backward."""
    dev = item_w.device
    N = ri_adj.shape[0]
    lib = native.lib()
    s = native.stream_of(item_w)
    mark = _persistent(ri_adj, ("front_mark", str(dev)), lambda: torch.zeros(I, dtype=torch.uint8, device=dev))
    lst = torch.empty(I, dtype=torch.int32, device=dev)
    cnt = torch.empty(1, dtype=torch.int32, device=dev)  # (reset by fr_rows_frontier)
    native.check(lib.fr_rows_frontier(ui_adj.rowptr.data_ptr(), ui_adj.col.data_ptr(), U, I, u.data_ptr(), p.data_ptr(),
                                      n.data_ptr(), int(u.numel()), mark.data_ptr(), lst.data_ptr(), cnt.data_ptr(), s),
                 "fr_rows_frontier")
    inv = 1.0 / 3.0
    out = torch.empty(N, 64, dtype=torch.float32, device=dev)
    E1 = torch.empty_like(out)
    spmm_range(ri_adj, item_w, I, N, X_hi=ingre_w, split=I, Y1=E1)  # layer 1, ingredient rows
    args = (ri_adj.rowptr.data_ptr(), ri_adj.col.data_ptr(), ri_adj.val.data_ptr(), N, I)
    nf = frontier_rows(ui_adj, int(u.numel()), I)
    # two row-list layers over the frontier's item rows: layer 1 writes E1, layer 2 writes out and
    # reads the two addends (item_w / ingre_w and E1)
    with profiling.region("spmm_rows", rows_bytes(ri_adj, nf, 64, 1) + rows_bytes(ri_adj, nf, 64, 3)):
        native.check(lib.fr_spmm_csr_list(*args, ctypes.byref(_tab(item_w, ingre_w)), ctypes.byref(_tab(E1)),
                                          ctypes.byref(_tab(None)), _f(1.0), ctypes.byref(_tab(None)), _f(0.0),
                                          ctypes.byref(_tab(None)), _f(0.0), lst.data_ptr(), cnt.data_ptr(), I, s),
                     "fr_spmm_csr_list")  # layer 1, listed item rows
        native.check(lib.fr_spmm_csr_list(*args, ctypes.byref(_tab(E1)), ctypes.byref(_tab(None)),
                                          ctypes.byref(_tab(out)), _f(inv), ctypes.byref(_tab(item_w, ingre_w)),
                                          _f(inv), ctypes.byref(_tab(E1)), _f(inv), lst.data_ptr(), cnt.data_ptr(), I,
                                          s), "fr_spmm_csr_list")  # layer 2, listed item rows
    return out, (lst, cnt, nf)


class _GraphBprForward:
    """The forward of _GraphBpr computed ahead of its autograd node (graph_bpr_begin), possibly on a
    branch stream: the outputs and the tensors the backward reads."""
    __slots__ = ("out", "item_rows", "ui_all", "u", "p", "n", "pn", "ws", "stream", "done", "args", "defer", "front")


@torch.no_grad()
def _graph_bpr_forward(user_w, item_w, ingre_w, u, p, n, pn, ri_adj, ui_adj, L_ri, L_ui, gamma, stream=None):
    U, I = user_w.shape[0], item_w.shape[0]
    dev = user_w.device
    native.require_device(user_w, item_w, ingre_w, u, p, n)
    for t in (user_w, item_w, ingre_w):
        if t.dtype != torch.float32 or t.shape[1] != 64 or not t.is_contiguous():
            raise native.EngineError("graph_bpr: contiguous fp32 [rows, 64] tables required")
    u, p, n, pn = (x.to(torch.int64).contiguous() for x in (u, p, n, pn))
    rows = [(u, 0), (p, U), (n, U)]
    if L_ui == 1 and L_ri == 2 and ri_adj.bipartite_split == I and ui_adj.bipartite_split == U and RI_FRONTIER:
        # the UI layer at the batch rows reads item_ir only at the batch users' items and the batch
        # items: the RI propagation's item rows are evaluated there only (device-built row list)
        ir_all, front = _ri_fwd_frontier(ri_adj, ui_adj, item_w, ingre_w, U, I, u, p, n)
    else:
        front = None
        # [I + NI, 64]; only the item rows are read (the reference discards the propagated ingredients)
        ir_all = _prop_fwd_split(ri_adj, item_w, ingre_w, I, L_ri, lo_rows_only=True)
    if L_ui == 1:
        ui_all = torch.empty(U + I, 64, dtype=torch.float32, device=dev)  # valid at the batch rows
        spmm_ex(ui_adj, user_w, ir_all, U, Y2=ui_all, alpha=0.5, A1=user_w, A1_hi=ir_all, beta1=0.5,
                rows=rows, region="spmm_rows")
    else:
        ui_all = _prop_fwd_split(ui_adj, user_w, ir_all, U, L_ui)
    B = int(u.numel())
    lib = native.lib()
    ws = native.workspace(lib.fr_bpr_workspace(B), dev)
    out = torch.empty(5, dtype=torch.float32, device=dev)
    items = ui_all[U:]
    item_rows = torch.empty(2 * B, 64, dtype=torch.float32, device=dev)  # [items[p] ; items[n]] (= items[pn])
    native.check(lib.fr_bpr_fwd_rows(ui_all.data_ptr(), 64, items.data_ptr(), 64, user_w.data_ptr(), 64,
                                     item_w.data_ptr(), 64, u.data_ptr(), p.data_ptr(), n.data_ptr(), B, 64,
                                     _f(gamma), out.data_ptr(), item_rows.data_ptr(), 64, ws.data_ptr(), ws.numel(),
                                     native.stream_of(user_w)), "fr_bpr_fwd_rows")
    f = _GraphBprForward()
    f.out, f.item_rows, f.ui_all, f.u, f.p, f.n, f.pn, f.ws, f.stream = out, item_rows, ui_all, u, p, n, pn, ws, stream
    f.defer = ingre_w.__dict__.get("_fr_defer_rows")
    f.front = front if RI_FRONTIER_BWD else None
    return f


class _GraphBpr(torch.autograd.Function):
    """HealthRec's propagation + BPR + user/item EmbLoss (cikm_model.py:182-208, 255-279) as one
    autograd node:

    forward   RI: mean over n_layers of A_RI^k [item ; ingre[:-1]]  (split-table reads, full graph)
              UI: (ego + A_UI ego) / 2 at the batch's users and items only (row-list mode: the
                  loss reads ui_all at u, U + pos, U + neg and nowhere else), ego = [user ; item_ir]
              fused BPR + EmbLoss on those rows; the [pos; neg] item rows returned for the KD term
    backward  BPR scatter into dUI (+ the KD rows' gradient); UI backward over the edges into the
              batch rows only (column mask), written straight into d user_embedding and the item
              block of the RI upstream gradient (its ingredient block is a persistent zero); RI
              backward written straight into d item_embedding and d ingre_embedding[:-1]; the
              EmbLoss ego-row gradients accumulated in place.  No concatenation, split, slice or
              gradient-sum kernels.
    ui_layers > 1: the UI propagation is evaluated in full (the loss rows' dependency cone spans
    the graph) with the same split-table reads and writes."""

    @staticmethod
    def forward(ctx, user_w, item_w, ingre_w, u, p, n, pn, ri_adj, ui_adj, L_ri, L_ui, gamma, det, pre=None):
        if pre is None:
            pre = _graph_bpr_forward(user_w, item_w, ingre_w, u, p, n, pn, ri_adj, ui_adj, L_ri, L_ui, gamma)
        out, item_rows, ui_all, u, p, n, pn, ws = pre.out, pre.item_rows, pre.ui_all, pre.u, pre.p, pre.n, pre.pn, pre.ws
        U, I, NI = user_w.shape[0], item_w.shape[0], ingre_w.shape[0] - 1
        ctx.save_for_backward(user_w, item_w, ui_all, u, p, n, pn)
        ctx.ingre_w = ingre_w  # the parameter itself (grad_buffer looks up its gradient destination)
        ctx.defer = pre.defer  # (taken at the forward's start: embedding_norms pops the slot meanwhile)
        ctx.branch = pre.stream  # the branch stream the forward ran on (None: the current stream)
        ctx.front = pre.front  # the RI frontier rows (list, count), or None
        ctx.meta = (ri_adj, ui_adj, L_ri, L_ui, gamma, int(bool(det)), ws, U, I, NI)
        return out[0], out[4:5], item_rows

    @staticmethod
    def backward(ctx, g_mf, g_emb, g_rows):
        side = ctx.branch
        if side is None:
            return _GraphBpr._backward_here(ctx, g_mf, g_emb, g_rows)
        # branch: the kernels go to the branch stream, which waits only for what the current stream
        # has issued so far (the loss heads' backward); the rest of the backward (encoder, fusion,
        # projections) proceeds on the current stream meanwhile.  The backward pass ends by joining
        # (_join_branch, an autograd final callback): the current stream waits for the branch, then
        # the deferred ingredient rows are added into its d ingre.
        main = torch.cuda.current_stream(side.device)
        side.wait_stream(main)
        for g in (g_mf, g_emb, g_rows):
            if g is not None:
                g.record_stream(side)
        with torch.cuda.stream(side):
            grads = _GraphBpr._backward_here(ctx, g_mf, g_emb, g_rows, drain=False)
            done = torch.cuda.Event()
            done.record(side)
        user_w, item_w = ctx.saved_tensors[:2]
        if ctx.defer is None or any(w.grad is not None for w in (user_w, item_w, ctx.ingre_w)):
            # autograd consumes the returned grads on the current stream right away when it has to
            # sum them (another gradient of the same table, or an existing .grad): join here
            main.wait_event(done)
        _BRANCH_PENDING.append((done, ctx.defer, ctx.ingre_w))  # (no reference to the returned grads:
        # AccumulateGrad adopts them as .grad only when nothing else holds them)
        # queued by every branch backward (idempotent: the first callback joins every pending entry),
        # so an entry left behind by a failed backward cannot keep later ones from being joined
        torch.autograd.Variable._execution_engine.queue_callback(_join_branch)
        return grads

    @staticmethod
    def _backward_here(ctx, g_mf, g_emb, g_rows, drain=True):
        user_w, item_w, ui_all, u, p, n, pn = ctx.saved_tensors
        ri_adj, ui_adj, L_ri, L_ui, gamma, det, ws, U, I, NI = ctx.meta
        dev = user_w.device
        if not det and L_ui == 1 and g_rows is not None and g_mf is not None and g_emb is not None:
            return _GraphBpr._backward_fast(ctx, g_mf, g_emb, g_rows, drain)
        g_mf = g_mf if g_mf is not None else torch.zeros((), device=dev)
        g_emb = g_emb if g_emb is not None else torch.zeros(1, device=dev)
        gscale = torch.cat([g_mf.reshape(1), g_emb.reshape(1)]).float().contiguous()
        B = int(u.numel())
        lib = native.lib()
        s = native.stream_of(user_w)
        items = ui_all[U:]
        dUI = torch.zeros(U + I, 64, dtype=torch.float32, device=dev)
        dI = dUI[U:]
        common = (ui_all.data_ptr(), 64, items.data_ptr(), 64, user_w.data_ptr(), 64, item_w.data_ptr(), 64,
                  u.data_ptr(), p.data_ptr(), n.data_ptr(), B, 64, _f(gamma), _f(1.0), _f(1.0), gscale.data_ptr())
        with profiling.region("bpr_bwd", bpr_bwd_bytes(int(u.numel()))):
            if g_rows is not None and not det:
                g_rows = g_rows.contiguous()
                native.check(lib.fr_bpr_bwd_ex(*common, dUI.data_ptr(), dI.data_ptr(), None, None, g_rows.data_ptr(),
                                               g_rows.stride(0), ws.data_ptr(), ws.numel(), s), "fr_bpr_bwd_ex")
            else:
                native.check(lib.fr_bpr_bwd(*common, dUI.data_ptr(), dI.data_ptr(), None, None, det, ws.data_ptr(),
                                            ws.numel(), s), "fr_bpr_bwd")
                if g_rows is not None:
                    dI.index_add_(0, pn, g_rows)
        d_user = torch.empty_like(user_w)
        # RI upstream gradient: [d item_ir ; 0] -- the ingredient block is never written (persistent zero)
        G_ri = _persistent(ri_adj, ("g_ri", str(dev)), lambda: torch.zeros(I + NI, 64, device=dev))
        if L_ui == 1:
            mask = _persistent(ui_adj, ("mask", str(dev)), lambda: torch.zeros(U + I, dtype=torch.uint8, device=dev))
            rows = [(u, 0), (p, U), (n, U)]
            rows_mark(mask, rows, 1)
            _prop_bwd_split(ui_adj, dUI, 1, d_user, G_ri, U, col_mask=mask)
            rows_mark(mask, rows, 0)
        else:
            _prop_bwd_split(ui_adj, dUI, L_ui, d_user, G_ri, U)
        d_item = torch.empty_like(item_w)
        d_ingre = torch.empty(NI + 1, 64, dtype=torch.float32, device=dev)
        _prop_bwd_ri(ri_adj, G_ri, L_ri, d_item, d_ingre, I)
        d_ingre[NI:].zero_()  # the padding row is not a graph node
        # EmbLoss on the ego rows, accumulated into the propagation gradients
        with profiling.region("bpr_bwd", bpr_bwd_bytes(int(u.numel()))):
            native.check(lib.fr_bpr_bwd(*common, None, None, d_user.data_ptr(), d_item.data_ptr(), det, ws.data_ptr(),
                                        ws.numel(), s), "fr_bpr_bwd")
        if ctx.defer is not None and drain:
            ctx.defer.drain(d_ingre)
        return (d_user, d_item, d_ingre) + (None,) * 11

    @staticmethod
    def _backward_fast(ctx, g_mf, g_emb, g_rows, drain=True):
        """Float-atomic path for one UI layer: mark the batch rows in the column mask and its bitmask
        and zero them in the persistent UI upstream gradient (no full fill: its other rows are never
        read, the backward gates its residual read by the same mask); the BPR scatter (+ the KD rows'
        gradient) with g_mf read on the device; the UI backward from those rows only
        (fr_spmm_sparse_upstream: edge scan against the bitmask, gathers at the marked columns) into
        d user_embedding and the item block of the RI upstream gradient; the RI backward into
        d item_embedding and d ingre_embedding[:-1]; fr_graph_bpr_finish: unmark, the ego rows'
        EmbLoss gradient, the padding row's zero."""
        user_w, item_w, ui_all, u, p, n, pn = ctx.saved_tensors
        ri_adj, ui_adj, L_ri, L_ui, gamma, det, ws, U, I, NI = ctx.meta
        dev = user_w.device
        B = int(u.numel())
        lib = native.lib()
        s = native.stream_of(user_w)
        items = ui_all[U:]
        g_mf = g_mf.float().contiguous()
        g_emb = g_emb.float().contiguous()
        g_rows = g_rows.contiguous()
        dUI = _persistent(ui_adj, ("g_ui", str(dev)), lambda: torch.empty(U + I, 64, device=dev))
        mask = _persistent(ui_adj, ("mask", str(dev)), lambda: torch.zeros(U + I, dtype=torch.uint8, device=dev))
        sparse = U + I <= SPARSE_UPSTREAM_MAX_ROWS
        bits = (_persistent(ui_adj, ("bits", str(dev)),
                            lambda: torch.zeros((U + I + 31) // 32, dtype=torch.int32, device=dev)) if sparse else None)
        rows = [(u, 0), (p, U), (n, U)]
        rows_mark(mask, rows, 1, zero=dUI, bits=bits)
        with profiling.region("bpr_bwd", bpr_bwd_bytes(int(u.numel()))):
            native.check(lib.fr_bpr_bwd_ex(ui_all.data_ptr(), 64, items.data_ptr(), 64, user_w.data_ptr(), 64,
                                           item_w.data_ptr(), 64, u.data_ptr(), p.data_ptr(), n.data_ptr(), B, 64,
                                           _f(gamma), _f(1.0), _f(0.0), g_mf.data_ptr(), dUI.data_ptr(),
                                           dUI[U:].data_ptr(), None, None, g_rows.data_ptr(), g_rows.stride(0),
                                           ws.data_ptr(), ws.numel(), s), "fr_bpr_bwd_ex")
        d_user = grad_buffer(user_w)
        G_ri = _persistent(ri_adj, ("g_ri", str(dev)), lambda: torch.zeros(I + NI, 64, device=dev))
        # (the scatter form, spmm_scatter_upstream, measured 362 us against this scan's 50 us at
        # Allrecipes shape: the batch items are popularity-drawn positives, so the marked rows' degree
        # sum is a large share of the edges and a heavy row serialises on one wave)
        d_item = grad_buffer(item_w)
        d_ingre = grad_buffer(ctx.ingre_w)
        # the RI backward's list scatter accumulates into d ingre's first NI rows: the UI backward's
        # launch zeroes them on the side (no memset node between the two)
        zero = d_ingre[:NI] if (SPARSE_ZERO_SIDE and sparse and ctx.front is not None and ri_adj.symmetric
                                and L_ri == 2 and d_ingre.is_contiguous() and d_ingre.data_ptr() % 16 == 0) else None
        if sparse:
            spmm_sparse_upstream(ui_adj, bits, dUI, d_user, G_ri, U, alpha=0.5, beta1=0.5, zero=zero)
        else:
            _prop_bwd_split(ui_adj, dUI, 1, d_user, G_ri, U, col_mask=mask, gate=True)
        # (the fast UI backward writes G_ri's item rows from the batch rows: non-zero at the frontier only)
        _prop_bwd_ri(ri_adj, G_ri, L_ri, d_item, d_ingre, I, front=ctx.front, zeroed=zero is not None)
        with profiling.region("bpr_bwd", bpr_finish_bytes(int(u.numel()))):
            native.check(lib.fr_graph_bpr_finish(mask.data_ptr(), U, user_w.data_ptr(), 64, item_w.data_ptr(), 64,
                                                 u.data_ptr(), p.data_ptr(), n.data_ptr(), B, 64, _f(1.0),
                                                 g_emb.data_ptr(), d_user.data_ptr(), d_item.data_ptr(),
                                                 d_ingre[NI:].data_ptr(), 64, native.ptr(bits), ws.data_ptr(),
                                                 ws.numel(), s),
                         "fr_graph_bpr_finish")
        if ctx.defer is not None and drain:
            ctx.defer.drain(d_ingre)  # the encoder input rows' gradient, atomically into d ingre
        return (d_user, d_item, d_ingre) + (None,) * 11


# FR_SPARSE_ZERO=0: HealthRec's d ingre rows zeroed by the list scatter's own memset node instead of on
# the side of the UI backward's launch
SPARSE_ZERO_SIDE = os.environ.get("FR_SPARSE_ZERO", "1") != "0"
UI_BPR = os.environ.get("FR_UI_BPR", "1") != "0"  # FR_UI_BPR=0: CLUSSL's UI layer + BPR unfused


class _UiBpr(torch.autograd.Function):
    """One UI propagation layer + BPR + EmbLoss as one node (CLUSSL, pricai_modelx.py:226-267 with
    n_ui_layers = 1): the propagation of [user ; item_hi] evaluated at the batch rows only (the loss
    reads nothing else), BPR on them, EmbLoss on the ego rows (user_w, item_w) times w_emb.  Backward:
    the batch rows marked and zeroed in a persistent upstream buffer, the BPR scatter into it, the UI
    backward from those rows only (fr_spmm_sparse_upstream) straight into d user_w and d item_hi,
    then fr_graph_bpr_finish (unmark, the ego rows' EmbLoss gradient).  Replaces the full-graph
    propagation forward and backward, the dense zero-filled upstream and the split / accumulation
    glue of propagate_mean + bpr_emb_loss."""

    @staticmethod
    def forward(ctx, user_w, item_hi, item_w, u, p, n, ui_adj, gamma, w_emb):
        U, I = user_w.shape[0], item_hi.shape[0]
        dev = user_w.device
        u, p, n = (x.to(torch.int64).contiguous() for x in (u, p, n))
        rows = [(u, 0), (p, U), (n, U)]
        ui_all = torch.empty(U + I, 64, dtype=torch.float32, device=dev)  # valid at the batch rows
        spmm_ex(ui_adj, user_w, item_hi, U, Y2=ui_all, alpha=0.5, A1=user_w, A1_hi=item_hi, beta1=0.5, rows=rows,
                region="spmm_rows")
        B = int(u.numel())
        lib = native.lib()
        ws = native.workspace(lib.fr_bpr_workspace(B), dev)
        out = torch.empty(5, dtype=torch.float32, device=dev)
        items = ui_all[U:]
        native.check(lib.fr_bpr_fwd_ex(ui_all.data_ptr(), 64, items.data_ptr(), 64, user_w.data_ptr(), 64,
                                       item_w.data_ptr(), 64, u.data_ptr(), p.data_ptr(), n.data_ptr(), B, 64,
                                       _f(gamma), _f(w_emb), out.data_ptr(), None, 0, ws.data_ptr(), ws.numel(),
                                       native.stream_of(user_w)), "fr_bpr_fwd_ex")
        ctx.save_for_backward(user_w, item_w, ui_all, u, p, n)
        ctx.meta = (ui_adj, float(gamma), float(w_emb), ws, U, I, tuple(item_hi.shape))
        sink = item_w.__dict__.get("_fr_emb_rows")
        ctx.sink = sink if sink is not None and sink.open else None  # (opened by this pass's item views)
        return out[0], out[4:5]

    @staticmethod
    def backward(ctx, g_mf, g_emb):
        user_w, item_w, ui_all, u, p, n = ctx.saved_tensors
        ui_adj, gamma, w_emb, ws, U, I, hi_shape = ctx.meta
        dev = user_w.device
        B = int(u.numel())
        lib = native.lib()
        s = native.stream_of(user_w)
        gm = None if g_mf is None or _is_unit(g_mf) else g_mf.float().contiguous()
        ge = None if g_emb is None or _is_unit(g_emb) else g_emb.float().contiguous()
        dUI = _persistent(ui_adj, ("g_ui", str(dev)), lambda: torch.empty(U + I, 64, device=dev))
        mask = _persistent(ui_adj, ("mask", str(dev)), lambda: torch.zeros(U + I, dtype=torch.uint8, device=dev))
        bits = _persistent(ui_adj, ("bits", str(dev)),
                           lambda: torch.zeros((U + I + 31) // 32, dtype=torch.int32, device=dev))
        rows = [(u, 0), (p, U), (n, U)]
        rows_mark(mask, rows, 1, zero=dUI, bits=bits)
        with profiling.region("bpr_bwd", bpr_bwd_bytes(int(u.numel()))):
            native.check(lib.fr_bpr_bwd(ui_all.data_ptr(), 64, ui_all[U:].data_ptr(), 64, user_w.data_ptr(), 64,
                                        item_w.data_ptr(), 64, u.data_ptr(), p.data_ptr(), n.data_ptr(), B, 64, _f(gamma),
                                        _f(0.0 if g_mf is None else 1.0), _f(0.0), native.ptr(gm), dUI.data_ptr(),
                                        dUI[U:].data_ptr(), None, None, 0, ws.data_ptr(), ws.numel(), s), "fr_bpr_bwd")
        d_user = grad_buffer(user_w)
        d_hi = torch.empty(hi_shape, dtype=torch.float32, device=dev)
        spmm_sparse_upstream(ui_adj, bits, dUI, d_user, d_hi, U, alpha=0.5, beta1=0.5)
        # the ego item rows' EmbLoss gradient: parked for the item views' backward (which adds it into
        # its d item), else a dense zero-filled gradient of its own
        sink = ctx.sink if ctx.sink is not None and ctx.sink.open and g_emb is not None else None
        d_item = None if sink is not None else torch.zeros_like(item_w)
        with profiling.region("bpr_bwd", bpr_finish_bytes(int(u.numel()))):
            native.check(lib.fr_graph_bpr_finish(mask.data_ptr(), U, user_w.data_ptr(), 64, item_w.data_ptr(), 64,
                                                 u.data_ptr(), p.data_ptr(), n.data_ptr(), B, 64,
                                                 _f(0.0 if g_emb is None else w_emb), native.ptr(ge), d_user.data_ptr(),
                                                 native.ptr(d_item), None, 0, bits.data_ptr(), ws.data_ptr(), ws.numel(),
                                                 s), "fr_graph_bpr_finish")
        if sink is not None:
            sink.entries.append((user_w, item_w, u, p, n, ws, w_emb, ge))
        return d_user, d_hi, d_item, None, None, None, None, None, None


def ui_bpr(ui_adj, user_w, item_hi, item_w, u, p, n, gamma: float = 1e-10, w_emb: float = 1.0):
    """(BPRLoss, w_emb * EmbLoss) of ``propagate_mean(ui_adj, cat([user_w, item_hi]), 1)`` at
    (u, U + p, U + n) with EmbLoss over the ego rows (user_w[u], item_w[p], item_w[n]) -- one node
    (_UiBpr) when the sparse-upstream backward applies, else propagate_mean_split + bpr_emb_loss."""
    U, I = user_w.shape[0], item_hi.shape[0]
    ok = (UI_BPR and not _DETERMINISTIC and user_w.is_cuda and all(t.dtype == torch.float32 and t.dim() == 2 and t.shape[1] == 64
                                                        and t.is_contiguous() for t in (user_w, item_hi, item_w))
          and U + I == ui_adj.shape[0] and U + I <= SPARSE_UPSTREAM_MAX_ROWS and getattr(ui_adj, "symmetric", False)
          and item_w.shape[0] == I)
    if not ok:
        ui = propagate_mean_split(ui_adj, user_w, item_hi, 1)
        return bpr_emb_loss(ui, None, user_w, item_w, u, p, n, gamma=gamma, item_offset=U, w_emb=w_emb)
    return _UiBpr.apply(user_w, item_hi, item_w, u, p, n, ui_adj, float(gamma), float(w_emb))


# graph_bpr_begin / _end on a branch stream (HealthRec's propagation beside its encoder); FR_BRANCH_STREAMS=0: off
BRANCH_STREAMS = os.environ.get("FR_BRANCH_STREAMS", "1") != "0"
AUX_STREAM = os.environ.get("FR_AUX_STREAM", "0") == "1"  # ops.aux_stream (FR_AUX_STREAM=1: on; measured no gain)
_BRANCH_STREAM = {}
_BRANCH_PENDING = []    # (event, deferred rows, ingredient table) of branch backwards not joined yet


# FR_STREAM_PRIO="branch=-1,loss=-1,...": HIP stream priorities of the engine's side streams (roles
# branch, aux, loss, side, rows; lower = higher priority; default: torch's default priority)
_STREAM_PRIO = {k: int(v) for k, v in (kv.split("=") for kv in os.environ.get("FR_STREAM_PRIO", "").split(",") if kv)}


def new_stream(device, role: str):
    """A side stream of the engine for ``role`` (its FR_STREAM_PRIO priority when set)."""
    if role in _STREAM_PRIO:
        return torch.cuda.Stream(device, priority=_STREAM_PRIO[role])
    return torch.cuda.Stream(device)


def _branch_stream(device):
    s = _BRANCH_STREAM.get(device)
    if s is None:
        s = new_stream(device, "branch")
        _BRANCH_STREAM[device] = s
    return s


def aux_stream(device):
    """A second branch stream (HealthRec's modal projections beside its encoder), or None when
    branching is off."""
    if not (BRANCH_STREAMS and AUX_STREAM):
        return None
    key = ("aux", str(device))
    s = _BRANCH_STREAM.get(key)
    if s is None:
        s = new_stream(device, "aux")
        _BRANCH_STREAM[key] = s
    return s


# FR_LATE_DRAIN=0: the deferred ingredient rows are always added at the end of the backward pass
LATE_DRAIN = os.environ.get("FR_LATE_DRAIN", "1") != "0"
_LATE_DRAIN = [False]   # set by the trainer around a backward whose gradients FusedAdam.step reads next
_PENDING_DRAINS = []    # (fork event, deferred rows, table) left by _join_branch in late mode


def late_drain(on: bool) -> None:
    """The trainer's promise for the next backward pass: nothing but FusedAdam.step reads its
    gradients.  The deferred ingredient rows are then not added at the end of the pass but by
    run_pending_drains, which FusedAdam.step calls after launching the update of every other
    tensor: the scatter runs on the branch stream beside that update instead of before it."""
    _LATE_DRAIN[0] = bool(on) and LATE_DRAIN


def pending_drain_params() -> set:
    return {id(w) for _, _, w in _PENDING_DRAINS}


def run_pending_drains(after=None) -> None:
    """Add the rows _join_branch left (late mode) into their tables' gradients on the branch stream,
    forked where the backward pass ended; the current stream waits for them (before the update of
    those tables).  ``after(stream)``: more work issued on the branch stream behind the last drain,
    before the current stream's join (FusedAdam: the drained tables' own update)."""
    pend = list(_PENDING_DRAINS)
    _PENDING_DRAINS.clear()
    for k, (fork, defer, ingre_w) in enumerate(pend):
        main = torch.cuda.current_stream(ingre_w.device)
        side = _branch_stream(ingre_w.device)
        side.wait_event(fork)
        for t in defer.tensors():
            t.record_stream(side)
        if ingre_w.grad is not None:
            ingre_w.grad.record_stream(side)
        with torch.cuda.stream(side):
            _drain_into(defer, ingre_w)
            if after is not None and k == len(pend) - 1:
                after(side)
            done = torch.cuda.Event()
            done.record(side)
        main.wait_event(done)


def _drain_into(defer, ingre_w):
    if defer.rows and ingre_w.grad is None:  # (no propagation gradient was adopted: the rows alone)
        ingre_w.grad = torch.zeros_like(ingre_w)
    if ingre_w.grad is not None:
        defer.drain(ingre_w.grad)
    else:
        defer.open = False


def _join_branch():
    """End of a backward pass that ran graph_bpr's backward on the branch stream: the current stream
    waits for it, then adds the deferred ingredient rows into d ingre (after both are complete) --
    or, in late mode (late_drain), leaves them to run_pending_drains."""
    pend = list(_BRANCH_PENDING)
    _BRANCH_PENDING.clear()
    for done, defer, ingre_w in pend:
        torch.cuda.current_stream(ingre_w.device).wait_event(done)
        if defer is not None and _LATE_DRAIN[0] and ingre_w.is_cuda:
            fork = torch.cuda.Event()
            fork.record(torch.cuda.current_stream(ingre_w.device))
            _PENDING_DRAINS.append((fork, defer, ingre_w))
            continue
        if defer is not None:
            _drain_into(defer, ingre_w)


def _drop_stale_branches():
    """Entries of a backward that never reached its final callback (it raised): wait for their
    kernels and forget them."""
    pend = list(_BRANCH_PENDING)
    _BRANCH_PENDING.clear()
    for done, defer, ingre_w in pend:
        torch.cuda.current_stream(ingre_w.device).wait_event(done)
        if defer is not None:
            defer.open, defer.rows = False, []


def graph_bpr_begin(user_w, item_w, ingre_w, u, p, n, pn, ri_adj, ui_adj, L_ri, L_ui, gamma=1e-10):
    """Start graph_bpr's forward (the RI + UI propagations and the fused BPR) on the branch stream,
    so that the caller's next work (HealthRec: the ingredient encoder, projections, modal fusion,
    which read none of its outputs) overlaps it; graph_bpr_end joins it and creates the autograd
    node, whose backward then runs on the branch stream too, beside the encoder backward.  Without a
    GPU, in the deterministic mode or with BRANCH_STREAMS off, the forward runs here."""
    args = (user_w, item_w, ingre_w, u, p, n, pn, ri_adj, ui_adj, int(L_ri), int(L_ui), gamma)
    if _BRANCH_PENDING:
        _drop_stale_branches()
    if _PENDING_DRAINS:  # (a late-mode pass whose optimiser step never ran: its rows still belong in .grad)
        run_pending_drains()
    if torch.is_grad_enabled() and ingre_w.requires_grad and not _DETERMINISTIC:
        ingre_w.__dict__["_fr_defer_rows"] = _DeferredRows()
    if not (BRANCH_STREAMS and user_w.is_cuda) or _DETERMINISTIC:
        f = _graph_bpr_forward(*args)
        f.done, f.args = None, args
        return f
    main = torch.cuda.current_stream(user_w.device)
    side = _branch_stream(user_w.device)
    side.wait_stream(main)
    for t in (u, p, n, pn):
        t.record_stream(side)
    with torch.cuda.stream(side):
        f = _graph_bpr_forward(*args, stream=side)
        f.done = torch.cuda.Event()
        f.done.record(side)
    f.args = args
    return f


def graph_bpr_end(f):
    """(BPRLoss, EmbLoss [1], [ui_items[pos]; ui_items[neg]]) of a graph_bpr_begin; see _GraphBpr."""
    if f.done is not None:
        main = torch.cuda.current_stream(f.out.device)
        main.wait_event(f.done)
        f.out.record_stream(main)
        f.item_rows.record_stream(main)
    return _GraphBpr.apply(*f.args, _DETERMINISTIC, f)


def graph_bpr(user_w, item_w, ingre_w, u, p, n, pn, ri_adj, ui_adj, L_ri, L_ui, gamma=1e-10):
    """HealthRec's propagation + BPR + EmbLoss(user, pos, neg) -> (BPRLoss, EmbLoss [1],
    [ui_items[pos]; ui_items[neg]]); see _GraphBpr.  Opens a deferred-rows slot on ``ingre_w``
    (_DeferredRows) that the next embedding_norms over the same table takes."""
    if torch.is_grad_enabled() and ingre_w.requires_grad and not _DETERMINISTIC:
        ingre_w.__dict__["_fr_defer_rows"] = _DeferredRows()
    return _GraphBpr.apply(user_w, item_w, ingre_w, u, p, n, pn, ri_adj, ui_adj, int(L_ri), int(L_ui), gamma,
                           _DETERMINISTIC, None)


class _DeferredRows:
    """Row gradients of a table whose dense gradient another backward writes in full later: HealthRec's
    ingredient table gets d ingre[:-1] from the RI propagation backward (graph_bpr, which runs last)
    and the encoder input's rows W[ids] (embedding_norms, which runs first).  Instead of a zero-filled
    dense scatter that autograd then adds to the propagation gradient (two PyTorch kernels over the
    table), the embedding backward hands its rows over (``put``) and returns no gradient; graph_bpr's
    backward scatters them atomically into the gradient it has just written (``drain``).  Either
    order is safe: rows handed over after the drain (``open`` False) are refused and scattered the
    usual way."""

    def __init__(self):
        self.open = True
        self.rows = []

    def put(self, idx, G, hot_row) -> bool:
        if not self.open:
            return False
        self.rows.append(("rows", (idx, G), hot_row))
        return True

    def put_norms(self, idx, G, E, gn, nrm, half, pad) -> bool:
        """Rows G + coef E of embedding_norms' backward, formed by the drain's scatter itself
        (fr_norms_bwd_scatter: no separate fr_norms_bwd_coef launch, no [n, 64] rows written)."""
        if not self.open:
            return False
        self.rows.append(("norms", (idx, G, E, gn, nrm), (half, pad)))
        return True

    def tensors(self):
        return [t for _, ts, _ in self.rows for t in ts]

    def drain(self, dW):
        self.open = False
        for kind, ts, meta in self.rows:
            if kind == "rows":
                scatter_rows_into(ts[0], ts[1], dW, meta)
            else:
                norms_scatter_into(*ts, *meta, dW)
        self.rows = []


# FR_NORMS_SCATTER=0: the deferred ingredient rows formed by fr_norms_bwd_coef at the end of the
# encoder backward and scattered by the drain (two launches) instead of fr_norms_bwd_scatter there
NORMS_SCATTER = os.environ.get("FR_NORMS_SCATTER", "1") != "0"


def norms_scatter_into(idx, G, E, gn, nrm, half, pad, dW) -> None:
    """``dW[idx[i]] += G[i] + [idx[i] != pad] (gn[h] / nrm[h]) E[i]`` (h: the position's half) with
    float atomics, the pad row pre-summed per workgroup (fr_norms_bwd_scatter)."""
    n = int(idx.numel())
    native.require_device(idx, G, E, gn, nrm, dW)
    if dW.dtype != torch.float32 or dW.shape[1] != 64 or dW.stride(1) != 1 or dW.stride(0) % 4 or dW.data_ptr() % 16:
        raise native.EngineError("norms_scatter_into: fp32 [rows, 64] table with 16-B aligned rows required")
    # the kernel reads G / E as dense [n, 64] rows (row stride 64), idx as n int64, gn[h * stride] and
    # nrm[h] for the two halves h = 0, 1
    for name, t in (("G", G), ("E", E)):
        if t.dtype != torch.float32 or not t.is_contiguous() or tuple(t.shape) != (n, 64):
            raise native.EngineError(f"norms_scatter_into: {name} must be a contiguous fp32 [{n}, 64] tensor")
    if idx.dtype != torch.int64 or not idx.is_contiguous():
        raise native.EngineError("norms_scatter_into: idx must be a contiguous int64 tensor")
    if gn.dtype != torch.float32 or gn.dim() < 1 or gn.shape[0] < 2 or nrm.dtype != torch.float32 \
            or not nrm.is_contiguous() or nrm.numel() < 2:
        raise native.EngineError("norms_scatter_into: gn and nrm must be fp32 with an entry per half (2)")
    if not 0 <= int(half) <= n:
        raise native.EngineError("norms_scatter_into: half must be in [0, n]")
    with profiling.region("embedding_bwd", embedding_bwd_bytes(n, int(dW.shape[0]), 64) + 4 * n * 64):
        native.check(native.lib().fr_norms_bwd_scatter(
            idx.data_ptr(), n, int(half), -1 if pad is None else int(pad), G.data_ptr(), E.data_ptr(), gn.data_ptr(),
            gn.stride(0), nrm.data_ptr(), int(dW.shape[0]), -1 if pad is None else int(pad), dW.data_ptr(),
            dW.stride(0), native.stream_of(G)), "fr_norms_bwd_scatter")


class _RegCombine(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, B, w):
        native.require_device(a, b)
        a, b = a.contiguous(), b.contiguous()
        out = torch.empty(1, dtype=torch.float32, device=a.device)
        native.check(native.lib().fr_reg_combine_fwd(a.data_ptr(), b.data_ptr(), b.numel(), _f(float(B)), _f(float(w)),
                                                     out.data_ptr(), native.stream_of(a)), "fr_reg_combine_fwd")
        ctx.meta = (a.shape, b.shape, float(B), float(w))
        return out

    @staticmethod
    def backward(ctx, g):
        sa, sb, B, w = ctx.meta
        key = (tuple(sa), tuple(sb), B, w, g.device)
        if _is_unit(g):  # the trainer's ones seed: the gradients are constants, computed once
            got = _REG_UNIT_GRADS.get(key)
            if got is not None:
                return got[0], got[1], None, None
        g = g.contiguous()
        da = torch.empty(sa, dtype=torch.float32, device=g.device)
        db = torch.empty(sb, dtype=torch.float32, device=g.device)
        native.check(native.lib().fr_reg_combine_bwd(g.data_ptr(), db.numel(), _f(B), _f(w), da.data_ptr(), db.data_ptr(),
                                                     native.stream_of(g)), "fr_reg_combine_bwd")
        if _is_unit(g) and not torch.cuda.is_current_stream_capturing():
            _REG_UNIT_GRADS[key] = (da, db)  # read-only from here on (consumers never write a grad input)
        return da, db, None, None


_REG_UNIT_GRADS = {}

# FR_LOSS_SIDE=1: the loss bookkeeping -- reg_combine's forward and the trainer's fr_step_book, which
# only the optimiser's NaN gate and the next step read -- on a side stream forked after the loss terms
# and joined after the backward, off the head -> backward chain.  Measured slower on MI355X (HealthRec
# 0.79-0.81 vs 0.755 ms/step, profiles/r4/ab_hr1_*): one more stream than the hardware queues the
# graph's branches map onto, so unrelated branches queue behind each other.  Default: main stream
LOSS_SIDE = os.environ.get("FR_LOSS_SIDE", "0") == "1"
_LOSS_STREAMS = {}
_LOSS_PENDING = [None]  # (main stream, side stream) with work not yet joined


def loss_side_stream(device=None, fork=False):
    """The loss side stream of this step (``fork``: fork it off the current stream now, creating it
    on first use); None when off, on the CPU, or outside a trainer step (which joins it: only the
    trainer's booked steps, under defer_counters, fork it)."""
    if not LOSS_SIDE or _DETERMINISTIC or not _DEFER[0]:
        return None
    if not fork:
        p = _LOSS_PENDING[0]
        return p[1] if p is not None else None
    if device is None or device.type != "cuda":
        return None
    s = _LOSS_STREAMS.get(device.index)
    if s is None:
        s = _LOSS_STREAMS[device.index] = new_stream(device, "loss")
    main = torch.cuda.current_stream(device)
    s.wait_stream(main)
    _LOSS_PENDING[0] = (main, s)
    return s


def loss_side_join() -> None:
    """The main stream waits for the loss side stream's work (after the backward is issued)."""
    p, _LOSS_PENDING[0] = _LOSS_PENDING[0], None
    if p is not None:
        p[0].wait_stream(p[1])


NORMS_DEFER = os.environ.get("FR_NORMS_DEFER", "1") != "0"
# FR_LOSS_FINALIZE=0: HealthRec's loss terms finalized by their own launches (head finalize, norms
# finalize + reg, the trainer's fr_step_book).  Default: inside a booked trainer step, one
# fr_healthrec_loss_finalize launch does all three (the loss chain after the encoder: 4 launches)
LOSS_FINALIZE = os.environ.get("FR_LOSS_FINALIZE", "1") != "0"

# outputs written by a later launch, keyed by their storage: a deferred norms finalize
# (embedding_norms(defer_norms=True)) and a deferred head finalize (modal_head inside a booked step)
_PENDING_NORMS = {}
_PENDING_HEAD = {}


def _storage(t) -> int:
    return t.untyped_storage().data_ptr()


def finalize_norms(nrm) -> None:
    """Write the norms an embedding_norms(..., defer_norms=True) left pending (one launch); no-op
    otherwise."""
    got = _PENDING_NORMS.pop(_storage(nrm), None) if nrm.is_cuda else None
    if got is not None:
        part, n, t = got
        native.check(native.lib().fr_reg_combine_norms_fwd(None, part.data_ptr(), n, _f(1.0), _f(1.0), t.data_ptr(),
                                                           None, native.stream_of(t)), "fr_reg_combine_norms_fwd")


def _finalize_head(out) -> None:
    got = _PENDING_HEAD.pop(_storage(out), None) if out.is_cuda else None
    if got is not None:
        part, n, thr, wh, wk, t = got
        native.check(native.lib().fr_healthrec_loss_finalize(
            part.data_ptr(), n, _f(thr), _f(wh), _f(wk), t.data_ptr(), None, 0, None, _f(1.0), _f(1.0), None, None,
            None, None, 0, None, None, 0, None, native.stream_of(t)), "fr_healthrec_loss_finalize")


def finalize_pending() -> None:
    """Run every deferred finalize not consumed by a loss op (the trainer calls this after the
    model's calculate_loss, before anything reads the loss terms)."""
    for _, (_, _, _, _, _, t) in list(_PENDING_HEAD.items()):
        _finalize_head(t)
    for _, (_, _, t) in list(_PENDING_NORMS.items()):
        finalize_norms(t)


def drop_pending_finalizes() -> None:
    """Forget every deferred finalize (the trainer's ``finally`` after calculate_loss): a loss that
    raised between a deferring op and its consumer must not leave partials keyed by an address a
    later tensor may reuse.  On the success path finalize_pending / the loss ops consumed them."""
    _PENDING_HEAD.clear()
    _PENDING_NORMS.clear()


# the trainer's request that a fused loss op book the step itself (fr_step_book's work in its launch)
_BOOK = {"request": None, "done": None}


def book_request(state, accumulate) -> None:
    _BOOK["request"], _BOOK["done"] = (state, bool(accumulate)), None


def book_taken():
    """(parts, loss) when a loss op booked the step since book_request, else None; clears both."""
    done = _BOOK["done"]
    _BOOK["request"], _BOOK["done"] = None, None
    return done


class _RegCombineNorms(torch.autograd.Function):
    """reg_combine over norms still pending (embedding_norms(defer_norms=True)): the norms' finalize
    and the combination in one launch; the norms tensor is written in place (it is the embedding_norms
    node's output, saved by it for its backward).  Backward as _RegCombine."""

    @staticmethod
    def forward(ctx, a, b, B, w):
        part, n, _ = _PENDING_NORMS.pop(_storage(b))
        a = a.contiguous()
        out = torch.empty(1, dtype=torch.float32, device=a.device)
        native.check(native.lib().fr_reg_combine_norms_fwd(a.data_ptr(), part.data_ptr(), n, _f(float(B)), _f(float(w)),
                                                           b.data_ptr(), out.data_ptr(), native.stream_of(a)),
                     "fr_reg_combine_norms_fwd")
        ctx.meta = (a.shape, b.shape, float(B), float(w))
        return out

    backward = _RegCombine.backward


class _HealthRecLossFinalize(torch.autograd.Function):
    """HealthRec's loss finalize (fr_healthrec_loss_finalize): the head's loss terms and the ingredient
    norms left pending, reg = w * (emb3 + sum(norms) / B), and the step's bookkeeping over
    [mf, health, kd, reg] when the trainer asked for it -- one launch.  Output: reg; gradients only
    to (emb3, norms), as reg_combine (the other inputs are read, not differentiated through)."""

    @staticmethod
    def forward(ctx, emb3, nrm, mf, health, kd, B, w, book):
        hp, n, thr, wh, wk, out = _PENDING_HEAD.pop(_storage(health))
        npart, nn, _ = _PENDING_NORMS.pop(_storage(nrm))
        reg = torch.empty(1, dtype=torch.float32, device=emb3.device)
        acc = nan = loss = None
        ctrs = []
        if book is not None:
            acc, nan, accumulate, loss = book
            ctrs = take_pending_counters()
        cptr = (ctypes.c_void_p * max(1, len(ctrs)))(*[c.data_ptr() for c in ctrs])
        native.check(native.lib().fr_healthrec_loss_finalize(
            hp.data_ptr(), n, _f(thr), _f(wh), _f(wk), out.data_ptr(), npart.data_ptr(), nn, emb3.data_ptr(),
            _f(float(B)), _f(float(w)), nrm.data_ptr(), reg.data_ptr(), native.ptr(mf) if book else None,
            native.ptr(acc), int(accumulate) if book else 0, native.ptr(nan), cptr, len(ctrs), native.ptr(loss),
            native.stream_of(emb3)), "fr_healthrec_loss_finalize")
        ctx.meta = (emb3.shape, nrm.shape, float(B), float(w))
        return reg

    @staticmethod
    def backward(ctx, g):
        da, db, _, _ = _RegCombine.backward(ctx, g)
        return da, db, None, None, None, None, None, None


def healthrec_loss_finalize(mf, health, kd, emb3, nrm, B, w):
    """``w * (emb3 + nrm.sum() / B)`` (HealthRec's EmbLoss assembly, cikm_model.py:267-279), finalizing
    in the same launch the modal head's loss terms and the ingredient norms a booked trainer step left
    pending, and booking the step ([mf, health, kd, reg]) when the trainer requested it."""
    if not (health.is_cuda and _storage(health) in _PENDING_HEAD and _storage(nrm) in _PENDING_NORMS
            and nrm.numel() == 2 and emb3.numel() == 1 and kd.untyped_storage().data_ptr() == _storage(health)):
        if health.is_cuda:
            _finalize_head(health)
        return reg_combine(emb3, nrm, B, w)
    book = None
    req = _BOOK["request"]
    if req is not None and mf.is_cuda and mf.dtype == torch.float32 and mf.numel() == 1:
        state, accumulate = req
        acc = state.get("acc")
        if acc is None:
            acc = state["acc"] = torch.zeros(4, dtype=torch.float64, device=mf.device)
            accumulate = False
        if acc.numel() == 4:
            loss = torch.empty((), dtype=torch.float32, device=mf.device)
            book = (acc, state["nan"], accumulate, loss)
    reg = _HealthRecLossFinalize.apply(emb3, nrm, mf, health, kd, B, w, book)
    if book is not None:
        _BOOK["done"] = ((mf, health, kd, reg), book[3])
    return reg


def reg_combine(a, b, B, w):
    """``w * (a + b.sum() / B)`` for a [1] and b [k] fp32 device tensors in one launch per direction
    (forward on the loss side stream when enabled: its value feeds only the step's bookkeeping).
    ``b`` = norms an embedding_norms(defer_norms=True) left pending: finalized in the same launch."""
    if not a.is_cuda:
        return w * (a + b.sum() / B)
    s = loss_side_stream(a.device, fork=True) if a.is_cuda else None
    if s is None:
        if _storage(b) in _PENDING_NORMS and b.numel() == 2:
            return _RegCombineNorms.apply(a, b, B, w)
        finalize_norms(b)
        return _RegCombine.apply(a, b, B, w)
    finalize_norms(b)
    a.record_stream(s)
    b.record_stream(s)
    with torch.cuda.stream(s):
        return _RegCombine.apply(a, b, B, w)


# ----------------------------------------------------------------------------- embedding
def embedding_bwd_bytes(n: int, rows: int, d: int) -> int:
    """Algorithmic HBM bytes of one fr_embedding_bwd: ids + gradient rows read, dW written."""
    return 8 * n + 4 * n * d + 4 * rows * d


def scatter_rows(ids: torch.Tensor, G: torch.Tensor, num_rows: int, padding_idx: int | None = None,
                 hot_row: int | None = None) -> torch.Tensor:
    """Dense ``dW[num_rows, d]`` with ``dW[ids[i]] += G[i]`` for ids in [0, num_rows) other than
    ``padding_idx`` (others skipped), zeros elsewhere -- the HIP ``fr_embedding_bwd`` (deterministic
    counting sort).  ``hot_row`` (d = 64, engine not in deterministic mode): a row id expected at many
    positions; the scatter then runs as fr_embedding_bwd_atomic (zero fill + one launch)."""
    d = G.shape[-1]
    if hot_row is not None and d == 64 and not _DETERMINISTIC and G.dtype == torch.float32:
        G2 = G.reshape(-1, d)
        if G2.stride(1) != 1 or G2.stride(0) % 4 or G2.data_ptr() % 16:
            G2 = G2.contiguous()
        ids2 = ids.reshape(-1)
        if ids2.dtype != torch.int64 or not ids2.is_contiguous():
            ids2 = ids2.to(torch.int64).contiguous()
        native.require_device(G2, ids2)
        n = int(ids2.numel())
        dW = torch.zeros(int(num_rows), d, dtype=torch.float32, device=G2.device)
        with profiling.region("embedding_bwd", embedding_bwd_bytes(n, int(num_rows), d)):
            native.check(native.lib().fr_embedding_bwd_atomic(
                ids2.data_ptr(), n, G2.data_ptr(), G2.stride(0), d, int(num_rows),
                -1 if padding_idx is None else int(padding_idx), int(hot_row), dW.data_ptr(), d,
                native.stream_of(G2)), "fr_embedding_bwd_atomic")
        return dW
    G = G.reshape(-1, d)
    if G.dtype != torch.float32:
        raise native.EngineError(f"engine ops compute in fp32 (got {G.dtype})")
    if G.stride(1) != 1 or G.stride(0) % 4 or G.data_ptr() % 16:
        G = G.contiguous()
    ids = ids.reshape(-1)
    if ids.dtype != torch.int64 or not ids.is_contiguous():
        ids = ids.to(torch.int64).contiguous()
    native.require_device(G, ids)
    n, R = int(ids.numel()), int(num_rows)
    dW = torch.empty(R, d, dtype=torch.float32, device=G.device)
    lib = native.lib()
    ws = native.workspace(lib.fr_embedding_bwd_workspace(n, R, d), G.device)
    with profiling.region("embedding_bwd", embedding_bwd_bytes(n, R, d)):
        native.check(lib.fr_embedding_bwd(ids.data_ptr(), n, G.data_ptr(), G.stride(0), d, R,
                                          -1 if padding_idx is None else int(padding_idx), dW.data_ptr(), d,
                                          ws.data_ptr(), ws.numel(), native.stream_of(G)), "fr_embedding_bwd")
    if _EMB_STATUS is not None:
        off = lib.fr_embedding_bwd_status_offset(R)
        _EMB_STATUS.append(ws[off:off + 4].view(torch.int32))
    return dW


def scatter_rows_into(ids: torch.Tensor, G: torch.Tensor, dW: torch.Tensor, hot_row: int | None = None) -> None:
    """``dW[ids[i]] += G[i]`` into an existing fp32 [rows, 64] table (fr_embedding_bwd_atomic without
    the zero fill; float-atomic order, the non-deterministic mode's scatter)."""
    G2 = G.reshape(-1, 64)
    if G2.stride(1) != 1 or G2.stride(0) % 4 or G2.data_ptr() % 16:
        G2 = G2.contiguous()
    ids2 = ids.reshape(-1)
    if ids2.dtype != torch.int64 or not ids2.is_contiguous():
        ids2 = ids2.to(torch.int64).contiguous()
    native.require_device(G2, ids2, dW)
    if dW.dtype != torch.float32 or dW.shape[1] != 64 or dW.stride(1) != 1 or dW.stride(0) % 4 or dW.data_ptr() % 16:
        raise native.EngineError("scatter_rows_into: fp32 [rows, 64] table with 16-B aligned rows required")
    n = int(ids2.numel())
    with profiling.region("embedding_bwd", embedding_bwd_bytes(n, int(dW.shape[0]), 64)):
        native.check(native.lib().fr_embedding_bwd_atomic(
            ids2.data_ptr(), n, G2.data_ptr(), G2.stride(0), 64, int(dW.shape[0]), -1,
            -1 if hot_row is None else int(hot_row), dW.data_ptr(), dW.stride(0),
            native.stream_of(G2)), "fr_embedding_bwd_atomic")


class _Embedding(torch.autograd.Function):
    @staticmethod
    def forward(ctx, idx, weight, padding_idx):
        native.require_device(weight, idx)
        ctx.save_for_backward(idx)
        ctx.rows, ctx.pad = weight.shape[0], padding_idx
        return torch.nn.functional.embedding(idx, weight)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        return None, scatter_rows(idx, g, ctx.rows, ctx.pad), None


class _EmbeddingExchanged(torch.autograd.Function):
    """Data-parallel row gather: backward stashes (ids, gradient rows) in the RowExchange
    (engine.dist) instead of producing a dense table gradient; after backward the exchange
    all-gathers every rank's rows and scatters their mean (GradAllReduce)."""

    @staticmethod
    def forward(ctx, idx, weight, padding_idx, exchange):
        _catch_up(exchange, weight, idx)
        native.require_device(weight, idx)
        ctx.save_for_backward(idx)
        ctx.weight, ctx.pad, ctx.exchange = weight, padding_idx, exchange
        return torch.nn.functional.embedding(idx, weight)

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        d = g.shape[-1]
        ctx.exchange.stash(ctx.weight, ctx.pad, idx.reshape(-1).to(torch.int64), g.reshape(-1, d))
        return None, None, None, None


class _EmbeddingNorms(torch.autograd.Function):
    """One gather serving two of the reference's uses of the same (table, ids): ``W[ids]`` (gradient
    to every row, cikm_model.py:230) and the Frobenius norms of the two halves of
    ``nn.Embedding(ids, padding_idx=pad)`` (EmbLoss over the pos / neg ingredient blocks,
    cikm_model.py:270-279; padding positions get no gradient).  Both gradients are combined before
    ONE deterministic scatter (fr_embedding_bwd)."""

    @staticmethod
    def forward(ctx, idx, weight, pad, half, defer_norms=False):
        native.require_device(weight, idx)
        n = idx.numel()
        hp = half * idx.shape[-1]  # positions in the first half
        ctx.fused = (weight.dtype == torch.float32 and weight.shape[1] == 64 and weight.stride(1) == 1
                     and weight.stride(0) % 4 == 0 and weight.data_ptr() % 16 == 0 and 0 <= hp <= n and n > 0)
        if ctx.fused:  # fr_gather_norms_fwd: gather + both halves' norms, 2 launches
            lib = native.lib()
            idx_c = idx.reshape(-1).contiguous()
            E = torch.empty(idx.shape + (64,), dtype=torch.float32, device=weight.device)
            nrm = torch.empty(2, dtype=torch.float32, device=weight.device)
            nparts = lib.fr_gather_norms_partials(n)
            part = torch.empty(nparts, dtype=torch.float32, device=weight.device)
            defer = bool(defer_norms) and NORMS_DEFER
            with profiling.region("gather_norms", 8 * n + 2 * 4 * n * 64):
                native.check(lib.fr_gather_norms_fwd(idx_c.data_ptr(), n, hp, weight.data_ptr(), weight.stride(0),
                                                     E.data_ptr(), part.data_ptr(), nparts,
                                                     None if defer else nrm.data_ptr(),
                                                     native.stream_of(weight)), "fr_gather_norms_fwd")
            if defer:  # finalized by the loss finalize / reg_combine (or finalize_pending) before any read
                _PENDING_NORMS[_storage(nrm)] = (part, n, nrm)
            ctx.save_for_backward(idx_c, E, nrm)
            ctx.rows, ctx.pad, ctx.half, ctx.hp = weight.shape[0], pad, half, hp
            ctx.defer = weight.__dict__.pop("_fr_defer_rows", None)
            return E, nrm
        weight.__dict__.pop("_fr_defer_rows", None)  # this path scatters its own rows
        E = torch.nn.functional.embedding(idx, weight)
        Ef = E.reshape(2, -1)  # full-tensor norms of each half (a 2-output dim reduction is slow)
        nrm = torch.stack([torch.linalg.vector_norm(Ef[0]), torch.linalg.vector_norm(Ef[1])])
        ctx.save_for_backward(idx, E, nrm)
        ctx.rows, ctx.pad, ctx.half = weight.shape[0], pad, half
        return E, nrm

    @staticmethod
    def backward(ctx, gE, gn):
        idx, E, nrm = ctx.saved_tensors
        if ctx.fused:
            G = torch.zeros_like(E) if gE is None else gE.contiguous()
            if (gn is not None and NORMS_SCATTER and ctx.defer is not None and ctx.hp <= idx.numel()
                    and ctx.defer.put_norms(idx.reshape(-1), G.reshape(-1, 64), E.reshape(-1, 64), gn, nrm, ctx.hp,
                                            ctx.pad)):
                return None, None, None, None, None  # formed and scattered by the drain (fr_norms_bwd_scatter)
            if gn is not None:
                out = torch.empty_like(G)
                with profiling.region("gather_norms", 8 * idx.numel() + 3 * 4 * G.numel()):
                    native.check(native.lib().fr_norms_bwd_coef(
                        idx.data_ptr(), idx.numel(), ctx.hp, -1 if ctx.pad is None else int(ctx.pad), G.data_ptr(),
                        E.data_ptr(), gn.data_ptr(), gn.stride(0), nrm.data_ptr(), out.data_ptr(),
                        native.stream_of(G)), "fr_norms_bwd_coef")
                G = out
            if ctx.defer is not None and ctx.defer.put(idx, G.reshape(-1, 64), ctx.pad):
                return None, None, None, None, None  # scattered into graph_bpr's d ingre (_DeferredRows)
            return None, scatter_rows(idx, G.reshape(-1, 64), ctx.rows, None, hot_row=ctx.pad), None, None, None
        G = torch.zeros_like(E) if gE is None else gE
        if gn is not None:
            coef = (gn / nrm).view(2, 1).expand(2, ctx.half * idx.shape[-1]).reshape(idx.shape)
            coef = torch.where(idx != ctx.pad, coef, torch.zeros((), dtype=coef.dtype, device=coef.device))
            G = torch.addcmul(G, coef.unsqueeze(-1), E)
        return None, scatter_rows(idx, G, ctx.rows, None), None, None, None


def embedding_norms(idx: torch.Tensor, weight: torch.Tensor, padding_idx: int, half: int, defer_norms: bool = False):
    """``(W[idx], stack(||Embedding(idx[:half], pad)||_F, ||Embedding(idx[half:], pad)||_F))`` with
    one gather and one scatter (see _EmbeddingNorms).  ``idx``: [2 * half, L]."""
    if idx.shape[0] != 2 * half:
        raise native.EngineError(f"embedding_norms: idx has {idx.shape[0]} rows, expected 2 x {half}")
    return _EmbeddingNorms.apply(idx, weight, int(padding_idx), int(half), bool(defer_norms))


_EMB_STATUS = None  # test hook: a list collecting each call's device status word (0 = consistent)


def embedding(idx: torch.Tensor, weight: torch.Tensor, padding_idx: int | None = None,
              exchange=None) -> torch.Tensor:
    """``F.embedding(idx, weight, padding_idx)`` whose weight gradient is the deterministic HIP
    scatter-add ``fr_embedding_bwd`` (rows == padding_idx receive no gradient, as in torch).
    ``exchange`` (an engine.dist.RowExchange, data-parallel training): the table's gradient is the
    mean over the ranks, exchanged as gathered rows after backward (see _EmbeddingExchanged)."""
    if padding_idx is not None and padding_idx < 0:
        padding_idx += weight.shape[0]
    if exchange is not None:
        return _EmbeddingExchanged.apply(idx, weight, padding_idx, exchange)
    return _Embedding.apply(idx, weight, padding_idx)


# ----------------------------------------------------------------------------- Linear
LINEAR_MIN_ROWS = 1024  # below this the library GEMM's weight gradient is already short


def _rows_operand(t: torch.Tensor, cols: int) -> torch.Tensor:
    t2 = t.reshape(-1, cols)
    if t2.stride(1) != 1 or t2.stride(0) % 4 or t2.data_ptr() % 16:
        t2 = t2.contiguous()
    return t2


def linear_wgrad_bytes(M: int, N: int, K: int) -> int:
    """Algorithmic bytes of fr_linear_wgrad: dY [M,N] and X [M,K] read once, dW + db written."""
    return 4 * (M * N + M * K + N * K + N)


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, W, b):
        ctx.save_for_backward(x, W)
        ctx.has_b = b is not None
        return torch.nn.functional.linear(x, W, b)

    @staticmethod
    def backward(ctx, gy):
        x, W = ctx.saved_tensors
        N, K = W.shape
        need = ctx.needs_input_grad
        gy2 = _rows_operand(gy, N)
        dx = dW = db = None
        if need[0]:
            dx = torch.mm(gy2, W).view(x.shape)
        if need[1] or (ctx.has_b and need[2]):
            x2 = _rows_operand(x, K)
            M = gy2.shape[0]
            dW = torch.empty(N, K, dtype=torch.float32, device=gy.device)
            db = torch.empty(N, dtype=torch.float32, device=gy.device) if ctx.has_b else None
            lib = native.lib()
            ws = native.workspace(lib.fr_linear_wgrad_workspace(M, N, K), gy.device)
            with profiling.region("linear_wgrad", linear_wgrad_bytes(M, N, K)):
                native.check(lib.fr_linear_wgrad(gy2.data_ptr(), gy2.stride(0), x2.data_ptr(), x2.stride(0), M,
                                                 N, K, dW.data_ptr(), K, native.ptr(db), ws.data_ptr(),
                                                 ws.numel(), native.stream_of(gy2)), "fr_linear_wgrad")
            if not need[1]:
                dW = None
            if not need[2]:
                db = None
        return dx, dW, db


def linear(x: torch.Tensor, W: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:
    """``F.linear(x, W, b)``; over >= LINEAR_MIN_ROWS rows of fp32 its weight/bias gradient is the
    split-K HIP kernel ``fr_linear_wgrad`` (the input gradient stays a library GEMM)."""
    N, K = W.shape
    rows = x.numel() // max(K, 1)
    if (rows < LINEAR_MIN_ROWS or N % 4 or K % 4 or x.dtype != torch.float32 or W.dtype != torch.float32
            or not torch.is_grad_enabled() or not (W.requires_grad or (b is not None and b.requires_grad))):
        return torch.nn.functional.linear(x, W, b)
    native.require_device(x, W)
    return _Linear.apply(x, W, b)


# ----------------------------------------------------------------------------- LayerNorm
def _ln_ok(x, weight, bias, d) -> bool:
    if not (x.is_cuda and x.dtype == torch.float32 and 4 <= d <= 256 and d % 4 == 0 and (d // 4) & (d // 4 - 1) == 0):
        return False
    for p in (weight, bias):
        if p is not None and (p.dtype != torch.float32 or not p.is_contiguous() or p.data_ptr() % 16):
            return False
    return True


def layernorm_bytes(rows: int, d: int, backward: bool) -> int:
    """Algorithmic bytes: forward reads x, writes y (+ mean/rstd); backward reads dy, x (+ stats),
    writes dx."""
    return (12 if backward else 8) * rows * d + 8 * rows


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, eps):
        d = x.shape[-1]
        x2 = _rows_operand(x, d)
        rows = x2.shape[0]
        y = torch.empty(rows, d, dtype=torch.float32, device=x.device)
        mean = torch.empty(rows, dtype=torch.float32, device=x.device)
        rstd = torch.empty_like(mean)
        with profiling.region("layernorm", layernorm_bytes(rows, d, False)):
            native.check(native.lib().fr_layernorm_fwd(x2.data_ptr(), x2.stride(0), rows, d, native.ptr(weight),
                                                       native.ptr(bias), float(eps), y.data_ptr(), d,
                                                       mean.data_ptr(), rstd.data_ptr(), native.stream_of(x2)),
                         "fr_layernorm_fwd")
        ctx.save_for_backward(x2, mean, rstd, weight)
        ctx.shape, ctx.has_bias = x.shape, bias is not None
        return y.view(x.shape)

    @staticmethod
    def backward(ctx, gy):
        x2, mean, rstd, weight = ctx.saved_tensors
        rows, d = x2.shape
        gy2 = _rows_operand(gy, d)
        need = ctx.needs_input_grad
        dx = torch.empty(rows, d, dtype=torch.float32, device=gy.device)
        dgamma = torch.empty(d, dtype=torch.float32, device=gy.device) if (weight is not None and need[1]) else None
        dbeta = torch.empty(d, dtype=torch.float32, device=gy.device) if (ctx.has_bias and need[2]) else None
        lib = native.lib()
        ws = native.workspace(lib.fr_layernorm_bwd_workspace(d), gy.device)
        with profiling.region("layernorm", layernorm_bytes(rows, d, True)):
            native.check(lib.fr_layernorm_bwd(gy2.data_ptr(), gy2.stride(0), x2.data_ptr(), x2.stride(0), rows, d,
                                              mean.data_ptr(), rstd.data_ptr(), native.ptr(weight), dx.data_ptr(), d,
                                              native.ptr(dgamma), native.ptr(dbeta), ws.data_ptr(), ws.numel(),
                                              native.stream_of(gy2)), "fr_layernorm_bwd")
        return dx.view(ctx.shape), dgamma, dbeta, None


def layer_norm(x: torch.Tensor, normalized_shape, weight=None, bias=None, eps: float = 1e-5) -> torch.Tensor:
    """``F.layer_norm`` over the last dimension through the HIP kernels ``fr_layernorm_fwd/_bwd``
    (other shapes / dtypes / host tensors: torch's own)."""
    shape = tuple(normalized_shape) if not isinstance(normalized_shape, int) else (normalized_shape,)
    d = x.shape[-1]
    if len(shape) != 1 or shape[0] != d or not _ln_ok(x, weight, bias, d):
        return torch.nn.functional.layer_norm(x, shape, weight, bias, eps)
    return _LayerNorm.apply(x, weight, bias, eps)


# ----------------------------------------------------------------------------- encoder layer
ENCODER_LENGTHS = (4, 5, 8, 10, 16, 20)


def encoder_flops(n_seq: int, L: int, backward: bool) -> int:
    """Algorithmic flops of one fused encoder-layer launch (d=64, 2 heads of 32, FF=256), all on
    the matrix cores: the four GEMMs per token (qkv 2*64*192, out-proj 2*64*64, FF1 2*64*256, FF2
    2*256*64 = 98,304 flops), twice in the backward (input and weight gradients); and attention's
    matrix products per (sequence, head): Q K^T and P' V (2 * 2 L L 32) forward, dP' = dctx V^T,
    dV = P'^T dctx, dQ = dS K, dK = dS^T Q (4 * 2 L L 32) backward.  The backward's recomputation of
    the scores is not counted (it is not algorithmic work)."""
    per_tok = 2 * 64 * 192 + 2 * 64 * 64 + 2 * 64 * 256 + 2 * 256 * 64
    att = n_seq * 2 * (4 if backward else 2) * 2 * L * L * 32
    return n_seq * L * per_tok * (2 if backward else 1) + att


def encoder_bytes(n_seq: int, L: int, backward: bool) -> int:
    """Algorithmic HBM bytes of one fused encoder-layer launch: the saved activations (qkv 192 +
    ctx 64 + y1 64 + fact 256 + dact 256 + y2 64 + 4 stats floats per token) written by the forward
    and read back by the backward, plus x / out (forward) or dout / x / dx (backward); weights are
    L2-resident.  The backward's weight-gradient partials are not counted (an implementation choice
    for the deterministic order, not algorithmic traffic)."""
    T = n_seq * L
    saved = 4 * T * (192 + 64 + 64 + 256 + 256 + 64 + 4)
    return (saved + 4 * T * 64 * 3) if backward else (saved + 4 * T * 64 * 2)


# FR_ENCODER_FOLD=1: layer k+1's ordered reduction folded into layer k's backward launch (measured 5-10 us
# slower per step than a separate reduction: the 200 KB per workgroup of partial reads at the launch
# start are not overlapped); default: every layer reduces its own partials
ENCODER_FOLD = os.environ.get("FR_ENCODER_FOLD", "0") == "1"


class _EncoderStack(torch.autograd.Function):
    """A stack of fused nn.TransformerEncoderLayer training steps (fr_encoder_fwd / fr_encoder_bwd),
    one autograd node: forward layer by layer; backward from the top layer down, each layer's
    ordered weight-gradient reduction folded into the next backward launch (d_prev_partials), the
    bottom layer's by fr_encoder_reduce."""

    @staticmethod
    def forward(ctx, x, mask, cfgs, *flat):
        nl = len(cfgs)
        NS, L, E = x.shape
        T = NS * L
        dev = x.device
        f32 = dict(dtype=torch.float32, device=dev)
        lib = native.lib()
        saved = []
        h = x
        for k, cfg in enumerate(cfgs):
            params = flat[12 * k:12 * (k + 1)]
            out = torch.empty(NS, L, E, **f32)
            qkv = torch.empty(T, 192, **f32)
            cx = torch.empty(T, 64, **f32)
            y1 = torch.empty(T, 64, **f32)
            fact = torch.empty(T, 256, **f32)
            dact = torch.empty(int(lib.fr_encoder_dact_numel(NS, L)), **f32)  # per-workgroup fragment layout
            y2 = torch.empty(T, 64, **f32)
            st1 = torch.empty(T, 2, **f32)
            st2 = torch.empty(T, 2, **f32)
            seed_used = torch.empty(1, dtype=torch.int64, device=dev)
            pp = (ctypes.c_void_p * 12)(*[p.data_ptr() for p in params])
            settle_counter(cfg.counter)  # a previous forward's increment not yet applied by a booked step
            with profiling.region("encoder_fwd", encoder_bytes(NS, L, False)):
                native.check(lib.fr_encoder_fwd(
                    h.data_ptr(), native.ptr(mask), NS, L, pp, cfg.eps, cfg.drop, cfg.seed, cfg.gelu,
                    cfg.counter.data_ptr(), seed_used.data_ptr(), out.data_ptr(), qkv.data_ptr(), cx.data_ptr(),
                    y1.data_ptr(), fact.data_ptr(), dact.data_ptr(), y2.data_ptr(), st1.data_ptr(), st2.data_ptr(),
                    native.stream_of(h)), "fr_encoder_fwd")
            defer_increment(cfg.counter)  # advanced by the step's fr_step_book (or before its next read)
            saved.append((h, qkv, cx, y1, fact, dact, y2, st1, st2, seed_used))
            h = out
        ctx.cfgs, ctx.saved, ctx.mask = cfgs, saved, mask
        ctx.save_for_backward(*flat)
        return h

    @staticmethod
    def backward(ctx, g):
        flat = ctx.saved_tensors
        cfgs, mask = ctx.cfgs, ctx.mask
        nl = len(cfgs)
        g = g.contiguous()
        NS, L, _ = g.shape
        lib = native.lib()
        dev = g.device
        nparts = lib.fr_encoder_partials(NS, L)
        grads = [None] * nl
        prev = None  # (partials, gradient) of the layer above, reduced by this layer's launch
        for k in range(nl - 1, -1, -1):
            h, qkv, cx, y1, fact, dact, y2, st1, st2, seed_used = ctx.saved[k]
            cfg = cfgs[k]
            params = flat[12 * k:12 * (k + 1)]
            dx = torch.empty_like(h)
            grad = torch.empty(lib.fr_encoder_grad_numel(), dtype=torch.float32, device=dev)
            part = torch.empty(nparts, dtype=torch.float32, device=dev)
            pp = (ctypes.c_void_p * 12)(*[p.data_ptr() for p in params])
            with profiling.region("encoder_bwd", encoder_bytes(NS, L, True)):
                native.check(lib.fr_encoder_bwd(
                    g.data_ptr(), h.data_ptr(), native.ptr(mask), NS, L, pp, cfg.eps, cfg.drop, cfg.seed, cfg.gelu,
                    seed_used.data_ptr(), qkv.data_ptr(), cx.data_ptr(), y1.data_ptr(), fact.data_ptr(),
                    dact.data_ptr(), y2.data_ptr(), st1.data_ptr(), st2.data_ptr(), dx.data_ptr(),
                    grad.data_ptr() if (k == 0 or not ENCODER_FOLD) else None,
                    part.data_ptr(), nparts, prev[0].data_ptr() if prev else None,
                    prev[1].data_ptr() if prev else None, native.stream_of(g)), "fr_encoder_bwd")
            grads[k] = grad
            prev = (part, grad) if ENCODER_FOLD else None
            g = dx
        out = []
        for k in range(nl):
            params = flat[12 * k:12 * (k + 1)]
            out += [gr.view(p.shape) for gr, p in zip(torch.split(grads[k], [p.numel() for p in params]), params)]
        ctx.saved = None
        return (g, None, None) + tuple(out)


def encoder_stack(x: torch.Tensor, mask, cfgs, params_list) -> torch.Tensor:
    """Fused post-norm encoder layers applied in order over batch-first x [n_seq, L, 64] (fp32);
    ``mask``: [n_seq, L] additive float key mask or None; ``cfgs`` / ``params_list``: one
    EncoderConfig and the 12 layer tensors (torch order, include/fr_engine.h) per layer."""
    native.require_device(x)
    if x.dim() != 3 or x.shape[2] != 64 or x.shape[1] not in ENCODER_LENGTHS or x.dtype != torch.float32:
        raise native.EngineError(f"fused encoder layer: unsupported input {tuple(x.shape)} {x.dtype}")
    if len(cfgs) != len(params_list) or not cfgs:
        raise native.EngineError("encoder_stack: one config per layer")
    x = x.contiguous()
    if mask is not None:
        mask = mask.to(torch.float32).contiguous()
    flat = [p for ps in params_list for p in ps]
    return _EncoderStack.apply(x, mask, tuple(cfgs), *flat)


class EncoderConfig:
    """Per-layer constants of the fused encoder: eps (2), dropout p (4), activation, the hash seed
    and the device step counter the forward reads (advanced after every forward)."""

    def __init__(self, eps, drop, gelu: bool, seed: int, device):
        self.eps = (ctypes.c_float * 2)(*[float(e) for e in eps])
        self.drop = (ctypes.c_float * 4)(*[float(p) for p in drop])
        self.gelu = 1 if gelu else 0
        self.seed = int(seed) & (2 ** 64 - 1)
        self.counter = torch.zeros(1, dtype=torch.int64, device=device)


def encoder_layer(x: torch.Tensor, mask, cfg: EncoderConfig, params) -> torch.Tensor:
    """One fused post-norm encoder layer over batch-first x [n_seq, L, 64] (fp32, contiguous);
    ``mask``: [n_seq, L] additive float key mask or None; ``params``: the 12 layer tensors in
    torch order (see include/fr_engine.h)."""
    return encoder_stack(x, mask, [cfg], [params])


# ----------------------------------------------------------------------------- modal fusion
def fusion_bytes(n: int, L: int, backward: bool) -> int:
    """Algorithmic HBM bytes: encoder rows, modal queries, ids, counts read; know / hin written
    (forward) or their gradients read and d_enc / d_query written (backward)."""
    base = 4 * n * (L * 64 + 2 * 64) + 8 * n * (L + 1)
    return base + (4 * n * 64 * 2) + ((4 * n * (L * 64 + 2 * 64)) if backward else 0)


class _ModalFusion(torch.autograd.Function):
    """fr_modal_fusion_fwd / _bwd: both HealthRec target attentions + the normalize heads."""

    @staticmethod
    def forward(ctx, enc, query, ids, num, pad_id, eps, ga, ba, gb, bb):
        n, L, _ = enc.shape
        know = torch.empty(n, 64, dtype=torch.float32, device=enc.device)
        hin = torch.empty_like(know)
        lnp = (ctypes.c_void_p * 4)(ga.data_ptr(), ba.data_ptr(), gb.data_ptr(), bb.data_ptr())
        with profiling.region("modal_fusion", fusion_bytes(n, L, False)):
            native.check(native.lib().fr_modal_fusion_fwd(enc.data_ptr(), query.data_ptr(), ids.data_ptr(),
                                                          num.data_ptr(), int(pad_id), n, L, lnp, float(eps),
                                                          know.data_ptr(), hin.data_ptr(), native.stream_of(enc)),
                         "fr_modal_fusion_fwd")
        ctx.save_for_backward(enc, query, ids, num, ga, ba, gb, bb)
        ctx.pad_id, ctx.eps = int(pad_id), float(eps)
        return know, hin

    @staticmethod
    def backward(ctx, dknow, dhin):
        enc, query, ids, num, ga, ba, gb, bb = ctx.saved_tensors
        n, L, _ = enc.shape
        dknow = torch.zeros(n, 64, dtype=torch.float32, device=enc.device) if dknow is None else dknow.contiguous()
        dhin = torch.zeros(n, 64, dtype=torch.float32, device=enc.device) if dhin is None else dhin.contiguous()
        denc = torch.empty_like(enc)
        dq = torch.empty_like(query)
        dln = torch.empty(4, 32, dtype=torch.float32, device=enc.device)
        lib = native.lib()
        nparts = lib.fr_modal_fusion_partials(n)
        part = torch.empty(nparts, dtype=torch.float32, device=enc.device)
        lnp = (ctypes.c_void_p * 4)(ga.data_ptr(), ba.data_ptr(), gb.data_ptr(), bb.data_ptr())
        with profiling.region("modal_fusion", fusion_bytes(n, L, True)):
            native.check(lib.fr_modal_fusion_bwd(enc.data_ptr(), query.data_ptr(), ids.data_ptr(), num.data_ptr(),
                                                 ctx.pad_id, n, L, lnp, ctx.eps, dknow.data_ptr(), dhin.data_ptr(),
                                                 denc.data_ptr(), dq.data_ptr(), dln.data_ptr(), part.data_ptr(),
                                                 nparts, native.stream_of(enc)), "fr_modal_fusion_bwd")
        return denc, dq, None, None, None, None, dln[0], dln[1], dln[2], dln[3]


def modal_fusion(enc, query, ids, num, pad_id, ln_a, ln_b):
    """HealthRec's two target attentions + F.normalize heads (cikm_model.py:245-249) fused:
    returns (item_know [n, 64], health-MLP input [n, 64]).  ``ln_a`` / ``ln_b``: the LayerNorm(32)
    modules of mm_target_atten / ingre_target_atten."""
    native.require_device(enc, query, ids)
    if ln_a.eps != ln_b.eps:
        raise native.EngineError("modal_fusion: both target-attention LayerNorms must share eps")
    return _ModalFusion.apply(enc.contiguous(), query.contiguous(), ids.contiguous(), num.contiguous(), pad_id,
                              ln_a.eps, ln_a.weight, ln_a.bias, ln_b.weight, ln_b.bias)


# ----------------------------------------------------------------------------- modal projections
def projection_bytes(n: int, K: int, backward: bool) -> int:
    """Algorithmic HBM bytes of one modality: the n gathered K-wide rows and W read, Y written
    (forward); dY and the gathered rows read again for dW (backward wgrad)."""
    return 4 * (n * K + 64 * K + n * 64) + (4 * (n * K + n * 64 + 64 * K) if backward else 0)


def factored_rows(ids, G, width: int, R: int, pad, Ws):
    """Row gradients of gathered Linear inputs: ``G`` holds len(Ws) adjacent 64-wide dY blocks
    ([n, width], row stride G.stride(0)); one fr_embedding_rowgrad over them gives the row map
    (rmap[r] = slot of id r, -1 if absent) and the per-id dY sums in ascending position order; then
    rows_t = sums_t W_t (fr_rows_matmul).  Returns (rmap [R] int32, [rows_t [n, K_t]])."""
    lib = native.lib()
    ids = ids.reshape(-1)
    n = ids.numel()
    dev = G.device
    rmap = torch.empty(R, dtype=torch.int32, device=dev)
    S = torch.empty(max(n, 1), width, dtype=torch.float32, device=dev)
    ws = native.workspace(lib.fr_embedding_rowgrad_workspace(n, R, width), dev)
    with profiling.region("embedding_rowgrad", 4 * R + 8 * n + 8 * n * width):
        native.check(lib.fr_embedding_rowgrad(ids.data_ptr(), n, G.data_ptr(), G.stride(0), width, R,
                                              -1 if pad is None else int(pad), rmap.data_ptr(), S.data_ptr(),
                                              ws.data_ptr(), ws.numel(), native.stream_of(G)), "fr_embedding_rowgrad")
    rows = [torch.empty(max(n, 1), W.shape[1], dtype=torch.float32, device=dev) for W in Ws]
    if n == 0:
        return rmap, rows
    T = len(Ws)
    nb = sum(4 * (n * 64 + 64 * W.shape[1] + n * W.shape[1]) for W in Ws)
    with profiling.region("rows_matmul", nb):  # every table in one launch (blockIdx.z = table)
        native.check(lib.fr_rows_matmul_multi(
            S.data_ptr(), width, n, T, (ctypes.c_void_p * T)(*[W.data_ptr() for W in Ws]),
            (ctypes.c_int * T)(*[W.shape[1] for W in Ws]), (ctypes.c_void_p * T)(*[c.data_ptr() for c in rows]),
            (ctypes.c_int64 * T)(*[c.shape[1] for c in rows]), native.stream_of(G)), "fr_rows_matmul_multi")
    return rmap, rows


def rows_to_dense(rmap, crow):
    """The dense table gradient of (rmap, compact rows), without a host synchronisation."""
    has = (rmap >= 0).unsqueeze(1)
    return torch.where(has, crow[rmap.clamp(min=0).long()], torch.zeros((), dtype=crow.dtype, device=crow.device))


class _ModalProjection(torch.autograd.Function):
    """fr_gather_linear_fwd per modality into one [n, T, 64] tensor; backward: dW / db by
    fr_linear_wgrad_gather, the feature tables' gradient factored as (ids, dY, W) -- stashed in the
    row-gradient exchange (FusedAdam: compact rows = per-id sum of dY x W, fr_rows_matmul), or, with
    no exchange, scattered densely."""

    @staticmethod
    def forward(ctx, ids, exchange, *flat):
        T = len(flat) // 3
        n = ids.numel()
        dev = ids.device
        lib = native.lib()
        out = torch.empty(n, T, 64, dtype=torch.float32, device=dev)
        Xs, Ws, bs = flat[0::3], flat[1::3], flat[2::3]
        for X in Xs:
            _catch_up(exchange, X, ids)
        nb = sum(projection_bytes(n, W.shape[1], False) for W in Ws)
        with profiling.region("modal_projection", nb):  # every modality in one launch (blockIdx.z = table)
            native.check(lib.fr_gather_linear_fwd_multi(
                ids.data_ptr(), n, T, (ctypes.c_void_p * T)(*[X.data_ptr() for X in Xs]),
                (ctypes.c_int64 * T)(*[X.stride(0) for X in Xs]), (ctypes.c_int * T)(*[W.shape[1] for W in Ws]),
                (ctypes.c_void_p * T)(*[W.data_ptr() for W in Ws]), (ctypes.c_void_p * T)(*[native.ptr(b) for b in bs]),
                out.data_ptr(), T * 64, native.stream_of(ids)), "fr_gather_linear_fwd_multi")
        ctx.save_for_backward(ids, *flat)
        ctx.exchange, ctx.T = exchange, T
        return out

    @staticmethod
    def backward(ctx, g):
        ids, *flat = ctx.saved_tensors
        T, n = ctx.T, ids.numel()
        g = g.contiguous()
        G2 = g.view(n, T * 64)
        lib = native.lib()
        grads = [None, None]
        dense = None
        if ctx.exchange is None and any(ctx.needs_input_grad[2 + 3 * t] for t in range(T)):
            # same kernels as the row-gradient path: dense and row modes see bit-identical table rows
            R = flat[0].shape[0]
            if all(flat[3 * t].shape[0] == R for t in range(T)) and (T * 64) & (T * 64 - 1) == 0:
                rmap, crows = factored_rows(ids, G2, T * 64, R, None, [flat[3 * t + 1] for t in range(T)])
                dense = [rows_to_dense(rmap, c) for c in crows]
            else:
                dense = []
                for t in range(T):
                    rmap, (c,) = factored_rows(ids, G2[:, 64 * t:], 64, flat[3 * t].shape[0], None, [flat[3 * t + 1]])
                    dense.append(rows_to_dense(rmap, c))
        Xs, Ws, bs = flat[0::3], flat[1::3], flat[2::3]
        dWs = [torch.empty_like(W) for W in Ws]
        dbs = [torch.empty_like(b) if b is not None else None for b in bs]
        Ks = (ctypes.c_int * T)(*[W.shape[1] for W in Ws])
        ws = native.workspace(lib.fr_linear_wgrad_gather_multi_workspace(n, 64, T, Ks), g.device)
        nb = sum(projection_bytes(n, W.shape[1], True) for W in Ws)
        with profiling.region("modal_projection", nb):  # dW / db of every modality: one slab + one reduce launch
            native.check(lib.fr_linear_wgrad_gather_multi(
                G2.data_ptr(), G2.stride(0), ids.data_ptr(), n, 64, T, (ctypes.c_void_p * T)(*[X.data_ptr() for X in Xs]),
                (ctypes.c_int64 * T)(*[X.stride(0) for X in Xs]), Ks, (ctypes.c_void_p * T)(*[d.data_ptr() for d in dWs]),
                (ctypes.c_int64 * T)(*[d.stride(0) for d in dWs]), (ctypes.c_void_p * T)(*[native.ptr(d) for d in dbs]),
                ws.data_ptr(), ws.numel(), native.stream_of(g)), "fr_linear_wgrad_gather_multi")
        for t in range(T):
            X, W, b = flat[3 * t], flat[3 * t + 1], flat[3 * t + 2]
            dW, db = dWs[t], dbs[t]
            dy = G2[:, 64 * t:64 * (t + 1)]
            dX = None
            if ctx.needs_input_grad[2 + 3 * t]:
                if ctx.exchange is not None:
                    ctx.exchange.stash_factored(X, None, ids, dy, W)
                else:
                    dX = dense[t]
            grads += [dX, dW if ctx.needs_input_grad[3 + 3 * t] else None,
                      db if (b is not None and ctx.needs_input_grad[4 + 3 * t]) else None]
        return tuple(grads)


def _catch_up(exchange, weight, ids):
    """A lazily updating optimiser (FusedAdam lazy rows) brings the rows about to be gathered up to
    date first; exchanges without one (or tables without lazy state) make this a no-op."""
    fn = getattr(exchange, "catch_up_rows", None)
    if fn is not None:
        fn(weight, ids)


def modal_projection(ids, pairs, exchange=None):
    """``torch.stack([lin(table[ids]) for table, lin in pairs], 1)`` -> [n, T, 64] (HealthRec's
    mm_query, cikm_model.py:240-243), the gathers folded into the projection GEMM.  ``pairs``:
    [(feature table [R, K], nn.Linear(K, 64)), ...]; ``exchange``: a RowGrads / RowExchange taking the
    tables' factored row gradients (else dense table gradients)."""
    native.require_device(ids, *[t for t, _ in pairs])
    flat = []
    for table, lin in pairs:
        if lin.out_features != 64 or table.shape[1] != lin.in_features or lin.in_features % 16:
            raise native.EngineError("modal_projection: Linear(K -> 64) with K a multiple of 16 required")
        flat += [table, lin.weight, lin.bias]
    return _ModalProjection.apply(ids.reshape(-1).contiguous(), exchange, *flat)


# ----------------------------------------------------------------------------- health / KD head
_HEAD_FWD_PARTS = {}  # device -> zero-initialised forward partials (+ ticket word; the kernel re-zeroes it)


def health_kd_bytes(n: int, H: int, backward: bool) -> int:
    """Algorithmic HBM bytes: hin / know / rows [n, 64] and labels [n, H] read (+ their three
    gradients written and the parameter-gradient partials written once and read once backward)."""
    base = 4 * n * (3 * 64 + H) + 4 * (64 * 64 + 64 + H * 64 + H)
    if not backward:
        return base
    nb = min((n + 3) // 4, 64)
    return base + 4 * n * 3 * 64 + 2 * 4 * nb * (64 * 64 + 64 + 16 * 64 + 16)


class _HealthKD(torch.autograd.Function):
    """fr_health_kd_fwd / _bwd: HealthRec's health MLP + BCE sum and the KD cosine term, weighted."""

    @staticmethod
    def forward(ctx, hin, know, rows, labels, w1, b1, w2, b2, thr, w_h, w_k):
        n, H = labels.shape
        dev = hin.device
        lib = native.lib()
        need = lib.fr_health_kd_partials(n, 0)
        part = _HEAD_FWD_PARTS.get(dev)
        if part is None or part.numel() < need:
            part = torch.zeros(max(need, 256), dtype=torch.float32, device=dev)
            _HEAD_FWD_PARTS[dev] = part
        out = torch.empty(3, dtype=torch.float32, device=dev)
        mlp = (ctypes.c_void_p * 4)(w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr())
        with profiling.region("health_kd", health_kd_bytes(n, H, False)):
            native.check(lib.fr_health_kd_fwd(hin.data_ptr(), know.data_ptr(), rows.data_ptr(), labels.data_ptr(), n, H,
                                              mlp, float(thr), float(w_h), float(w_k), out.data_ptr(),
                                              part.data_ptr(), part.numel(), native.stream_of(hin)),
                         "fr_health_kd_fwd")
        ctx.save_for_backward(hin, know, rows, labels, w1, b1, w2, b2)
        ctx.out, ctx.cfg = out, (float(thr), float(w_h), float(w_k))
        return out[0], out[1]

    @staticmethod
    def backward(ctx, gh, gk):
        hin, know, rows, labels, w1, b1, w2, b2 = ctx.saved_tensors
        n, H = labels.shape
        dev = hin.device
        zero = None
        if gh is None or gk is None:
            zero = torch.zeros((), dtype=torch.float32, device=dev)
        gh = zero if gh is None else gh.to(torch.float32).contiguous()
        gk = zero if gk is None else gk.to(torch.float32).contiguous()
        dhin, dknow, drows = torch.empty_like(hin), torch.empty_like(know), torch.empty_like(rows)
        dw1, db1, dw2, db2 = (torch.empty_like(t) for t in (w1, b1, w2, b2))
        lib = native.lib()
        nparts = lib.fr_health_kd_partials(n, 1)
        part = torch.empty(nparts, dtype=torch.float32, device=dev)
        mlp = (ctypes.c_void_p * 4)(w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr())
        dmlp = (ctypes.c_void_p * 4)(dw1.data_ptr(), db1.data_ptr(), dw2.data_ptr(), db2.data_ptr())
        thr, w_h, w_k = ctx.cfg
        with profiling.region("health_kd", health_kd_bytes(n, H, True)):
            native.check(lib.fr_health_kd_bwd(hin.data_ptr(), know.data_ptr(), rows.data_ptr(), labels.data_ptr(), n, H,
                                              mlp, thr, w_h, w_k, ctx.out.data_ptr(), gh.data_ptr(), gk.data_ptr(),
                                              dhin.data_ptr(), dknow.data_ptr(), drows.data_ptr(), dmlp,
                                              part.data_ptr(), nparts, native.stream_of(hin)), "fr_health_kd_bwd")
        return dhin, dknow, drows, None, dw1, db1, dw2, db2, None, None, None


def health_kd_loss(hin, know, rows, labels, mlp, kd_threshold, w_health, w_kd):
    """HealthRec's loss head (cikm_model.py:249-264, 304-308) in one HIP launch per direction:
    returns (w_health * BCELoss-sum of sigmoid(mlp(hin)) vs labels,
             w_kd * max(0, 1 - cosine_similarity(know, rows).mean() - kd_threshold)).
    ``mlp``: nn.Sequential(Linear(64, 64), ReLU, Linear(64, H)), H <= 16."""
    native.require_device(hin, know, rows, labels)
    l1, l2 = mlp[0], mlp[2]
    return _HealthKD.apply(hin.contiguous(), know.contiguous(), rows.contiguous(),
                           labels.to(torch.float32).contiguous(), l1.weight, l1.bias, l2.weight, l2.bias,
                           kd_threshold, w_health, w_kd)


# ----------------------------------------------------------------------------- fused loss head
_TICKETS = {}
# FR_HEAD_TICKET=1: the modal head's finalize run by the forward's last-arriving block instead of its
# own launch.  Measured ~5 us/step slower on MI355X (profiles/r4/ab_hr2_*: every block's fence +
# arrival atomic and the serial finalize at the tail cost more than the launch they save): off
HEAD_TICKET = os.environ.get("FR_HEAD_TICKET", "0") == "1"


def _arrival_ticket(device) -> torch.Tensor:
    """A zero int32 per device for kernels whose last-arriving block finalises (the kernel resets it
    to 0): one allocation and fill, ever, not per step.  Launches sharing it must be stream-ordered."""
    t = _TICKETS.get(device)
    if t is None:
        t = _TICKETS[device] = torch.zeros(1, dtype=torch.int32, device=device)
    return t


class _ModalHead(torch.autograd.Function):
    """fr_modal_head_fwd / _bwd: HealthRec's target attentions + normalize heads feeding the health
    MLP / BCE and KD cosine terms, one node (see include/fr_engine.h)."""

    @staticmethod
    def forward(ctx, enc, query, ids, num, rows, labels, pad_id, eps, thr, w_h, w_k, ga, ba, gb, bb, w1, b1, w2, b2):
        n, L, _ = enc.shape
        H = labels.shape[1]
        dev = enc.device
        lib = native.lib()
        part = torch.empty(lib.fr_modal_head_partials(n, 0), dtype=torch.float32, device=dev)
        out = torch.empty(3, dtype=torch.float32, device=dev)
        lnp = (ctypes.c_void_p * 4)(ga.data_ptr(), ba.data_ptr(), gb.data_ptr(), bb.data_ptr())
        mlp = (ctypes.c_void_p * 4)(w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr())
        defer = LOSS_FINALIZE and _DEFER[0] and not HEAD_TICKET
        with profiling.region("modal_head", fusion_bytes(n, L, False) + health_kd_bytes(n, H, False)):
            if defer:  # the finalize is left to healthrec_loss_finalize (or finalize_pending)
                native.check(lib.fr_modal_head_fwd_items(
                    enc.data_ptr(), query.data_ptr(), ids.data_ptr(), num.data_ptr(), int(pad_id), n, L, lnp, float(eps),
                    rows.data_ptr(), labels.data_ptr(), H, mlp, float(thr), float(w_h), float(w_k), part.data_ptr(),
                    part.numel(), native.stream_of(enc)), "fr_modal_head_fwd_items")
                _PENDING_HEAD[_storage(out)] = (part, n, float(thr), float(w_h), float(w_k), out)
            else:
                native.check(lib.fr_modal_head_fwd(enc.data_ptr(), query.data_ptr(), ids.data_ptr(), num.data_ptr(),
                                                   int(pad_id), n, L, lnp, float(eps), rows.data_ptr(), labels.data_ptr(),
                                                   H, mlp, float(thr), float(w_h), float(w_k), out.data_ptr(),
                                                   part.data_ptr(), part.numel(),
                                                   _arrival_ticket(enc.device).data_ptr() if HEAD_TICKET else None,
                                                   native.stream_of(enc)), "fr_modal_head_fwd")
        ctx.save_for_backward(enc, query, ids, num, rows, labels, ga, ba, gb, bb, w1, b1, w2, b2)
        ctx.out, ctx.cfg = out, (int(pad_id), float(eps), float(thr), float(w_h), float(w_k))
        return out[0], out[1]

    @staticmethod
    def backward(ctx, gh, gk):
        enc, query, ids, num, rows, labels, ga, ba, gb, bb, w1, b1, w2, b2 = ctx.saved_tensors
        pad_id, eps, thr, w_h, w_k = ctx.cfg
        n, L, _ = enc.shape
        H = labels.shape[1]
        dev = enc.device
        zero = None
        if gh is None or gk is None:
            zero = torch.zeros((), dtype=torch.float32, device=dev)
        gh = zero if gh is None else gh.to(torch.float32).contiguous()
        gk = zero if gk is None else gk.to(torch.float32).contiguous()
        lib = native.lib()
        denc, dq, drows = torch.empty_like(enc), torch.empty_like(query), torch.empty_like(rows)
        part = torch.empty(lib.fr_modal_head_partials(n, 1), dtype=torch.float32, device=dev)
        grad = torch.empty(lib.fr_modal_head_grad_numel(), dtype=torch.float32, device=dev)
        lnp = (ctypes.c_void_p * 4)(ga.data_ptr(), ba.data_ptr(), gb.data_ptr(), bb.data_ptr())
        mlp = (ctypes.c_void_p * 4)(w1.data_ptr(), b1.data_ptr(), w2.data_ptr(), b2.data_ptr())
        with profiling.region("modal_head", fusion_bytes(n, L, True) + health_kd_bytes(n, H, True)):
            native.check(lib.fr_modal_head_bwd(enc.data_ptr(), query.data_ptr(), ids.data_ptr(), num.data_ptr(), pad_id, n,
                                               L, lnp, eps, rows.data_ptr(), labels.data_ptr(), H, mlp, thr, w_h, w_k,
                                               ctx.out.data_ptr(), gh.data_ptr(), gk.data_ptr(), denc.data_ptr(),
                                               dq.data_ptr(), drows.data_ptr(), part.data_ptr(), part.numel(),
                                               native.stream_of(enc)), "fr_modal_head_bwd")
            native.check(lib.fr_modal_head_reduce(part.data_ptr(), n, grad.data_ptr(), native.stream_of(enc)),
                         "fr_modal_head_reduce")
        D, HM = 64, 16
        o = 0
        dw1 = grad[o:o + D * D].view(D, D); o += D * D
        db1 = grad[o:o + D]; o += D
        dw2 = grad[o:o + H * D].view(H, D); o += HM * D
        db2 = grad[o:o + H]; o += HM
        dln = grad[o:o + 128].view(4, 32)
        return (denc, dq, None, None, drows, None, None, None, None, None, None, dln[0], dln[1], dln[2], dln[3],
                dw1, db1, dw2, db2)


def modal_head(enc, query, ids, num, pad_id, rows, labels, ln_a, ln_b, mlp, kd_threshold, w_health, w_kd):
    """modal_fusion + health_kd_loss as one node (cikm_model.py:245-264): returns (w_health * BCE sum,
    w_kd * max(0, 1 - mean cos(know, rows) - kd_threshold)).  ``mlp``: Linear(64, 64), ReLU,
    Linear(64, H <= 16); ``ln_a`` / ``ln_b``: the target attentions' LayerNorm(32) modules."""
    native.require_device(enc, query, ids, rows, labels)
    if ln_a.eps != ln_b.eps:
        raise native.EngineError("modal_head: both target-attention LayerNorms must share eps")
    l1, l2 = mlp[0], mlp[2]
    return _ModalHead.apply(enc.contiguous(), query.contiguous(), ids.contiguous(), num.contiguous(), rows.contiguous(),
                            labels.to(torch.float32).contiguous(), int(pad_id), ln_a.eps,
                            kd_threshold, w_health, w_kd, ln_a.weight, ln_a.bias, ln_b.weight, ln_b.bias,
                            l1.weight, l1.bias, l2.weight, l2.bias)


# ----------------------------------------------------------------------------- dCor
class _DCor(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pairs, weight, *views):
        views = tuple(_rowmajor(v, f32_only=True) for v in views)
        native.require_device(*views)
        V = len(views)
        n, d = views[0].shape
        lib = native.lib()
        ws = native.workspace(lib.fr_dcor_workspace(n, V), views[0].device)
        vp = (ctypes.c_void_p * V)(*[v.data_ptr() for v in views])
        pa = (ctypes.c_int32 * (2 * len(pairs)))(*[x for pr in pairs for x in pr])
        out = torch.empty(len(pairs) + 1, dtype=torch.float32, device=views[0].device)
        # out[P] = weight * sum of the pairs (the model's loss_cl applied in the kernel)
        native.check(lib.fr_dcor_fwd_ex(vp, V, n, d, pa, len(pairs), _f(weight), out.data_ptr(), ws.data_ptr(),
                                        ws.numel(), native.stream_of(views[0])), "fr_dcor_fwd_ex")
        ctx.save_for_backward(*views)
        ctx.ws, ctx.pairs, ctx.weight = ws, pairs, float(weight)
        return out[len(pairs):]

    @staticmethod
    def backward(ctx, g):
        views = ctx.saved_tensors
        V = len(views)
        n, d = views[0].shape
        # written in full by the kernel (overwrite): no zero-filled buffers
        grads = [torch.empty_like(v) if ctx.needs_input_grad[2 + i] else None for i, v in enumerate(views)]
        vp = (ctypes.c_void_p * V)(*[v.data_ptr() for v in views])
        gp = (ctypes.c_void_p * V)(*[native.ptr(x) for x in grads])
        pa = (ctypes.c_int32 * (2 * len(ctx.pairs)))(*[x for pr in ctx.pairs for x in pr])
        gs = None if _is_unit(g) else g.reshape(1).float().contiguous()
        native.check(native.lib().fr_dcor_bwd_ex(vp, V, n, d, pa, len(ctx.pairs), _f(ctx.weight), native.ptr(gs),
                                                 gp, 1, ctx.ws.data_ptr(), ctx.ws.numel(),
                                                 native.stream_of(views[0])), "fr_dcor_bwd_ex")
        return (None, None, *grads)


def dcor_loss(views, pairs, weight: float = 1.0) -> torch.Tensor:
    """weight * sum over pairs (a,b) of correlation_distance(views[a], views[b]) -> shape [1]."""
    return _DCor.apply(tuple(tuple(p) for p in pairs), float(weight), *views)


class _ViewsSumGather(torch.autograd.Function):
    """(v_0 + v_1 + ... , v_0[ids], v_1[ids], ...) for V equally shaped tables (CLUSSL: item_emb =
    item_ingre + item_image + item_text and the SSL views gathered at the batch items,
    pricai_modelx.py:227-263).  Backward: d v_k = g_sum + scatter_add(ids, g_k) for all k at once --
    a broadcast and one float-atomic row add per id and view (deterministic mode: an id sort and an
    ordered add per distinct id) instead of, per view, a
    zero-filled scatter and autograd's accumulation add."""

    @staticmethod
    def forward(ctx, ids, *views):
        ctx.save_for_backward(ids)
        ctx.V, ctx.shape = len(views), views[0].shape
        views = [_rowmajor(v) for v in views]
        native.require_device(ids, *views)
        n, d = views[0].shape
        m = ids.numel()
        total = torch.empty_like(views[0])
        gathered = [torch.empty(m, d, dtype=views[0].dtype, device=ids.device) for _ in views]
        V = len(views)
        # the sum (torch's add order) and the gathers in one launch (fr_views_sum_gather)
        native.check(native.lib().fr_views_sum_gather(
            (ctypes.c_void_p * V)(*[v.data_ptr() for v in views]), V, n, d, ids.data_ptr(), m, total.data_ptr(),
            (ctypes.c_void_p * V)(*[g.data_ptr() for g in gathered]), native.stream_of(total)), "fr_views_sum_gather")
        return (total, *gathered)

    @staticmethod
    def backward(ctx, g_sum, *g_rows):
        (ids,) = ctx.saved_tensors
        V, (n, d) = ctx.V, ctx.shape
        dev = ids.device
        out = [torch.empty(n, d, dtype=torch.float32, device=dev) for _ in range(V)]
        m = ids.numel()
        g_rows = [(_rowmajor(g) if g is not None else torch.zeros(m, d, dtype=torch.float32, device=dev))
                  for g in g_rows]
        g_sum = _rowmajor(g_sum) if g_sum is not None else None
        # d v_k = g_sum + the rows of g_k scattered at ids: a broadcast and one float-atomic row add per
        # id and view (deterministic mode: an id sort and one ordered add per distinct id instead)
        lib = native.lib()
        det = int(_DETERMINISTIC)
        ws = native.workspace(lib.fr_views_sum_gather_bwd_workspace(m) if det else 16, dev)
        native.check(lib.fr_views_sum_gather_bwd(
            native.ptr(g_sum), (ctypes.c_void_p * V)(*[g.data_ptr() for g in g_rows]), V, n, d, ids.data_ptr(), m,
            (ctypes.c_void_p * V)(*[o.data_ptr() for o in out]), det, ws.data_ptr(), ws.numel(),
            native.stream_of(out[0])), "fr_views_sum_gather_bwd")
        return (None, *out)


def views_sum_gather(views, ids):
    """(sum(views) in list order, [v[ids] for v in views]); see _ViewsSumGather.  More than 8,192 ids:
    the separate sum and row gathers."""
    ids = ids.reshape(-1).to(torch.int64)
    if not all(v.is_cuda and v.dtype == torch.float32 and v.dim() == 2 for v in views) or ids.numel() > 8192 \
            or len({tuple(v.shape) for v in views}) != 1 or len(views) > 4 or views[0].shape[1] % 4:
        total = views[0]
        for v in views[1:]:
            total = total + v
        return total, [embedding(ids, v) for v in views]
    out = _ViewsSumGather.apply(ids, *views)
    return out[0], list(out[1:])


# ----------------------------------------------------------------------------- InfoNCE
class _InfoNCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, H, tau):
        H = _rowmajor(H, f32_only=True)
        native.require_device(H)
        m, d = H.shape
        if m % 2:
            raise native.EngineError("InfoNCE expects an even number of rows (two halves)")
        b = m // 2
        lib = native.lib()
        ws = native.workspace(lib.fr_infonce_workspace(b), H.device)
        out = torch.empty(1, dtype=torch.float32, device=H.device)
        native.check(lib.fr_infonce_fwd(H.data_ptr(), b, d, _f(tau), out.data_ptr(), ws.data_ptr(),
                                        ws.numel(), native.stream_of(H)), "fr_infonce_fwd")
        ctx.save_for_backward(H)
        ctx.ws, ctx.tau, ctx.b = ws, tau, b
        return out[0]

    @staticmethod
    def backward(ctx, g):
        (H,) = ctx.saved_tensors
        dH = torch.empty_like(H)  # written in full by fr_infonce_bwd
        gs = g.reshape(1).float().contiguous()
        native.check(native.lib().fr_infonce_bwd(H.data_ptr(), ctx.b, H.shape[1], _f(ctx.tau), _f(1.0),
                                                 gs.data_ptr(), dH.data_ptr(), ctx.ws.data_ptr(),
                                                 ctx.ws.numel(), native.stream_of(H)), "fr_infonce_bwd")
        return dH, None


def infonce_loss(H: torch.Tensor, tau: float = 0.5) -> torch.Tensor:
    return _InfoNCE.apply(H, float(tau))


class _InfoNCEMulti(torch.autograd.Function):
    @staticmethod
    def forward(ctx, pairs, tau, weight, *views):
        views = tuple(_rowmajor(v, f32_only=True) for v in views)
        native.require_device(*views)
        V = len(views)
        b, d = views[0].shape
        if any(v.shape != (b, d) for v in views):
            raise native.EngineError("infonce_pairs: views of one shape [b, d] required")
        lib = native.lib()
        ws = native.workspace(lib.fr_infonce_multi_workspace(V, b, d, len(pairs)), views[0].device)
        vp = (ctypes.c_void_p * V)(*[v.data_ptr() for v in views])
        pa = (ctypes.c_int32 * (2 * len(pairs)))(*[x for pr in pairs for x in pr])
        out = torch.empty(1 + len(pairs), dtype=torch.float32, device=views[0].device)
        native.check(lib.fr_infonce_multi_fwd_ex(vp, V, b, d, pa, len(pairs), _f(tau), _f(weight), out.data_ptr(),
                                                 ws.data_ptr(), ws.numel(), native.stream_of(views[0])),
                     "fr_infonce_multi_fwd_ex")
        ctx.save_for_backward(*views)
        ctx.ws, ctx.pairs, ctx.tau, ctx.weight = ws, pairs, tau, float(weight)
        return out[0]

    @staticmethod
    def backward(ctx, g):
        views = ctx.saved_tensors
        V = len(views)
        b, d = views[0].shape
        grads = [torch.empty_like(v) if ctx.needs_input_grad[3 + i] else None for i, v in enumerate(views)]
        vp = (ctypes.c_void_p * V)(*[v.data_ptr() for v in views])
        gp = (ctypes.c_void_p * V)(*[native.ptr(x) for x in grads])
        pa = (ctypes.c_int32 * (2 * len(ctx.pairs)))(*[x for pr in ctx.pairs for x in pr])
        gs = None if _is_unit(g) else g.reshape(1).float().contiguous()
        native.check(native.lib().fr_infonce_multi_bwd(vp, V, b, d, pa, len(ctx.pairs), _f(ctx.tau), _f(ctx.weight),
                                                       native.ptr(gs), gp, ctx.ws.data_ptr(), ctx.ws.numel(),
                                                       native.stream_of(views[0])), "fr_infonce_multi_bwd")
        return (None, None, None, *grads)


def infonce_pairs(views, pairs, tau: float = 0.5, weight: float = 1.0) -> torch.Tensor:
    """sum over pairs (a, b) of infonce_loss(cat([views[a], views[b]]), tau) (CLUSSL's ssl_mode
    infonce, pricai_modelx.py:263 with CL_loss :354-378) in one forward and one backward node: no
    concatenation, each view normalised once, all pairs in the same launches.  0-dim result, times
    ``weight`` (the model's loss_cl) in the kernel."""
    return _InfoNCEMulti.apply(tuple(tuple(int(x) for x in p) for p in pairs), float(tau), float(weight), *views)


def infonce_flops(n: int, d: int, n_pairs: int, backward: bool = True) -> int:
    """Algorithmic FLOPs of infonce_pairs over ``n_pairs`` pairs of [n, d] views (CL_loss,
    pricai_modelx.py:354-378, hidden = [2n, d]): the logits aa / ab / ba / bb form one (2n)^2 Gram
    (2 (2n)^2 d) forward; the backward's dH = S H and S^T H are two more.  Normalisation, exp and the
    log-sum-exp are not counted."""
    N = 2 * n
    return n_pairs * 2 * N * N * d * (3 if backward else 1)


def dcor_flops(n: int, d: int, n_views: int, backward: bool = True) -> int:
    """Algorithmic FLOPs of dcor_loss over ``n_views`` [n, d] views (correlation_distance,
    pricai_modelx.py:409-437): one X X^T Gram (2 n^2 d) per view forward -- every pair reuses the
    views' distance matrices -- and the backward's m X product (2 n^2 d) per view.  The
    centring sums and square roots are not counted; nor is the backward's recomputation of the
    distances (not algorithmic work)."""
    return n_views * 2 * n * n * d * (2 if backward else 1)


# ----------------------------------------------------------------------------- full-sort top-k
def topk_flops(n_users: int, n_items: int, d: int) -> int:
    """Algorithmic FLOPs of one fr_topk_scores call: the dense n_users x n_items x d score GEMM."""
    return 2 * n_users * n_items * d


def full_sort_topk(user_rows: torch.Tensor, item_table: torch.Tensor, k: int, user_ids=None,
                   exclude=None, held_out=None):
    """Top-k items per query user over ALL items, scored <user, item> on the matrix cores, with
    the running top-k fused (the n_users x n_items score matrix is never written).

    user_rows [n, d] and item_table [I, d]: both fp32 (d in {64, 128}) or both bf16
    (d in {64, 128, 256}).  ``exclude`` / ``held_out``: optional (rowptr int64, col int32, base)
    CSRs indexed by ``user_ids`` (int64 [n], default 0..n-1); items ``base + i`` in a user's
    ``exclude`` row are skipped (history masking), and ``hits[u, j]`` flags top-k entries found in
    the user's ``held_out`` row.  Order: score descending, item id ascending on ties.
    Returns (scores f32 [n, k], items int64 [n, k], hits uint8 [n, k] or None).
    Replaces full_sort_predict + torch.topk (common/trainer.py:476-503, topk_evaluator.py:45-66)."""
    U = _rowmajor(user_rows)
    It = _rowmajor(item_table)
    dt = _same_dtype(U, It)
    native.require_device(U, It)
    n, d = U.shape
    nI = It.shape[0]
    if It.shape[1] != d:
        raise native.EngineError(f"full_sort_topk: user d={d} vs item d={It.shape[1]}")
    dev = U.device
    scores = torch.empty(n, k, dtype=torch.float32, device=dev)
    items = torch.empty(n, k, dtype=torch.int64, device=dev)
    hits = torch.empty(n, k, dtype=torch.uint8, device=dev) if held_out is not None else None
    if n == 0:
        return scores, items, hits
    lib = native.lib()
    ws = native.workspace(lib.fr_topk_workspace(n, nI, k), dev)
    uid = user_ids.to(device=dev, dtype=torch.int64).contiguous() if user_ids is not None else None

    def csr(c):
        if c is None:
            return None, None, 0
        rp, col, base = c
        return rp, col, int(base)

    ep, ec, eb = csr(exclude)
    tp, tc, tb = csr(held_out)
    for t in (ep, ec, tp, tc):
        if t is not None:
            native.require_device(t)
    if (ep is not None and (ep.dtype != torch.int64 or ec.dtype != torch.int32)) or \
            (tp is not None and (tp.dtype != torch.int64 or tc.dtype != torch.int32)):
        raise native.EngineError("CSR rows must be int64 rowptr + int32 columns")
    with profiling.region("topk", topk_flops(n, nI, d)):
        native.check(lib.fr_topk_scores(
            U.data_ptr(), U.stride(0), n, It.data_ptr(), It.stride(0), nI, d,
            1 if dt == torch.bfloat16 else 0, int(k), native.ptr(uid),
            native.ptr(ep), native.ptr(ec), eb, native.ptr(tp), native.ptr(tc), tb,
            scores.data_ptr(), items.data_ptr(), native.ptr(hits), ws.data_ptr(), ws.numel(),
            native.stream_of(U)), "fr_topk_scores")
    return scores, items, hits


# ----------------------------------------------------------------------------- evaluation ranking
def score_segments_ok(user_table, item_table) -> bool:
    """The tables fr_score_segments takes: fp32, 2-D, 64 wide, unit column stride (any row stride)."""
    return all(torch.is_tensor(t) and t.dim() == 2 and t.shape[1] == 64 and t.dtype == torch.float32
               and t.stride(1) == 1 for t in (user_table, item_table))


def score_segments(user_table: torch.Tensor, item_table: torch.Tensor, uid: torch.Tensor, offsets: torch.Tensor,
                   items: torch.Tensor) -> torch.Tensor:
    """``(user_table[u] * item_table[items[e]]).sum()`` for every candidate e of every user segment
    (fr_score_segments): uid [S] user ids, offsets [S + 1] segment bounds, items [n] (int64 device
    tensors).  The graph models' inference_fast over the evaluation lists without the [n, 64] gathers."""
    native.require_device(user_table, item_table, uid, offsets, items)
    d = user_table.shape[1]
    if not score_segments_ok(user_table, item_table):
        raise native.EngineError("score_segments: fp32 [*, 64] row-major tables required")
    out = torch.empty(items.numel(), dtype=torch.float32, device=items.device)
    native.check(native.lib().fr_score_segments(user_table.data_ptr(), user_table.stride(0), item_table.data_ptr(),
                                                item_table.stride(0), uid.data_ptr(), offsets.data_ptr(), uid.numel(),
                                                items.data_ptr(), d, out.data_ptr(), native.stream_of(items)),
                 "fr_score_segments")
    return out


def rank_metrics(scores: torch.Tensor, lens, npos, k: int = 20):
    """fr_rank_metrics over the per-user candidate scores (device fp32, users' lists back to back,
    positives first): numpy (hits uint32, auc counts int64, flags uint8) per user.  Replaces the
    per-user argsort / metrics_by_user / get_auc_fast loop (trainer.py:231-282, 49-69)."""
    native.require_device(scores)
    dev = scores.device
    lens = np.asarray(lens, np.int64)
    U = len(lens)
    off = torch.zeros(U + 1, dtype=torch.int64)
    torch.cumsum(torch.from_numpy(lens), 0, out=off[1:])
    if int(off[-1]) != scores.numel():
        raise ValueError("candidate lengths do not add up to the score count")
    off_d = off.to(dev)
    npos_d = torch.from_numpy(np.asarray(npos, np.int32)).to(dev)
    hits = torch.empty(U, dtype=torch.int32, device=dev)
    auc = torch.empty(U, dtype=torch.int64, device=dev)
    flags = torch.empty(U, dtype=torch.uint8, device=dev)
    sc = scores.float().contiguous()
    native.check(native.lib().fr_rank_metrics(sc.data_ptr(), off_d.data_ptr(), npos_d.data_ptr(), U, int(k),
                                              hits.data_ptr(), auc.data_ptr(), flags.data_ptr(),
                                              native.stream_of(sc)), "fr_rank_metrics")
    return hits.cpu().numpy().view(np.uint32), auc.cpu().numpy(), flags.cpu().numpy()
