"""Row-sharded LightGCN-ID over P GPUs: the config-4 step on 1/2/4/8 MI355X.

Partition.  Users are split into P contiguous blocks balanced by interactions (nnz); rank r holds
its users' ego rows and two CSR slices of the symmetric normalised adjacency (values with the GLOBAL
degrees, identical to the single-GPU Adjacency's entries):

  A_ui[r]  [n_r x I]  user rows of rank r -> item columns       (user -> item block)
  A_iu[r]  [I x n_r]  item rows -> rank r's users (its transpose slice)

Item tables are replicated (1M x 64 fp32 = 256 MB).

Forward, layer k:   E_u^{k+1} = A_ui[r] E_i^k                     (local)
                    E_i^{k+1} = sum_r A_iu[r] E_u^k[r]             (one RCCL all-reduce of I x d)
the item-partial SpMM is launched first and its all-reduce overlaps the user SpMM.  The layer
mean is fused into the last user SpMM's epilogue; the item mean is one pass after the reduce.

Loss.  Every rank samples the same global batch (same seeds).  The batch's user rows (propagated
and ego) are gathered from their owners with one B x d all-reduce (exactly one non-zero
contribution per row), after which BPRLoss + EmbLoss over the global batch are evaluated
redundantly on every rank on identical inputs: the item gradients come out identical everywhere
(no dense gradient all-reduce), and each rank keeps the gradient rows of its own users.

Backward mirrors the forward (H_L = G/(L+1); H_k = A^T H_{k+1} + G/(L+1)): one item all-reduce per
layer.  Per step: 2L collectives of I x d (4 x 256 MB at config 4) + two B x d gathers.  Adam: local
user rows, replicated item rows (bit-identical across ranks, since every rank applies the same
all-reduced gradient).

With P = 1 the step is exactly the single-GPU LightGCN_ID step (up to fp32 summation order).
"""
from __future__ import annotations

import contextlib
import math

import torch
import torch.distributed as dist
from torch import nn

from . import ops
from .graph import DEFAULT_CHUNK, Adjacency


_FORCE = [False]


@contextlib.contextmanager
def collectives_at_world_one():
    """Issue every collective even in a one-rank group (normally skipped as the identity), so a
    single-GPU run exercises the RCCL path (tests on a one-GPU box)."""
    _FORCE[0] = True
    try:
        yield
    finally:
        _FORCE[0] = False


def _all_reduce(t, group, async_op=False):
    """Sum ``t`` over ``group`` in place: a torch.distributed group (backend "nccl" = RCCL) or an
    engine.comm.RcclComm (the C-ABI communicator).  Returns a handle with ``wait()`` for async_op."""
    if group is None:
        return None
    from .comm import RcclComm
    if isinstance(group, RcclComm):
        if group.world == 1 and not _FORCE[0]:
            return None
        return group.all_reduce(t, async_op=async_op)
    if dist.get_world_size(group) == 1 and not _FORCE[0]:
        return None
    return dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group, async_op=async_op)


def _group_rank_world(group):
    from .comm import RcclComm
    if isinstance(group, RcclComm):
        return group.rank, group.world
    return dist.get_rank(group), dist.get_world_size(group)


def check_same_count(n: int, group, what: str, device):
    """Fail fast when the ranks disagree on a row count the next collectives are sized by (the
    rows form's |S|): one all-reduce of a P-slot vector, rank r's count in slot r, so every rank
    sees every count exactly (fp32 is exact below 2^24).  A mismatch would otherwise make the
    |S|-row all-reduces of different lengths hang or read past a buffer; here every rank raises."""
    if group is None:
        return
    rank, world = _group_rank_world(group)
    if world == 1 and not _FORCE[0]:
        return
    slots = torch.zeros(world, dtype=torch.float32, device=device)
    slots[rank] = float(n)
    _all_reduce(slots, group)
    counts = [int(c) for c in slots.cpu().tolist()]
    if any(c != counts[0] for c in counts):
        raise RuntimeError(f"row-sharded step: ranks disagree on {what}: {counts} (rank {rank} has {n})")


class ShardedGraph:
    """Rank ``rank``'s slice of the bipartite interaction graph (u, i) of n_users x n_items."""

    def __init__(self, n_users, n_items, u, i, rank, world, device, chunk=DEFAULT_CHUNK, item_blocks=4):
        U, I = int(n_users), int(n_items)
        dev = torch.device(device)
        u = torch.as_tensor(u, dtype=torch.int64, device=dev)
        i = torch.as_tensor(i, dtype=torch.int64, device=dev)
        key = torch.unique(u * I + i, sorted=True)  # duplicates collapse (binary graph)
        uu = torch.div(key, I, rounding_mode="floor")
        ii = key - uu * I
        # every rank keeps the sorted interaction keys: the global triple sampler below draws the
        # same batch on every rank from them (8 B per interaction)
        self.keys = key
        deg_u = torch.bincount(uu, minlength=U)
        deg_i = torch.bincount(ii, minlength=I)
        dinv_u = torch.pow(deg_u.to(torch.float64) + 1e-7, -0.5)
        dinv_i = torch.pow(deg_i.to(torch.float64) + 1e-7, -0.5)
        E = int(uu.numel())
        # nnz-balanced contiguous user blocks: block r ends at the first user whose prefix count
        # reaches E * (r+1) / P
        cum = torch.cumsum(deg_u, 0)
        targets = torch.tensor([E * (r + 1) // world for r in range(world)], dtype=torch.int64, device=dev)
        ends = torch.searchsorted(cum, targets, right=False) + 1
        ends[-1] = U
        bounds = torch.cat([torch.zeros(1, dtype=torch.int64, device=dev), ends.clamp(max=U)])
        bounds = torch.cummax(bounds, 0).values
        self.bounds = [int(x) for x in bounds.cpu()]
        lo, hi = self.bounds[rank], self.bounds[rank + 1]
        self.lo, self.hi, self.n_local = lo, hi, hi - lo
        self.n_users, self.n_items, self.n_edges = U, I, E
        self.rank, self.world = rank, world
        # local interactions (key order = (u, i) sorted, so user rows come out CSR-ordered)
        a = int(torch.searchsorted(uu, torch.tensor([lo], device=dev)).item())
        b = int(torch.searchsorted(uu, torch.tensor([hi], device=dev)).item())
        lu, li = uu[a:b] - lo, ii[a:b]
        del uu, ii
        val = (dinv_u[lu + lo] * dinv_i[li]).to(torch.float32)
        rp_u = torch.zeros(self.n_local + 1, dtype=torch.int64, device=dev)
        torch.cumsum(torch.bincount(lu, minlength=self.n_local), 0, out=rp_u[1:])
        self.A_ui = Adjacency(rp_u, li.to(torch.int32), val, (self.n_local, I), device=dev, chunk=chunk,
                              symmetric=False)
        order = torch.argsort(li * max(self.n_local, 1) + lu)
        rp_i = torch.zeros(I + 1, dtype=torch.int64, device=dev)
        torch.cumsum(torch.bincount(li, minlength=I), 0, out=rp_i[1:])
        col_iu, val_iu = lu[order].to(torch.int32), val[order]
        self.A_iu = Adjacency(rp_i, col_iu, val_iu, (I, self.n_local), device=dev, chunk=chunk, symmetric=False)
        # the transpose slice cut into nnz-balanced item-row blocks: each block's partial item rows are
        # all-reduced as soon as they are computed, while the next block is still gathering
        self.iu_blocks = self._row_blocks(rp_i, col_iu, val_iu, torch.cumsum(deg_i, 0), max(1, int(item_blocks)),
                                          chunk, dev)
        self.local_nnz = int(lu.numel())

    def _row_blocks(self, rp, col, val, gcum, nb, chunk, dev):
        """[(row_lo, row_hi, Adjacency of rows [row_lo, row_hi))]: item-row blocks balanced by the GLOBAL
        item degrees (``gcum`` = their prefix sums, the same on every rank), so every rank cuts the
        item table at the same rows and the per-block all-reduces match across ranks."""
        R = rp.numel() - 1
        total = int(gcum[-1].item()) if R else 0
        if nb == 1 or R == 0 or total == 0:
            return [(0, R, self.A_iu)]
        targets = torch.tensor([total * (b + 1) // nb for b in range(nb - 1)], dtype=torch.int64, device=gcum.device)
        cuts = (torch.searchsorted(gcum, targets) + 1).clamp(0, R).cpu().tolist()
        bounds = sorted(set([0] + [int(c) for c in cuts] + [R]))
        out = []
        for lo, hi in zip(bounds, bounds[1:]):
            e0, e1 = int(rp[lo].item()), int(rp[hi].item())
            out.append((lo, hi, Adjacency(rp[lo:hi + 1] - e0, col[e0:e1], val[e0:e1], (hi - lo, self.n_local),
                                          device=dev, chunk=chunk, symmetric=False)))
        return out

    # ------------------------------------------------------------------ global triple sampler
    def triples(self, batch_size: int, seed: int, epoch_step: int):
        """Batch ``epoch_step`` of the epoch permutation seeded by ``seed`` -- identical on every rank
        (same seeds, same keys).  Positives: interactions in permutation order (the shuffled
        positive list); negatives: uniform items redrawn while (u, n) is an interaction
        (get_random_neg, dataloader.py:145-151), at most 64 rounds."""
        B = int(batch_size)
        E = self.n_edges
        per_epoch = E // B
        epoch, k = divmod(int(epoch_step), per_epoch)
        dev = self.keys.device
        if getattr(self, "_perm_epoch", None) != (seed, epoch):
            gen = torch.Generator(device=dev).manual_seed(seed * 1_000_003 + epoch)
            self._perm = torch.randperm(E, device=dev, generator=gen)
            self._perm_epoch = (seed, epoch)
        key = self.keys[self._perm[k * B:(k + 1) * B]]
        I = self.n_items
        u = torch.div(key, I, rounding_mode="floor")
        p = key - u * I
        gen = torch.Generator(device=dev).manual_seed((seed * 7_919 + int(epoch_step)) & 0x7FFFFFFFFFFF)
        n = torch.randint(0, I, (B,), device=dev, generator=gen)
        for _ in range(64):  # every rank takes the same rounds (same data), so draws stay in step
            cand = u * I + n
            pos = torch.searchsorted(self.keys, cand).clamp_(max=E - 1)
            hit = self.keys[pos] == cand
            if not bool(hit.any()):
                break
            n = torch.where(hit, torch.randint(0, I, (B,), device=dev, generator=gen), n)
        return u, p, n

    def owner_index(self, users: torch.Tensor):
        """(mask of batch users owned by this rank, their local row index)."""
        own = (users >= self.lo) & (users < self.hi)
        return own, torch.where(own, users - self.lo, torch.full_like(users, -1))


def _item_partial(g: ShardedGraph, Eu, out, group):
    """out = A_iu[rank] Eu (this rank's contribution to every item row), one launch per item-row block,
    each block's all-reduce issued (async) right after its launch.  Returns the pending handles."""
    works = []
    for lo, hi, blk in g.iu_blocks:
        ops.spmm_launch(blk, Eu, Y1=out[lo:hi])
        works.append(_all_reduce(out[lo:hi], group, async_op=True))
    return works


def _wait(works):
    for w in works:
        if w is not None:
            w.wait()


class _ShardedPropagate(torch.autograd.Function):
    """Layer k: E_u^{k+1} = A_ui E_i^k (local) and E_i^{k+1} = sum_r A_iu[r] E_u^k[r] (all-reduce).
    The item partial of layer k only needs E_u^k, so it is launched first, block by block with each
    block's all-reduce issued behind it; the all-reduce of layer k is waited for only right before
    the user SpMM of layer k + 1 needs E_i^{k+1} -- it overlaps the rest of the item partial, the
    user SpMM of layer k and the item partial of layer k + 1.  Backward mirrors it."""

    @staticmethod
    def forward(ctx, ego_u, ego_i, g: ShardedGraph, L: int, group):
        ctx.g, ctx.L, ctx.group = g, L, group
        inv = 1.0 / (L + 1)
        Eu, Ei = ego_u, ego_i
        out_u = torch.empty_like(ego_u)
        acc_i = ego_i.clone()
        prev_u = []
        pending = None  # (handles, table) of the previous layer's item all-reduce
        for k in range(L):
            pi = torch.empty_like(ego_i)
            works = _item_partial(g, Eu, pi, group)               # E_i^{k+1}, reduce in flight
            if pending is not None:                              # E_i^k for this layer's user SpMM
                _wait(pending[0])
                acc_i.add_(pending[1])
                Ei = pending[1]
            if k == L - 1:                                        # last user layer: mean in the epilogue
                terms = [ego_u] + prev_u
                A1 = terms[0]
                A2 = terms[1] if len(terms) > 1 else None
                if len(terms) <= 2:
                    ops.spmm_launch(g.A_ui, Ei, Y2=out_u, alpha=inv, A1=A1, beta1=inv, A2=A2, beta2=inv)
                else:
                    ops.spmm_launch(g.A_ui, Ei, Y1=out_u)
                    out_u.add_(torch.stack(terms).sum(0)).mul_(inv)
            else:
                nu = torch.empty_like(ego_u)
                ops.spmm_launch(g.A_ui, Ei, Y1=nu)
                prev_u.append(nu)
                Eu = nu
            pending = (works, pi)
        _wait(pending[0])
        acc_i.add_(pending[1])
        out_i = acc_i.mul_(inv)
        return out_u, out_i

    @staticmethod
    def backward(ctx, g_u, g_i):
        g, L, group = ctx.g, ctx.L, ctx.group
        inv = 1.0 / (L + 1)
        g_u = g_u.contiguous() if g_u is not None else None
        g_i = g_i.contiguous() if g_i is not None else None
        dev_u = g_u if g_u is not None else torch.zeros(g.n_local, g_i.shape[1], device=g_i.device)
        dev_i = g_i if g_i is not None else torch.zeros(g.n_items, g_u.shape[1], device=g_u.device)
        Hu = dev_u * inv
        Hi = dev_i * inv
        pending = None
        for _ in range(L):
            pi = torch.empty_like(Hi)
            works = _item_partial(g, Hu, pi, group)
            if pending is not None:
                _wait(pending[0])
                Hi = pending[1].add_(dev_i, alpha=inv)
            nHu = torch.empty_like(Hu)
            ops.spmm_launch(g.A_ui, Hi, Y2=nHu, alpha=1.0, A1=dev_u, beta1=inv)
            pending = (works, pi)
            Hu = nHu
        _wait(pending[0])
        Hi = pending[1].add_(dev_i, alpha=inv)
        return Hu, Hi, None, None, None


def _marks(g, key, n, dev):
    """Persistent (uint8 mask, int32 bitmask) over ``n`` rows, kept on the graph (all clear between uses)."""
    cache = g.__dict__.setdefault("_marks", {})
    m = cache.get(key)
    if m is None:
        m = (torch.zeros(n, dtype=torch.uint8, device=dev), torch.zeros((n + 31) // 32, dtype=torch.int32, device=dev))
        cache[key] = m
    return m


def _neighbour_items(g: ShardedGraph, loc: torch.Tensor) -> torch.Tensor:
    """Item columns of this rank's batch users (rows ``loc`` >= 0 of A_ui), duplicates kept."""
    own = loc[loc >= 0]
    rp = g.A_ui.rowptr
    starts, ends = rp[own], rp[own + 1]
    lens = ends - starts
    total = int(lens.sum().item())
    if total == 0:
        return torch.zeros(0, dtype=torch.int64, device=loc.device)
    first = torch.cumsum(lens, 0) - lens
    pos = torch.repeat_interleave(starts - first, lens) + torch.arange(total, device=loc.device)
    return g.A_ui.col[pos].to(torch.int64)


class _ShardedRowsStep(torch.autograd.Function):
    """_ShardedPropagate (L = 2) for a loss that reads the propagated tables at the batch rows only
    (the rows form of ops.propagate_rows, single-GPU config 4), with the owner gathers of the batch
    users' propagated and ego rows folded in.  The item table of layer 1 is needed only at S = the
    items adjacent to the batch users (for their layer-2 rows) plus the batch items (for theirs),
    and the first backward layer's item rows are non-zero only on the first part of S:
      forward   S agreed on by every rank (an all-reduce of per-item flags, then the same nonzero
                list everywhere); layer-1 item partial at S only (row list), its |S| rows all-reduced
                (|S| x d instead of I x d); the user layer 1 in full (local); layer 2 at this rank's
                batch users (row list, users owned elsewhere carry id -1) and at the batch items (row
                list on the transpose slice, the 2B partial rows all-reduced); the batch users'
                propagated and ego rows gathered from their owners by ONE [2B x d] all-reduce;
      backward  the batch users' upstream stays B rows: the first layer from the sparse upstream
                gradients (users: A_ui at the batch items' columns; items: A_iu at this rank's batch
                users' columns, all-reduced at S only), the second in full (item partial per item-row
                block, all-reduced as before); the user rows' own terms (g / 3 and the ego rows'
                gradient) are added at the batch rows after each user SpMM, so no dense
                [n_local x d] upstream table is zero-filled, read as an epilogue addend, or summed
                with a second dense ego gradient by autograd.
    Collectives per step: one all-reduce of I x d (the last backward layer, in blocks) + |S| x d
    twice + 2B x d twice + the flags (I floats).  Returns (propagated user rows [B, d], ego user
    rows [B, d], propagated item table valid at the batch items).  Float-atomic row additions."""

    @staticmethod
    def forward(ctx, ego_u, ego_i, g: ShardedGraph, group, loc, p, n):
        inv = 1.0 / 3.0
        ctx.g, ctx.group = g, group
        dev = ego_u.device
        pn = torch.cat([p, n])
        # fp32 flags (the C-ABI communicator reduces fp32): every rank the same sums, the same list
        flags = torch.zeros(g.n_items, dtype=torch.float32, device=dev)
        flags[_neighbour_items(g, loc)] = 1.0
        flags[pn] = 1.0
        _all_reduce(flags, group)
        S = torch.nonzero(flags > 0).reshape(-1)
        del flags
        check_same_count(S.numel(), group, "|S| (layer-1 item rows)", dev)
        pi1 = torch.empty_like(ego_i)                              # valid at S
        ops.spmm_ex(g.A_iu, ego_u, Y1=pi1, rows=[(S, 0)], region="spmm_rows")
        part1 = pi1.index_select(0, S)
        work = _all_reduce(part1, group, async_op=True)
        E1u = torch.empty_like(ego_u)
        ops.spmm_launch(g.A_ui, ego_i, Y1=E1u)                    # E_u^1 (local, in flight beside the reduce)
        _wait([work])
        E1i = pi1
        E1i.index_copy_(0, S, part1)                               # E_i^1, valid at S
        out_u = torch.empty_like(ego_u)                            # valid at this rank's batch users
        ops.spmm_ex(g.A_ui, E1i, Y2=out_u, alpha=inv, A1=ego_u, beta1=inv, A2=E1u, beta2=inv, rows=[(loc, 0)],
                    region="spmm_rows")
        pi2 = torch.empty_like(ego_i)                              # valid at the batch items
        ops.spmm_ex(g.A_iu, E1u, Y1=pi2, rows=[(p, 0), (n, 0)], region="spmm_rows")
        part2 = pi2.index_select(0, pn)
        _all_reduce(part2, group)
        del E1u
        out_i = torch.empty_like(ego_i)                            # valid at the batch items
        out_i.index_copy_(0, pn, (ego_i.index_select(0, pn) + E1i.index_select(0, pn) + part2) * inv)
        # owner gathers: [out_u[loc] ; ego_u[loc]], rows owned elsewhere zero, one all-reduce
        B = loc.numel()
        safe = loc.clamp(min=0)
        rows = torch.cat([out_u.index_select(0, safe), ego_u.index_select(0, safe)])
        # rows owned elsewhere read row 0 of a table valid only at this rank's batch users: select,
        # not multiply (0 * a NaN / Inf bit pattern would reach every rank through the all-reduce)
        rows.masked_fill_((loc < 0).repeat(2).unsqueeze(1), 0.0)
        _all_reduce(rows, group)
        ctx.save_for_backward(loc, p, n, S)
        ctx.n_local = ego_u.shape[0]
        return rows[:B], rows[B:], out_i

    @staticmethod
    def backward(ctx, g_ub, g_eb, g_i):
        g, group = ctx.g, ctx.group
        loc, p, n, S = ctx.saved_tensors
        inv = 1.0 / 3.0
        dev = loc.device
        B = loc.numel()
        own = (loc >= 0).to(torch.float32).unsqueeze(1)
        safe = loc.clamp(min=0)
        g_ub = g_ub.contiguous() * own if g_ub is not None else torch.zeros(B, 64, device=dev)
        g_eb = g_eb.contiguous() * own if g_eb is not None else torch.zeros(B, 64, device=dev)
        g_i = g_i.contiguous() if g_i is not None else torch.zeros(g.n_items, 64, device=dev)
        # items of the first backward layer: A_iu at this rank's batch users (non-zero inside S only),
        # all-reduced at S.  The users' upstream rows go into a persistent table read only at the
        # marked rows (those rows zeroed by the mark, then summed: a user may occur twice)
        mu, bu = _marks(g, "users", g.n_local, dev)
        Gu = g.__dict__.get("_g_rows")
        if Gu is None or Gu.device != dev:
            Gu = torch.empty(g.n_local, 64, device=dev)
            g.__dict__["_g_rows"] = Gu
        ops.rows_mark(mu, [(loc, 0)], 1, zero=Gu, bits=bu)
        Gu.index_add_(0, safe, g_ub)                                 # rows owned elsewhere add 0 to an unread row
        piH = torch.empty_like(g_i)
        ops.spmm_sparse_rect(g.A_iu, bu, Gu, piH, alpha=1.0)
        ops.rows_mark(mu, [(loc, 0)], 0, bits=bu)
        partH = piH.index_select(0, S)
        work = _all_reduce(partH, group, async_op=True)
        # users of the first backward layer (local): A_ui at the batch items' columns, + g / 3 at the rows
        mi, bi = _marks(g, "items", g.n_items, dev)
        ops.rows_mark(mi, [(p, 0), (n, 0)], 1, bits=bi)
        Hu = torch.empty(ctx.n_local, 64, device=dev)
        ops.spmm_sparse_rect(g.A_ui, bi, g_i, Hu, alpha=inv)
        ops.rows_mark(mi, [(p, 0), (n, 0)], 0, bits=bi)
        Hu.index_add_(0, safe, g_ub * inv)
        _wait([work])
        Hi = g_i * inv
        Hi.index_copy_(0, S, partH.mul_(inv).add_(Hi.index_select(0, S)))
        # second layer in full; the user rows' own terms (g / 3 + the ego rows' gradient) added after
        pi = piH
        works = _item_partial(g, Hu, pi, group)
        d_u = torch.empty(ctx.n_local, 64, device=dev)
        ops.spmm_launch(g.A_ui, Hi, Y1=d_u)
        d_u.index_add_(0, safe, g_ub * inv + g_eb)
        _wait(works)
        d_i = pi.add_(g_i, alpha=inv)
        return d_u, d_i, None, None, None, None, None


class _OwnerGather(torch.autograd.Function):
    """rows[b] = local_table[loc[b]] on the owning rank, assembled on every rank by one all-reduce
    (exactly one rank contributes each row).  Backward: every rank holds the full gradient of the
    gathered rows (the loss is evaluated redundantly), so each scatters its own rows -- no
    communication (deterministic fr_embedding_bwd; rows owned elsewhere are skipped)."""

    @staticmethod
    def forward(ctx, local_table, loc, group):
        ctx.save_for_backward(loc)
        ctx.n = local_table.shape[0]
        safe = loc.clamp(min=0)
        rows = local_table.index_select(0, safe) * (loc >= 0).unsqueeze(1).to(local_table.dtype)
        _all_reduce(rows, group)
        return rows

    @staticmethod
    def backward(ctx, grad):
        (loc,) = ctx.saved_tensors
        return ops.scatter_rows(loc, grad, ctx.n), None, None


class ShardedLightGCN(nn.Module):
    """LightGCN_ID's parameters and step, row-sharded.  ``ego_u``: this rank's user rows; ``ego_i``:
    the replicated item table.  Initialised from the same seed as the single-GPU model (the full
    user table is drawn on every rank and sliced), so P ranks start from identical global tables."""

    # the rows form sizes its launches from host reads (the agreed row set S): Trainer steps it eagerly
    graph_capturable = False

    def __init__(self, graph: ShardedGraph, d=64, n_layers=2, reg_weight=0.1, group=None, seed=999):
        super().__init__()
        self.g, self.L, self.reg_weight, self.group, self.d = graph, int(n_layers), float(reg_weight), group, d
        dev = graph.A_ui.rowptr.device
        U, I = graph.n_users, graph.n_items
        gen = torch.Generator(device=dev).manual_seed(seed)
        bu, bi = math.sqrt(6.0 / (U + d)), math.sqrt(6.0 / (I + d))  # xavier_uniform_ of [U,d], [I,d]
        full_u = torch.empty(U, d, device=dev).uniform_(-bu, bu, generator=gen)
        self.ego_u = nn.Parameter(full_u[graph.lo:graph.hi].clone())
        del full_u
        self.ego_i = nn.Parameter(torch.empty(I, d, device=dev).uniform_(-bi, bi, generator=gen))

    def calculate_loss(self, batch):
        u, p, n = batch["u_id"], batch["pos_i_id"], batch["neg_i_id"]
        _, loc = self.g.owner_index(u)
        if (self.L == 2 and self.ego_u.is_cuda and self.d == 64 and not ops._DETERMINISTIC
                and not torch.cuda.is_current_stream_capturing()):
            # the loss reads the propagated tables at the batch rows only (rows form)
            p, n = p.to(torch.int64).contiguous(), n.to(torch.int64).contiguous()
            out_ub, ego_ub, out_i = _ShardedRowsStep.apply(self.ego_u, self.ego_i, self.g, self.group,
                                                           loc.contiguous(), p, n)
        else:
            out_u, out_i = _ShardedPropagate.apply(self.ego_u, self.ego_i, self.g, self.L, self.group)
            out_ub = _OwnerGather.apply(out_u, loc, self.group)
            ego_ub = _OwnerGather.apply(self.ego_u, loc, self.group)
        B = u.numel()
        ar = torch.arange(B, device=u.device)
        # replicated item gradients must come out bit-identical on every rank: deterministic BPR
        # scatter (owner slots) and deterministic row gathers for the EmbLoss item rows
        mf, _ = ops.bpr_emb_loss(out_ub, out_i, None, None, ar, p, n, deterministic=True)
        ego_ib = ops.embedding(torch.cat([p, n]), self.ego_i)
        reg = (torch.norm(ego_ub) + torch.norm(ego_ib[:B]) + torch.norm(ego_ib[B:])) / B
        return mf, self.reg_weight * reg.reshape(1)
