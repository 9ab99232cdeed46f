"""Fused multi-tensor Adam on the HIP kernels ``fr_adam_step_dev`` / ``fr_adam_step``.

Drop-in for ``torch.optim.Adam`` as the reference trainer builds it (common/trainer.py:143-144):
same param_groups and per-parameter state keys (``step``, ``exp_avg``, ``exp_avg_sq``), so
``state_dict()`` round-trips.  Parameters whose ``.grad`` is None are skipped, as in torch.

The step counters and the learning rate live in device memory (like torch's capturable Adam): the
kernel increments each tensor's counter and derives the bias corrections on the device, so a
whole training step (forward, backward, optimiser) can be captured in a HIP graph and replayed.
After changing ``group['lr']`` outside of step() (LR scheduler), call :meth:`sync_lr`.

Row gradients (``row_grads``): a table whose only use on the step is a row gather (HealthRec's
45,630 x 2048 image and x 512 text tables) can hand its gradient to the optimiser as the gathered
(ids, rows) instead of a dense zero-filled table (``ops.embedding(..., exchange=opt.row_grads)``).
``step()`` reduces them with ``fr_embedding_rowgrad`` (a row -> slot map plus one summed row per
distinct id) and ``fr_adam_step_rows`` applies Adam to every row with the gradient read from the
compact rows (zero elsewhere): the same arithmetic as the dense update, bit for bit, without the
dense table's zero fill and gradient read (8 of 32 bytes per parameter).
"""
from __future__ import annotations

import ctypes
import os

import torch

from . import native, profiling


ROW_GRAD_MAX = 1 << 18  # positions per table per step the row-gradient reduction takes (fr_embedding_rowgrad)


def adam_rows_bytes(numel: int, rows: int, compact: int) -> int:
    """Algorithmic HBM bytes of the row-gradient Adam on one table: p, m, v read + written (24 B per
    parameter), the row map (4 B per row) and the compact gradient rows (read once)."""
    return 24 * numel + 4 * rows + 4 * compact


# FusedAdam.step: the factored row gradients and the row tables' update on a side stream (forked
# at the projection backward); FR_ROWS_SIDE_STREAM=0: on the current stream after the backward
ROWS_SIDE_STREAM = os.environ.get("FR_ROWS_SIDE_STREAM", "1") != "0"


# FR_SLICE_PARTS: the per-step background slice in this many launches -- the first beside the step's
# start (as with 1), the others where the model calls RowGrads.background_rest
SLICE_PARTS = max(1, int(os.environ.get("FR_SLICE_PARTS", "1")))


class RowGrads:
    """Pending row gradients of row-gathered tables: ``stash`` is called from the backward of
    ``ops.embedding(..., exchange=self)``; several stashes of one table before a step (repeated
    backward passes) accumulate, exactly as dense gradients would."""

    def __init__(self):
        self.pending = {}   # id(weight) -> [weight, padding_idx, [ids], [rows]]
        # id(weight) -> (weight, padding_idx, ids, dY [n, 64], W [64, K]): gradient rows dY[i] W of a
        # gathered Linear input (ops.modal_projection), materialised by FusedAdam before any update
        self.factored = {}
        self.catch_up = None  # set by a FusedAdam with lazy_rows
        self.catch_up_slice = None  # set by a FusedAdam with lazy_rows and lazy_slices > 0
        self._bg_join = None  # joins the background slice replay into the main stream
        self._bg_rest = None  # issues the slice's remaining parts (background_rest)
        # (weight, ids) pairs caught up by prefetch_rows this step.  The ids tensors are held here, so
        # their memory cannot be handed to another tensor by the caching allocator before clear():
        # a (weight, pointer, numel) match below therefore names the same ids
        self._prefetched = []
        self._side = None
        self.factored_event = None

    def stash_factored(self, weight, padding_idx, ids, dY, W):
        if id(weight) in self.pending or id(weight) in self.factored:  # repeated backward: explicit rows
            e = self.factored.pop(id(weight), None)
            if e is not None:
                self.stash(e[0], e[1], e[2], e[3] @ e[4])
            self.stash(weight, padding_idx, ids, dY @ W)
            return
        self.factored[id(weight)] = (weight, padding_idx, ids, dY, W)
        if dY.is_cuda:  # where the backward stream stood when dY was written (FusedAdam.step forks here)
            self.factored_event = torch.cuda.Event()
            self.factored_event.record(torch.cuda.current_stream(dY.device))

    def stash(self, weight, padding_idx, ids, G):
        e = self.pending.get(id(weight))
        if e is None:
            self.pending[id(weight)] = [weight, padding_idx, [ids], [G]]
        else:
            e[2].append(ids)
            e[3].append(G)

    def clear(self):
        self.join_background()
        self.pending.clear()
        self.factored.clear()
        self.factored_event = None
        self._prefetched.clear()

    def catch_up_rows(self, weight, ids):
        """Called before ``weight`` is gathered at ``ids``: a lazily updating optimiser brings those
        rows up to the current step (FusedAdam.catch_up_rows).  Skipped when ``prefetch_rows``
        already covered (weight, ids)."""
        if self.catch_up is not None and not any(
                w is weight and (i is ids or (i.data_ptr() == ids.data_ptr() and i.numel() == ids.numel()
                                              and i.dtype == ids.dtype)) for w, i in self._prefetched):
            self.catch_up(weight, ids)

    def prefetch_rows(self, pairs):
        """Catch up [(weight, ids), ...] on a side stream, overlapping whatever the caller runs next
        (HealthRec: the SpMM propagation, which reads none of these tables).  Returns a callable that
        makes a stream (default: the current one) wait for it; call it before the gathers.
        Graph-capturable (fork / join of the capture stream)."""
        if self.catch_up is None or not pairs or not pairs[0][0].is_cuda:
            return lambda stream=None: None
        main = torch.cuda.current_stream(pairs[0][0].device)
        if self._side is None:
            from . import ops
            self._side = ops.new_stream(pairs[0][0].device, "side")
        side = self._side
        side.wait_stream(main)
        with torch.cuda.stream(side):
            multi = getattr(self.catch_up, "__self__", None)
            same_ids = all(ids is pairs[0][1] for _, ids in pairs)
            if multi is not None and same_ids and len(pairs) <= 4:
                multi.catch_up_rows_multi([w for w, _ in pairs], pairs[0][1])
            else:
                for w, ids in pairs:
                    self.catch_up(w, ids)
            self._prefetched.extend(pairs)
            caught = torch.cuda.Event()
            caught.record(side)
            if self.catch_up_slice is not None and self._bg_join is None:
                # then one row slice of the lazily updated tables replays its backlog behind the
                # catch-up (the batch's rows are current by then and skip), overlapping the rest of
                # the step; joined before the optimiser touches any lazy state (join_background).
                # With SLICE_PARTS > 1 only its first part here; background_rest issues the others
                ws = [w for w, _ in pairs]
                self.catch_up_slice(ws, 0, SLICE_PARTS)
                self._bg_join = lambda: main.wait_stream(side)
                if SLICE_PARTS > 1:
                    def rest(ws=ws, side=side, main=main):
                        side.wait_stream(main)
                        with torch.cuda.stream(side):
                            for part in range(1, SLICE_PARTS):
                                self.catch_up_slice(ws, part, SLICE_PARTS)
                    self._bg_rest = rest
        return lambda stream=None: (stream if stream is not None else main).wait_event(caught)

    def background_rest(self):
        """Issue the background slice's remaining parts behind everything the current stream has
        issued so far (a model calls this where the step leaves the chip idle enough: HealthRec after
        its encoder forward); join_background issues them if nobody did."""
        if self._bg_rest is not None:
            r, self._bg_rest = self._bg_rest, None
            r()

    def join_background(self):
        """Make the current stream wait for the background slice replay (before any optimiser
        kernel reads or advances the lazy step counters / history)."""
        self.background_rest()
        if self._bg_join is not None:
            j, self._bg_join = self._bg_join, None
            j()

    def __bool__(self):
        return bool(self.pending or self.factored)

    def take(self, weight):
        e = self.pending.pop(id(weight), None)
        if e is None:
            return None
        ids = e[2][0] if len(e[2]) == 1 else torch.cat(e[2])
        G = e[3][0] if len(e[3]) == 1 else torch.cat(e[3])
        return ids, G, e[1]


def _row_grad_ok(p, ids, G) -> bool:
    d = p.shape[-1] if p.dim() == 2 else 0
    return (p.dim() == 2 and p.dtype == torch.float32 and p.is_contiguous() and d >= 4 and d & (d - 1) == 0
            and ids.numel() <= ROW_GRAD_MAX and G.dtype == torch.float32 and p.data_ptr() % 16 == 0)


# a late-drained table's update on the branch stream right behind the scatter of its deferred rows
# (no cross-queue hop between them).  Slower while that scatter was a chain of dependent load rounds
# (0.694 / 0.691 vs 0.688 / 0.689 ms per step); with the one-round scatter formed from the norms'
# backward in the same launch (fr_norms_bwd_scatter) 0.682 / 0.673 vs 0.685 / 0.684 ms, on.
# FR_HELD_ON_BRANCH=0: the held update on the current stream after the join (round 4)
HELD_ON_BRANCH = os.environ.get("FR_HELD_ON_BRANCH", "1") == "1"


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, lazy_rows=False,
                 hist_cap=8192, lazy_slices=0):
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("invalid Adam hyper-parameters")
        if hist_cap < 4:
            raise ValueError("hist_cap < 4")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      amsgrad=False, maximize=False))
        self._d_lr = {}   # group index -> (device float64 lr, host value it holds)
        self.row_grads = RowGrads()
        # lazy_rows: row-gradient tables defer their zero-gradient steps (fr_adam_step_rows_lazy);
        # flush() brings them up to date (bit-identical to the dense update).  _lazy_pending counts
        # executed lazy steps since the last flush (graph replays report theirs via note_replay).
        self.lazy_rows = bool(lazy_rows)
        self.hist_cap = int(hist_cap)
        self._lazy_pending = 0
        self._lazy_launched = False
        self.lazy_slices = int(lazy_slices)
        if self.lazy_slices < 0:
            raise ValueError("lazy_slices < 0")
        if self.lazy_rows:
            self.row_grads.catch_up = self.catch_up_rows
            if self.lazy_slices:
                self.row_grads.catch_up_slice = self.catch_up_slice

    @torch.no_grad()
    def catch_up_rows_multi(self, ps, ids):
        """catch_up_rows for several tables gathered at the same ids, one launch
        (fr_adam_catch_up_rows_multi).  Tables without lazy state are skipped."""
        ps = [p for p in ps if "lazy_last" in self.state.get(p, {})]
        if not ps:
            return
        groups = {id(p): g for g in self.param_groups for p in g["params"]}
        g0 = groups[id(ps[0])]
        if any(groups[id(p)] is not g0 for p in ps):  # differing hyper-parameters: one launch per table
            for p in ps:
                self.catch_up_rows(p, ids)
            return
        beta1, beta2 = g0["betas"]
        ids = ids.reshape(-1)
        if ids.dtype != torch.int64:
            ids = ids.to(torch.int64)
        n = len(ps)
        st = [self.state[p] for p in ps]
        arr = lambda xs: (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])  # noqa: E731
        with profiling.region("adam_rows_catch_up", sum(28 * ids.numel() * p.shape[1] for p in ps) + 8 * ids.numel()):
            native.check(native.lib().fr_adam_catch_up_rows_multi(
                n, arr(ps), arr([s_["exp_avg"] for s_ in st]), arr([s_["exp_avg_sq"] for s_ in st]),
                arr([s_["step"] for s_ in st]), (ctypes.c_int64 * n)(*[p.shape[0] for p in ps]),
                (ctypes.c_int32 * n)(*[p.shape[1] for p in ps]), arr([s_["lazy_last"] for s_ in st]),
                arr([s_["lazy_hist"] for s_ in st]), ids.data_ptr(), ids.numel(), self.hist_cap, float(beta1),
                float(beta2), float(g0["eps"]), float(g0["weight_decay"]), native.stream_of(ps[0])),
                "fr_adam_catch_up_rows_multi")

    @torch.no_grad()
    def catch_up_slice(self, ps, part=0, n_parts=1):
        """One background slice (fr_adam_catch_up_slice_part): rows [R s / K, R (s + 1) / K) of the
        lazily updated tables ``ps``, s = device step counter mod K = ``lazy_slices``, replay their
        backlog through the current step (``part`` of ``n_parts`` even row ranges of it).  Tables
        without lazy state are skipped."""
        ps = [p for p in ps if "lazy_last" in self.state.get(p, {})]
        groups = {id(p): g for g in self.param_groups for p in g["params"]}
        by_group = {}
        for p in ps:
            by_group.setdefault(id(groups[id(p)]), (groups[id(p)], []))[1].append(p)
        for group, tabs in by_group.values():
            beta1, beta2 = group["betas"]
            for k in range(0, len(tabs), 4):
                chunk = tabs[k:k + 4]
                n = len(chunk)
                st = [self.state[p] for p in chunk]
                arr = lambda xs: (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])  # noqa: E731
                rows = sum(-(-p.shape[0] // self.lazy_slices) * p.shape[1] for p in chunk) // n_parts
                with profiling.region("adam_rows_slice", 24 * rows):
                    native.check(native.lib().fr_adam_catch_up_slice_part(
                        n, arr(chunk), arr([s_["exp_avg"] for s_ in st]), arr([s_["exp_avg_sq"] for s_ in st]),
                        arr([s_["step"] for s_ in st]), (ctypes.c_int64 * n)(*[p.shape[0] for p in chunk]),
                        (ctypes.c_int32 * n)(*[p.shape[1] for p in chunk]), arr([s_["lazy_last"] for s_ in st]),
                        arr([s_["lazy_hist"] for s_ in st]), self.lazy_slices, int(part), int(n_parts), self.hist_cap,
                        float(beta1), float(beta2), float(group["eps"]), float(group["weight_decay"]),
                        native.stream_of(chunk[0])), "fr_adam_catch_up_slice_part")

    @torch.no_grad()
    def catch_up_rows(self, p, ids):
        """Rows ``ids`` of a lazily updated table replay their deferred steps (fr_adam_catch_up_rows)
        so a gather reads dense-Adam values.  No-op for tables without lazy state."""
        st = self.state.get(p)
        if not st or "lazy_last" not in st:
            return
        group = next(g for g in self.param_groups if any(q is p for q in g["params"]))
        beta1, beta2 = group["betas"]
        ids = ids.reshape(-1)
        if ids.dtype != torch.int64:
            ids = ids.to(torch.int64)
        with profiling.region("adam_rows_catch_up", 28 * ids.numel() * p.shape[1] + 8 * ids.numel()):
            native.check(native.lib().fr_adam_catch_up_rows(
                p.data_ptr(), st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr(), st["step"].data_ptr(),
                ids.data_ptr(), ids.numel(), p.shape[0], p.shape[1], st["lazy_last"].data_ptr(),
                st["lazy_hist"].data_ptr(), self.hist_cap, float(beta1), float(beta2), float(group["eps"]),
                float(group["weight_decay"]), native.stream_of(p)), "fr_adam_catch_up_rows")

    @torch.no_grad()
    def flush(self):
        """Bring every lazily updated table (and its moments) up to the current step.  Call before
        reading those tables in full (evaluation, checkpoints, comparisons); cheap when nothing is
        pending."""
        self.row_grads.join_background()
        if self._lazy_pending == 0:
            return
        for group in self.param_groups:
            self._flush_tables(group, [p for p in group["params"] if "lazy_last" in self.state.get(p, {})])
        self._lazy_pending = 0

    def _flush_tables(self, group, ps):
        """fr_adam_flush_rows over ``ps`` (tables of ``group`` with lazy state), unconditionally."""
        if not ps:
            return
        lib = native.lib()
        beta1, beta2 = group["betas"]
        for k in range(0, len(ps), 16):
            chunk = ps[k:k + 16]
            n = len(chunk)
            st = [self.state[p] for p in chunk]
            arr = lambda xs: (ctypes.c_void_p * n)(*[x.data_ptr() for x in xs])  # noqa: E731
            with profiling.region("adam_rows_flush", sum(24 * p.numel() + 4 * p.shape[0] for p in chunk)):
                native.check(lib.fr_adam_flush_rows(
                    arr(chunk), arr([s["exp_avg"] for s in st]), arr([s["exp_avg_sq"] for s in st]),
                    arr([s["step"] for s in st]), (ctypes.c_int64 * n)(*[p.numel() for p in chunk]),
                    (ctypes.c_int32 * n)(*[p.shape[1] for p in chunk]), arr([s["lazy_last"] for s in st]),
                    arr([s["lazy_hist"] for s in st]), self.hist_cap, n, float(beta1), float(beta2),
                    float(group["eps"]), float(group["weight_decay"]),
                    torch.cuda.current_stream(chunk[0].device).cuda_stream), "fr_adam_flush_rows")

    def load_state_dict(self, state_dict):
        """torch's loader casts every non-``step`` state tensor to the parameter's dtype and leaves
        ``step`` where the file put it.  The per-row lazy bookkeeping is dropped (``state_dict()``
        flushed it: every row was current), moments and bf16 masters are kept in fp32 and ``step``
        becomes the device int64 counter the kernels read."""
        slim = {"param_groups": state_dict["param_groups"], "state": {}}
        keep = {}
        for k, st in state_dict["state"].items():
            slim["state"][k] = {n: v for n, v in st.items() if n not in ("lazy_last", "lazy_hist")}
            keep[k] = {n: v for n, v in st.items()
                       if n in ("exp_avg", "exp_avg_sq", "master") and torch.is_tensor(v)}
        super().load_state_dict(slim)
        for g_sd, group in zip(state_dict["param_groups"], self.param_groups):
            for idx, p in zip(g_sd["params"], group["params"]):
                st = self.state.get(p)
                if not st:
                    continue
                if "step" in st:
                    st["step"] = torch.as_tensor(st["step"]).to(device=p.device, dtype=torch.int64).reshape(())
                for n, v in keep.get(idx, {}).items():
                    st[n] = v.to(device=p.device, dtype=torch.float32).contiguous()
        self._d_lr.clear()
        self._lazy_pending = 0
        self._lazy_launched = False

    def note_replay(self):
        """A captured step containing a lazy row update was replayed: count it, and flush before
        the per-step history ring (hist_cap steps) could wrap."""
        if self._lazy_launched:
            self._lazy_pending += 1
            if self._lazy_pending >= self.hist_cap - 2:
                self.flush()

    def reserve_replays(self, n: int):
        """``n`` captured lazy steps are about to run in one replay (an unrolled graph) before
        note_replay sees them: flush first when they would carry the pending count past the ring's
        bound (hist_cap - 2), so no row ever replays from an overwritten history slot."""
        if int(n) > self.hist_cap - 2:
            raise ValueError(f"{n} steps per replay exceed the lazy history ring (hist_cap {self.hist_cap})")
        if self._lazy_launched and self._lazy_pending + int(n) > self.hist_cap - 2:
            self.flush()

    def state_dict(self):
        self.flush()
        return super().state_dict()

    def zero_grad(self, set_to_none: bool = True):
        super().zero_grad(set_to_none=set_to_none)
        self.row_grads.clear()

    @torch.no_grad()
    def materialize_row_grads(self):
        """Turn pending row gradients into dense ``.grad`` tensors (accumulating), for callers that
        read or clip gradients between backward and step."""
        from . import ops
        for w, pad, ids, dY, W in list(self.row_grads.factored.values()):
            self.row_grads.stash(w, pad, ids, dY @ W)
        self.row_grads.factored.clear()
        for w, pad, ids, G in list(self.row_grads.pending.values()):
            ids, G, pad = self.row_grads.take(w)
            dense = ops.scatter_rows(ids.reshape(-1), G.reshape(-1, w.shape[-1]), w.shape[0], pad)
            w.grad = dense if w.grad is None else w.grad.add_(dense)

    def _ticket(self, device) -> int:
        """This optimiser's arrival words for the device-scalar launches (fr_adam_step_dev's d_ticket):
        its own, so two optimisers stepping concurrently never share them."""
        tk = self.__dict__.setdefault("_tickets", {})
        t = tk.get(device)
        if t is None:
            t = tk[device] = torch.zeros(32, dtype=torch.int32, device=device)  # FR_ADAM_TICKET_WORDS
        return t.data_ptr()

    def _lr_tensor(self, gi, group, device):
        """The group's device lr scalar and whether this call wrote it (on the current stream)."""
        t, held = self._d_lr.get(gi, (None, None))
        if t is None:
            t = torch.full((), float(group["lr"]), dtype=torch.float64, device=device)
            self._d_lr[gi] = (t, float(group["lr"]))
            return t, True
        if held != float(group["lr"]):
            t.fill_(float(group["lr"]))
            self._d_lr[gi] = (t, float(group["lr"]))
            return t, True
        return t, False

    def _ticket_created(self, device) -> bool:
        """Create the ticket words for ``device`` now (on the current stream); True if created."""
        new = device not in self.__dict__.get("_tickets", {})
        self._ticket(device)
        return new

    @torch.no_grad()
    def sync_lr(self):
        """Push every group's current lr to its device copy (call after an LR-scheduler step when
        the optimiser step itself is replayed from a captured graph)."""
        for gi, group in enumerate(self.param_groups):
            if gi in self._d_lr:
                t, _ = self._d_lr[gi]
                t.fill_(float(group["lr"]))
                self._d_lr[gi] = (t, float(group["lr"]))

    @torch.no_grad()
    def step(self, closure=None, skip_flag: torch.Tensor | None = None, part: str = "all"):
        """One Adam update.  ``skip_flag`` (device int32 scalar): when non-zero on the device the
        kernels leave every tensor (and step counter) untouched — the trainer's NaN guard
        without a host synchronisation.  ``part``: "rows" updates only the tables with pending row
        gradients, "dense" only the others (a data-parallel step runs the row update while the
        dense gradients are still being all-reduced)."""
        if part not in ("all", "rows", "dense"):
            raise ValueError(f"part must be all, rows or dense (got {part!r})")
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = native.lib()
        self.row_grads.join_background()
        from . import ops
        # tables whose gradient still waits for rows a late-mode backward left (ops.late_drain): the
        # other tensors' update is launched first, then the rows are added (beside it, on the branch
        # stream), then these tables' update
        late = ops.pending_drain_params() if part != "rows" else set()
        if late and any(p.grad is None for group in self.param_groups for p in group["params"] if id(p) in late):
            ops.run_pending_drains()  # (a table whose whole gradient is the rows: added before collecting)
            late = set()
        late_plans = []
        # factored row gradients read the projection weights: materialise them before any update.
        # A full step runs them, and then the row tables' update, on a side stream that forks where
        # the backward wrote dY (the projection backward, before the encoder backward): both leave
        # the tail of the step and overlap the encoder backward and the dense update
        side = self._rows_side() if (part == "all" and self.row_grads.factored) else None
        w_read = None
        if side is not None:
            side.wait_event(self.row_grads.factored_event)
            if self.row_grads._side is not None:  # the background slice replay (lazy state) first
                side.wait_stream(self.row_grads._side)
            for w, _, ids, dY, W in self.row_grads.factored.values():
                ids.record_stream(side)
                dY.record_stream(side)
            with torch.cuda.stream(side):
                prepared = self._prepare_factored(lib)
                w_read = torch.cuda.Event()
                w_read.record(side)
        else:
            prepared = self._prepare_factored(lib) if (self.row_grads.factored and part != "dense") else {}
        # pass 1, on the current stream: collect the tensors and create any state the launches read.
        # When the row tables' update runs on the side stream, everything this pass writes on the
        # current stream (zero-filled moments / step counters / lazy bookkeeping on a first step, the
        # lr scalar, the ticket words, rows stashed after the fork event) must be ordered before it:
        # ``dirty`` makes the side stream wait for the current one before the row launches
        main = torch.cuda.current_stream(side.device) if side is not None else None
        dirty = False
        plans = []
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            plist, rows = [], []
            for p in group["params"]:
                if id(p) in prepared:
                    rows.append((p, prepared.pop(id(p))))
                    dirty |= self._init_state(p)
                    continue
                if part == "dense" and (id(p) in self.row_grads.pending or id(p) in self.row_grads.factored):
                    continue
                rg = self.row_grads.take(p) if (self.row_grads.pending and part != "dense") else None
                if part == "rows" and rg is None:
                    continue
                if rg is not None and (p.grad is not None or not _row_grad_ok(p, rg[0], rg[1])):
                    from . import ops  # dense fallback: scatter the rows into (or onto) .grad
                    dense = ops.scatter_rows(rg[0].reshape(-1), rg[1].reshape(-1, p.shape[-1]), p.shape[0], rg[2])
                    p.grad = dense if p.grad is None else p.grad.add_(dense)
                    rg = None
                if p.grad is None and rg is None:
                    continue
                if p.grad is not None and p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                native.require_device(p)
                if not p.is_contiguous():
                    raise RuntimeError("FusedAdam needs contiguous parameters")
                created = self._init_state(p)
                st = self.state[p]
                if not created and (st["step"].device != p.device or st["step"].dtype != torch.int64):
                    st["step"] = st["step"].to(device=p.device, dtype=torch.int64)
                if p.dtype == torch.bfloat16:
                    self._step_bf16(p, group, lib, skip_flag, gi)
                    continue
                if p.dtype != torch.float32:
                    raise RuntimeError(f"FusedAdam supports fp32 and bf16 parameters (got {p.dtype})")
                if rg is not None:
                    rows.append((p, rg))
                    dirty = True  # its rows were written by the backward, possibly after the fork event
                    dirty |= created
                else:
                    plist.append(p)
            if not plist and not rows:
                continue
            dev = (plist or [rows[0][0]])[0].device
            d_lr, lr_written = self._lr_tensor(gi, group, dev)
            dirty |= lr_written
            if rows:
                dirty |= self._ticket_created(dev)
                if self.lazy_rows:
                    for p, _ in rows:
                        dirty |= self._init_lazy(p)
            hyper = (d_lr.data_ptr(), float(group["lr"]), float(beta1), float(beta2), float(group["eps"]),
                     float(group["weight_decay"]), native.ptr(skip_flag), torch.cuda.current_stream(dev).cuda_stream)
            plans.append((group, plist, rows, hyper))
        if side is not None and dirty:
            side.wait_stream(main)
        # pass 2: the launches.  ``before_dense``: everything pass 1 wrote on the current stream, before
        # the first update launch (a held table's update on the branch stream waits for it, not for them)
        before_dense = None
        if late and HELD_ON_BRANCH:
            before_dense = torch.cuda.Event()
            before_dense.record()
        for group, plist, rows, hyper in plans:
            lazy_dense = [p for p in plist if "lazy_last" in self.state[p]]
            # a lazily updated table taking a dense step (a dense .grad: more ids than the row path
            # takes, a gradient hook, clipping): its deferred steps are replayed first and its rows
            # are marked current through the new step afterwards, so no later replay reads a history
            # slot this step never wrote
            self._flush_tables(group, lazy_dense)
            if late:
                # a late table waits for its deferred gradient rows (ops.run_pending_drains below),
                # also when it is a lazily updated table taking a dense step
                held = [p for p in plist if id(p) in late]
                if held:
                    # the branch stream's update of a held table must also follow its backlog flush
                    # (_flush_tables above, on the current stream after ``before_dense``): such a
                    # table's plan waits for an event recorded behind that flush instead
                    ready = before_dense
                    if before_dense is not None and any(id(p) in {id(q) for q in lazy_dense} for p in held):
                        ready = torch.cuda.Event()
                        ready.record()
                    late_plans.append((held, hyper, ready))
                    plist = [p for p in plist if id(p) not in late]
            if plist:
                if w_read is not None:
                    torch.cuda.current_stream(plist[0].device).wait_event(w_read)  # (long done: forked early)
                with profiling.region("adam", 28 * sum(p.numel() for p in plist)):
                    self._launch_dense(lib, plist, hyper)
            self._mark_current([p for p in lazy_dense if id(p) not in late])
            if rows:
                if side is not None:
                    with torch.cuda.stream(side):
                        self._launch_rows(lib, rows, hyper[:-1] + (side.cuda_stream,))
                else:
                    self._launch_rows(lib, rows, hyper)
        def launch_held(stream=None):
            for held, hyper, ready in late_plans:
                if stream is not None:
                    stream.wait_event(ready)
                    hyper = hyper[:-1] + (stream.cuda_stream,)
                with profiling.region("adam", 28 * sum(p.numel() for p in held)):
                    self._launch_dense(lib, held, hyper)
                self._mark_current([p for p in held if "lazy_last" in self.state[p]])

        if late or ops.pending_drain_params():
            if late_plans and before_dense is not None:
                # the held tables' update right behind their rows' scatter on the branch stream: no
                # cross-queue hop between the scatter and the update; the current stream joins after
                ops.run_pending_drains(after=launch_held)
                late_plans = []
            else:
                ops.run_pending_drains()
        launch_held()
        if side is not None:
            torch.cuda.current_stream(side.device).wait_stream(side)
        return loss

    def _mark_current(self, ps):
        """Lazily updated tables that just took a dense step: every row is current through it."""
        for p in ps:
            st = self.state[p]
            st["lazy_last"].copy_(st["step"].to(torch.int32).expand(p.shape[0]))

    def _init_state(self, p) -> bool:
        """Create ``p``'s Adam state (on the current stream) if it has none; True if created."""
        st = self.state[p]
        if len(st):
            return False
        st["step"] = torch.zeros((), dtype=torch.int64, device=p.device)
        # fp32 moments (and, for bf16 parameters, an fp32 master copy: config 5)
        st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.preserve_format)
        st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.preserve_format)
        if p.dtype == torch.bfloat16:
            st["master"] = p.detach().float()
        return True

    def _init_lazy(self, p) -> bool:
        """The lazy-row bookkeeping of a row table (on the current stream); True if created."""
        st = self.state[p]
        if "lazy_last" in st:
            return False
        # every row is current through the table's present step (0, or the dense steps so far)
        st["lazy_last"] = st["step"].to(torch.int32).expand(p.shape[0]).contiguous()
        # per step: neg_step, bc2_sqrt (fp32) and RN64(1 / bc2_sqrt) (a double in floats 2-3)
        st["lazy_hist"] = torch.zeros(self.hist_cap, 4, dtype=torch.float32, device=p.device)
        return True

    def _rows_side(self):
        """The stream of the row tables' part of a full step (None: not on a GPU, or no fork point)."""
        ev = self.row_grads.factored_event
        if ev is None or not ROWS_SIDE_STREAM:
            return None
        dev = next(iter(self.row_grads.factored.values()))[3].device
        if dev.type != "cuda":
            return None
        if getattr(self, "_rows_stream", None) is None or self._rows_stream.device != dev:
            from . import ops
            self._rows_stream = ops.new_stream(dev, "rows")
        return self._rows_stream

    def _arrays(self, plist, grads):
        n = len(plist)
        P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in plist])
        G = (ctypes.c_void_p * n)(*[g.data_ptr() for g in grads])
        M = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg"].data_ptr() for p in plist])
        V = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg_sq"].data_ptr() for p in plist])
        S = (ctypes.c_void_p * n)(*[self.state[p]["step"].data_ptr() for p in plist])
        N = (ctypes.c_int64 * n)(*[p.numel() for p in plist])
        return P, G, M, V, S, N

    def _launch_dense(self, lib, plist, hyper):
        grads = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in plist]
        P, G, M, V, S, N = self._arrays(plist, grads)
        native.check(lib.fr_adam_step_dev(P, G, M, V, S, N, len(plist), *hyper[:-1], self._ticket(plist[0].device),
                                          hyper[-1]), "fr_adam_step_dev")

    def _prepare_factored(self, lib) -> dict:
        """Compact rows + row map of every factored entry: one fr_embedding_rowgrad over the entries'
        dY rows (entries with the same ids whose dY views are adjacent columns of one buffer share it),
        then rows = (per-id sum of dY) W by fr_rows_matmul.  Entries that cannot take the row path
        (a dense gradient already present, an unsupported table) become dense gradients."""
        from . import ops
        groups = {}
        for key, (w, pad, ids, dY, W) in list(self.row_grads.factored.items()):
            if w.grad is not None or not _row_grad_ok(w, ids, w) or dY.stride(1) != 1 or w.shape[1] != W.shape[1]:
                dense = ops.scatter_rows(ids.reshape(-1), dY @ W, w.shape[0], pad)
                w.grad = dense if w.grad is None else w.grad.add_(dense)
                continue
            groups.setdefault((id(ids), w.shape[0], pad, dY.stride(0)), []).append((w, ids, dY, W))
        self.row_grads.factored.clear()
        out = {}
        for (_, R, pad, ld), ents in groups.items():
            ents.sort(key=lambda e: e[2].data_ptr())
            base = ents[0][2]
            adjacent = all(e[2].data_ptr() == base.data_ptr() + 4 * 64 * k for k, e in enumerate(ents))
            width = 64 * len(ents)
            if not (adjacent and width & (width - 1) == 0 and ld >= width):
                for e in ents:  # one row pass per table
                    out.update(self._factored_rows(lib, [e], e[2], 64, R, pad))
                continue
            out.update(self._factored_rows(lib, ents, base, width, R, pad))
        return out

    def _factored_rows(self, lib, ents, G, width, R, pad):
        from . import ops
        rmap, crows = ops.factored_rows(ents[0][1], G, width, R, pad, [e[3] for e in ents])
        ids = ents[0][1].reshape(-1)
        return {id(e[0]): ("prepared", rmap, c, ids) for e, c in zip(ents, crows)}

    def _launch_rows(self, lib, rows, hyper):
        plist, compact, maps, dims, idl = [], [], [], [], []
        for p, entry in rows:
            if entry[0] == "prepared":
                plist.append(p)
                compact.append(entry[2])
                maps.append(entry[1])
                dims.append(p.shape[1])
                idl.append(entry[3])
                continue
            ids, G, pad = entry
            R, d = p.shape
            ids = ids.reshape(-1)
            G = G.reshape(-1, d)
            if G.stride(1) != 1 or G.stride(0) % 4 or G.data_ptr() % 16:
                G = G.contiguous()
            rmap = torch.empty(R, dtype=torch.int32, device=p.device)
            crow = torch.empty(max(ids.numel(), 1), d, dtype=torch.float32, device=p.device)
            ws = native.workspace(lib.fr_embedding_rowgrad_workspace(ids.numel(), R, d), p.device)
            with profiling.region("embedding_rowgrad", 4 * R + 8 * ids.numel() + 8 * G.numel()):
                native.check(lib.fr_embedding_rowgrad(ids.data_ptr(), ids.numel(), G.data_ptr(), G.stride(0), d, R,
                                                      -1 if pad is None else int(pad), rmap.data_ptr(),
                                                      crow.data_ptr(), ws.data_ptr(), ws.numel(),
                                                      native.stream_of(p)), "fr_embedding_rowgrad")
            plist.append(p)
            compact.append(crow)
            maps.append(rmap)
            dims.append(d)
            idl.append(ids if ids.dtype == torch.int64 else ids.to(torch.int64))
        P, G, M, V, S, N = self._arrays(plist, compact)
        n = len(plist)
        RM = (ctypes.c_void_p * n)(*[m.data_ptr() for m in maps])
        RD = (ctypes.c_int32 * n)(*dims)
        if self.lazy_rows:
            for p in plist:
                self._init_lazy(p)  # (created in step()'s first pass; kept for direct callers)
            idl = [i if i.is_contiguous() else i.contiguous() for i in idl]
            for k in range(0, n, 16):  # the kernel's argument block takes 16 tables per launch
                m = min(16, n - k)
                sl = slice(k, k + m)
                arr = lambda xs: (ctypes.c_void_p * m)(*[x.data_ptr() for x in xs])  # noqa: E731
                sts = [self.state[p] for p in plist[sl]]
                LA, LH = arr([s_["lazy_last"] for s_ in sts]), arr([s_["lazy_hist"] for s_ in sts])
                ID = arr(idl[sl])
                NI = (ctypes.c_int64 * m)(*[i.numel() for i in idl[sl]])
                # algorithmic bytes: p, m, v of the touched rows (bounded by the compact rows' count)
                # read and written, the compact gradient rows read, the ids / map / last-step entries
                with profiling.region("adam_rows", sum(28 * c.numel() + 16 * i.numel()
                                                       for c, i in zip(compact[sl], idl[sl]))):
                    native.check(lib.fr_adam_step_rows_lazy(
                        arr(plist[sl]), arr(compact[sl]), arr([s_["exp_avg"] for s_ in sts]),
                        arr([s_["exp_avg_sq"] for s_ in sts]), arr([s_["step"] for s_ in sts]),
                        (ctypes.c_int64 * m)(*[p.numel() for p in plist[sl]]), arr(maps[sl]), ID, NI,
                        (ctypes.c_int32 * m)(*dims[sl]), LA, LH, self.hist_cap, m, *hyper), "fr_adam_step_rows_lazy")
            self._lazy_launched = True
            if not torch.cuda.is_current_stream_capturing():
                self._lazy_pending += 1
                if self._lazy_pending >= self.hist_cap - 2:
                    self.flush()
            return
        with profiling.region("adam_rows", sum(adam_rows_bytes(p.numel(), p.shape[0], c.numel())
                                              for p, c in zip(plist, compact))):
            native.check(lib.fr_adam_step_rows(P, G, M, V, S, N, RM, RD, n, *hyper[:-1], self._ticket(plist[0].device),
                                               hyper[-1]), "fr_adam_step_rows")

    def _step_bf16(self, p, group, lib, skip_flag, gi):
        """bf16 parameter: update the fp32 master with fp32 moments, re-round the parameter."""
        st = self.state[p]
        g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
        if g.dtype != torch.bfloat16:
            raise RuntimeError("a bf16 parameter needs a bf16 gradient")
        beta1, beta2 = group["betas"]
        d_lr, _ = self._lr_tensor(gi, group, p.device)
        with profiling.region("adam", 30 * p.numel()):
            native.check(lib.fr_adam_step_bf16(
                p.data_ptr(), st["master"].data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                st["exp_avg_sq"].data_ptr(), st["step"].data_ptr(), p.numel(), d_lr.data_ptr(),
                float(group["lr"]), float(beta1), float(beta2), float(group["eps"]),
                float(group["weight_decay"]), native.ptr(skip_flag), native.stream_of(p)), "fr_adam_step_bf16")
