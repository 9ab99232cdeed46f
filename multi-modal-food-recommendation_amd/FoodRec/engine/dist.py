"""Multi-GPU: one process per GPU, torch.distributed over RCCL (backend "nccl") on xGMI.

Round-1 scheme: data-parallel replicas.  Each rank trains on its own triple batch; after the
backward pass the dense gradient buffer (every parameter that received a gradient, packed into
one fp32 buffer) is all-reduced once per step and averaged, then every rank applies the same
fused Adam update, so the replicas stay bit-identical.  (The row-sharded graph scheme of SURVEY
8(e) is for the 10M-user synthetic graph; at Allrecipes shape the graph is replicated.)
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def pg_timeout() -> datetime.timedelta:
    """Collective timeout of the engine's process groups: FR_PG_TIMEOUT_S seconds (default 300), so
    a collective that one rank never joins ends the job with an error instead of hanging until
    torch's default watchdog (10 minutes for RCCL, 30 for gloo)."""
    return datetime.timedelta(seconds=float(os.environ.get("FR_PG_TIMEOUT_S", "300")))


def init_process_group(backend, device=None, **kw):
    """torch.distributed.init_process_group with the engine's timeout; for RCCL ("nccl") also the
    asynchronous error handling that tears the process down when a collective times out or fails
    (TORCH_NCCL_ASYNC_ERROR_HANDLING, unless the caller's environment sets it)."""
    if backend == "nccl":
        os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
        if device is not None:
            kw["device_id"] = device
    dist.init_process_group(backend, timeout=pg_timeout(), **kw)


def init_from_env(backend=None):
    """Initialise the default process group from torchrun's env (RANK/WORLD_SIZE/LOCAL_RANK)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and not dist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
            init_process_group(backend, torch.device("cuda", local))
        else:
            init_process_group(backend)
    return rank, world, local


class RowExchange:
    """Data-parallel gradient of row-gathered tables, exchanged as rows.

    In backward, ``ops.embedding(..., exchange=self)`` (or ``ops.modal_projection``, whose rows are
    the 64-wide dY of the factored gradient) stashes its ids and gradient rows into static buffers
    (and gives the table no dense gradient); ``exchange()`` all-gathers every rank's stash -- all
    tables packed into one buffer, ONE collective, P x sum(n x (8 + 4d)) bytes; ``apply()`` sets
    each table's gradient to the deterministic scatter of the gathered rows / P (or hands them to
    FusedAdam's row gradients) -- identical on every rank and equal to the mean of the ranks' dense
    gradients."""

    def __init__(self, group, world):
        self.group, self.world = group, int(world)
        self.slots = {}  # id(weight) -> dict(weight, pad, ids, G, ids_all, G_all)
        # every slot's ids and rows packed into ONE send buffer (one all-gather per step); built at
        # the first exchange, after which the stashes write straight into their views of it
        self._send = self._recv = None
        self._groups = []
        self._ids_done = set()  # ids groups whose region this step's stashes already wrote
        self._comb = {}  # per ids group: [world * n, 64 * tables] scaled rows handed to the sink
        # optional FusedAdam.row_grads: apply() hands it the gathered mean rows (fr_adam_step_rows)
        # instead of scattering a dense table gradient
        self.sink = None

    def catch_up_rows(self, weight, ids):
        """Before this rank gathers ``ids``: the sink's lazily updating optimiser brings the rows up
        to date (rows other ranks touch are replayed inside their own row update)."""
        if self.sink is not None:
            self.sink.catch_up_rows(weight, ids)

    def prefetch_rows(self, pairs):
        """The sink's side-stream catch-up of this rank's batch rows (+ its background slice replay),
        overlapping the propagation as in the single-GPU step; returns the join callable."""
        if self.sink is not None and hasattr(self.sink, "prefetch_rows"):
            return self.sink.prefetch_rows(pairs)
        for w, ids in pairs:
            self.catch_up_rows(w, ids)
        return lambda stream=None: None  # caught up inline on the current stream

    def join_background(self):
        """Join the sink's background slice replay (the end of a graphed step's part A: a captured
        stream may not end with unjoined side-stream work)."""
        if self.sink is not None and hasattr(self.sink, "join_background"):
            self.sink.join_background()

    def stash(self, weight, padding_idx, ids, G, W=None):
        # tables stashed with the same ids tensor (HealthRec's image / text) share one ids region.
        # The key is the ids' memory, and the slot holds a reference to them until the exchange, so
        # no other ids tensor can occupy that memory meanwhile (a Python id() of a freed temporary
        # can be recycled within one backward)
        key = (ids.data_ptr(), tuple(ids.shape), ids.dtype)
        src = ids
        ids = ids.to(torch.int64)
        G = G.to(torch.float32)
        s = self.slots.get(id(weight))
        if s is None or s["ids"].shape != ids.shape or s["G"].shape != G.shape or s["W"] is not W:
            s = {"weight": weight, "pad": padding_idx, "ids": torch.empty_like(ids),
                 "G": torch.empty(G.shape, dtype=G.dtype, device=G.device), "W": W,
                 "ids_all": torch.empty((self.world,) + tuple(ids.shape), dtype=ids.dtype, device=ids.device),
                 "G_all": torch.empty((self.world,) + tuple(G.shape), dtype=G.dtype, device=G.device)}
            self.slots[id(weight)] = s
            self._send = self._recv = None  # layout changed: repack at the next exchange
        s["key"] = key
        s["ids_src"] = src
        if not (s.get("shared") and key in self._ids_done):  # a shared ids region is written once
            s["ids"].copy_(ids)
            self._ids_done.add(key)
        s["G"].copy_(G)

    def stash_factored(self, weight, padding_idx, ids, dY, W):
        """Gradient rows dY[i] W of a gathered Linear input (ops.modal_projection): only the 64-wide
        dY rows and the ids cross the interconnect; W is replicated on every rank."""
        self.stash(weight, padding_idx, ids, dY, W)

    def _pack(self):
        """One float32 send buffer [ids(int64 as 2 words) | rows ...] -- one ids region per group of
        slots stashed with the same ids tensor -- and the matching [world, total] receive buffer;
        slot tensors become views of them."""
        groups = {}
        for s in self.slots.values():
            groups.setdefault((s["key"], tuple(s["ids"].shape)), []).append(s)
        total = 0
        layout = []
        for slots in groups.values():
            ni = 2 * slots[0]["ids"].numel()
            regs = []
            off_g = total + ni
            for s in slots:
                ng = s["G"].numel()
                regs.append((s, off_g, ng))
                off_g += ng + ng % 2  # keep every region 8-byte aligned
            layout.append((slots, total, ni, regs))
            total = off_g
        dev = next(iter(self.slots.values()))["G"].device
        send = torch.empty(total, dtype=torch.float32, device=dev)
        recv = torch.empty(self.world, total, dtype=torch.float32, device=dev)
        for slots, off, ni, regs in layout:
            ids_v = send[off:off + ni].view(torch.int64).view(slots[0]["ids"].shape)
            ids_v.copy_(slots[0]["ids"])
            ids_all = recv[:, off:off + ni].view(torch.int64)  # [world, n]
            for s, og, ng in regs:
                g_v = send[og:og + ng].view(s["G"].shape)
                g_v.copy_(s["G"])
                s["ids"], s["G"], s["ids_all"] = ids_v, g_v, ids_all
                s["G_all"] = recv[:, og:og + ng]  # [world, n * d]
                s["shared"] = len(slots) > 1
        self._send, self._recv = send, recv
        self._groups = [slots for slots, _, _, _ in layout]

    def exchange(self):
        import torch.distributed as dist
        if self._send is not None and any(len(slots) > 1 and len({s["key"] for s in slots}) > 1
                                          for slots in self._groups):
            # tables packed as sharing ids were stashed with different ids this step: every slot
            # takes its own ids again and the buffers are repacked by this step's keys
            for s in self.slots.values():
                s["ids"] = s["ids_src"].to(torch.int64).clone()
                s["G"] = s["G"].clone()
            self._send = None
        if self._send is None:
            self._pack()
        self._ids_done.clear()
        for s in self.slots.values():
            s.pop("ids_src", None)
        # one collective for every table (views of these static buffers are what graph B reads)
        if dist.get_backend(self.group) == "nccl":
            dist.all_gather_into_tensor(self._recv, self._send, group=self.group)
        else:
            dist.all_gather(list(self._recv.unbind(0)), self._send, group=self.group)

    def apply(self):
        """The gathered rows, scaled by 1 / world, handed to the sink (or scattered).  Factored
        tables of one ids group go to the sink as adjacent 64-column views of one buffer with one
        ids tensor, so FusedAdam builds their row gradients in one pass (as on a single GPU)."""
        from . import ops
        inv = 1.0 / self.world
        for slots in self._groups:
            ids = slots[0]["ids_all"].reshape(-1).contiguous()
            fac = [s for s in slots if s["W"] is not None and s["G"].shape[-1] == 64] if self.sink is not None else []
            if len(fac) > 1:
                n = ids.numel()
                comb = self._comb.get(id(slots[0]["ids_all"]))
                if comb is None or comb.shape != (n, 64 * len(fac)):
                    comb = torch.empty(n, 64 * len(fac), dtype=torch.float32, device=ids.device)
                    self._comb[id(slots[0]["ids_all"])] = comb
                for t, s in enumerate(fac):
                    dst = comb[:, 64 * t:64 * (t + 1)]
                    torch.mul(s["G_all"].view(self.world, -1, 64), inv, out=dst.view(self.world, -1, 64))
                    self.sink.stash_factored(s["weight"], s["pad"], ids, dst, s["W"])
            for s in slots:
                if len(fac) > 1 and any(s is f for f in fac):
                    continue
                w = s["weight"]
                d = s["G"].shape[-1]
                rows = s["G_all"].reshape(-1, d) * inv
                if s["W"] is not None:  # factored: rows are dY, the table gradient rows are dY W
                    if self.sink is not None:
                        self.sink.stash_factored(w, s["pad"], ids, rows, s["W"])
                    else:
                        w.grad = ops.scatter_rows(ids, rows @ s["W"], w.shape[0], s["pad"])
                elif self.sink is not None:
                    self.sink.stash(w, s["pad"], ids, rows)
                else:
                    w.grad = ops.scatter_rows(ids, rows, w.shape[0], s["pad"])


def _shares(t, buf):
    return t.untyped_storage().data_ptr() == buf.untyped_storage().data_ptr()


class GradAllReduce:
    """Trainer.grad_hook: average gradients over ranks with ONE dense collective per step.

    Parameters a model lists in ``row_sparse_tables`` (tables whose only use on the step is a row
    gather through ``ops.embedding``) are exchanged as rows instead (``RowExchange``; the model's
    ``_fr_exchange`` is set here) and are left out of the dense buffer: for HealthRec that is the
    45,630 x 2048 image and 45,630 x 512 text tables, 466 MB of the 503 MB gradient.

    ``pack()`` (copy gradients into the flat buffer) and ``unpack()`` (average, copy back, apply the
    row exchange) are collective-free, so a graphed step captures them; ``communicate()`` issues the
    collectives eagerly between the two graphs (Trainer.GraphedDPStep)."""

    def __init__(self, model, world: int, group=None, exchange_rows: bool | None = None):
        import torch.distributed as dist
        self.world = int(world)
        self.group = group
        sparse = {id(p) for p in getattr(model, "row_sparse_tables", lambda: [])()}
        self.rows = None
        # exchange_rows: route the row tables through RowExchange (default: when there is more than
        # one rank; True at world 1 exercises the exchange on a single GPU)
        if sparse and (self.world > 1 if exchange_rows is None else exchange_rows):
            self.rows = RowExchange(group if group is not None else dist.group.WORLD, self.world)
            model._fr_exchange = self.rows
        else:
            sparse = set()
        self.params = [p for p in model.parameters() if p.requires_grad and id(p) not in sparse]
        self.flat = None
        self._avg_in_collective = False
        self.layout = None
        self.views = []

    def pack(self):
        """Every live gradient into the flat buffer: ONE batched-copy launch (torch.cat into the
        buffer), not one copy per parameter (78 copies, 0.37 ms/step at HealthRec's 39 tensors)."""
        if self.rows is not None:
            self.rows.join_background()
        live = [p for p in self.params if p.grad is not None]
        if self.flat is None or self.layout != [id(p) for p in live]:
            # every slot starts on a 256-B boundary (the optimiser's vector path needs 16-B aligned
            # gradients; the gaps are zero and stay zero through the sum)
            self.offs, total = [], 0
            for p in live:
                self.offs.append(total)
                total += -(-p.numel() // 64) * 64
            self.flat = torch.zeros(total, dtype=torch.float32, device=live[0].grad.device)
            self.layout = [id(p) for p in live]
            # the gradients land in views of the buffer: one batched copy (torch.cat into the
            # slot views when the slots are dense, else per-slot copies)
            self._dense = all(o == sum(q.numel() for q in live[:k]) for k, o in enumerate(self.offs))
            # backward kernels that know their gradient's destination (ops.grad_buffer) write straight
            # into the slot from the next step on
            for p, o in zip(live, self.offs):
                p.__dict__["_fr_grad_dest"] = self._slot_view(p, o)
        base = self.flat.data_ptr()
        todo = []
        for p, o in zip(live, self.offs):
            if p.grad.data_ptr() == base + 4 * o and p.grad.dtype == torch.float32:
                continue  # already in its slot
            if _shares(p.grad, self.flat):
                raise RuntimeError("GradAllReduce.pack: a gradient views the flat buffer outside its slot "
                                   "(zero_grad(set_to_none=False) after unpack?): use set_to_none=True")
            todo.append((p, o))
        if todo and self._dense and len(todo) == len(live):
            torch.cat([p.grad.reshape(-1).to(torch.float32) for p in live], out=self.flat[:sum(p.numel() for p in live)])
        elif todo:
            torch._foreach_copy_([self.flat[o:o + p.numel()] for p, o in todo],
                                 [p.grad.reshape(-1).to(torch.float32) for p, _ in todo])
        self.views = [(p, self.flat[o:o + p.numel()].view(p.shape)) for p, o in zip(live, self.offs)]

    def _slot_view(self, p, o):
        n, shape = p.numel(), p.shape
        return lambda: self.flat[o:o + n].view(shape) if self.flat is not None and self.flat.numel() >= o + n else None

    def communicate(self):
        self.communicate_rows()
        self.communicate_dense()

    def communicate_rows(self):
        if self.rows is not None:
            self.rows.exchange()

    def communicate_dense(self, async_op: bool = False):
        """The flat all-reduce; with ``async_op`` the returned work's ``wait()`` orders the current
        stream after it, so work enqueued in between (the row-table Adam update) overlaps it."""
        # RCCL averages inside the collective (ncclAvg); other backends sum and unpack scales
        self._avg_in_collective = self.world > 1 and dist.get_backend(self.group) == "nccl"
        op = dist.ReduceOp.AVG if self._avg_in_collective else dist.ReduceOp.SUM
        return dist.all_reduce(self.flat, op=op, group=self.group, async_op=async_op)

    def unpack(self):
        self.unpack_dense()
        self.unpack_rows()

    def unpack_dense(self):
        """Average in place; each parameter's gradient becomes its view of the flat buffer (no copy
        back: the optimiser reads the buffer)."""
        if self.world > 1 and not self._avg_in_collective:
            self.flat.mul_(1.0 / self.world)
        for p, v in self.views:
            if p.grad is not None and p.grad.dtype == torch.float32:
                p.grad = v
            elif p.grad is not None:
                p.grad.copy_(v)

    def unpack_rows(self):
        if self.rows is not None:
            self.rows.apply()

    def __call__(self, model):
        self.pack()
        self.communicate()
        self.unpack()
