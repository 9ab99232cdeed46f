"""Multi-GPU: one process per GPU, torch.distributed over RCCL (backend "nccl") on xGMI.

Round-1 scheme: data-parallel replicas.  Each rank trains on its own triple batch; after the
backward pass the dense gradient buffer (every parameter that received a gradient, packed into
one fp32 buffer) is all-reduced once per step and averaged, then every rank applies the same
fused Adam update, so the replicas stay bit-identical.  (The row-sharded graph scheme of SURVEY
8(e) is for the 10M-user synthetic graph; at Allrecipes shape the graph is replicated.)
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


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
            dist.init_process_group(backend, device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
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
        # optional FusedAdam.row_grads: apply() hands it the gathered mean rows (fr_adam_step_rows)
        # instead of scattering a dense table gradient
        self.sink = None

    def catch_up_rows(self, weight, ids):
        """Before this rank gathers ``ids``: the sink's lazily updating optimiser brings the rows up
        to date (rows other ranks touch are replayed inside their own row update)."""
        if self.sink is not None:
            self.sink.catch_up_rows(weight, ids)

    def stash(self, weight, padding_idx, ids, G, W=None):
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
        s["ids"].copy_(ids)
        s["G"].copy_(G)

    def stash_factored(self, weight, padding_idx, ids, dY, W):
        """Gradient rows dY[i] W of a gathered Linear input (ops.modal_projection): only the 64-wide
        dY rows and the ids cross the interconnect; W is replicated on every rank."""
        self.stash(weight, padding_idx, ids, dY, W)

    def _pack(self):
        """One float32 send buffer [ids(int64 as 2 words) | rows] per slot, and the matching
        [world, total] receive buffer; slot tensors become views of them."""
        layout, total = [], 0
        for s in self.slots.values():
            ni, ng = 2 * s["ids"].numel(), s["G"].numel()
            ng += ng % 2  # keep every region 8-byte aligned
            layout.append((s, total, ni, ng))
            total += ni + ng
        dev = next(iter(self.slots.values()))["G"].device
        send = torch.empty(total, dtype=torch.float32, device=dev)
        recv = torch.empty(self.world, total, dtype=torch.float32, device=dev)
        for s, off, ni, ng in layout:
            ids_v = send[off:off + ni].view(torch.int64).view(s["ids"].shape)
            ids_v.copy_(s["ids"])
            g_v = send[off + ni:off + ni + s["G"].numel()].view(s["G"].shape)
            g_v.copy_(s["G"])
            s["ids"], s["G"] = ids_v, g_v
            s["ids_all"] = recv[:, off:off + ni].view(torch.int64)  # [world, n]
            s["G_all"] = recv[:, off + ni:off + ni + s["G"].numel()]  # [world, n * d]
        self._send, self._recv = send, recv

    def exchange(self):
        import torch.distributed as dist
        if self._send is None:
            self._pack()
        # one collective for every table (views of these static buffers are what graph B reads)
        dist.all_gather(list(self._recv.unbind(0)), self._send, group=self.group)

    def apply(self):
        from . import ops
        for s in self.slots.values():
            w = s["weight"]
            d = s["G"].shape[-1]
            rows = s["G_all"].reshape(-1, d) * (1.0 / self.world)
            ids = s["ids_all"].reshape(-1).contiguous()
            if s["W"] is not None:  # factored: rows are dY, the table gradient rows are dY W
                if self.sink is not None:
                    self.sink.stash_factored(w, s["pad"], ids, rows, s["W"])
                else:
                    w.grad = ops.scatter_rows(ids, rows @ s["W"], w.shape[0], s["pad"])
            elif self.sink is not None:
                self.sink.stash(w, s["pad"], ids, rows)
            else:
                w.grad = ops.scatter_rows(ids, rows, w.shape[0], s["pad"])


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
        self.layout = None
        self.views = []

    def pack(self):
        live = [p for p in self.params if p.grad is not None]
        if self.flat is None or self.layout != [id(p) for p in live]:
            total = sum(p.numel() for p in live)
            self.flat = torch.empty(total, dtype=torch.float32, device=live[0].grad.device)
            self.layout = [id(p) for p in live]
        off = 0
        self.views = []
        for p in live:
            n = p.numel()
            v = self.flat[off:off + n]
            v.copy_(p.grad.reshape(-1))
            self.views.append((p, v))
            off += n

    def communicate(self):
        self.communicate_rows()
        self.communicate_dense()

    def communicate_rows(self):
        if self.rows is not None:
            self.rows.exchange()

    def communicate_dense(self, async_op: bool = False):
        """The flat all-reduce; with ``async_op`` the returned work's ``wait()`` orders the current
        stream after it, so work enqueued in between (the row-table Adam update) overlaps it."""
        return dist.all_reduce(self.flat, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)

    def unpack(self):
        self.unpack_dense()
        self.unpack_rows()

    def unpack_dense(self):
        self.flat.mul_(1.0 / self.world)
        for p, v in self.views:
            p.grad.copy_(v.view_as(p.grad))

    def unpack_rows(self):
        if self.rows is not None:
            self.rows.apply()

    def __call__(self, model):
        self.pack()
        self.communicate()
        self.unpack()
