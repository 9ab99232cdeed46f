"""RCCL communicator through the engine's C-ABI (fr_comm_*, include/fr_engine.h).

One communicator per process and GPU.  ``RcclComm.from_process_group()`` draws the 128-byte RCCL id
on rank 0 and hands it to the other ranks over an existing torch.distributed group (any backend;
only the id travels there), then every rank joins with ``fr_comm_init``.  Collectives are issued on
the caller's current HIP stream, or -- ``async_op=True`` -- on the communicator's own stream after
the current one, returning a handle whose ``wait()`` orders the current stream after the collective
(so the caller overlaps it with independent kernels: the sharded step's user SpMM).  Both forms are
graph-capturable (no host synchronisation).

This is the exchange layer of engine/sharded.py for a process that wants RCCL without torch's
ProcessGroup bookkeeping (``ShardedLightGCN(group=RcclComm...)``); torch.distributed with backend
"nccl" (= RCCL) remains the default group type there and in engine/dist.py.
"""
from __future__ import annotations

import ctypes

import torch

from . import native


class _Pending:
    def __init__(self, stream, comm_stream):
        self.stream, self.comm_stream = stream, comm_stream

    def wait(self):
        self.stream.wait_stream(self.comm_stream)


class RcclComm:
    def __init__(self, rank: int, world: int, unique_id: bytes, device=None):
        lib = native.lib()
        if not lib.fr_comm_available():
            raise native.EngineError("RCCL is not available to the engine library")
        nbytes = int(lib.fr_comm_unique_id_bytes())
        if len(unique_id) != nbytes:
            raise ValueError(f"RCCL unique id must be {nbytes} bytes")
        self.rank, self.world = int(rank), int(world)
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        buf = ctypes.create_string_buffer(bytes(unique_id), nbytes)
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            native.check(lib.fr_comm_init(self.rank, self.world, buf, ctypes.byref(h)), "fr_comm_init")
        self._h = h
        self._stream = None

    @staticmethod
    def unique_id() -> bytes:
        lib = native.lib()
        n = int(lib.fr_comm_unique_id_bytes())
        buf = ctypes.create_string_buffer(n)
        native.check(lib.fr_comm_unique_id(buf, n), "fr_comm_unique_id")
        return buf.raw

    @classmethod
    def from_process_group(cls, group=None):
        import torch.distributed as dist
        rank, world = dist.get_rank(group), dist.get_world_size(group)
        box = [cls.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(box, src=dist.get_global_rank(group, 0) if group is not None else 0, group=group)
        return cls(rank, world, box[0])

    def _comm_stream(self):
        if self._stream is None:
            self._stream = torch.cuda.Stream(self.device)
        return self._stream

    def _run(self, fn, tensors, async_op):
        cur = torch.cuda.current_stream(self.device)
        if not async_op:
            fn(cur.cuda_stream)
            return None
        side = self._comm_stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            fn(side.cuda_stream)
        for t in tensors:
            t.record_stream(side)
        return _Pending(cur, side)

    def all_reduce(self, t: torch.Tensor, async_op: bool = False):
        """In-place float32 sum over the ranks."""
        if t.dtype != torch.float32 or not t.is_contiguous() or not t.is_cuda:
            raise native.EngineError("all_reduce needs a contiguous float32 device tensor")
        lib = native.lib()
        return self._run(lambda s: native.check(lib.fr_allreduce_f32(self._h, t.data_ptr(), t.numel(), s),
                                                "fr_allreduce_f32"), [t], async_op)

    def all_gather(self, recv: torch.Tensor, send: torch.Tensor, async_op: bool = False):
        """recv [world, n] = every rank's send [n] (float32, contiguous)."""
        if send.dtype != torch.float32 or recv.dtype != torch.float32 or not (send.is_contiguous() and recv.is_contiguous()):
            raise native.EngineError("all_gather needs contiguous float32 device tensors")
        if recv.numel() != self.world * send.numel():
            raise ValueError("recv must hold world x send elements")
        lib = native.lib()
        return self._run(lambda s: native.check(lib.fr_allgather_f32(self._h, send.data_ptr(), recv.data_ptr(),
                                                                     send.numel(), s), "fr_allgather_f32"),
                         [send, recv], async_op)

    def close(self):
        if self._h is not None and self._h.value:
            native.check(native.lib().fr_comm_destroy(self._h), "fr_comm_destroy")
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
