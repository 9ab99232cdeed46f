"""Fused multi-tensor Adam on the HIP kernels ``fr_adam_step_dev`` / ``fr_adam_step``.

Drop-in for ``torch.optim.Adam`` as the reference trainer builds it (common/trainer.py:143-144):
same param_groups and per-parameter state keys (``step``, ``exp_avg``, ``exp_avg_sq``), so
``state_dict()`` round-trips.  Parameters whose ``.grad`` is None are skipped, as in torch.

The step counters and the learning rate live in device memory (like torch's capturable Adam): the
kernel increments each tensor's counter and derives the bias corrections on the device, so a
whole training step (forward, backward, optimiser) can be captured in a HIP graph and replayed.
After changing ``group['lr']`` outside of step() (LR scheduler), call :meth:`sync_lr`.
"""
from __future__ import annotations

import ctypes

import torch

from . import native, profiling


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        if lr < 0.0 or eps < 0.0 or not (0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0):
            raise ValueError("invalid Adam hyper-parameters")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay,
                                      amsgrad=False, maximize=False))
        self._d_lr = {}   # group index -> (device float64 lr, host value it holds)

    def _lr_tensor(self, gi, group, device):
        t, held = self._d_lr.get(gi, (None, None))
        if t is None:
            t = torch.full((), float(group["lr"]), dtype=torch.float64, device=device)
            self._d_lr[gi] = (t, float(group["lr"]))
        elif held != float(group["lr"]):
            t.fill_(float(group["lr"]))
            self._d_lr[gi] = (t, float(group["lr"]))
        return t

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
    def step(self, closure=None, skip_flag: torch.Tensor | None = None):
        """One Adam update.  ``skip_flag`` (device int32 scalar): when non-zero on the device the
        kernels leave every tensor (and step counter) untouched — the trainer's NaN guard
        without a host synchronisation."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = native.lib()
        for gi, group in enumerate(self.param_groups):
            beta1, beta2 = group["betas"]
            plist = []
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                native.require_device(p)
                if not p.is_contiguous():
                    raise RuntimeError("FusedAdam needs contiguous parameters")
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.zeros((), dtype=torch.int64, device=p.device)
                    # fp32 moments (and, for bf16 parameters, an fp32 master copy: config 5)
                    st["exp_avg"] = torch.zeros_like(p, dtype=torch.float32, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, dtype=torch.float32,
                                                        memory_format=torch.preserve_format)
                    if p.dtype == torch.bfloat16:
                        st["master"] = p.detach().float()
                elif st["step"].device != p.device or st["step"].dtype != torch.int64:
                    st["step"] = st["step"].to(device=p.device, dtype=torch.int64)
                if p.dtype == torch.bfloat16:
                    self._step_bf16(p, group, lib, skip_flag, gi)
                    continue
                if p.dtype != torch.float32:
                    raise RuntimeError(f"FusedAdam supports fp32 and bf16 parameters (got {p.dtype})")
                plist.append(p)
            if not plist:
                continue
            grads = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in plist]
            n = len(plist)
            P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in plist])
            G = (ctypes.c_void_p * n)(*[g.data_ptr() for g in grads])
            M = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg"].data_ptr() for p in plist])
            V = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg_sq"].data_ptr() for p in plist])
            S = (ctypes.c_void_p * n)(*[self.state[p]["step"].data_ptr() for p in plist])
            N = (ctypes.c_int64 * n)(*[p.numel() for p in plist])
            d_lr = self._lr_tensor(gi, group, plist[0].device)
            with profiling.region("adam", 28 * sum(p.numel() for p in plist)):
                native.check(lib.fr_adam_step_dev(
                    P, G, M, V, S, N, n, d_lr.data_ptr(), float(group["lr"]), float(beta1), float(beta2),
                    float(group["eps"]), float(group["weight_decay"]), native.ptr(skip_flag),
                    native.stream_of(plist[0])), "fr_adam_step_dev")
        return loss

    def _step_bf16(self, p, group, lib, skip_flag, gi):
        """bf16 parameter: update the fp32 master with fp32 moments, re-round the parameter."""
        st = self.state[p]
        g = p.grad if p.grad.is_contiguous() else p.grad.contiguous()
        if g.dtype != torch.bfloat16:
            raise RuntimeError("a bf16 parameter needs a bf16 gradient")
        beta1, beta2 = group["betas"]
        d_lr = self._lr_tensor(gi, group, p.device)
        with profiling.region("adam", 30 * p.numel()):
            native.check(lib.fr_adam_step_bf16(
                p.data_ptr(), st["master"].data_ptr(), g.data_ptr(), st["exp_avg"].data_ptr(),
                st["exp_avg_sq"].data_ptr(), st["step"].data_ptr(), p.numel(), d_lr.data_ptr(),
                float(group["lr"]), float(beta1), float(beta2), float(group["eps"]),
                float(group["weight_decay"]), native.ptr(skip_flag), native.stream_of(p)), "fr_adam_step_bf16")
