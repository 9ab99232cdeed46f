"""Fused multi-tensor Adam on the HIP kernel ``fr_adam_step``.

Drop-in for ``torch.optim.Adam`` as the reference trainer builds it (common/trainer.py:143-144):
same param_groups, same per-parameter state keys (``step``, ``exp_avg``, ``exp_avg_sq``), so
``state_dict()`` round-trips with torch.  Parameters whose ``.grad`` is None are skipped, as in
torch.  One kernel launch per 24 tensors; the step count is a host integer (no device sync).
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

    @torch.no_grad()
    def step(self, closure=None, skip_flag: torch.Tensor | None = None):
        """One Adam update.  ``skip_flag`` (device int32 scalar): when non-zero on the device,
        the kernels leave every tensor untouched (used by the trainer's NaN guard without a
        host sync)."""
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = native.lib()
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            by_step: dict[int, list] = {}
            for p in group["params"]:
                if p.grad is None:
                    continue
                if p.grad.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                native.require_device(p)
                st = self.state[p]
                if len(st) == 0:
                    st["step"] = torch.tensor(0.0)
                    st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["step"] += 1
                by_step.setdefault(int(st["step"].item()), []).append(p)
            for step, plist in by_step.items():
                grads = [p.grad if p.grad.is_contiguous() else p.grad.contiguous() for p in plist]
                for p in plist:
                    if not p.is_contiguous():
                        raise RuntimeError("FusedAdam needs contiguous parameters")
                n = len(plist)
                P = (ctypes.c_void_p * n)(*[p.data_ptr() for p in plist])
                G = (ctypes.c_void_p * n)(*[g.data_ptr() for g in grads])
                M = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg"].data_ptr() for p in plist])
                V = (ctypes.c_void_p * n)(*[self.state[p]["exp_avg_sq"].data_ptr() for p in plist])
                N = (ctypes.c_int64 * n)(*[p.numel() for p in plist])
                with profiling.region("adam", 28 * sum(p.numel() for p in plist)):
                    native.check(lib.fr_adam_step(
                        P, G, M, V, N, n, max(p.numel() for p in plist), float(group["lr"]),
                        float(beta1), float(beta2), float(group["eps"]),
                        float(group["weight_decay"]), step, native.ptr(skip_flag),
                        native.stream_of(plist[0])), "fr_adam_step")
        return loss
