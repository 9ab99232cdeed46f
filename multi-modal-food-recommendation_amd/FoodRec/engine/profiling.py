"""Per-launch kernel timing with HIP events (torch.cuda.Event on the launch stream).

Every engine launch goes to torch's current stream, so events recorded there bracket exactly
that kernel (plus its launch gap).  bench.py enables this over its timed steps to report the
dominant kernel's average duration and algorithmic bytes per launch (roofline.achieved);
when disabled the hooks cost one attribute check.
"""
from __future__ import annotations

import contextlib
from collections import defaultdict

import torch

_ACTIVE = None
SPIN_CYCLES = 200_000  # ~0.1 ms busy-wait before each timed region (not part of the measurement)


class KernelTimer:
    def __init__(self):
        self.records = []  # (name, start_event, end_event, algorithmic_bytes)

    @contextlib.contextmanager
    def region(self, name: str, nbytes: int):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        # keep the GPU busy while the host records the start event and launches the kernel: with
        # a starved queue the start event would fire before the launch and count the host's
        # launch latency as kernel time
        torch.cuda._sleep(SPIN_CYCLES)
        s.record()
        try:
            yield
        finally:
            e.record()
            self.records.append((name, s, e, int(nbytes)))

    def summary(self) -> dict:
        torch.cuda.synchronize()
        agg = defaultdict(lambda: [0, 0.0, 0, []])
        for name, s, e, b in self.records:
            a = agg[name]
            ms = s.elapsed_time(e)
            a[0] += 1
            a[1] += ms
            a[2] += b
            a[3].append(ms)
        # median_ms: robust to a launch stretched by a host stall between its events (dominance)
        return {k: {"launches": n, "total_ms": t, "avg_ms": t / n, "median_ms": sorted(v)[len(v) // 2],
                    "bytes_per_launch": b / n, "gbps": (b / n) / (t / n * 1e-3) / 1e9 if t > 0 else 0.0}
                for k, (n, t, b, v) in agg.items()}


class StampTimer:
    """Region timing inside a captured HIP graph (timing events cannot be recorded during capture):
    each region is bracketed by two fr_stamp launches writing the device's constant-rate wall
    clock into its own slot of a device buffer.  Capture one step with this active, replay the graph,
    then ``read`` the per-region durations of that replay (the stamp kernels' own launch gaps, ~1-2
    µs per region, are included: an upper bound on the kernels' time)."""

    def __init__(self, device, capacity: int = 1024):
        from . import native
        self.lib = native.lib()
        self.hz = int(self.lib.fr_stamp_hz())
        self.buf = torch.zeros(capacity, 2, dtype=torch.int64, device=device)
        self.names = []  # (name, algorithmic bytes) per slot, in issue order

    @contextlib.contextmanager
    def region(self, name: str, nbytes: int):
        from . import native
        i = len(self.names)
        if i >= self.buf.shape[0]:
            yield
            return
        self.names.append((name, int(nbytes), torch.cuda.is_current_stream_capturing()))
        st = torch.cuda.current_stream(self.buf.device).cuda_stream
        native.check(self.lib.fr_stamp(self.buf[i, 0].data_ptr(), st), "fr_stamp")
        try:
            yield
        finally:
            native.check(self.lib.fr_stamp(self.buf[i, 1].data_ptr(), st), "fr_stamp")

    def read(self) -> list:
        """[(name, microseconds, bytes)] of the captured regions' last replay, in issue order."""
        torch.cuda.synchronize()
        t = self.buf[:len(self.names)].cpu()
        return [(n, float(t[i, 1] - t[i, 0]) * 1e6 / self.hz, b) for i, (n, b, cap) in enumerate(self.names) if cap]


def active():
    return _ACTIVE


@contextlib.contextmanager
def timing():
    global _ACTIVE
    prev, _ACTIVE = _ACTIVE, KernelTimer()
    try:
        yield _ACTIVE
    finally:
        _ACTIVE = prev


@contextlib.contextmanager
def stamping(device):
    """StampTimer active (for a capture): the regions issued meanwhile are stamped."""
    global _ACTIVE
    prev, _ACTIVE = _ACTIVE, StampTimer(device)
    try:
        yield _ACTIVE
    finally:
        _ACTIVE = prev


def region(name: str, nbytes: int):
    t = _ACTIVE
    if t is None:
        return contextlib.nullcontext()
    if isinstance(t, StampTimer):
        return t.region(name, nbytes)
    if torch.cuda.is_current_stream_capturing():
        return contextlib.nullcontext()
    return t.region(name, nbytes)
