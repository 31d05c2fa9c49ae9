"""Tracing / profiling helpers.

* :class:`StepTimer` — per-phase device time of a training step
  (forward / backward / all-reduce wait / optimizer) from HIP events
  recorded on the compute stream; no host sync until :meth:`summary`.
* :func:`torch_trace` — ``torch.profiler`` with HIP kernel activity for a
  window of steps, exported as a Chrome trace (``chrome://tracing`` /
  Perfetto), one file per rank.
* Kernel-level numbers come from ``rocprofv3 --kernel-trace --stats``;
  ``tools/rocprof_summary.py`` turns its output into the tables under
  ``profiles/``.

The reference has no tracing beyond per-sync log lines and TensorBoardX
scalars (``controller.go:291-295``, ``examples/mnist/mnist.py:44-49``).
"""
from __future__ import annotations

import contextlib
import os
from collections import defaultdict

import torch


class StepTimer:
    def __init__(self, device=None, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available() and (device is None or torch.device(device).type == "cuda")
        self.device = device
        self._events: dict[str, list] = defaultdict(list)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            yield
            return
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        a.record()
        try:
            yield
        finally:
            b.record()
            self._events[name].append((a, b))

    def summary(self, reset: bool = True) -> dict:
        """Mean milliseconds per phase (device time between the events)."""
        if not self.enabled:
            return {}
        torch.cuda.synchronize(self.device)
        out = {k: round(sum(a.elapsed_time(b) for a, b in v) / len(v), 3) for k, v in self._events.items() if v}
        if reset:
            self._events.clear()
        return out


@contextlib.contextmanager
def torch_trace(out_dir: str | None, rank: int = 0, active_steps: int = 10):
    """Yield a ``step()`` callable; with ``out_dir`` set, profile (HIP
    kernels + host ops) for ``active_steps`` steps after 2 warmup steps and
    write ``out_dir/trace_rank{rank}.json``."""
    if not out_dir:
        yield lambda: None
        return
    from torch.profiler import ProfilerActivity, profile, schedule

    os.makedirs(out_dir, exist_ok=True)
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if torch.cuda.is_available() else [])

    def on_ready(p):
        p.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}.json"))

    with profile(activities=acts, schedule=schedule(wait=0, warmup=2, active=active_steps, repeat=1),
                 on_trace_ready=on_ready) as prof:
        yield prof.step
