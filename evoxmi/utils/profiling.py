"""Tracing and per-phase timing.

The reference has no built-in profiling (``run/run_de.py:77,87-88`` times whole
runs with ``time.time()``).  evoxmi provides:

* :func:`trace_range` — a roctx range (``torch.cuda.nvtx`` maps to roctx on ROCm,
  so ``rocprofv3 --marker-trace`` shows it) plus a ``torch.profiler`` label.  The
  workflow opens one around ``ask`` / ``evaluate`` / ``tell`` when
  ``evoxmi.config`` knob ``trace`` is on (``EVOXMI_TRACE=1``) and one around each
  graph replay.
* :class:`PhaseTimer` — stream-ordered hipEvent timers: ``start``/``stop`` only
  *record* events, so timing a generation never synchronises the host; the
  elapsed times are resolved when :meth:`PhaseTimer.summary` is called.  On CPU
  tensors it falls back to ``time.perf_counter``.
"""
from __future__ import annotations

import contextlib
import time
from collections import defaultdict
from typing import Dict, List, Optional

import torch

from .. import config


def _markers_available() -> bool:
    return torch.cuda.is_available() and hasattr(torch.cuda, "nvtx")


@contextlib.contextmanager
def trace_range(name: str, enabled: Optional[bool] = None):
    """roctx + torch.profiler range; a no-op unless tracing is enabled."""
    if enabled is None:
        enabled = config.get("trace")
    if not enabled:
        yield
        return
    pushed = False
    if _markers_available():
        try:
            torch.cuda.nvtx.range_push(name)
            pushed = True
        except RuntimeError:
            pushed = False
    try:
        with torch.profiler.record_function(name):
            yield
    finally:
        if pushed:
            torch.cuda.nvtx.range_pop()


_ACTIVE_TIMER = None


def phase(name: str):
    """Time ``name`` on the workflow's active :class:`PhaseTimer` (eager steps with a
    ``phase_timer``); a no-op otherwise.  Lets algorithms expose inner phases (e.g. the
    CMA-ES eigensolve inside ``tell``) in the same per-phase breakdown."""
    t = _ACTIVE_TIMER
    if t is None:
        return contextlib.nullcontext()
    return t.phase(name)


class PhaseTimer:
    """Accumulate per-phase wall time without host synchronisation.

    >>> timer = PhaseTimer()
    >>> with timer.phase("ask"):
    ...     ...
    >>> timer.summary()   # {'ask': {'count': 1, 'total_ms': ..., 'mean_ms': ...}}
    """

    def __init__(self, device=None):
        self.device = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
        self._pending: Dict[str, List] = defaultdict(list)
        self._done: Dict[str, List[float]] = defaultdict(list)

    @property
    def on_gpu(self) -> bool:
        return self.device.type == "cuda"

    @contextlib.contextmanager
    def phase(self, name: str):
        if self.on_gpu and not torch.cuda.is_current_stream_capturing():
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            try:
                yield
            finally:
                b.record()
                self._pending[name].append((a, b))
        else:
            t = time.perf_counter()
            try:
                yield
            finally:
                self._done[name].append((time.perf_counter() - t) * 1e3)

    def _resolve(self):
        for name, evs in self._pending.items():
            for a, b in evs:
                b.synchronize()
                self._done[name].append(a.elapsed_time(b))
        self._pending.clear()

    def summary(self) -> Dict[str, Dict[str, float]]:
        self._resolve()
        out = {}
        for name, ts in self._done.items():
            out[name] = {"count": len(ts), "total_ms": float(sum(ts)), "mean_ms": float(sum(ts) / max(len(ts), 1))}
        return out

    def reset(self):
        self._pending.clear()
        self._done.clear()
