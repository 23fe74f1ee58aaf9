"""Segmented hipGraph capture: graph segments with host-orchestrated phases between them.

A generation is captured once and replayed (``StdWorkflow(graph=True)``).  Some steps
need host decisions in the middle of a generation — the CMA-ES eigensolver reads its
device-side convergence statistics to decide how many Jacobi sweeps / refinement
iterations to run (``evoxmi/ops/sbr.py``).  Such a step calls :func:`host_phase`:

* eagerly (no capture active) it simply runs ``fn(*args)``;
* while a :class:`SegmentedGraph` is capturing, it closes the current graph segment,
  records ``(fn, args)`` plus static output buffers shaped like ``out_like`` and opens
  the next segment, which reads those buffers.  :meth:`SegmentedGraph.replay` then
  replays segment 0, runs ``fn`` eagerly on the (now valid) static inputs and copies
  its results into the static outputs, replays segment 1, and so on.

All segments share one private memory pool and are replayed in capture order (the
condition under which PyTorch allows a pool to be shared), so tensors produced by one
segment stay valid for the host phase and the segments after it.
"""
from __future__ import annotations

import gc
from typing import Callable, List, Sequence

import torch

_ACTIVE = None


def capturing() -> bool:
    return _ACTIVE is not None and torch.cuda.is_current_stream_capturing()


def _words(t: torch.Tensor):
    """A contiguous tensor whose size is a whole number of 32-bit words, viewed as int32 words."""
    if t.is_contiguous() and t.element_size() in (4, 8) and t.numel() > 0:
        return t.reshape(-1).view(torch.int32)
    return None


def copy_into(dst: Sequence[torch.Tensor], src: Sequence[torch.Tensor]):
    """dst[i].copy_(src[i]) for all i.  Same-dtype pairs on one device share one multi-tensor launch
    (``torch._foreach_copy_``); pairs of different 4- and 8-byte dtypes are copied as int32 words so
    that, e.g., a float32 / int64 / float64 state write-back is still one launch."""
    dst, src = list(dst), list(src)
    if not dst:
        return
    if len(dst) > 1 and hasattr(torch, "_foreach_copy_") and len({d.dtype for d in dst}) > 1:
        wd, ws, rest = [], [], []
        for d, s_ in zip(dst, src):
            a, b = _words(d), _words(s_)
            if a is not None and b is not None and d.dtype == s_.dtype and d.device == s_.device == dst[0].device:
                wd.append(a)
                ws.append(b)
            else:
                rest.append((d, s_))
        if len(wd) > 1:
            torch._foreach_copy_(wd, ws)
            for d, s_ in rest:
                d.copy_(s_)
            return
    same = all(d.dtype == dst[0].dtype and d.device == dst[0].device and s.dtype == d.dtype and s.device == d.device
               for d, s in zip(dst, src))
    if same and len(dst) > 1 and hasattr(torch, "_foreach_copy_"):
        torch._foreach_copy_(dst, src)
    else:
        for d, s in zip(dst, src):
            d.copy_(s)


def host_phase(fn: Callable, *args, out_like: Sequence[torch.Tensor]):
    """Run ``fn(*args)`` (returning tensors shaped like ``out_like``) as a host phase."""
    sess = _ACTIVE
    if sess is None or not torch.cuda.is_current_stream_capturing():
        return tuple(fn(*args))
    return sess._split(fn, args, out_like)


class SegmentedGraph:
    """A generation captured as hipGraph segments separated by host phases."""

    def __init__(self):
        self.items: List = []  # ("graph", CUDAGraph) | ("host", fn, args, outs)
        self.pool = None
        self._cur = None

    # ------------------------------------------------------------------ capture
    def _begin(self):
        g = torch.cuda.CUDAGraph()
        g.capture_begin(pool=self.pool)
        self._cur = g

    def _end(self):
        self._cur.capture_end()
        self.items.append(("graph", self._cur))
        self._cur = None

    def _split(self, fn, args, out_like):
        self._end()
        outs = tuple(torch.empty_like(t) for t in out_like)
        self.items.append(("host", fn, args, outs))
        self._begin()
        return outs

    def capture(self, body: Callable, stream: torch.cuda.Stream):
        """Capture ``body()`` on ``stream`` (a side stream, as hipGraph capture requires)."""
        global _ACTIVE
        torch.cuda.synchronize()
        gc.collect()
        self.pool = torch.cuda.graph_pool_handle()
        with torch.cuda.stream(stream):
            self._begin()
            _ACTIVE = self
            try:
                out = body()
            except BaseException:
                _ACTIVE = None
                if self._cur is not None:
                    try:
                        self._cur.capture_end()
                    except Exception:
                        pass
                raise
            _ACTIVE = None
            self._end()
        return out

    @property
    def n_segments(self) -> int:
        return sum(1 for it in self.items if it[0] == "graph")

    # ------------------------------------------------------------------ replay
    def replay(self):
        for it in self.items:
            if it[0] == "graph":
                it[1].replay()
            else:
                _, fn, args, outs = it
                res = fn(*args)
                groups = {}
                for o, r in zip(outs, res):
                    g = groups.setdefault((o.dtype, o.device), ([], []))
                    g[0].append(o)
                    g[1].append(r.to(o.device) if r.device != o.device else r)
                for dst, src in groups.values():
                    copy_into(dst, src)
