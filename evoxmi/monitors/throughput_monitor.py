"""Throughput and per-generation logging monitors.

The reference exposes no speed counter; the north-star metric (generations/s and
evaluations/s) is built in here.  Both monitors keep the generation pipeline
asynchronous: they record hipEvents / device scalars and only synchronise when a
getter runs (``ThroughputMonitor``) or every ``flush_every`` generations
(``JSONLLogger``).
"""
from __future__ import annotations

import json
import time
from typing import List, Optional

import torch

from ..core import Monitor


class ThroughputMonitor(Monitor):
    """Generations/s and evaluations/s over the steps seen so far.

    ``pre_step``/``post_step`` record events on the current stream; ``post_ask``
    counts the candidate rows (for sharded workflows: the local rows of this rank)."""

    def __init__(self, skip_first: int = 1):
        super().__init__()
        self.skip_first = skip_first
        self._events: List = []
        self._evals: List[int] = []
        self._cur_evals = 0
        self._t0 = None

    def hooks(self):
        return ["pre_step", "post_ask", "post_step"]

    def _mark(self):
        if torch.cuda.is_available() and torch.cuda.is_initialized():
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            return e
        return time.perf_counter()

    def pre_step(self, state):
        self._cur_evals = 0
        self._t0 = self._mark()

    def post_ask(self, state, cand_sol):
        leaf = cand_sol if isinstance(cand_sol, torch.Tensor) else torch.utils._pytree.tree_leaves(cand_sol)[0]
        self._cur_evals += int(leaf.shape[0])

    def post_step(self, state):
        self._events.append((self._t0, self._mark()))
        self._evals.append(self._cur_evals)

    def _elapsed_ms(self, a, b) -> float:
        if isinstance(a, float):
            return (b - a) * 1e3
        b.synchronize()
        return a.elapsed_time(b)

    def step_times_ms(self) -> List[float]:
        return [self._elapsed_ms(a, b) for a, b in self._events]

    def summary(self) -> dict:
        ts = self.step_times_ms()[self.skip_first:]
        ev = self._evals[self.skip_first:]
        total = sum(ts)
        if not ts or total <= 0:
            return {"generations": len(ts), "gens_per_sec": None, "evals_per_sec": None, "ms_per_gen": None}
        return {"generations": len(ts), "ms_per_gen": total / len(ts), "gens_per_sec": 1e3 * len(ts) / total,
                "evals_per_sec": 1e3 * sum(ev) / total}


class JSONLLogger(Monitor):
    """Append one JSON line per generation: generation, best fitness so far (in the
    user's optimisation direction), best of this generation, wall time.

    Per-generation values stay on the device until ``flush_every`` generations
    have accumulated (one host sync per flush, not per generation)."""

    def __init__(self, path: str, flush_every: int = 16, extra: Optional[dict] = None):
        super().__init__()
        self.path = path
        self.flush_every = flush_every
        self.extra = dict(extra or {})
        self.opt_direction = 1
        self._buf = []
        self._best = None
        self._gen = 0
        self._t0 = time.time()

    def hooks(self):
        return ["post_eval", "post_step"]

    def set_opt_direction(self, opt_direction):
        self.opt_direction = opt_direction

    def post_eval(self, state, cand_sol, transformed, fitness):
        f = fitness if fitness.dim() == 1 else fitness[:, 0]
        cur = f.min().detach().reshape(1)
        self._best = cur.clone() if self._best is None else torch.minimum(self._best, cur)
        self._buf.append((self._gen, torch.cat([cur, self._best]), time.time() - self._t0))

    def post_step(self, state):
        self._gen += 1
        if len(self._buf) >= self.flush_every:
            self.flush()

    def flush(self):
        if not self._buf:
            return
        vals = torch.stack([v for _, v, _ in self._buf]).cpu()
        od = self.opt_direction if not isinstance(self.opt_direction, torch.Tensor) else float(self.opt_direction.reshape(-1)[0])
        with open(self.path, "a") as fh:
            for (g, _, t), v in zip(self._buf, vals):
                rec = {"generation": g, "best_in_generation": float(v[0]) * od, "best_so_far": float(v[1]) * od, "wall_s": round(t, 6)}
                rec.update(self.extra)
                fh.write(json.dumps(rec) + "\n")
        self._buf.clear()
