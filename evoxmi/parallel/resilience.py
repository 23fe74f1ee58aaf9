"""Failure detection, elastic recovery and fault injection.

The reference has none of these (a Ray worker failure simply raises in
``ray.get``; ``distributed.py:205-208``).  evoxmi's SPMD design makes recovery
simple: the algorithm state is *replicated* on every rank and only the population
slice depends on the world size (``balanced_slices``), so

* any surviving rank holds everything needed to continue;
* a restarted job with a different number of ranks re-shards automatically.

Pieces:

* :class:`Heartbeat` — each rank stamps ``evoxmi/hb/<rank>`` in the job's
  ``TCPStore`` from a daemon thread; :meth:`Heartbeat.dead_ranks` lists ranks
  whose stamp is older than the timeout (a rank watchdog that needs no
  collective, so it still works while a peer is hung inside RCCL).
* :func:`run_elastic` — step a workflow with periodic atomic checkpoints written
  by rank 0 and resume from the newest one on (re)start, with whatever world
  size the restarted job has (use with ``torchrun --max-restarts``).
* :class:`FaultInjector` — a monitor that poisons fitness values (NaN/Inf) or
  raises :class:`InjectedFault` on a chosen rank at a chosen generation, for
  testing the NaN policy, the watchdog and the restart path.
"""
from __future__ import annotations

import glob
import os
import re
import threading
import time
from typing import Callable, Iterable, List, Optional

import torch
import torch.distributed as dist

from .. import config
from ..core import Monitor
from ..core.checkpoint import load_state, save_state


# ----------------------------------------------------------------------------- watchdog
def default_store():
    """The TCPStore of the default process group (None without one)."""
    if not (dist.is_available() and dist.is_initialized()):
        return None
    try:
        return dist.distributed_c10d._get_default_store()
    except Exception:  # pragma: no cover - private API moved
        return None


class Heartbeat:
    KEY = "evoxmi/hb/{}"

    def __init__(self, store=None, rank: Optional[int] = None, world_size: Optional[int] = None,
                 interval: Optional[float] = None, timeout: Optional[float] = None):
        self.store = store if store is not None else default_store()
        if self.store is None:
            raise RuntimeError("Heartbeat needs a TCPStore (initialise torch.distributed or pass store=)")
        self.rank = dist.get_rank() if rank is None else rank
        self.world_size = dist.get_world_size() if world_size is None else world_size
        self.interval = config.get("heartbeat_interval") if interval is None else interval
        self.timeout = config.get("heartbeat_timeout") if timeout is None else timeout
        self._stop = threading.Event()
        self._thread = None

    def beat(self):
        self.store.set(self.KEY.format(self.rank), repr(time.time()))

    def _loop(self):
        while not self._stop.wait(self.interval):
            try:
                self.beat()
            except Exception:
                return  # store gone: the job is shutting down

    def start(self):
        self.beat()
        self._thread = threading.Thread(target=self._loop, name=f"evoxmi-heartbeat-{self.rank}", daemon=True)
        self._thread.start()
        return self

    def stop(self):
        self._stop.set()
        if self._thread is not None:
            self._thread.join(timeout=self.interval + 1.0)

    def last_seen(self, rank: int) -> Optional[float]:
        key = self.KEY.format(rank)
        try:
            if not self.store.check([key]):
                return None
            return float(self.store.get(key).decode())
        except Exception:
            return None

    def dead_ranks(self, now: Optional[float] = None) -> List[int]:
        now = time.time() if now is None else now
        dead = []
        for r in range(self.world_size):
            t = self.last_seen(r)
            if t is None or now - t > self.timeout:
                dead.append(r)
        return dead


# ----------------------------------------------------------------------------- fault injection
class InjectedFault(RuntimeError):
    pass


class FaultInjector(Monitor):
    """Deterministic faults for tests.

    * ``poison={generation: [indices]}`` — overwrite those fitness entries with
      ``poison_value`` (NaN by default) right after evaluation (eager steps);
    * ``crash_at=(rank, generation)`` — raise :class:`InjectedFault` on that rank
      before the given generation starts.
    """

    def __init__(self, poison: Optional[dict] = None, poison_value: float = float("nan"), crash_at=None):
        super().__init__()
        self.poison = dict(poison or {})
        self.poison_value = poison_value
        self.crash_at = crash_at
        self._gen = None

    def hooks(self):
        return ["pre_step", "post_eval"]

    def pre_step(self, state):
        self._gen = int(state.generation)
        if self.crash_at is not None:
            rank = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
            if (rank, self._gen) == tuple(self.crash_at):
                raise InjectedFault(f"injected crash on rank {rank} at generation {self._gen}")

    def post_eval(self, state, cand_sol, transformed, fitness):
        idx = self.poison.get(self._gen)
        if idx:
            fitness[torch.as_tensor(list(idx), device=fitness.device)] = self.poison_value


# ----------------------------------------------------------------------------- elastic run loop
_CKPT_RE = re.compile(r"state_(\d+)\.safetensors$")


def checkpoints(ckpt_dir: str) -> List[str]:
    files = [(int(m.group(1)), f) for f in glob.glob(os.path.join(ckpt_dir, "state_*.safetensors"))
             if (m := _CKPT_RE.search(f))]
    return [f for _, f in sorted(files)]


def latest_checkpoint(ckpt_dir: str) -> Optional[str]:
    c = checkpoints(ckpt_dir)
    return c[-1] if c else None


def _atomic_save(state, path: str):
    tmp = path + ".tmp"
    save_state(state, tmp)
    os.replace(tmp, path)


def run_elastic(make_workflow: Callable, key: torch.Tensor, n_steps: int, ckpt_dir: str, every: int = 10,
                keep: int = 2, distributed: Optional[bool] = None, map_location=None, on_step: Callable = None):
    """Run ``n_steps`` generations of ``make_workflow()`` with crash-safe resume.

    On start the newest ``state_<gen>.safetensors`` in ``ckpt_dir`` (if any) is
    loaded and stepping continues from its generation.  With an initialised
    process group the workflow is population-sharded across the *current* ranks
    (rank 0's state is broadcast), so a job restarted with fewer or more ranks
    resumes seamlessly.  Rank 0 writes a checkpoint every ``every`` generations
    (write-to-temp + rename, so a crash never leaves a torn file) and keeps the
    newest ``keep``.  Returns ``(workflow, state)``.
    """
    os.makedirs(ckpt_dir, exist_ok=True)
    wf = make_workflow()
    state = wf.init(key)
    path = latest_checkpoint(ckpt_dir)
    if path is not None:
        loaded = load_state(path, map_location=map_location)
        if map_location is None:
            dev = next((x.device for x in torch.utils._pytree.tree_leaves(state) if isinstance(x, torch.Tensor)), None)
            if dev is not None:
                loaded = torch.utils._pytree.tree_map(lambda x: x.to(dev) if isinstance(x, torch.Tensor) else x, loaded)
        state = loaded
    use_dist = (dist.is_available() and dist.is_initialized()) if distributed is None else distributed
    if use_dist:
        state = wf.enable_distributed(state)
    rank = dist.get_rank() if use_dist else 0
    start = int(state.generation)
    for g in range(start, n_steps):
        state = wf.step(state)
        if on_step is not None:
            on_step(g, state)
        if (g + 1) % every == 0 or g + 1 == n_steps:
            if rank == 0:
                _atomic_save(state, os.path.join(ckpt_dir, f"state_{g + 1}.safetensors"))
                for old in checkpoints(ckpt_dir)[:-keep]:
                    os.remove(old)
            if use_dist:
                dist.barrier()
    return wf, state
