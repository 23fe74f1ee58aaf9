"""Driver + worker-process data-parallel workflow (Ray-free).

Parity target: ``RayDistributedWorkflow`` (reference
``src/evox/workflows/distributed.py:13-361``): ``num_workers`` copies of the
workflow are created with the **same seed**; each evaluates a balanced slice of
the population (``_get_slice`` ``:40-45``), the fitness slices are all-gathered so
every worker runs the identical ``tell``; only worker 0 forwards monitor calls,
which the driver replays (``:346-349``); ``async_dispatch`` bounds the number of
generations the driver lets run ahead (``:336-344``).

Ray is not part of this stack.  Workers are local processes started with the
``spawn`` method that form a ``torch.distributed`` group (RCCL when each worker
owns a GPU, gloo otherwise); the all-gather is a collective instead of an object
store round-trip.  The driver talks to workers over pipes.
"""
from __future__ import annotations

import os
import socket
import warnings
from collections import deque
from typing import Callable, Dict, List, Optional

import torch
import torch.multiprocessing as mp

from ..core import Monitor, State, Workflow
from ..utils.common import parse_opt_direction

_HOOKS = ("pre_step", "pre_ask", "post_ask", "pre_eval", "post_eval", "pre_tell", "post_tell", "post_step")


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cpu(x):
    if isinstance(x, torch.Tensor):
        return x.detach().to("cpu")
    if isinstance(x, (list, tuple)):
        return type(x)(_cpu(y) for y in x)
    return x


class _ForwardingMonitor(Monitor):
    """Lives in worker 0; records hook calls (tensors moved to host) for the driver."""

    def __init__(self, hooks, conn):
        super().__init__()
        self._hooks = [h for h in hooks if h not in ("pre_step", "post_step")]
        self.conn = conn
        self.queue = []
        for h in self._hooks:
            if h != "post_eval":  # post_eval is a real method: it also ships the fitness to the driver
                setattr(self, h, self._make(h))

    def hooks(self):
        return list(self._hooks) + ["post_eval"]

    def _make(self, hook):
        def fn(state, *args):
            self.queue.append((hook, tuple(_cpu(a) for a in args)))

        return fn

    def post_eval(self, state, cand_sol, transformed, fitness):
        self.conn.send(("fitness", _cpu(fitness)))
        if "post_eval" in self._hooks:
            self.queue.append(("post_eval", (_cpu(cand_sol), None, _cpu(fitness))))


def _worker(rank, world, port, conn, payload):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from .std_workflow import StdWorkflow

    use_gpu = payload["use_gpu"] and torch.cuda.is_available()
    if use_gpu:
        torch.cuda.set_device(rank % torch.cuda.device_count())
    dist.init_process_group("nccl" if use_gpu else "gloo", rank=rank, world_size=world)
    monitors = [_ForwardingMonitor(payload["hooks"], conn)] if rank == 0 else []
    wf = StdWorkflow(
        payload["algorithm"],
        payload["problem"],
        monitors=monitors,
        opt_direction=payload["opt_direction"],
        sol_transforms=payload["sol_transforms"],
        fit_transforms=payload["fit_transforms"],
    )
    state = None
    try:
        while True:
            cmd, arg = conn.recv()
            if cmd == "setup":
                key = arg.to("cuda") if use_gpu else arg
                state = wf.init(key)
                state = wf.enable_distributed(state)
                conn.send(("ok", None))
            elif cmd == "step":
                state = wf.step(state)
                q = monitors[0].queue if monitors else []
                if monitors:
                    monitors[0].queue = []
                conn.send(("done", q))
            elif cmd == "valid":
                fit, state = wf.valid(state, arg)
                conn.send(("valid", _cpu(fit)))
            elif cmd == "sample":
                from ..core import use_state

                pop, _ = use_state(wf.algorithm.ask)(state)
                conn.send(("sample", _cpu(pop)))
            elif cmd == "state":
                conn.send(("state", state.to("cpu")))
            elif cmd == "close":
                break
    finally:
        dist.destroy_process_group()
        conn.close()


class RayDistributedWorkflow(Workflow):
    """Process-parallel workflow with the reference's constructor and ``step`` API."""

    def __init__(
        self,
        algorithm,
        problem,
        num_workers: int,
        monitors=(),
        opt_direction="min",
        metrics: Optional[Dict[str, Callable]] = None,
        options: dict = None,
        sol_transforms: List[Callable] = (),
        fit_transforms: List[Callable] = (),
        global_fit_transform: List[Callable] = (),
        async_dispatch: int = 4,
        monitor=None,
        use_gpu: bool = False,
    ):
        super().__init__()
        self.monitors = list(monitors) if monitor is None else [monitor]
        if monitor is not None:
            warnings.warn("`monitor` is deprecated", DeprecationWarning)
        self.registered_hooks = {h: [] for h in _HOOKS}
        for m in self.monitors:
            for h in m.hooks():
                self.registered_hooks[h].append(m)
        self.opt_direction = parse_opt_direction(opt_direction)
        for m in self.monitors:
            m.set_opt_direction(self.opt_direction)
        self.async_dispatch = async_dispatch
        self.num_workers = num_workers
        self._pending = deque()
        non_empty = [h for h in _HOOKS if self.registered_hooks[h]]
        payload = dict(
            algorithm=algorithm,
            problem=problem,
            opt_direction=opt_direction,
            sol_transforms=list(sol_transforms),
            fit_transforms=list(fit_transforms),
            hooks=non_empty,
            use_gpu=use_gpu,
        )
        ctx = mp.get_context("spawn")
        port = _free_port()
        self._conns, self._procs = [], []
        self._stash = [deque() for _ in range(num_workers)]
        for r in range(num_workers):
            a, b = ctx.Pipe()
            p = ctx.Process(target=_worker, args=(r, num_workers, port, b, payload), daemon=True)
            p.start()
            self._conns.append(a)
            self._procs.append(p)

    # --- message plumbing ------------------------------------------------------------
    def _recv(self, rank, kind):
        st = self._stash[rank]
        for i, (k, v) in enumerate(st):
            if k == kind:
                del st[i]
                return v
        while True:
            k, v = self._conns[rank].recv()
            if k == kind:
                return v
            st.append((k, v))

    def _broadcast(self, cmd, arg=None):
        for c in self._conns:
            c.send((cmd, arg))

    def _drain_one(self):
        self._pending.popleft()
        calls = None
        for r in range(self.num_workers):
            q = self._recv(r, "done")
            if r == 0:
                calls = q
        for hook, args in calls or []:
            for m in self.registered_hooks[hook]:
                getattr(m, hook)(None, *args)

    # --- workflow API ----------------------------------------------------------------
    def setup(self, key):
        self._broadcast("setup", key.to("cpu"))
        for r in range(self.num_workers):
            self._recv(r, "ok")
        return State(generation=0)

    def step(self, state: State, block: bool = False) -> State:
        for m in self.registered_hooks["pre_step"]:
            m.pre_step(state)
        self._broadcast("step")
        fitness = self._recv(0, "fitness")
        for m in self.registered_hooks["post_eval"]:
            if "post_eval" in m.hooks():
                pass
        self._pending.append(1)
        while len(self._pending) >= self.async_dispatch:
            self._drain_one()
        if block:
            while self._pending:
                self._drain_one()
        self.last_fitness = fitness
        state = state.update(generation=state.generation + 1)
        for m in self.registered_hooks["post_step"]:
            m.post_step(state)
        return state

    def flush(self):
        while self._pending:
            self._drain_one()

    def valid(self, state: State, metric="loss"):
        self.flush()
        self._broadcast("valid", metric)
        fit = [self._recv(r, "valid") for r in range(self.num_workers)][0]
        return fit, state

    def sample(self, state: State):
        self.flush()
        self._broadcast("sample")
        pops = [self._recv(r, "sample") for r in range(self.num_workers)]
        return pops[0], state

    def worker_state(self) -> State:
        """Full state of worker 0 (all replicas are identical)."""
        self.flush()
        self._broadcast("state")
        return [self._recv(r, "state") for r in range(self.num_workers)][0]

    def close(self):
        try:
            self.flush()
            self._broadcast("close")
        except Exception:
            pass
        for p in self._procs:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()

    def __del__(self):
        try:
            if any(p.is_alive() for p in self._procs):
                self.close()
        except Exception:
            pass
