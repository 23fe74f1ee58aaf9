"""Single-node rank launcher for the benchmark entry points (``bench.py``, ``tools/bench_*.py``).

``python bench.py --gpus N`` must run N ranks, one per GPU, or fail — never silently
measure one GPU.  The reference spans every visible device in ``enable_distributed``
(``/root/reference/src/evox/workflows/std_workflow.py:329-345``); here the same job is one
process per GPU over RCCL, so a launch without ``torchrun`` spawns the ranks itself:

* ``WORLD_SIZE`` set (``torchrun`` / ``torch.distributed.run``): this process IS a rank; the
  requested N must equal ``WORLD_SIZE``;
* ``WORLD_SIZE`` unset and N > 1: the parent checks the visible device count (without
  initialising HIP: ``torch.cuda.device_count()`` does not on this image), spawns N fresh
  child processes with the torchrun environment (``RANK`` / ``LOCAL_RANK`` / ``WORLD_SIZE``,
  ``MASTER_ADDR=127.0.0.1``, a free ``MASTER_PORT``), forwards their output and exits with the
  status of the first child to fail — the other ranks are then terminated (they would block in
  a collective with the dead rank), and so are all of them when the parent is interrupted.  The parent never touches the GPU, so no HIP context is forked
  or exec'd.
* ``device="cpu"``: the ranks run on gloo (tests of the launcher on a GPU-less host).
"""
from __future__ import annotations

import os
import socket
import subprocess
import sys
from typing import List, Optional


class LaunchError(RuntimeError):
    pass


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return int(s.getsockname()[1])


def visible_devices() -> int:
    import torch

    return int(torch.cuda.device_count())


def _stop(procs, grace: float = 5.0) -> None:
    """Terminate every live child, then kill whatever is still running after ``grace`` s."""
    import time

    live = [p for p in procs if p.poll() is None]
    for p in live:
        p.terminate()
    t_end = time.monotonic() + grace
    for p in live:
        try:
            p.wait(timeout=max(0.0, t_end - time.monotonic()))
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()


def spawn_ranks(n: int, argv: List[str], device: str = "cuda", env: Optional[dict] = None, timeout: Optional[float] = None,
                poll_s: float = 0.05) -> int:
    """Run ``python argv…`` as N ranks of one job; returns the job's exit status: 0 when every
    rank exited 0, else the status of the FIRST rank to fail (in time, not rank order).

    All children are polled together: when one exits non-zero the others are terminated at
    once (a surviving rank would otherwise block forever in a collective with the dead one),
    and a ``timeout`` (seconds) or an interrupt of the parent (SIGINT / SIGTERM) ends every
    child too, so no rank is left holding a GPU."""
    import signal
    import time

    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                EVOXMI_LAUNCHED="1")
    procs = []

    def _on_signal(signum, _frame):
        _stop(procs)
        raise SystemExit(128 + signum)

    old = {}
    for sig in (signal.SIGINT, signal.SIGTERM):
        try:
            old[sig] = signal.signal(sig, _on_signal)
        except ValueError:  # not the main thread: the finally below still cleans up
            pass
    try:
        for r in range(n):
            e = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
            if device == "cpu":
                e["EVOXMI_DIST_BACKEND"] = "gloo"
            procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
        t_end = None if timeout is None else time.monotonic() + timeout
        while True:
            codes = [p.poll() for p in procs]
            bad = [c for c in codes if c is not None and c != 0]
            if bad:
                _stop(procs)
                return bad[0]
            if all(c == 0 for c in codes):
                return 0
            if t_end is not None and time.monotonic() > t_end:
                _stop(procs)
                return 124
            time.sleep(poll_s)
    finally:
        _stop(procs)
        for sig, h in old.items():
            signal.signal(sig, h)


def ensure_ranks(n: int, device: str = "cuda", argv: Optional[List[str]] = None) -> None:
    """Make the current invocation an N-rank job.  Returns in a rank process (or when N = 1);
    otherwise spawns the ranks and exits the parent with their status."""
    if n < 1:
        raise LaunchError(f"--gpus must be >= 1, got {n}")
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != n:
            raise LaunchError(f"--gpus {n} but the launcher started WORLD_SIZE={ws} ranks")
        return
    if n == 1:
        return
    if device != "cpu":
        have = visible_devices()
        if have < n:
            raise LaunchError(f"--gpus {n} requested but only {have} GPU(s) are visible; refusing to run fewer ranks")
    argv = list(sys.argv if argv is None else argv)
    sys.exit(spawn_ranks(n, argv, device=device))
