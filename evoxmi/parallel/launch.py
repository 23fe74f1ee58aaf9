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
  first non-zero child status.  The parent never touches the GPU, so no HIP context is forked
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


def spawn_ranks(n: int, argv: List[str], device: str = "cuda", env: Optional[dict] = None, timeout: Optional[float] = None) -> int:
    """Run ``python argv…`` as N ranks of one job; returns the job's exit status (0 when
    every rank exited 0, else the first non-zero status in rank order)."""
    base = dict(os.environ if env is None else env)
    base.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                EVOXMI_LAUNCHED="1")
    procs = []
    for r in range(n):
        e = dict(base, RANK=str(r), LOCAL_RANK=str(r), GROUP_RANK="0")
        if device == "cpu":
            e["EVOXMI_DIST_BACKEND"] = "gloo"
        procs.append(subprocess.Popen([sys.executable] + list(argv), env=e))
    codes = []
    for p in procs:
        try:
            codes.append(p.wait(timeout=timeout))
        except subprocess.TimeoutExpired:
            for q in procs:
                if q.poll() is None:
                    q.kill()
            codes.append(124)
    for c in codes:
        if c != 0:
            return c
    return 0


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
