"""Process-group bootstrap for one-process-per-GPU SPMD runs.

Reads the torchrun contract (``RANK``, ``LOCAL_RANK``, ``WORLD_SIZE``,
``MASTER_ADDR``, ``MASTER_PORT``), binds the process to ``cuda:LOCAL_RANK`` and
initialises ``torch.distributed`` with RCCL (backend ``"nccl"``) on GPUs or gloo
on CPU.  The reference relied on ``jax.distributed.initialize``
(docs ``guide/user/3-distributed.md:90-125``) or a Ray cluster.
"""
from __future__ import annotations

import datetime
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


def init_distributed(backend: str = None, timeout_s: int = 600, force: bool = False):
    """Initialise the default process group if the env describes >1 rank (or always,
    with ``force=True`` — a one-rank RCCL group exercises the distributed code path,
    including hipGraph capture of the collectives, on a single GPU).

    Returns ``(rank, world_size, device)``.
    """
    world, rank, local = env_world()
    backend = backend or os.environ.get("EVOXMI_DIST_BACKEND") or None
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    if use_gpu:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    else:
        device = torch.device("cpu")
    if (world > 1 or force) and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29511")
        be = backend or ("nccl" if use_gpu else "gloo")
        kw = dict(backend=be, rank=rank, world_size=world, timeout=datetime.timedelta(seconds=timeout_s))
        if be == "nccl":
            kw["device_id"] = device
        dist.init_process_group(**kw)
    return rank, world, device


def destroy():
    if dist.is_initialized():
        dist.destroy_process_group()
