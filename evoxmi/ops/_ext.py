"""Loader for the in-tree HIP extension ``evoxmi/_C.so``.

Device tensors go through ``torch.ops.evoxmi.*`` HIP kernels; CPU tensors use the
plain-PyTorch reference implementations in the sibling modules (those are also
the numerics oracles the GPU tests compare against).  On a machine with a GPU the
extension is **required**: if it cannot be loaded, every device op raises instead
of silently falling back to an eager PyTorch path.
"""
from __future__ import annotations

import os
import threading

import torch

_LOCK = threading.Lock()
_LOADED = False
_ERROR = None
SO_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")


def load(build_if_missing: bool = True) -> bool:
    global _LOADED, _ERROR
    if _LOADED:
        return True
    with _LOCK:
        if _LOADED:
            return True
        try:
            if not os.path.exists(SO_PATH) and build_if_missing:
                from .build import build

                build(verbose=False)
            torch.ops.load_library(SO_PATH)
            _LOADED = True
        except Exception as e:  # pragma: no cover - depends on the box
            _ERROR = e
    return _LOADED


def available() -> bool:
    return load()


def ops():
    if not load():
        raise RuntimeError(
            f"evoxmi HIP extension could not be loaded from {SO_PATH}: {_ERROR!r}. "
            "Build it with `python -m evoxmi.ops.build` (device ops never fall back to eager PyTorch)."
        )
    return torch.ops.evoxmi


def philox_fill(key: torch.Tensor, n: int, dist: int, offset: int = 0) -> torch.Tensor:
    return ops().philox_fill(key, int(n), int(dist), int(offset))
