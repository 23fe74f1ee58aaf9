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
SO_PATH = os.environ.get("EVOXMI_SO") or os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "_C.so")
# EVOXMI_SO: an alternative build of the same extension (compiler-flag A/B runs)


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


# ---------------------------------------------------------------- sticky kernel error word
# Kernels that can detect a failure they cannot report synchronously (out-of-range
# indices, a persistent kernel's grid barrier timing out) OR a bit into one int32 word per
# device.  It is read at host sync points: monitor getters, ``check_kernel_errors()``,
# and after every launch when EVOXMI_DEBUG=1.
KERNEL_ERROR_BITS = {1: "de_trial: out-of-range row index", 2: "de_trial: out-of-range target row",
                     4: "nds: persistent peel grid barrier timed out (workgroups not co-resident)"}
_ERR = {}


def error_flag(dev) -> torch.Tensor:
    dev = torch.device(dev)
    if dev not in _ERR:
        _ERR[dev] = torch.zeros(1, dtype=torch.int32, device=dev)
    return _ERR[dev]


def kernel_error_flags() -> int:
    v = 0
    for f in _ERR.values():
        v |= int(f.item())
    return v


def check_kernel_errors(reset: bool = True) -> None:
    """Raise if any kernel has set the sticky error word (one host sync per device)."""
    v = kernel_error_flags()
    if v:
        if reset:
            for f in _ERR.values():
                f.zero_()
        msgs = [m for b, m in KERNEL_ERROR_BITS.items() if v & b] or [f"flag {v}"]
        raise RuntimeError("evoxmi kernel error: " + "; ".join(msgs))
