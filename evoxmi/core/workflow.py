"""Workflow marker class (reference ``src/evox/core/workflow.py:4-5``)."""
from .module import Stateful


class Workflow(Stateful):
    pass


# ---------------------------------------------------------------------------- capture warm-ups
_WARMUP = [0]


class capture_warmup:
    """Context of a hipGraph capture's warm-up step: it runs on a COPY of the state (allocator
    and lazy initialisation before capture), so components that record per-step diagnostics
    (e.g. the device eigensolver's per-solve log) skip them inside it — a warm-up is not a
    generation of the run."""

    def __enter__(self):
        _WARMUP[0] += 1
        return self

    def __exit__(self, *exc):
        _WARMUP[0] -= 1
        return False


def in_capture_warmup() -> bool:
    return _WARMUP[0] > 0
