"""vmap rules that fold a batch of independent runs into ONE launch of each HIP op.

``BatchedRuns`` (``evoxmi/algorithms/containers/batched.py``) executes n independent
runs of an algorithm under ``torch.func.vmap``.  PyTorch's own ops batch natively; the
evoxmi HIP ops below would otherwise hit functorch's per-sample fallback (one launch
per run).  Each rule moves the run axis to the front and calls the op's batched form:

* ``philox_words`` / ``philox_fill``: keys (B, 2) → grid.y = run (``rng.hip``);
* ``argsort_f32`` / ``radix_argsort_f32`` / ``rank_argsort_f32``: keys (B, n) → one workgroup
  (row of workgroups, rank kernel) per run (``sort.hip``);
* ``de_trial``: P (B, rows, d), idx (B, R, K), per-row vectors (B, R), keys (B, 2) →
  grid.y = run, all indices run-local (``evo_ops.hip``).

Each run's words/trials are bit-identical to the single-run op with that run's key
(``tests/test_batched_runs.py``).  This mirrors the reference's use of ``jax.vmap`` for
independent copies of a workflow (``run/run_de.py:54-114`` runs 32 seeds per function).
"""
from __future__ import annotations

import torch

from . import _ext

_REGISTERED = False


def _front(x, bdim, B):
    """Run axis first (broadcast an unbatched operand), contiguous."""
    if bdim is None:
        return x.unsqueeze(0).expand((B,) + tuple(x.shape)).contiguous()
    return x.movedim(bdim, 0).contiguous()


def _philox_words(info, in_dims, key, nblocks, domain, offset, words=4):
    if in_dims[0] is None:
        return _ext.ops().philox_words(key, nblocks, domain, offset, words), None
    return _ext.ops().philox_words(_front(key, in_dims[0], info.batch_size), nblocks, domain, offset, words), 0


def _philox_fill(info, in_dims, key, n, dist, offset):
    if in_dims[0] is None:
        return _ext.ops().philox_fill(key, n, dist, offset), None
    return _ext.ops().philox_fill(_front(key, in_dims[0], info.batch_size), n, dist, offset), 0


def _argsort_f32(info, in_dims, keys, descending):
    if in_dims[0] is None:
        return tuple(_ext.ops().argsort_f32(keys, descending)), (None, None)
    k = _front(keys, in_dims[0], info.batch_size)
    if k.dim() != 2:
        raise NotImplementedError("argsort_f32 vmap rule: per-run keys must be 1-D")
    ok, oi = _ext.ops().argsort_f32(k, descending)
    return (ok, oi), (0, 0)


def _radix_argsort_f32(info, in_dims, keys, descending):
    if in_dims[0] is None:
        return tuple(_ext.ops().radix_argsort_f32(keys, descending)), (None, None)
    k = _front(keys, in_dims[0], info.batch_size)
    if k.dim() != 2:
        raise NotImplementedError("radix_argsort_f32 vmap rule: per-run keys must be 1-D")
    ok, oi = _ext.ops().radix_argsort_f32(k, descending)
    return (ok, oi), (0, 0)


def _rank_argsort_f32(info, in_dims, keys, descending):
    if in_dims[0] is None:
        return tuple(_ext.ops().rank_argsort_f32(keys, descending)), (None, None)
    k = _front(keys, in_dims[0], info.batch_size)
    if k.dim() != 2:
        raise NotImplementedError("rank_argsort_f32 vmap rule: per-run keys must be 1-D")
    ok, oi = _ext.ops().rank_argsort_f32(k, descending)
    return (ok, oi), (0, 0)


def _de_trial(info, in_dims, P, idx, coef, cur, mode, CR, jr, L, key, lb, ub, repair, err, col0=0, d_total=0):
    B = info.batch_size
    if any(d is not None for d in in_dims[9:11]) or in_dims[12] is not None:
        raise NotImplementedError("de_trial vmap rule: bounds and the error word must be shared by all runs")
    args = [_front(t, d, B) for t, d in zip((P, idx, coef, cur, mode, CR, jr, L, key), in_dims[:9])]
    return _ext.ops().de_trial(*args, lb, ub, repair, err, col0, d_total), 0


def register():
    """Install the rules (idempotent).  Without the compiled extension there is nothing to
    batch: CPU tensors never reach the HIP ops, and a device op raises on its own."""
    global _REGISTERED
    if _REGISTERED or not _ext.load(build_if_missing=False):
        return
    for name, fn in (("philox_words", _philox_words), ("philox_fill", _philox_fill), ("argsort_f32", _argsort_f32),
                     ("radix_argsort_f32", _radix_argsort_f32), ("rank_argsort_f32", _rank_argsort_f32), ("de_trial", _de_trial)):
        torch.library.register_vmap(f"evoxmi::{name}", fn)
    _REGISTERED = True
