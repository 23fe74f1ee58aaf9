"""Symmetric eigendecomposition (K4 of SURVEY §2.10).

CMA-ES at the north-star shape decomposes a 1000×1000 covariance **every
generation**.  The ROCm library ``syevd`` takes ≈23 ms for that on MI355X
(measured, ``profiles/probe_gpu.json``) — 10× the rest of the generation.  The
device path here is a **warm-started block Jacobi** solver
(``csrc/kernels/eigh_jacobi.hip``): the previous generation's eigenbasis ``B``
turns the new covariance into a nearly diagonal ``A = Bᵀ C B`` (two MFMA GEMMs),
block-Jacobi sweeps annihilate the small off-diagonal mass, and the accumulated
rotation ``V`` gives ``B_new = B V``.  Sweeps stop on a device-side convergence
flag, so the whole solve is graph-capturable (no host round trip).  It is truncated at
a fixed sweep count; the default ``sbr`` solver (:mod:`evoxmi.ops.sbr`) instead runs until
the relative off-norm reaches ``EVOXMI_EIGH_TOL`` every generation.
"""
from __future__ import annotations

import collections


import torch

from . import _ext


def eigh_reference(C: torch.Tensor):
    """Library eigendecomposition (ascending eigenvalues)."""
    w, V = torch.linalg.eigh(C)
    return w, V


def symmetrize_upper(C: torch.Tensor) -> torch.Tensor:
    """``triu(C) + triu(C, 1)ᵀ`` — the reference's symmetrisation (``cma_es.py:193-195``)."""
    U = torch.triu(C)
    return U + torch.triu(C, 1).T


# EigInfo of the most recent converged decompositions (host-side diagnostics for benches/monitors)
HISTORY = collections.deque(maxlen=4096)


def sbr_phase(C: torch.Tensor, B_prev: torch.Tensor, plans: dict = None):
    """Host phase of the converged solver: ``(w, B, stats)`` with stats =
    float64[off_rel, jacobi_sweeps, refine_iters, fallback] (evoxmi.ops.sbr)."""
    from .. import config
    from . import sbr

    w, B, info = sbr.eigh_warm(C, B_prev, sbr.SBRConfig(tol=config.get("eigh_tol"), block=config.get("sbr_block")), plans)
    HISTORY.append(info)
    st = torch.tensor([info.off_rel, info.jacobi_sweeps, info.refine_iters, float(info.fallback)], dtype=torch.float64)
    return w, B, st.to(C.device, non_blocking=True)


def warm_eigh(C: torch.Tensor, B_prev: torch.Tensor, max_sweeps: int = None, tol: float = None, plans: dict = None):
    """Eigen-decomposition of symmetric ``C`` warm-started from basis ``B_prev``.

    Returns ``(w, B)`` with ``C ≈ B diag(w) Bᵀ`` (eigenvalues not sorted).
    """
    from .. import config

    impl = config.get("eigh")
    if not C.is_cuda or impl in ("library", "torch"):
        return eigh_reference(C)
    if impl == "sbr":
        from ..runtime import host_phase

        w, B, _ = host_phase(sbr_phase, C, B_prev, plans, out_like=(C.new_empty(C.shape[0]), C, C.new_empty(4, dtype=torch.float64)))
        return w, B
    from . import jacobi

    return jacobi.warm_eigh(C, B_prev, max_sweeps=max_sweeps, tol=tol)
