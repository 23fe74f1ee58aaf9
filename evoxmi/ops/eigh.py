"""Symmetric eigendecomposition (K4 of SURVEY §2.10).

CMA-ES at the north-star shape decomposes a 1000×1000 covariance **every
generation**.  The ROCm library ``syevd`` takes ≈23 ms for that on MI355X
(measured, ``profiles/probe_gpu.json``) — 10× the rest of the generation.  The
device path here is a **warm-started block Jacobi** solver
(``csrc/kernels/eigh_jacobi.hip``): the previous generation's eigenbasis ``B``
turns the new covariance into a nearly diagonal ``A = Bᵀ C B`` (two MFMA GEMMs),
block-Jacobi sweeps annihilate the small off-diagonal mass, and the accumulated
rotation ``V`` gives ``B_new = B V``.  Sweeps stop on a device-side convergence
flag, so the whole solve is graph-capturable (no host round trip).
"""
from __future__ import annotations


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


def warm_eigh(C: torch.Tensor, B_prev: torch.Tensor, max_sweeps: int = None, tol: float = None):
    """Eigen-decomposition of symmetric ``C`` warm-started from basis ``B_prev``.

    Returns ``(w, B)`` with ``C ≈ B diag(w) Bᵀ`` (eigenvalues not sorted).
    """
    from .. import config

    impl = config.get("eigh")
    if not C.is_cuda or impl in ("library", "torch"):
        return eigh_reference(C)
    from . import jacobi

    return jacobi.warm_eigh(C, B_prev, max_sweeps=max_sweeps, tol=tol)
