"""Host orchestration of the block-Jacobi eigensolver (kernels: ``eigh_jacobi.hip``).

``warm_eigh(C, B_prev)``: pad to np = 16·nb (nb even; pad block = identity, which
never mixes with the real indices because its couplings are exact zeros), form
``A = B_padᵀ C_pad B_pad`` with two MFMA GEMMs, run tournament sweeps until the
device-side flag reports ‖offdiag(A)‖_F ≤ tol·‖diag(A)‖_F, and return
``(diag(A)[:n], B_pad[:n, :n])``.
"""
from __future__ import annotations

import functools

import torch

from . import _ext
from .linalg import matmul, matmul_tn

from .. import config

COLD_SWEEPS = 12
# (round 6: fixed here instead of EVOXMI_JACOBI_* knobs)
TOL_FACTOR = 4.0      # convergence: ‖offdiag‖ ≤ factor·eps_f32·sqrt(n)·‖diag‖
INNER_TOL = 1e-6      # per-subproblem skip threshold of the solve kernel
INNER = 1             # inner sweeps per 32×32 subproblem (2 / 3 do not speed the outer convergence)
REORTHO = True        # Newton–Schulz re-orthonormalisation of the warm-start basis
# round pipeline: 2 = B update of round t−1 inside round t's solve launch (default); 0 = split
# solve / apply launches; 1 = fused apply + next solve (bit-identical, 27 vs 17.4 µs per round)
FUSED = 2
# convergence is judged against the f32 floor of ‖offdiag‖/‖diag‖ ≈ eps·sqrt(n)
# (sweeps / tolerance / inner sweeps are evoxmi.config knobs: EVOXMI_JACOBI_*)


@functools.lru_cache(maxsize=16)
def _schedule_cpu(nb: int) -> torch.Tensor:
    """Row 0: the within-block phase pairing (0,1),(2,3),...; rows 1..nb−1: circle-method
    round robin of the nb blocks (pairs = consecutive entries)."""
    assert nb % 2 == 0
    rounds = [list(range(nb))]
    others = list(range(1, nb))
    for r in range(nb - 1):
        L = [0] + others[r:] + others[:r]
        row = []
        for i in range(nb // 2):
            row += [L[i], L[nb - 1 - i]]
        rounds.append(row)
    return torch.tensor(rounds, dtype=torch.int32)


def round_pairing(t: int, nb: int) -> list:
    """Row ``t`` of :func:`_schedule_cpu` in closed form — the formula the HIP kernels
    evaluate in registers (``round_blk`` in csrc/kernels/eigh_jacobi.hip) instead of
    loading the table: round 0 pairs (2P, 2P+1); round t ≥ 1 pairs (L[P], L[nb−1−P]) with
    L[0] = 0 and L[i] = ((i − 2 + t) mod (nb − 1)) + 1."""
    def blk(P, side):
        if t == 0:
            return 2 * P + side
        i = nb - 1 - P if side else P
        return 0 if i == 0 else (i - 2 + t) % (nb - 1) + 1

    return [blk(P, side) for P in range(nb // 2) for side in (0, 1)]


_DEV_SCHED = {}


def schedule(nb: int, device) -> torch.Tensor:
    k = (nb, str(device))
    if k not in _DEV_SCHED:
        _DEV_SCHED[k] = _schedule_cpu(nb).to(device)
    return _DEV_SCHED[k]


def padded_size(n: int) -> int:
    nb = -(-n // 16)
    nb += nb % 2
    return nb * 16


def reorthonormalize(B: torch.Tensor) -> torch.Tensor:
    """One Newton–Schulz step toward the nearest orthonormal matrix,
    ``B ← 1.5·B − 0.5·B(BᵀB)`` (two MFMA GEMMs, error e → ≈1.5e²).

    The eigenbasis is carried from generation to generation as a product of f32
    rotations, so its orthogonality error grows by ≈eps·sweeps·sqrt(n) per
    decomposition; restoring it first keeps ``A = BᵀCB`` similar to C."""
    from .linalg import Operand, gemm

    n = B.shape[0]
    B = B.contiguous()
    if config.get("plain_gemm") == "blas":
        return torch.addmm(B, B, B.t() @ B, beta=1.5, alpha=-0.5)
    if not B.is_cuda:
        X = gemm(Operand(B, rc=True), Operand(B, rc=True), n, n, n)
        return gemm(Operand(B), Operand(X), n, n, n, alpha=-0.5, beta=1.5, Cin=B)
    from .linalg import mm

    G = mm(B, B, ta=True, mode=1)  # BᵀB, symmetric: upper tiles only
    return mm(B, G, tb=True, alpha=-0.5, beta=1.5, Cin=B)


def _btcb(C: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """Bᵀ C B for symmetric C: framework GEMMs on the device (Bᵀ·C with C's rows, then a
    symmetric-output product), the GEMM oracle path on the CPU."""
    if C.is_cuda:
        from .linalg import mm

        return mm(mm(B, C, ta=True, tb=True), B, mode=1)
    return matmul_tn(B, matmul(C, B)).contiguous()


def warm_eigh(C: torch.Tensor, B_prev: torch.Tensor = None, max_sweeps: int = None, tol: float = None, return_stats: bool = False,
              fused: int = None):
    n = C.shape[0]
    np_ = padded_size(n)
    dev = C.device
    eye_pad = torch.eye(np_ - n, device=dev)
    Cp = torch.zeros(np_, np_, device=dev)
    Cp[:n, :n] = C
    Cp[n:, n:] = eye_pad
    Bp = torch.zeros(np_, np_, device=dev)
    if B_prev is None:
        Bp.fill_diagonal_(1.0)
        A = Cp
        sweeps = COLD_SWEEPS if max_sweeps is None else max_sweeps
    else:
        Bp[:n, :n] = reorthonormalize(B_prev) if REORTHO else B_prev
        Bp[n:, n:] = eye_pad
        if config.get("plain_gemm") == "blas":
            A = (Bp.t() @ (Cp @ Bp)).contiguous()
        else:
            A = _btcb(Cp, Bp)
        sweeps = config.get("jacobi_sweeps") if max_sweeps is None else max_sweeps
    tol = tol or TOL_FACTOR * 1.1920929e-07 * max(n, 16) ** 0.5
    w, stats = _ext.ops().jacobi_sweeps(A, Bp, schedule(np_ // 16, dev), int(sweeps), float(tol),
                                        float(INNER_TOL), int(INNER), int(FUSED if fused is None else fused))
    out = (w[:n].contiguous(), Bp[:n, :n].contiguous())
    return (*out, stats) if return_stats else out


def warm_eigh_padded(Cp: torch.Tensor, Bp: torch.Tensor, n: int, max_sweeps: int = None, tol: float = None, fused: int = None):
    """``warm_eigh`` on operands that are already padded to ``padded_size(n)`` with an
    identity block (``Cp`` symmetric; ``Bp`` the previous basis, e.g. from the fused
    CMA-ES epilogue).  Returns ``(w_padded, Bp_rotated)``; the first ``n`` entries /
    the leading n×n block are the decomposition of the unpadded matrix."""
    np_ = Cp.shape[0]
    assert np_ == padded_size(n) and Bp.shape == Cp.shape
    if REORTHO:
        # Newton–Schulz on the padded basis: the identity block is a fixed point
        Bp = torch.addmm(Bp, Bp, Bp.t() @ Bp, beta=1.5, alpha=-0.5) if config.get("plain_gemm") == "blas" else reorthonormalize(Bp)
    if config.get("plain_gemm") == "blas":
        A = (Bp.t() @ (Cp @ Bp)).contiguous()
    else:
        A = _btcb(Cp, Bp)
    Bp = Bp.contiguous()
    sweeps = config.get("jacobi_sweeps") if max_sweeps is None else max_sweeps
    tol = tol or TOL_FACTOR * 1.1920929e-07 * max(n, 16) ** 0.5
    w, _ = _ext.ops().jacobi_sweeps(A, Bp, schedule(np_ // 16, Cp.device), int(sweeps), float(tol),
                                    float(INNER_TOL), int(INNER), int(FUSED if fused is None else fused))
    return w, Bp


def eigh(C: torch.Tensor, max_sweeps: int = None):
    """Cold-start symmetric eigendecomposition on the GPU (eigenvalues ascending)."""
    w, V = warm_eigh(C, None, max_sweeps=max_sweeps)
    order = torch.argsort(w)
    return w[order], V[:, order]
