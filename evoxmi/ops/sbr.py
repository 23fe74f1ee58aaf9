"""Converged per-generation eigendecomposition for CMA-ES: sorted-block refinement (K4).

Why not plain Jacobi.  The reference decomposes C with ``jnp.linalg.eigh`` every
generation at the north-star shape (``cma_es.py:155-160,193-198``; decomp_per_iter = 1
at d = 1000, λ = 10⁴).  Warm-started from the previous eigenbasis B, A = Bᵀ C B is
nearly diagonal, but the rank-μ perturbation (entries ≈1e-4) is as large as the
eigenvalue gaps (≈1e-4), so eigenvectors mix over windows of ~60 neighbours every
generation and cyclic Jacobi converges only linearly (≈0.5× per 1.1 ms sweep; 2 sweeps
left a 5e-4 residual in round 1, profiles/r1_jacobi_convergence_probe.log).

Sorted-block refinement (SBR, ``csrc/kernels/eigh_sbr.hip``).  One iteration
  1. sorts diag(A), cuts the sorted order into 64-blocks (offset 0 / 32 alternately) and
     diagonalises each block with two cyclic Jacobi sweeps (near, clustered pairs;
     ``sbr_block2_kernel``: double-buffered S, one barrier per round, Q in registers);
  2. builds the rotation generator X_ij = ½·atan(2·A1_ij / (d_j − d_i)) (the exact 2×2
     Jacobi angle, = A1_ij / (d_j − d_i) to first order) for pairs in different blocks
     whose gap exceeds ``thr_fac·32·spread/n`` (far pairs);
  3. caps the step at ‖αX‖₂ ≤ 1 while κ is large (``damping``: 3 block power steps on
     −X²), V = exp(αX) (Paterson–Stockmeyer Taylor, 3 GEMMs), B ← B[:, perm]·Qblk·V,
     Newton–Schulz re-orthonormalisation after large steps, A ← Bᵀ C B (plain GEMMs).
Far pairs converge quadratically once the step is small, so 4 iterations take the
relative off-norm from 3e-3 to ≤1e-5 in steady state.  Early generations (C ≈ I) start
from a basis whose couplings are as large as the spectral spread (κ = ‖offdiag A‖_F /
(max diag − min diag) up to ~4): the undamped step diverges there (‖X‖₂ ≈ 2–7), the
damped one contracts (generation 1: 9 iterations, generation 4: 6; measured on CMA-ES
matrices at d = 1000).  If an iteration ever increases the off-norm the solver restores
the basis and finishes with block-Jacobi sweeps (``eigh_jacobi.hip``), so every
generation ends converged (``EigInfo.off_rel``).

Everything here is host-orchestrated (a few ``.item()`` reads of the device stats per
generation): StdWorkflow's hipGraph capture runs it as a *host phase* between graph
segments (``evoxmi.runtime.segments``).
"""
from __future__ import annotations

import functools
import math
from dataclasses import dataclass, field
from typing import List

import torch

from . import _ext
from .linalg import mm

BK = 64


def block_starts(n: int, off: int) -> List[int]:
    starts = ([0] + list(range(off, n, BK))) if off else list(range(0, n, BK))
    return starts + [n]


def nblocks(n: int, off: int) -> int:
    return len(block_starts(n, off)) - 1


# ---------------------------------------------------------------------------- reference
@functools.lru_cache(maxsize=None)
def _rr_rounds(m: int = BK):
    """Circle-method round robin on m slots: round r pairs (m−1, r) and
    ((r+i) mod (m−1), (r−i) mod (m−1)), i = 1..m/2−1 — the kernel's pairing."""
    out = []
    for r in range(m - 1):
        pairs = [(m - 1, r)] + [((r + i) % (m - 1), (r - i) % (m - 1)) for i in range(1, m // 2)]
        out.append((torch.tensor([min(a, b) for a, b in pairs]), torch.tensor([max(a, b) for a, b in pairs])))
    return out


def _block_jacobi_ref(S: torch.Tensor, sweeps: int):
    nb, m, _ = S.shape
    Q = torch.eye(m, dtype=S.dtype, device=S.device).repeat(nb, 1, 1)
    ar = torch.arange(nb, device=S.device)[:, None]
    fmin = torch.finfo(torch.float32).tiny
    for _ in range(sweeps):
        for p, q in _rr_rounds(m):
            p = p.to(S.device)
            q = q.to(S.device)
            app, aqq, apq = S[:, p, p], S[:, q, q], S[:, p, q]
            rot = apq.abs() >= fmin
            theta = (aqq - app) / (2 * torch.where(rot, apq, torch.ones_like(apq)))
            t = torch.where(theta >= 0, 1.0, -1.0) / (theta.abs() + torch.sqrt(theta * theta + 1))
            t = torch.where(rot, t, torch.zeros_like(t))
            c = torch.rsqrt(t * t + 1)
            s = t * c
            # S' = Jᵀ S J, Q' = Q J with J = [[c, s], [−s, c]] on every (p, q): row then column
            # updates of the 32 disjoint pairs (index form of the dense product)
            cb, sb = c[:, :, None], s[:, :, None]
            Sp, Sq = S[:, p, :], S[:, q, :]
            S = S.clone()
            S[:, p, :], S[:, q, :] = cb * Sp - sb * Sq, sb * Sp + cb * Sq
            Sp, Sq = S[:, :, p], S[:, :, q]
            cr, sr = c[:, None, :], s[:, None, :]
            S[:, :, p], S[:, :, q] = cr * Sp - sr * Sq, sr * Sp + cr * Sq
            S[ar, p, p] = app - t * apq
            S[ar, q, q] = aqq + t * apq
            S[ar, p, q] = 0
            S[ar, q, p] = 0
            Qp, Qq = Q[:, :, p], Q[:, :, q]
            Q = Q.clone()
            Q[:, :, p], Q[:, :, q] = cr * Qp - sr * Qq, sr * Qp + cr * Qq
    return S, Q


def stats_ref(A: torch.Tensor) -> torch.Tensor:
    d = torch.diagonal(A).double()
    off = (A.double() ** 2).sum() - (d**2).sum()
    return torch.stack([off, (d**2).sum(), d.min(), d.max()])


def block_solve_ref(A: torch.Tensor, off: int, sweeps: int):
    n = A.shape[0]
    d = torch.diagonal(A)
    perm = torch.argsort(d, stable=True).to(torch.int32)
    st = block_starts(n, off)
    nb = len(st) - 1
    S = torch.zeros(nb, BK, BK, dtype=A.dtype, device=A.device)
    for k in range(nb):
        idx = perm[st[k] : st[k + 1]].long()
        m = idx.numel()
        S[k, :m, :m] = A[idx][:, idx]
    S, Q = _block_jacobi_ref(S, sweeps)
    dq = torch.cat([torch.diagonal(S[k])[: st[k + 1] - st[k]] for k in range(nb)])
    return perm, Q.contiguous(), dq


def _blockdiag(Q: torch.Tensor, n: int, off: int) -> torch.Tensor:
    st = block_starts(n, off)
    Qf = torch.zeros(n, n, dtype=Q.dtype, device=Q.device)
    for k in range(len(st) - 1):
        m = st[k + 1] - st[k]
        Qf[st[k] : st[k + 1], st[k] : st[k + 1]] = Q[k, :m, :m]
    return Qf


def far_ref(A, off, perm, Q, dq, stats, thr_fac):
    n = A.shape[0]
    p = perm.long()
    Qf = _blockdiag(Q, n, off)
    A1 = Qf.T @ A[p][:, p] @ Qf
    st = block_starts(n, off)
    blk = torch.zeros(n, dtype=torch.long, device=A.device)
    for k in range(len(st) - 1):
        blk[st[k] : st[k + 1]] = k
    den = dq[None, :] - dq[:, None]
    thr = thr_fac * (0.5 * BK) * float(stats[3] - stats[2]) / n
    mask = (blk[None, :] != blk[:, None]) & (den.abs() > thr)
    # the 2×2 Jacobi angle ½·atan(2a/den): first-order a/den for separated pairs, ≤ π/4
    return torch.where(mask, 0.5 * torch.atan(2 * A1 / torch.where(mask, den, torch.ones_like(den))), torch.zeros_like(A1))


def bq_ref(B, off, perm, Q):
    return B[:, perm.long()] @ _blockdiag(Q, B.shape[1], off)


# ------------------------------------------------- 16-wide blocks, shifted sorted order
# (csrc/kernels/eigh_sbr16.hip): position j of the order is index argsort(diag)[(j + shift)
# mod n] and blocks are always [16k, 16k + 16) — shift 0 / 8 on alternate iterations.
SB = 16


def perm_shift_ref(A: torch.Tensor, shift: int) -> torch.Tensor:
    d = torch.diagonal(A)
    d = torch.where(torch.isnan(d), torch.full_like(d, float("inf")), d)
    perm = torch.argsort(d, stable=True).to(torch.int32)
    return torch.roll(perm, -(shift % A.shape[0]))


SHIFT_BLOCKS = (16, 32)  # block sizes of the shifted layout (eigh_sbr16.hip templates)


def block_solve16_ref(A: torch.Tensor, shift: int, sweeps: int, sb: int = SB):
    n = A.shape[0]
    perm = perm_shift_ref(A, shift)
    nb = (n + sb - 1) // sb
    S = torch.zeros(nb, sb, sb, dtype=A.dtype, device=A.device)
    for k in range(nb):
        idx = perm[k * sb : (k + 1) * sb].long()
        m = idx.numel()
        S[k, :m, :m] = A[idx][:, idx]
    S, Q = _block_jacobi_ref(S, sweeps)
    dq = torch.diagonal(S, dim1=1, dim2=2).reshape(-1)[:n]
    return perm, Q.contiguous(), dq.contiguous()


def _blockdiag16(Q: torch.Tensor, n: int) -> torch.Tensor:
    return torch.block_diag(*Q.unbind(0))[:n, :n]


# local threshold factor of the far mask: 0 (global threshold only) by default; the driver
# switches it on for the rest of a solve when a far iteration stalls (pairs in clusters
# denser than the global threshold assumes are then neither in a block nor far)
LOCAL_THETA = 0.0


def local_threshold(dq: torch.Tensor, theta: float = None, sb: int = SB) -> torch.Tensor:
    """θ·min(|d[j+8] − d[j]|, |d[j] − d[j−8]|) at every position j of the order.  A pair whose
    gap is below both ends' local thresholds is less than half a block apart, so one of
    the two shifts puts it in a common block: every pair is either rotated by a block solve
    or by the far step, even inside clusters denser than the global threshold assumes."""
    theta = LOCAL_THETA if theta is None else theta
    n = dq.shape[0]
    h = sb // 2
    inf = torch.full((h,), float("inf"), dtype=dq.dtype, device=dq.device)
    up = torch.cat([(dq[h:] - dq[:-h]).abs(), inf]) if n > h else torch.full_like(dq, float("inf"))
    dn = torch.cat([inf, (dq[h:] - dq[:-h]).abs()]) if n > h else torch.full_like(dq, float("inf"))
    return theta * torch.minimum(up, dn)


def far16_ref(A, perm, Q, dq, stats, thr_fac, theta: float = None):
    theta = LOCAL_THETA if theta is None else theta
    sb = Q.shape[1]
    n = A.shape[0]
    p = perm.long()
    Qf = _blockdiag16(Q, n)
    A1 = Qf.T @ A[p][:, p] @ Qf
    blk = torch.arange(n, device=A.device) // sb
    den = dq[None, :] - dq[:, None]
    thr = thr_fac * (0.5 * sb) * float(stats[3] - stats[2]) / n
    thr = torch.full_like(dq, thr)
    if theta > 0:
        thr = torch.minimum(thr, local_threshold(dq, theta, sb))
    mask = (blk[None, :] != blk[:, None]) & (den.abs() > torch.minimum(thr[:, None], thr[None, :]))
    return torch.where(mask, 0.5 * torch.atan(2 * A1 / torch.where(mask, den, torch.ones_like(den))), torch.zeros_like(A1))


def bq16_ref(B, perm, Q):
    return B[:, perm.long()] @ _blockdiag16(Q, B.shape[1])


# ---------------------------------------------------------------------------- dispatch
def _dev(t):
    return t.is_cuda


def _rowmajor(t):
    return t if t.stride(-1) == 1 else t.contiguous()


def stats(A):
    return _ext.ops().sbr_stats(_rowmajor(A)) if _dev(A) else stats_ref(A)


def block_solve(A, off, sweeps, bk: int = BK):
    if bk in SHIFT_BLOCKS:
        if _dev(A):
            return tuple(_ext.ops().sbr16_block(_rowmajor(A), int(off) % A.shape[0], int(sweeps), int(bk)))
        return block_solve16_ref(A, off, sweeps, bk)
    if _dev(A):
        perm, Q, dq = _ext.ops().sbr_block(_rowmajor(A), int(off), int(sweeps))
        return perm, Q, dq
    return block_solve_ref(A, off, sweeps)


def far(A, off, perm, Q, dq, st, thr_fac, bk: int = BK, theta: float = None):
    theta = LOCAL_THETA if theta is None else theta
    if bk in SHIFT_BLOCKS:
        if _dev(A):
            return _ext.ops().sbr16_far(_rowmajor(A), perm, Q, dq, st, float(thr_fac), float(theta))
        return far16_ref(A, perm, Q, dq, st, thr_fac, theta)
    if _dev(A):
        return _ext.ops().sbr_far(_rowmajor(A), int(off), perm, Q, dq, st, float(thr_fac))
    return far_ref(A, off, perm, Q, dq, st, thr_fac)


def bq(B, off, perm, Q, bk: int = BK):
    if bk in SHIFT_BLOCKS:
        return _ext.ops().sbr16_bq(_rowmajor(B), perm, Q) if _dev(B) else bq16_ref(B, perm, Q)
    return _ext.ops().sbr_bq(_rowmajor(B), int(off), perm, Q) if _dev(B) else bq_ref(B, off, perm, Q)


def expm_taylor6(X: torch.Tensor, X2: torch.Tensor = None, alpha: torch.Tensor = None) -> torch.Tensor:
    """exp(αX) to 6th order with 3 GEMMs (Paterson–Stockmeyer), Y = αX:
    I + Y + Y²/2 + Y³/6 + Y³(Y/24 + Y²/120 + Y³/720).  ``alpha`` is a 1-element device
    tensor (no host sync), folded into the elementwise prep."""
    if X.is_cuda:
        X2 = mm(X, X, tb=True, mode=1, alpha=-1.0) if X2 is None else X2
        X3 = mm(X2, X, tb=True, mode=2, alpha=-1.0)
        P, M = _ext.ops().sbr_taylor_prep(X.contiguous(), X2, X3, alpha)
        return mm(X3, P, beta=1.0, Cin=M, out=M)  # in place: no copy of M into a fresh output
    X2 = X @ X if X2 is None else X2
    X3 = X2 @ X
    a = 1.0 if alpha is None else alpha.reshape(())
    Y, Y2, Y3 = a * X, (a * a) * X2, (a * a * a) * X3
    P = Y / 24 + Y2 / 120 + Y3 / 720
    V = Y3 @ P
    V += Y + Y2 / 2 + Y3 / 6
    V.diagonal().add_(1.0)
    return V


def expm_taylor4(X: torch.Tensor, X2: torch.Tensor, alpha: torch.Tensor = None) -> torch.Tensor:
    """exp(αX) to 4th order with one GEMM on top of X² (Paterson–Stockmeyer), Y = αX:
    I + Y + Y²/2 + Y²(Y/6 + Y²/24).  Orthogonal to ‖Y‖⁵/120: used where
    ‖Y‖ is small (κ below ``SBRConfig.t4_kappa``)."""
    if X.is_cuda:
        P, M = _ext.ops().sbr_taylor4_prep(X.contiguous(), X2, alpha)
        return mm(X2, P, beta=1.0, Cin=M, out=M)
    a = 1.0 if alpha is None else alpha.reshape(())
    Y, Y2 = a * X, (a * a) * X2
    V = Y2 @ (Y / 6 + Y2 / 24)
    V += Y + Y2 / 2
    V.diagonal().add_(1.0)
    return V


def expm_t_device(X: torch.Tensor, X2: torch.Tensor, alpha: torch.Tensor = None, order: int = 6) -> torch.Tensor:
    """Vᵀ = exp(αX)ᵀ = exp(−αX) on the device, every product an A·Bᵀ GEMM on row-major
    operands (gemm_ks K-contiguous loads): with P = P(α) of the Taylor prep and
    M(−α) (the prep's ``mt`` flag, odd terms negated), Pᵀ(α) = −P(−α) for order 6 and
    +P(−α) for order 4 (X skew), so

        order 6:  Vᵀ = M(−α) − X³·P(α)ᵀ      (X³ = X²·X = −X²·Xᵀ, skew: upper tiles only)
        order 4:  Vᵀ = M(−α) + X²·P(α)ᵀ

    and the basis update B·V = B·(Vᵀ)ᵀ reads Vᵀ's rows too."""
    ops = _ext.ops()
    if order == 6:
        X3 = mm(X2, X, tb=True, mode=2, alpha=-1.0)
        P, MT = ops.sbr_taylor_prep(X.contiguous(), X2, X3, alpha, 1)
        return mm(X3, P, tb=True, alpha=-1.0, beta=1.0, Cin=MT, out=MT)
    P, MT = ops.sbr_taylor4_prep(X.contiguous(), X2, alpha, 1)
    return mm(X2, P, tb=True, alpha=1.0, beta=1.0, Cin=MT, out=MT)


@functools.lru_cache(maxsize=8)
def _probe_vectors(n: int, dev: str) -> torch.Tensor:
    i = torch.arange(n, dtype=torch.float64)[:, None]
    j = torch.arange(8, dtype=torch.float64)[None, :]
    return torch.cos(0.7 * i * (j + 1) + j).to(device=dev, dtype=torch.float32).contiguous()


def damping(X2: torch.Tensor, tau: float, out: torch.Tensor = None) -> torch.Tensor:
    """α = min(1, τ / ‖X‖₂) for the skew generator X, with ‖X‖₂² = λmax(−X²) estimated
    by three block power steps on 8 fixed probe vectors (device-only, graph-capturable).

    Early generations (C ≈ I) warm-start from a basis whose far couplings are as large as
    the spectral spread: the undamped generator has ‖X‖₂ ≈ 2–7 and the step diverges;
    capping ‖αX‖₂ at τ = 1 turns it into a contraction (measured: generation 1 converges
    in 10 iterations instead of needing block-Jacobi sweeps first)."""
    V = _probe_vectors(X2.shape[0], str(X2.device))
    if X2.is_cuda:
        return _ext.ops().sbr_damping(_rowmajor(X2), V, float(tau), out)
    V1 = -(X2 @ V)
    V2 = -(X2 @ V1)
    V3 = -(X2 @ V2)
    lam = (torch.linalg.vector_norm(V3, dim=0) / torch.linalg.vector_norm(V2, dim=0).clamp_min(1e-30)).max()
    return torch.clamp(tau / torch.sqrt(lam.clamp_min(1e-30)), max=1.0).reshape(1).to(torch.float32)


def newton_schulz(B: torch.Tensor, out: torch.Tensor = None) -> torch.Tensor:
    """One step toward the nearest orthonormal matrix, B(1.5 I − 0.5 BᵀB)."""
    if B.is_cuda:
        G = mm(B, B, ta=True, mode=1)  # BᵀB: symmetric, upper tiles only
        return mm(B, G, tb=True, alpha=-0.5, beta=1.5, Cin=B, out=out)
    return torch.addmm(B, B, B.t() @ B, beta=1.5, alpha=-0.5)


def _btcb_device(C: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """Bᵀ C B on the device as two framework GEMMs: W = Bᵀ·C (C symmetric: its rows are
    read K-contiguous) and T = W·B with a symmetric output (upper tiles only)."""
    W = mm(B, C, ta=True, tb=True)
    return mm(W, B, mode=1)


def sym_product(C: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """A = Bᵀ C B, symmetrised."""
    if C.is_cuda:
        return _btcb_device(C, B)
    A = B.t() @ (C @ B)
    return (A + A.t()) * 0.5


def sym_product_stats(C: torch.Tensor, B: torch.Tensor):
    """(A = sym(Bᵀ C B), stats(A)); on the device symmetrisation and stats are one kernel."""
    if C.is_cuda:
        A, st = _ext.ops().sbr_symstats(_btcb_device(C, B))
        return A, st
    T = B.t() @ (C @ B)
    A = (T + T.t()) * 0.5
    return A, stats_ref(A)


# ---------------------------------------------------------------------------- driver
@dataclass
class EigInfo:
    off_rel: float = float("nan")
    jacobi_sweeps: int = 0
    refine_iters: int = 0
    kappa0: float = float("nan")
    fallback: bool = False
    damped: int = 0            # iterations whose step was capped (α < 1)
    history: list = field(default_factory=list)


@dataclass
class SBRConfig:
    tol: float = 1e-5          # relative off-norm ‖offdiag‖_F / ‖diag‖_F to reach
    kappa_max: float = math.inf  # optional hand-off from Jacobi sweeps to refinement (the
                                 # damped generator converges from any warm start)
    max_iters: int = 16
    damp_tau: float = 1.0      # cap on ‖αX‖₂ (0: undamped)
    ns_kappa: float = 0.3      # Newton–Schulz also while κ exceeds this (large undamped steps
                               # early in a cold start: Taylor-6 loses orthogonality at ‖X‖₂ ≈ 1)
    t4_kappa: float = 0.05     # Taylor-4 exponential once κ is below this (‖X‖₂ small)
    damp_kappa: float = 1.0    # estimate ‖X‖₂ in the first iteration and while κ exceeds this
                               # (steady-state CMA-ES: κ ≈ 1.3 → 0.45 → 0.1: only iteration 0)
    near_only: float = 3.0     # near-only (no far step) iteration once off_rel ≤ near_only·tol
    theta0: float = 0.0        # local far threshold factor once κ ≤ theta_kappa (0: after a stall only)
    theta_kappa: float = 0.05
    max_jacobi: int = 16
    block_sweeps: int = 2
    block: int = 32            # 16 / 32: blocks in a shifted sorted order (eigh_sbr16.hip; 16 = one
                               # wave per block, 32 = four); 64: the 64-wide offset layout (eigh_sbr.hip)
    thr_fac: float = None      # far-pair threshold factor (default 0.3)
    ns_iters: int = 2          # Newton–Schulz re-orthonormalisation in the first iterations and
                               # after every damped one (undamped later ones have ‖X‖₂ ≲ 0.5:
                               # Taylor-6 is orthogonal to ~1e-6 there)
    graphs: bool = True        # replay each device iteration as a captured hipGraph
    plan: bool = True          # graphs: replay the previous solve's iteration sequence, one stats read

    def __post_init__(self):
        if self.thr_fac is None:
            self.thr_fac = 0.3
        if self.block not in SHIFT_BLOCKS + (BK,):
            raise ValueError(f"SBR block size must be one of {SHIFT_BLOCKS + (BK,)}, got {self.block}")


def _read(st: torch.Tensor):
    """(off_rel, κ[, α]) from [off², diag², dmin, dmax(, α)] (one device→host copy)."""
    v = [float(x) for x in st.cpu()]
    off, dg, mn, mx = v[:4]
    off_rel = math.sqrt(max(off, 0.0) / dg) if dg > 0 else float("nan")
    kappa = math.sqrt(max(off, 0.0)) / (mx - mn) if mx > mn else float("inf")
    return (off_rel, kappa) if len(v) == 4 else (off_rel, kappa, v[4])


def _refine_core(C, A, B, st, off: int, ns: bool, damp: bool, cfg: SBRConfig, out=None, far_on: bool = True,
                 theta: float = None, order: int = 6):
    """One iteration; returns (A, B, stats, α).  ``out = (A, B, st, α)`` static buffers to
    write the results into (the workspace graphs: no copies; ``st`` may be a row of the
    stats history).  ``damp``: estimate ‖X‖₂ and cap the step (the host enables it while κ
    is large).  ``far_on = False``: a near-only iteration (block solves, B ← B[:, perm]·Qblk,
    A ← BᵀCB) for the last step, when the residual is almost entirely near pairs (4 GEMMs
    fewer)."""
    perm, Q, dq = block_solve(A, off, cfg.block_sweeps, cfg.block)
    alpha = None
    dev = A.is_cuda
    if not far_on:
        Bn = bq(B, off, perm, Q, cfg.block)
        if out:
            out[1].copy_(Bn)
            Bn = out[1]
    else:
        X = far(A, off, perm, Q, dq, st, cfg.thr_fac, cfg.block, theta)
        # X is skew: X² = −X·Xᵀ is symmetric (upper tiles only)
        X2 = mm(X, X, tb=True, mode=1, alpha=-1.0) if dev else X @ X
        if damp and cfg.damp_tau > 0:
            alpha = damping(X2, cfg.damp_tau, out=out[3] if out else None)
        Bq = bq(B, off, perm, Q, cfg.block)
        if dev:
            # every product A·Bᵀ on row-major operands: Bq·V = Bq·(Vᵀ)ᵀ (expm_t_device)
            VT = expm_t_device(X, X2, alpha, order)
            if ns:
                Bn = mm(Bq, VT, tb=True)
                Bn = newton_schulz(Bn, out=out[1] if out else None)
            else:
                Bn = mm(Bq, VT, tb=True, out=out[1] if out else None)
        else:
            V = expm_taylor6(X, X2, alpha) if order == 6 else expm_taylor4(X, X2, alpha)
            Bn = newton_schulz(Bq @ V) if ns else Bq @ V
    if out and dev:
        _ext.ops().sbr_symstats_out(_btcb_device(C, Bn), out[0], out[2])
        A, st = out[0], out[2]
    else:
        A, st = sym_product_stats(C, Bn)
    if alpha is None:
        alpha = out[3] if out else torch.ones(1, device=Bn.device)
    return A, Bn, st, alpha


def refine_step(C, A, B, st, it: int, cfg: SBRConfig, ns: bool = None, damp: bool = True, far_on: bool = True,
                theta: float = None, order: int = 6):
    ns = it < cfg.ns_iters if ns is None else ns
    return _refine_core(C, A, B, st, (it % 2) * (cfg.block // 2), ns, damp, cfg, far_on=far_on, theta=theta, order=order)


def decide(cfg: SBRConfig, it: int, off_rel: float, kappa: float, alpha_prev: float, last_far: bool, theta: float) -> tuple:
    """Flags of refinement iteration ``it`` from the stats before it: (Newton–Schulz, damping,
    far step, local-threshold θ, Taylor order)."""
    # re-orthonormalise in the first iterations, after a damped (large) step and while κ is
    # large; the ‖X‖₂ estimate runs in iteration 0 and while κ is very large
    ns = it < cfg.ns_iters or alpha_prev < 1.0 or kappa > cfg.ns_kappa
    damp = it == 0 or kappa > cfg.damp_kappa
    # close to the tolerance the residual is near pairs only: skip the far step (once: if a
    # near-only iteration did not reach the tolerance, far pairs are left)
    far_on = not (it > 0 and off_rel <= cfg.near_only * cfg.tol and last_far)
    # Taylor-4 (one GEMM fewer) only for small steps: a damped ‖αX‖₂ ≈ 1 step loses ~1e-2 of
    # orthogonality at 4th order, more than one Newton–Schulz step repairs
    order = 4 if kappa < cfg.t4_kappa else 6
    # the local far threshold from the start once the step is undamped (the device schedule's
    # rule, eigh_sbr_dev.hip)
    if cfg.theta0 > 0 and kappa <= cfg.theta_kappa:
        theta = max(theta, cfg.theta0)
    return (ns, damp, far_on, theta, order)


class _Workspace:
    """Static device buffers + captured hipGraphs of the refinement iteration (one per
    (iteration index, block offset, flags) variant) and of the initial Bᵀ C B.  Iteration
    j reads its stats from row j of ``hist`` and writes row j + 1 (and its step size to
    ``alpha[j + 1]``), so a planned solve is a chain of graph launches with no copies and
    a single device→host read at the end."""

    def __init__(self, n: int, dev, cfg: SBRConfig):
        self.n, self.cfg = n, cfg
        z = lambda: torch.zeros(n, n, device=dev)  # noqa: E731
        self.C, self.A, self.B = z(), z(), z()
        self.hist = torch.zeros(cfg.max_iters + 1, 4, dtype=torch.float64, device=dev)
        self.alpha = torch.ones(cfg.max_iters + 1, dtype=torch.float32, device=dev)
        self.graphs = {}
        self.pool = torch.cuda.graph_pool_handle()  # graphs replay one at a time: one memory pool
        self.warm = False

    def precapture(self, n_iters: int = 9):
        """Capture the iteration variants of the first tens of generations up front
        (iteration j: Newton–Schulz always for j < 2 and optionally later, damping at j = 0,
        with and without the far step, Taylor order 6 for j < 2 and 4 / 6 later) so plan
        changes replay existing graphs instead of capturing new ones mid-run.  Capture
        warm-ups leave the buffers unchanged (``_capture``)."""
        for j in range(min(n_iters, self.cfg.max_iters)):
            for ns in ((True,) if j < self.cfg.ns_iters else (True, False)):
                for far_on in ((True, False) if j > 0 else (True,)):
                    for order in ((6,) if j < 2 else (4, 6)):
                        self.iterate(j, ns, j == 0, far_on, 0.0, order, replay=False)
        self.warm = True

    def _capture(self, key, body):
        if key not in self.graphs:
            # the bodies update A / B / hist / alpha in place: the warm-up run must not
            # count as an iteration, so the buffers are restored before capturing
            saved = [t.clone() for t in (self.A, self.B, self.hist, self.alpha)]
            s = torch.cuda.Stream(device=self.C.device)
            s.wait_stream(torch.cuda.current_stream(self.C.device))
            with torch.cuda.stream(s):  # warm-up (allocator, lazy init) outside the capture
                body()
                for t, v in zip((self.A, self.B, self.hist, self.alpha), saved):
                    t.copy_(v)
            torch.cuda.current_stream(self.C.device).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s, pool=self.pool):
                body()
            self.graphs[key] = g
        return self.graphs[key]

    def init(self):
        # no re-orthonormalisation here: iteration 0 always applies Newton–Schulz to its result
        def body():
            _ext.ops().sbr_symstats_out(_btcb_device(self.C, self.B), self.A, self.hist[0])
            self.alpha.fill_(1.0)

        self._capture(("init",), body).replay()

    def _body(self, it: int, ns: bool, damp: bool, far_on: bool, theta: float, order: int):
        off = (it % 2) * (self.cfg.block // 2)
        j = min(it, self.cfg.max_iters - 1)

        def body():
            # A, B are written in place (fully read before the last GEMM/kernel of the
            # iteration overwrites them); stats row j → row j + 1
            _refine_core(self.C, self.A, self.B, self.hist[j], off, ns, damp, self.cfg,
                         out=(self.A, self.B, self.hist[j + 1], self.alpha[j + 1 : j + 2]), far_on=far_on, theta=theta,
                         order=order)

        return ("it", j, off, ns, damp, far_on, theta, order), body

    def iterate(self, it: int, ns: bool, damp: bool, far_on: bool = True, theta: float = 0.0, order: int = 6,
                replay: bool = True):
        key, body = self._body(it, ns, damp, far_on, theta, order)
        g = self._capture(key, body)
        if replay:
            g.replay()

    def run_plan(self, plan):
        """The iterations of a plan, one graph launch each.  (One graph per plan would save
        ≈8 µs of launch gap per iteration, but plans keep changing in the first tens of
        generations and a capture costs ≈2.7 ms: measured as a net loss over 50
        generations, profiles/NOTES.md.)"""
        for j, stp in enumerate(plan):
            k, b = self._body(j, *stp)
            self._capture(k, b).replay()

    def read(self, it: int):
        """(off_rel, κ, α) after iteration ``it`` (−1: the initial product)."""
        return _decode(list(self.hist[it + 1].cpu()) + [float(self.alpha[it + 1])])

    def read_all(self, k: int):
        h = torch.cat([self.hist[: k + 1], self.alpha[: k + 1, None].double()], 1).cpu()
        return [_decode(r) for r in h]


_WS = {}


def _workspace(n, dev, cfg) -> _Workspace:
    k = (n, str(dev), cfg.block, cfg.block_sweeps, cfg.thr_fac, cfg.ns_iters, cfg.damp_tau)
    if k not in _WS:
        _WS[k] = _Workspace(n, dev, cfg)
    return _WS[k]


def _jacobi_sweep(A, B, tol):
    """One block-Jacobi sweep on padded copies of (A, B); returns unpadded (A, B)."""
    from . import jacobi

    n = A.shape[0]
    np_ = jacobi.padded_size(n)
    dev = A.device
    Ap = torch.zeros(np_, np_, device=dev)
    Bp = torch.zeros(np_, np_, device=dev)
    Ap[:n, :n] = A
    Bp[:n, :n] = B
    if np_ > n:
        Ap[n:, n:] = torch.eye(np_ - n, device=dev)
        Bp[n:, n:] = torch.eye(np_ - n, device=dev)
    _ext.ops().jacobi_sweeps(Ap, Bp, jacobi.schedule(np_ // 16, dev), 1, float(tol), float(jacobi.INNER_TOL), int(jacobi.INNER),
                             int(jacobi.FUSED))
    return Ap[:n, :n].contiguous(), Bp[:n, :n].contiguous()


_PLANS = {}


def _decode(row) -> tuple:
    """(off_rel, κ, α) of a history row [off², diag², dmin, dmax, α]."""
    off, dg, mn, mx, a = (float(x) for x in row)
    off_rel = math.sqrt(max(off, 0.0) / dg) if dg > 0 else float("nan")
    kappa = math.sqrt(max(off, 0.0)) / (mx - mn) if mx > mn else float("inf")
    return off_rel, kappa, a


def eigh_warm(C: torch.Tensor, B_prev: torch.Tensor, cfg: SBRConfig = None, plans: dict = None):
    """Converged eigendecomposition of symmetric ``C`` warm-started from ``B_prev``.

    Returns ``(w, B, info)`` with ``C ≈ B diag(w) Bᵀ`` to ``info.off_rel ≤ cfg.tol``
    (eigenvalues in no particular order).

    Planned solves: with device graphs the iteration sequence of the previous solve of
    the same workspace ((Newton–Schulz, damping, far step, local threshold) per
    iteration) is replayed without reading anything back (``plans``: the dict that holds
    the sequence — one per optimiser run, so the decomposition of a run depends only on
    that run's own history; the module-level default is shared), then the per-iteration stats
    history is read once; a sequence that fell short continues adaptively (one stats read
    per iteration), one that converged early is shortened for the next solve.  Consecutive
    CMA-ES covariances differ by one rank-μ update, so the sequence is stable and a
    generation costs one host synchronisation instead of one per iteration."""
    cfg = cfg or SBRConfig()
    info = EigInfo()
    use_graphs = cfg.graphs and C.is_cuda and not torch.cuda.is_current_stream_capturing()
    ws = wkey = None
    if use_graphs:
        ws = _workspace(C.shape[0], C.device, cfg)
        wkey = (C.shape[0], str(C.device), cfg.block, cfg.block_sweeps, cfg.thr_fac, cfg.ns_iters, cfg.damp_tau,
                cfg.tol, cfg.damp_kappa, cfg.near_only)
        ws.C.copy_(C)
        ws.B.copy_(B_prev)
        if not ws.warm and cfg.plan:
            ws.precapture()
        ws.init()
        A, B, st = ws.A, ws.B, ws.hist[0]
    else:
        B = newton_schulz(B_prev.contiguous())
        A, st = sym_product_stats(C, B)
    use_jacobi = C.is_cuda  # the CPU path has no Jacobi kernels: refinement only
    steps = []                 # executed (ns, damp, far_on, θ) per iteration
    plans = _PLANS if plans is None else plans
    plan = plans.get(wkey) if (ws is not None and cfg.plan) else None
    it = 0
    diverged = False
    if plan:
        ws.run_plan(plan)
        rows = ws.read_all(len(plan))  # the one host sync
        r0, k0 = rows[0][0], rows[0][1]
        info.kappa0 = k0
        info.history.append(("init", r0, k0))
        prev = r0
        for j, (r, k, a) in enumerate(rows[1:]):
            info.history.append(("refine", r, k))
            info.damped += a < 1.0
            if not math.isfinite(r) or r > 1.5 * prev:
                diverged = True
                break
            prev = r
        it = len(plan)
        off_rel, kappa, alpha = rows[-1]
        # next plan: the decisions the adaptive loop would take on these stats (the replayed
        # flags came from an earlier generation), cut at the first converged iteration
        steps = []
        last_far, theta = True, plan[0][3]
        for j in range(len(plan)):
            r, k, a_prev = rows[j]
            stp = decide(cfg, j, r, k, a_prev, last_far, max(theta, plan[j][3]))
            steps.append(stp)
            last_far = stp[2]
            if rows[j + 1][0] <= cfg.tol:
                break
        last_far = plan[-1][2]
        theta = plan[-1][3]
    else:
        off_rel, kappa = _read(st)
        info.kappa0 = kappa
        info.history.append(("init", off_rel, kappa))
        r0, k0 = off_rel, kappa
        prev = off_rel
        alpha = 1.0
        last_far = True
        theta = 0.0

    def jacobi_until(A, B, off_rel, kappa, kappa_target):
        st = None
        while off_rel > cfg.tol and kappa > kappa_target and info.jacobi_sweeps < cfg.max_jacobi:
            A, B = _jacobi_sweep(A, B, cfg.tol)
            info.jacobi_sweeps += 1
            st = stats(A)
            off_rel, kappa = _read(st)
            info.history.append(("jacobi", off_rel, kappa))
        return A, B, st, off_rel, kappa

    while not diverged and off_rel > cfg.tol and it < cfg.max_iters:
        # re-orthonormalise in the first iterations and after a damped (large) step; the
        # ‖X‖₂ estimate runs only while the off-diagonal mass is large against the spread
        # (κ > damp_kappa: converging iterations have ‖X‖₂ ≪ 1 and are never capped)
        stp = decide(cfg, it, off_rel, kappa, alpha, last_far, theta)
        far_on = stp[2]
        if ws is not None:
            ws.iterate(it, *stp)
            A, B, st = ws.A, ws.B, ws.hist[min(it + 1, cfg.max_iters)]
            off_rel, kappa, alpha = ws.read(it)
        else:
            A, B, st, a = refine_step(C, A, B, st, it, cfg, *stp)
            off_rel, kappa, alpha = _read(torch.cat([st.double(), a.double().reshape(1)]))
        steps.append(stp)
        it += 1
        info.damped += alpha < 1.0
        info.history.append(("refine", off_rel, kappa))
        if not math.isfinite(off_rel) or off_rel > 1.5 * prev:
            diverged = True
            break
        # an undamped far iteration close to the tolerance that barely helps: pairs inside a
        # cluster denser than the global threshold assumes are neither far nor in a block —
        # the local threshold takes them into the far step for the rest of the solve
        if far_on and alpha >= 1.0 and off_rel < 100 * cfg.tol and off_rel > 0.6 * prev and cfg.block in SHIFT_BLOCKS:
            theta = 1.0
        last_far = far_on
        prev = off_rel
    info.refine_iters = it
    if (diverged or off_rel > cfg.tol) and use_jacobi:
        # safety net: back to the pre-refinement basis, finish with Jacobi sweeps
        info.fallback = True
        B0 = newton_schulz(B_prev.contiguous())
        A0, _ = sym_product_stats(C, B0)
        A, B, _, off_rel, kappa = jacobi_until(A0, B0, r0, k0, 0.0)
    if wkey is not None:
        if info.fallback:
            plans.pop(wkey, None)
        else:
            plans[wkey] = steps
    info.off_rel = off_rel
    return torch.diagonal(A).clone(), B.clone() if ws is not None and B is ws.B else B, info
