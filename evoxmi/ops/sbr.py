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
     diagonalises each block with two cyclic Jacobi sweeps (near, clustered pairs);
  2. builds the Newton rotation generator X_ij = A1_ij / (d_j − d_i) for pairs in
     different blocks whose gap exceeds ``thr_fac·32·spread/n`` (far pairs);
  3. V = exp(X) (Paterson–Stockmeyer Taylor, 3 GEMMs), B ← B[:, perm]·Qblk·V, one
     Newton–Schulz re-orthonormalisation, A ← Bᵀ C B (plain GEMMs).
Far pairs converge quadratically, so 3–5 iterations take the relative off-norm from
3e-3 to ≤1e-5.  The iteration needs the off-diagonal mass to be small against the
spectral spread — κ = ‖offdiag A‖_F / (max diag − min diag) ≲ 1.9 (measured on
CMA-ES matrices, tools/eig_probe.py); early generations (C ≈ I, κ up to ~4) first run
block-Jacobi sweeps (``eigh_jacobi.hip``) until κ is small enough.  If an iteration
ever increases the off-norm the solver restores the basis and finishes with Jacobi
sweeps, so every generation ends converged (``EigInfo.off_rel``).

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
            J = torch.eye(m, dtype=S.dtype, device=S.device).repeat(nb, 1, 1)
            J[ar, p, p] = c
            J[ar, q, q] = c
            J[ar, p, q] = s
            J[ar, q, p] = -s
            S = J.transpose(1, 2) @ S @ J
            S[ar, p, p] = app - t * apq
            S[ar, q, q] = aqq + t * apq
            S[ar, p, q] = 0
            S[ar, q, p] = 0
            Q = Q @ J
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
    return torch.where(mask, A1 / torch.where(mask, den, torch.ones_like(den)), torch.zeros_like(A1))


def bq_ref(B, off, perm, Q):
    return B[:, perm.long()] @ _blockdiag(Q, B.shape[1], off)


# ---------------------------------------------------------------------------- dispatch
def _dev(t):
    return t.is_cuda


def _rowmajor(t):
    return t if t.stride(-1) == 1 else t.contiguous()


def stats(A):
    return _ext.ops().sbr_stats(_rowmajor(A)) if _dev(A) else stats_ref(A)


def block_solve(A, off, sweeps):
    if _dev(A):
        perm, Q, dq = _ext.ops().sbr_block(_rowmajor(A), int(off), int(sweeps))
        return perm, Q, dq
    return block_solve_ref(A, off, sweeps)


def far(A, off, perm, Q, dq, st, thr_fac):
    if _dev(A):
        return _ext.ops().sbr_far(_rowmajor(A), int(off), perm, Q, dq, st, float(thr_fac))
    return far_ref(A, off, perm, Q, dq, st, thr_fac)


def bq(B, off, perm, Q):
    return _ext.ops().sbr_bq(_rowmajor(B), int(off), perm, Q) if _dev(B) else bq_ref(B, off, perm, Q)


def expm_taylor6(X: torch.Tensor) -> torch.Tensor:
    """exp(X) to 6th order with 3 GEMMs (Paterson–Stockmeyer):
    I + X + X²/2 + X³/6 + X³(X/24 + X²/120 + X³/720)."""
    X2 = X @ X
    X3 = X2 @ X
    if X.is_cuda:
        P, M = _ext.ops().sbr_taylor_prep(X.contiguous(), X2, X3)
        return torch.addmm(M, X3, P)
    P = X / 24 + X2 / 120 + X3 / 720
    V = X3 @ P
    V += X + X2 / 2 + X3 / 6
    V.diagonal().add_(1.0)
    return V


def newton_schulz(B: torch.Tensor) -> torch.Tensor:
    """One step toward the nearest orthonormal matrix, B(1.5 I − 0.5 BᵀB)."""
    return torch.addmm(B, B, B.t() @ B, beta=1.5, alpha=-0.5)


def sym_product(C: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """A = Bᵀ C B, symmetrised."""
    A = B.t() @ (C @ B)
    return (A + A.t()) * 0.5


def sym_product_stats(C: torch.Tensor, B: torch.Tensor):
    """(A = sym(Bᵀ C B), stats(A)); on the device symmetrisation and stats are one kernel."""
    T = B.t() @ (C @ B)
    if T.is_cuda:
        A, st = _ext.ops().sbr_symstats(T)
        return A, st
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
    history: list = field(default_factory=list)


@dataclass
class SBRConfig:
    tol: float = 1e-5          # relative off-norm ‖offdiag‖_F / ‖diag‖_F to reach
    kappa_max: float = 1.9     # hand-off from Jacobi sweeps to refinement
    max_iters: int = 8
    max_jacobi: int = 16
    block_sweeps: int = 2
    thr_fac: float = 0.3
    ns_iters: int = 2          # Newton–Schulz re-orthonormalisation in the first iterations
                               # (later ones have ‖X‖ ≤ 0.2: Taylor-6 is orthogonal to ~1e-10)
    graphs: bool = True        # replay each device iteration as a captured hipGraph


def _read(st: torch.Tensor):
    off, dg, mn, mx = (float(v) for v in st.cpu())
    off_rel = math.sqrt(max(off, 0.0) / dg) if dg > 0 else float("nan")
    kappa = math.sqrt(max(off, 0.0)) / (mx - mn) if mx > mn else float("inf")
    return off_rel, kappa


def _refine_core(C, A, B, st, off: int, ns: bool, cfg: SBRConfig):
    perm, Q, dq = block_solve(A, off, cfg.block_sweeps)
    X = far(A, off, perm, Q, dq, st, cfg.thr_fac)
    Bn = bq(B, off, perm, Q) @ expm_taylor6(X)
    if ns:
        Bn = newton_schulz(Bn)
    A, st = sym_product_stats(C, Bn)
    return A, Bn, st


def refine_step(C, A, B, st, it: int, cfg: SBRConfig):
    return _refine_core(C, A, B, st, (it % 2) * (BK // 2), it < cfg.ns_iters, cfg)


class _Workspace:
    """Static device buffers + captured hipGraphs of the refinement iteration (one per
    (block offset, Newton–Schulz) variant) and of the initial Bᵀ C B, so a generation's
    solve costs one graph launch + one 32-byte stats read per iteration."""

    def __init__(self, n: int, dev, cfg: SBRConfig):
        self.n, self.cfg = n, cfg
        z = lambda: torch.zeros(n, n, device=dev)  # noqa: E731
        self.C, self.A, self.B = z(), z(), z()
        self.st = torch.zeros(4, dtype=torch.float64, device=dev)
        self.graphs = {}

    def _capture(self, key, body):
        if key not in self.graphs:
            s = torch.cuda.Stream(device=self.C.device)
            s.wait_stream(torch.cuda.current_stream(self.C.device))
            with torch.cuda.stream(s):  # warm-up (allocator, lazy init) outside the capture
                body()
            torch.cuda.current_stream(self.C.device).wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                body()
            self.graphs[key] = g
        return self.graphs[key]

    def init(self):
        def body():
            B = newton_schulz(self.B)
            A, st = sym_product_stats(self.C, B)
            self.B.copy_(B)
            self.A.copy_(A)
            self.st.copy_(st)

        self._capture(("init",), body).replay()

    def iterate(self, it: int):
        off, ns = (it % 2) * (BK // 2), it < self.cfg.ns_iters

        def body():
            A, B, st = _refine_core(self.C, self.A, self.B, self.st, off, ns, self.cfg)
            self.A.copy_(A)
            self.B.copy_(B)
            self.st.copy_(st)

        self._capture(("it", off, ns), body).replay()


_WS = {}


def _workspace(n, dev, cfg) -> _Workspace:
    k = (n, str(dev), cfg.block_sweeps, cfg.thr_fac, cfg.ns_iters)
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
    from .. import config

    _ext.ops().jacobi_sweeps(Ap, Bp, jacobi.schedule(np_ // 16, dev), 1, float(tol), float(config.get("jacobi_inner_tol")),
                             int(config.get("jacobi_inner")), int(config.get("jacobi_fused")))
    return Ap[:n, :n].contiguous(), Bp[:n, :n].contiguous()


def eigh_warm(C: torch.Tensor, B_prev: torch.Tensor, cfg: SBRConfig = None):
    """Converged eigendecomposition of symmetric ``C`` warm-started from ``B_prev``.

    Returns ``(w, B, info)`` with ``C ≈ B diag(w) Bᵀ`` to ``info.off_rel ≤ cfg.tol``
    (eigenvalues in no particular order)."""
    cfg = cfg or SBRConfig()
    info = EigInfo()
    use_graphs = cfg.graphs and C.is_cuda and not torch.cuda.is_current_stream_capturing()
    ws = None
    if use_graphs:
        ws = _workspace(C.shape[0], C.device, cfg)
        ws.C.copy_(C)
        ws.B.copy_(B_prev)
        ws.init()
        A, B, st = ws.A, ws.B, ws.st
    else:
        B = newton_schulz(B_prev.contiguous())
        A, st = sym_product_stats(C, B)
    off_rel, kappa = _read(st)
    info.kappa0 = kappa
    info.history.append(("init", off_rel, kappa))
    use_jacobi = C.is_cuda  # the CPU path has no Jacobi kernels: refinement only

    def jacobi_until(A, B, off_rel, kappa, kappa_target):
        st = None
        while off_rel > cfg.tol and kappa > kappa_target and info.jacobi_sweeps < cfg.max_jacobi:
            A, B = _jacobi_sweep(A, B, cfg.tol)
            info.jacobi_sweeps += 1
            st = stats(A)
            off_rel, kappa = _read(st)
            info.history.append(("jacobi", off_rel, kappa))
        return A, B, st, off_rel, kappa

    if use_jacobi and kappa > cfg.kappa_max and off_rel > cfg.tol:
        A, B, st_j, off_rel, kappa = jacobi_until(A, B, off_rel, kappa, cfg.kappa_max)
        if st_j is not None:
            st = st_j
            if ws is not None:
                ws.A.copy_(A)
                ws.B.copy_(B)
                ws.st.copy_(st)
                A, B, st = ws.A, ws.B, ws.st
    A0, B0, r0, k0 = A.clone(), B.clone(), off_rel, kappa
    it = 0
    prev = off_rel
    diverged = False
    while off_rel > cfg.tol and it < cfg.max_iters:
        if ws is not None:
            ws.iterate(it)
            A, B, st = ws.A, ws.B, ws.st
        else:
            A, B, st = refine_step(C, A, B, st, it, cfg)
        it += 1
        off_rel, kappa = _read(st)
        info.history.append(("refine", off_rel, kappa))
        if not math.isfinite(off_rel) or off_rel > 1.5 * prev:
            diverged = True
            break
        prev = off_rel
    info.refine_iters = it
    if (diverged or off_rel > cfg.tol) and use_jacobi:
        # safety net: back to the pre-refinement basis, finish with Jacobi sweeps
        info.fallback = True
        A, B, _, off_rel, kappa = jacobi_until(A0, B0, r0, k0, 0.0)
    info.off_rel = off_rel
    return torch.diagonal(A).clone(), B.clone() if ws is not None and B is ws.B else B, info
