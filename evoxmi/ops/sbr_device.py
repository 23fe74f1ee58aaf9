"""Device-controlled sorted-block refinement: the converged eigensolver as one capturable schedule.

The host-driven solver (:func:`evoxmi.ops.sbr.eigh_warm`) chooses every refinement
iteration's variant from statistics it reads back, so a CMA-ES generation was split into
graph segments around a host phase (``runtime.host_phase``) with a device→host read per
generation.  The reference decomposes C inside its one jitted step
(``/root/reference/src/evox/algorithms/so/es_variants/cma_es.py:155-160,193-198`` under
``std_workflow.py:203-216``); this module restores that property on MI355X:

* the solve is a FIXED schedule of ``K`` iterations (``EVOXMI_SBR_DEVICE_ITERS``), each
  the same kernel sequence as the host driver's iteration (block solves, far generator,
  X², damping, Taylor exponential, Bq·V, Newton–Schulz, Bᵀ C B) —
  ``csrc/kernels/eigh_sbr_dev.hip`` + ``gemm_ks.hip``;
* every kernel reads a device control word and returns at once when its variant is off
  for this iteration or the solve has already converged (a skipped kernel costs one
  launch boundary, ≈1.5 µs);
* the Bᵀ C B GEMM writes the convergence statistics' partials in its epilogue and one
  single-workgroup kernel per iteration reduces them and writes the next iteration's
  control words with :func:`evoxmi.ops.sbr.decide`'s rules (tolerance stop, Newton–Schulz
  while κ is large or after a damped step, damping at iteration 0 / large κ, near-only
  close to the tolerance, Taylor order 4 once κ is small, the sticky local threshold, and
  the divergence stop — which restores the warm-start basis).

No host read, no iteration plan, no state outside the algorithm's ``State``: a solve
depends only on (C, B_prev), so a checkpoint-resumed run is bitwise identical
(``tests/test_sbr_device_gpu.py``).  The per-solve [off_rel, 0, iterations, fallback]
also go to a device ring (:meth:`DeviceSBR.history`) that benches read after timing.
"""
from __future__ import annotations

import torch

from . import _ext
from .linalg import mm
from .sbr import SBRConfig, _probe_vectors

LOG_LEN = 4096


class DeviceSBR:
    """Persistent buffers + the fixed iteration schedule for one (n, device, config)."""

    def __init__(self, n: int, device, cfg: SBRConfig, iters: int, lean_from: int = None, xgate: bool = None,
                 damp_from: int = None):
        if cfg.block not in (16, 32):
            raise ValueError("the device schedule uses the shifted-layout blocks (16 / 32)")
        self.n, self.cfg, self.K = n, cfg, int(iters)
        # slots ≥ lean_from launch no damping / Newton–Schulz / X³ kernels (their variants are
        # only chosen in the first iterations of a warm-started solve): a skipped lean slot
        # costs 7 launch boundaries fewer
        self.lean_from = self.K if lean_from is None else min(int(lean_from), self.K)
        # slots ≥ damp_from launch no damping power steps (the late schedule keeps them in slot 0:
        # in settled solves they return at once, ≈6 launches per generation); the control kernel
        # stops the solve (capped, escalated by the host) where the κ rule would damp there
        self.damp_from = self.lean_from if damp_from is None else min(int(damp_from), self.lean_from)
        dev = torch.device(device)
        ops = _ext.ops()

        def mat():
            return torch.zeros(n, n, device=dev)

        (self.A, self.B, self.T, self.W, self.X, self.X2, self.X3, self.P, self.VT, self.Bq,
         self.G) = (mat() for _ in range(11))
        from .. import config

        # opt-in: A[perm, perm] and B[:, perm] gathered row-wise first (measured no faster)
        self.prepermute = bool(config.get("sbr_prepermute"))
        # a block already diagonal to this relative off-norm skips its remaining Jacobi sweeps
        self.sweep_tol = float(config.get("sbr_sweep_tol"))
        self.Ap, self.Bp = (mat(), mat()) if self.prepermute else (None, None)
        sb = cfg.block
        nb = -(-n // sb)
        self.perm = torch.zeros(n, dtype=torch.int32, device=dev)
        self.Q = torch.zeros(nb * sb * sb, device=dev)
        self.dq = torch.zeros(n, device=dev)
        self.nparts = int(ops.gemm_ks_grid(n, n, 1))
        self.part = torch.zeros(4 * self.nparts, dtype=torch.float64, device=dev)
        # stats partials of X² = −X·Xᵀ: the free ‖X‖_F bound that gates every step size (sbr_dev_prep)
        self.xgate = bool(config.get("sbr_xgate") == 1) if xgate is None else bool(xgate)
        self.part2 = torch.zeros(4 * self.nparts, dtype=torch.float64, device=dev) if self.xgate else None
        K = self.K
        self.hist = torch.zeros(4 * (K + 1), dtype=torch.float64, device=dev)
        self.alpha = torch.ones(K + 1, device=dev)
        self.theta = torch.zeros(max(K, 1), device=dev)
        self.ctrl = torch.ones(8 * max(K, 1), dtype=torch.int32, device=dev)
        self.st = torch.zeros(8, dtype=torch.int32, device=dev)
        self.never = torch.zeros(1, dtype=torch.int32, device=dev)
        self.V = _probe_vectors(n, str(dev))
        self.work = torch.zeros(24 * n, device=dev)
        self.w = torch.zeros(n, device=dev)
        self.w_init = torch.zeros(n, device=dev)
        self.eig_stats = torch.zeros(4, dtype=torch.float64, device=dev)
        self.log = torch.zeros(LOG_LEN, 4, dtype=torch.float64, device=dev)
        self.log_count = torch.zeros(1, dtype=torch.int32, device=dev)
        # precision tiers (round 6): the residual products (Bᵀ C B, BᵀB) stay f32-accurate
        # (bf16x6); the products that only form a correction of an exactly held matrix —
        # X², X³ and the Taylor terms of exp(αX) − I, the basis update Bq + Bq·(V − I), and
        # Newton–Schulz's T − ½T·(TᵀT − I) — run at bf16x3 (≈1e-5 of the correction's own size)
        self.corr = "x3" if config.get("sbr_corr_prec") == "x3" else None
        self.prm = [float(cfg.tol), float(cfg.ns_kappa), float(cfg.damp_kappa), float(cfg.t4_kappa), float(cfg.near_only),
                    float(cfg.theta0), float(cfg.theta_kappa), float(self.lean_from), float(config.get("sbr_recover")),
                    float(config.get("sbr_lean_guard")), float(self.xgate), float(self.damp_from)]

    # ------------------------------------------------------------------ pieces
    def _btcb(self, C, skip):
        """A = Bᵀ C B (symmetric output, stats partials in the epilogue)."""
        mm(self.B, C, ta=True, tb=True, out=self.W, skip=skip)
        mm(self.W, self.B, mode=1, out=self.A, skip=skip, stat_part=self.part)

    def _ctrl(self, j, C):
        from ..core import in_capture_warmup

        # a graph capture's warm-up step (on a copy of the state) is not a solve of the run: unlogged
        log = self.log[:0] if in_capture_warmup() else self.log  # log_len 0: the ctrl kernel writes no row
        _ext.ops().sbr_dev_ctrl(self.part, self.nparts, j, self.K, self.hist, self.alpha, self.theta, self.ctrl, self.st, self.prm,
                                int(self.cfg.ns_iters), self.A, self.w, self.eig_stats, self.w_init, log, self.log_count)

    def _iteration(self, j, C):
        ops = _ext.ops()
        cfg = self.cfg
        sb = cfg.block
        c = self.ctrl[8 * j : 8 * j + 8]
        sk_all, sk_far, sk_damp, sk_x3, sel6, sk_ns, sel_ns, sk_copy = (c[i : i + 1] for i in range(8))
        shift = (j % 2) * (sb // 2)
        full = j < self.lean_from
        damp_slot = j < self.damp_from
        ops.sbr16_block_out(self.A, shift, int(cfg.block_sweeps), sb, self.perm, self.Q, self.dq, sk_all, self.sweep_tol)
        # far generator X and Bq = B[:, perm]·blockdiag(Q) in one launch
        if self.prepermute:
            # A[perm, perm] and B[:, perm] row by row first, so that the tiles read contiguous blocks —
            # far+Bq 30.0 instead of 28 µs plus 6 µs for the gather (profiles/NOTES.md): off by default
            ops.sbr16_permute_out(self.A, self.perm, self.B, self.Ap, self.Bp, sk_far, sk_all)
            ops.sbr16_far_bq_out(self.Ap, self.perm, self.Q, self.dq, self.hist[4 * j : 4 * j + 4], float(cfg.thr_fac),
                                 self.theta[j : j + 1], self.X, self.Bp, self.Bq, sb, sk_far, sk_all, True)
        else:
            ops.sbr16_far_bq_out(self.A, self.perm, self.Q, self.dq, self.hist[4 * j : 4 * j + 4], float(cfg.thr_fac),
                                 self.theta[j : j + 1], self.X, self.B, self.Bq, sb, sk_far, sk_all)
        corr = self.corr
        # X skew ⇒ X² = −X·Xᵀ, symmetric (upper tiles only)
        mm(self.X, self.X, tb=True, mode=1, alpha=-1.0, out=self.X2, skip=sk_far, stat_part=self.part2, stat_diag_only=True,
           prec=corr)
        if cfg.damp_tau > 0 and damp_slot:
            # three power-step launches (they return at once when the free Frobenius bound already
            # gives α = 1); α itself is formed by the prep kernel below (no_final)
            ops.sbr_damping_out(self.X2, self.V, float(cfg.damp_tau), self.alpha[j + 1 : j + 2], self.work, sk_damp, None, True,
                                self.part2)
        if full:
            # order 6 only: X³ = X²·X = −X²·Xᵀ (skew)
            mm(self.X2, self.X, tb=True, mode=2, alpha=-1.0, out=self.X3, skip=sk_x3, prec=corr)
        damp_here = cfg.damp_tau > 0 and damp_slot
        # near-only iterations (no far step): the block-rotated basis is the new basis — Bq → B
        # copied by this launch (it returns at once otherwise), no copy launch of its own
        ops.sbr_dev_prep(self.X, self.X2, self.X3, self.alpha[j + 1 : j + 2], self.P, self.VT, c, self.work if damp_here else None,
                         float(cfg.damp_tau), self.part2, self.Bq, self.B, int(corr is not None))
        # Vᵀ = M(−α) + X²·Pᵀ (order 4) or M(−α) − X³·Pᵀ (order 6): the control word selects
        # (with the tiered precision the prep wrote M − I, so this is Vᵀ − I)
        mm(self.X2, self.P, tb=True, alpha=1.0, beta=1.0, Cin=self.VT, out=self.VT, skip=sk_far, sel=sel6, A2=self.X3, alpha2=-1.0,
           prec=corr)
        # B·V → B, or into T when Newton–Schulz follows
        if corr is not None:
            # Bq + Bq·(V − I): the exact basis plus an x3 correction product
            mm(self.Bq, self.VT, tb=True, beta=1.0, Cin=self.Bq, out=self.B, skip=sk_far, sel=sel_ns, C2=self.T, prec=corr)
        else:
            mm(self.Bq, self.VT, tb=True, out=self.B, skip=sk_far, sel=sel_ns, C2=self.T)
        if full:
            if corr is not None:
                # E = TᵀT − I at full precision (the orthogonality residual), then T − ½T·E
                mm(self.T, self.T, ta=True, mode=1, out=self.G, skip=sk_ns, diag_add=-1.0)
                mm(self.T, self.G, tb=True, alpha=-0.5, beta=1.0, Cin=self.T, out=self.B, skip=sk_ns, prec=corr)
            else:
                mm(self.T, self.T, ta=True, mode=1, out=self.G, skip=sk_ns)
                mm(self.T, self.G, tb=True, alpha=-0.5, beta=1.5, Cin=self.T, out=self.B, skip=sk_ns)
        self._btcb(C, sk_all)
        self._ctrl(j, C)

    # ------------------------------------------------------------------ solve
    def solve(self, C: torch.Tensor, B_prev: torch.Tensor):
        """(w, B, eig_stats) with C ≈ B diag(w) Bᵀ — device buffers of this workspace, valid
        until the next solve.  Nothing is read back; capturable into a hipGraph."""
        ops = _ext.ops()
        n = self.n
        assert C.shape == (n, n) and B_prev.shape == (n, n)
        B_prev = B_prev if B_prev.is_contiguous() else B_prev.contiguous()
        ops.sbr_dev_copy(B_prev, self.B, self.never)
        self._btcb(C, self.never)
        self._ctrl(-1, C)
        for j in range(self.K):
            self._iteration(j, C)
        # the refinement diverged (st[5] = 0): back to the warm-start basis
        ops.sbr_dev_copy(B_prev, self.B, self.st[5:6])
        return self.w, self.B, self.eig_stats

    def history(self, last: int = None):
        """[off_rel, 0, refinement iterations, fallback] of the most recent solves (one
        device→host read — call it outside timed loops)."""
        cnt = int(self.log_count.item())
        k = min(cnt, LOG_LEN) if last is None else min(cnt, LOG_LEN, int(last))
        if k == 0:
            return torch.zeros(0, 4, dtype=torch.float64)
        idx = [(cnt - k + i) % LOG_LEN for i in range(k)]
        return self.log.cpu()[idx]


_WS = {}


def workspace(n: int, device, cfg: SBRConfig, iters: int, lean_from: int = None, xgate: bool = False,
              damp_from: int = None) -> DeviceSBR:
    from .. import config

    key = (n, str(device), cfg.block, cfg.block_sweeps, cfg.thr_fac, cfg.ns_iters, cfg.damp_tau, cfg.tol, cfg.ns_kappa,
           cfg.damp_kappa, cfg.t4_kappa, cfg.near_only, cfg.theta0, cfg.theta_kappa, int(iters), lean_from,
           bool(config.get("sbr_prepermute")), float(config.get("sbr_sweep_tol")), int(config.get("sbr_recover")),
           int(config.get("sbr_lean_guard")), bool(xgate), damp_from, config.get("sbr_corr_prec"))
    if key not in _WS:
        _WS[key] = DeviceSBR(n, device, cfg, iters, lean_from, xgate, damp_from)
    return _WS[key]


def schedule_iters(n: int, iters: int) -> int:
    """Refinement slots a schedule of ``iters`` slots actually runs at order ``n`` (larger
    matrices get at least ``sbr_large_n_iters``; see :func:`eigh_device`)."""
    from .. import config

    if n > int(config.get("sbr_lean_max_n")) and iters < int(config.get("sbr_cold_iters")):
        return max(int(iters), int(config.get("sbr_large_n_iters")))
    return int(iters)


def eigh_device(C: torch.Tensor, B_prev: torch.Tensor, cfg: SBRConfig = None, iters: int = None):
    """Converged-or-capped eigendecomposition of symmetric ``C`` warm-started from
    ``B_prev``, entirely on the device (see module docstring).  Returns ``(w, B, stats)``."""
    from .. import config

    cfg = cfg or SBRConfig(tol=config.get("eigh_tol"), block=config.get("sbr_block"), near_only=config.get("sbr_near_only"),
                           theta0=config.get("sbr_theta0"), theta_kappa=config.get("sbr_theta_kappa"),
                           thr_fac=config.get("sbr_thr_fac"), block_sweeps=config.get("sbr_sweeps"),
                           damp_tau=config.get("sbr_damp_tau"), damp_kappa=config.get("sbr_damp_kappa"),
                           ns_kappa=config.get("sbr_ns_kappa"), ns_iters=config.get("sbr_ns_iters"))
    if iters is None:
        iters = config.get("sbr_device_iters")
        # lean tail slots only in a schedule that does not start cold (CMA-ES's cold-start
        # variant passes a longer schedule with every slot full)
        lean = config.get("sbr_full_slots") if iters < config.get("sbr_cold_iters") else None
        # larger matrices stay above the damping / Newton–Schulz thresholds for more iterations
        # (d = 2000: the lean-slot guard capped warm solves at slot 5): every slot full there,
        # and at least sbr_large_n_iters slots (a 7-slot warm schedule capped one d = 2000 solve
        # at 7 iterations, off_rel 1.39e-5)
        if C.shape[0] > int(config.get("sbr_lean_max_n")):
            lean = None
            iters = max(iters, int(config.get("sbr_large_n_iters")))
    else:
        lean = None
    # the bounds-gated damping: everywhere (1) or in the cold-start schedule only (2): the
    # large generators of a cold start are where an undamped step diverged (d = 2000), and in
    # settled solves the extra power iterations cost ≈3 % of a generation (profiles/r5_eigh_recover.txt)
    xg = int(config.get("sbr_xgate"))
    xgate = xg == 1 or (xg == 2 and iters >= config.get("sbr_cold_iters"))
    ds = int(config.get("sbr_damp_slots"))
    damp_from = ds if (lean is not None and ds > 0) else None
    return workspace(C.shape[0], C.device, cfg, iters, lean, xgate, damp_from).solve(C, B_prev)


def all_histories():
    """Concatenated per-solve histories of every device workspace (bench diagnostics)."""
    out = [ws.history() for ws in _WS.values()]
    out = [h for h in out if h.shape[0]]
    return torch.cat(out) if out else torch.zeros(0, 4, dtype=torch.float64)


def history_count() -> int:
    return sum(int(ws.log_count.item()) for ws in _WS.values())


def histories_since(counts: dict):
    """Per-solve rows appended since ``counts`` (a {key: count} snapshot from
    :func:`snapshot_counts`), all workspaces concatenated."""
    rows = []
    for k, ws in _WS.items():
        new = int(ws.log_count.item()) - counts.get(k, 0)
        if new > 0:
            rows.append(ws.history(new))
    return torch.cat(rows) if rows else torch.zeros(0, 4, dtype=torch.float64)


def snapshot_counts() -> dict:
    return {k: int(ws.log_count.item()) for k, ws in _WS.items()}
