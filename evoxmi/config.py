"""Runtime knobs.

The reference has no flag system: every parameter is a constructor kwarg and a few
behaviours follow environment variables (``XLA_PYTHON_CLIENT_PREALLOCATE``,
``CUDA_VISIBLE_DEVICES``; ``docs/source/miscellaneous/*.md``).  evoxmi keeps kwargs
as the API and gathers the process-wide *implementation* choices here, each
readable from an ``EVOXMI_*`` environment variable and overridable in code:

>>> from evoxmi import config
>>> config.get("eigh")
'sbr'
>>> with config.override(jacobi_sweeps=3):
...     ...

Device selection uses ``HIP_VISIBLE_DEVICES`` (or ``ROCR_VISIBLE_DEVICES``) as
usual for ROCm; multi-process runs read ``RANK``/``LOCAL_RANK``/``WORLD_SIZE``.
"""
from __future__ import annotations

import contextlib
import os
from dataclasses import dataclass
from typing import Any, Callable, Dict


@dataclass(frozen=True)
class Knob:
    env: str
    default: Any
    parse: Callable[[str], Any]
    doc: str


def _bool(s: str) -> bool:
    return s.strip().lower() in ("1", "true", "yes", "on")


KNOBS: Dict[str, Knob] = {
    "eigh": Knob("EVOXMI_EIGH", "sbr", str, "symmetric eigensolver for CMA-ES: 'sbr' (converged: Jacobi hand-off + sorted-block refinement, ops/sbr.py), 'jacobi' (fixed-sweep warm block Jacobi) or 'torch' (rocSOLVER)"),
    "eigh_tol": Knob("EVOXMI_EIGH_TOL", 1e-5, float, "sbr: target relative off-norm ‖offdiag(BᵀCB)‖_F / ‖diag‖_F of every decomposition"),
    "sbr_prepermute": Knob("EVOXMI_SBR_PREPERMUTE", 0, int, "device eigensolver: gather A[perm, perm] and B[:, perm] row-wise before the far / Bq tiles (1) — measured no faster (far+Bq 30.0 vs 28 µs, plus 6 µs for the gather)"),
    "sbr_damp_tau": Knob("EVOXMI_SBR_DAMP_TAU", 1.0, float, "device eigensolver: cap on ‖αX‖₂ of a damped refinement step"),
    "sbr_damp_kappa": Knob("EVOXMI_SBR_DAMP_KAPPA", 1.0, float, "device eigensolver: estimate ‖X‖₂ (damping) while κ exceeds this"),
    "sbr_ns_kappa": Knob("EVOXMI_SBR_NS_KAPPA", 0.3, float, "device eigensolver: Newton–Schulz re-orthonormalisation while κ exceeds this"),
    "sbr_sweep_tol": Knob("EVOXMI_SBR_SWEEP_TOL", 0.0, float, "device eigensolver: a 32×32 block whose relative off-diagonal norm is at most this before a Jacobi sweep skips its remaining sweeps (0: always every sweep)"),
    "sbr_sweeps": Knob("EVOXMI_SBR_SWEEPS", 2, int, "sbr: cyclic Jacobi sweeps of the near-pair block solve per refinement iteration"),
    "sbr_block": Knob("EVOXMI_SBR_BLOCK", 32, int, "sbr: near-pair block size — 32 or 16 (blocks in a shifted sorted order, eigh_sbr16.hip; 32 converges in fewer iterations on the bench matrices) or 64 (eigh_sbr.hip)"),
    "sbr_mode": Knob("EVOXMI_SBR_MODE", "device", str, "sbr: 'device' — fixed device-controlled iteration schedule inside the generation's graph (ops/sbr_device.py, no host read); 'host' — host-driven iterations with planned solves as a host phase between graph segments (ops/sbr.py)"),
    "sbr_device_iters": Knob("EVOXMI_SBR_DEVICE_ITERS", 7, int, "sbr device mode: refinement iterations in the fixed (warm) schedule (kernels of iterations past convergence return at once; round 5: 8 → 7 slots, 1.644-1.656 → 1.630 ms at 20 steps — warm solves at d ≤ 1000 take at most 6 iterations on F1 / F4 / F6 / F12 over 200 generations, and a capped solve escalates the schedule)"),
    "sbr_large_n_iters": Knob("EVOXMI_SBR_LARGE_N_ITERS", 8, int, "device eigensolver: least warm-schedule slots for matrices larger than sbr_lean_max_n"),
    "sbr_cold_iters": Knob("EVOXMI_SBR_COLD_ITERS", 16, int, "CMA-ES device eigensolver: refinement slots of the cold-start schedule (every run starts on it; CMAES moves down to the warm / late schedules after consecutive solves that fit them with a slot to spare)"),
    "sbr_late_iters": Knob("EVOXMI_SBR_LATE_ITERS", 5, int, "refinement slots of the late (settled) eigensolver schedule (settled solves take 4; a capped or slow solve moves the run back up two generations later — round 5: 6 → 5 slots, 1.439 → 1.424 ms over 50 steps)"),
    "sbr_late_full_slots": Knob("EVOXMI_SBR_LATE_FULL_SLOTS", 3, int, "late-generation eigensolver schedule: slots that carry the damping / Newton–Schulz / order-6 kernels (the rest are lean); settled generations need them in slots 0-2 only (profiles/r4_near_only_ab.txt detail)"),
    "sbr_late_damp_slots": Knob("EVOXMI_SBR_LATE_DAMP_SLOTS", 1, int, "late-generation eigensolver schedule: slots that carry the damping power steps (slot 0 always damps by the κ rule; in settled solves the later slots' power steps return at once — 6 launches per generation; a later slot whose step the κ rule would damp stops the solve, capped, and the host escalates)"),
    "sbr_damp_slots": Knob("EVOXMI_SBR_DAMP_SLOTS", 0, int, "device eigensolver: slots that carry the damping power steps in a schedule with lean slots (0: every full slot; the late CMA-ES variant sets sbr_late_damp_slots)"),
    "sbr_ns_iters": Knob("EVOXMI_SBR_NS_ITERS", 2, int, "device eigensolver: refinement iterations that always re-orthonormalise B (Newton–Schulz, two 1000³ GEMMs each); later ones only when κ or a damped step asks for it"),
    "sbr_late_ns_iters": Knob("EVOXMI_SBR_LATE_NS_ITERS", 2, int, "late-generation eigensolver schedule: iterations that always take the Newton–Schulz step (sbr_ns_iters of the late variant).  2: ‖BᵀB − I‖_F 1.4-2e-5 over 600 generations; 1 holds it at 2-3e-5 and saves two 1000³ GEMMs per generation (100 steps 1.320 vs 1.349 ms) but moved the 5-seed trajectory-parity test against the library eigh (tests/test_eigh_sbr.py) to 5.8 % against its 5 % bound, so it stays opt-in; 0 drifts linearly (3.8e-3 at generation 600) — profiles/r5_late_ns_orthogonality.txt"),
    "sbr_full_slots": Knob("EVOXMI_SBR_FULL_SLOTS", 5, int, "sbr device schedule (warm, 8 slots): slots past this carry no damping / Newton–Schulz / X³ kernels (those variants are chosen only in the first iterations of a warm-started solve), so a skipped tail slot costs 7 launches fewer"),
    "sbr_near_only": Knob("EVOXMI_SBR_NEAR_ONLY", 1.5, float, "sbr: a refinement iteration skips the far step once off_rel ≤ near_only·tol (after a far iteration).  1.5: with 3.0 a near-only step taken at off_rel 1.5-3e-5 often barely helped (far pairs left) and cost a further far iteration — 20 / 50-step bench 1.830 / 1.686 vs 1.850 / 1.694 ms, mean iterations 4.75 vs 5.0 (profiles/r4_near_only_ab.txt)"),
    "sbr_theta0": Knob("EVOXMI_SBR_THETA0", 1.0, float, "sbr: local far-pair threshold factor θ in every iteration whose κ ≤ sbr_theta_kappa (0: switched on only after a stalled far iteration). θ = 1 keeps steady-state CMA-ES solves at 4 iterations where θ = 0 stalls at ≈1.3e-5 for tens of generations (profiles/r4_sbr_threshold_variants.txt)"),
    "sbr_theta_kappa": Knob("EVOXMI_SBR_THETA_KAPPA", 0.05, float, "sbr: κ below which the local far threshold θ applies (larger far steps with it diverged in cold-start solves)"),
    "sbr_thr_fac": Knob("EVOXMI_SBR_THR_FAC", 0.3, float, "sbr: global far-pair threshold factor (gap > thr_fac·(block/2)·spread/n)"),
    "sbr_corr_prec": Knob("EVOXMI_SBR_CORR_PREC", "x3", str, "device eigensolver: precision of the correction products (X², X³, the Taylor terms of exp(αX) − I, Bq·(V − I), Newton–Schulz T·(TᵀT − I)) — 'x3' (bf16x3, ≈1e-5 of the correction's size; the residual products Bᵀ C B and TᵀT stay bf16x6) or 'x6' (every product f32-accurate, the round-5 solver)"),
    "cma_fused": Knob("EVOXMI_CMA_FUSED", 1, int, "CMA-ES tell epilogue as the fused cmaes.hip kernels (0: reference-shaped torch ops)"),
    "sbr_recover": Knob("EVOXMI_SBR_RECOVER", 2, int, "device eigensolver: divergences (off-norm up > 1.5× in one iteration) answered by a forced damped + re-orthonormalised step from the current basis before the solve gives up and keeps the better of the current and the warm-start basis (0: give up at the first, the round-4 behaviour)"),
    "sbr_lean_guard": Knob("EVOXMI_SBR_LEAN_GUARD", 1, int, "device eigensolver: a lean slot (no damping / Newton–Schulz / order-6 kernels) whose step the full rules would damp, re-orthonormalise or take to order 6 stops the solve as capped instead of taking an unguarded order-4 step (the host then escalates the schedule)"),
    "sbr_lean_max_n": Knob("EVOXMI_SBR_LEAN_MAX_N", 1024, int, "device eigensolver: lean tail slots only for matrices up to this order (larger ones keep the damping / Newton–Schulz kernels in every slot)"),
    "sbr_xgate": Knob("EVOXMI_SBR_XGATE", 2, int, "device eigensolver: the damping's power iteration also follows free bounds of the generator (the X² GEMM's diagonal stats): skipped when ‖X‖₂ ≤ τ is proven, run when a row of X is longer than τ/2 whatever κ says — 1 in every schedule, 2 in the cold-start schedule only (where an undamped step on a large generator diverged the d = 2000 cold start; in settled solves it costs ≈3 % of a generation), 0 off"),
    "cec_stack": Knob("EVOXMI_CEC_STACK", 1, int, "CEC'22 compositions (F9–F12) on the device: every rotated component from ONE GEMM over the stacked rotations with per-block exact shifts (1) or one GEMM per component (0)"),
    "cec_compose_fused": Knob("EVOXMI_CEC_COMPOSE_FUSED", 1, int, "CEC'22 compositions on the device: every component's basic function, the distances and the weighted sum in one kernel after the stacked GEMM (cec2022.hip: cec_compose_kernel) (1) or per-component launches (0)"),
    "cec_fused": Knob("EVOXMI_CEC_FUSED", 0, int, "CEC'22 F1 / F4 on the device: 1 = row terms from the rotation GEMM's epilogue (rotated population never written), 0 = GEMM + basic-function kernel (default: the fused epilogue measured 7 µs slower at pop 10 000 × d 1000, profiles/r3_cec_fused_epilogue.txt)"),
    "cec_rowterms_h3": Knob("EVOXMI_CEC_ROWTERMS_H3", 1, int, "CEC'22 F1 / F4 on the device with the f16x3 rotation: the basic function's row terms reduced in the GEMM epilogue (1; the rotated population is never written) or the GEMM + basic-function kernel (0)"),
    "gemm_prec": Knob("EVOXMI_GEMM_PREC", "x6", str, "framework f32 GEMMs (gemm_ks.hip): 'x6' — each f32 operand split exactly into three bf16 parts, six bf16 MFMA products (f32-accurate, 3/8 of the f32 MFMA time) — or 'f32' (v_mfma_f32_16x16x4_f32)"),
    "gemm_nw8_tiles": Knob("EVOXMI_GEMM_NW8_TILES", 384, int, "gemm_ks: grids of at most this many 64×64 (or smaller) tiles with K ≥ 3072 run 8-wave workgroups (K split 8 ways, two waves per SIMD: one wave's loads overlap the other's MFMAs; the rank-μ product 55.8 → 47.8 µs); 0 = always 4 waves"),
    "gemm_planes": Knob("EVOXMI_GEMM_PLANES", 0, int, "x6 GEMMs: the d×d operand that is constant (CEC rotations) or produced once per generation (CMA-ES B·D) pre-split into bf16 fragment planes (1) — alone 162.6 vs 174.3 µs for the 10k sampling GEMM, but in the flagship generation 175.8 vs 172.6 µs (the planes leave L2 between calls) and 1.825 vs 1.811 ms/gen, so off by default; 2 also generates the CMA-ES noise into planes (205 µs); 0 splits both inside the GEMM (profiles/r4_gemm_planes.log)"),
    "gemm_tall": Knob("EVOXMI_GEMM_TALL", "h3", str, "tall f32 NT products that fill the chip with 320×128 tiles (CMA-ES sampling 10 000×1000×1000, the CEC'22 rotation): 'h3' — operands split once into per-row-scaled f16 pairs (h + m, |x − h − m| ≤ 2⁻²²|x|) and multiplied by the LDS-staged gemm_blk.hip kernel as three f16 MFMA products (hh + hm + mh; ≤ 3·2⁻²²|ab| per product, inside the 2e-6·Σ|ab| bound of tests/test_gemm_blk.py; 73 µs vs 174-200 µs for gemm_ks at 10 000×1000×1000, profiles/r5_gemm_tall.jsonl) — or 'ks' (gemm_ks bf16x6)"),
    "plain_gemm": Knob("EVOXMI_PLAIN_GEMM", "evoxmi", str, "flagship GEMMs: 'evoxmi' (framework MFMA kernels, csrc/kernels/gemm_ks.hip) or 'blas' (hipBLASLt via torch, an A/B baseline only)"),
    "jacobi_sweeps": Knob("EVOXMI_JACOBI_SWEEPS", 2, int, "maximum warm-started Jacobi sweeps per decomposition (stops early once converged)"),
    "jacobi_tol_factor": Knob("EVOXMI_JACOBI_TOL_FACTOR", 4.0, float, "convergence: ‖offdiag‖ ≤ factor·eps_f32·sqrt(n)·‖diag‖"),
    "jacobi_inner_tol": Knob("EVOXMI_JACOBI_INNER_TOL", 1e-6, float, "per-subproblem skip threshold of the Jacobi solve kernel"),
    "jacobi_reortho": Knob("EVOXMI_JACOBI_REORTHO", 1, int, "Newton–Schulz re-orthonormalisation of the warm-start basis before each decomposition"),
    "jacobi_fused": Knob("EVOXMI_JACOBI_FUSED", 2, int, "Jacobi round pipeline: 2 = B update of round t-1 inside round t's solve launch; 0 = split solve/apply launches; 1 = experimental fused apply + next solve (slower, see profiles/NOTES.md)"),
    "jacobi_inner": Knob("EVOXMI_JACOBI_INNER", 1, int, "inner sweeps per 32×32 Jacobi subproblem"),
    "debug": Knob("EVOXMI_DEBUG", False, _bool, "synchronous kernel error-flag checks after fused kernels (not while capturing)"),
    "trace": Knob("EVOXMI_TRACE", False, _bool, "emit roctx ranges around ask / evaluate / tell in eager workflow steps"),
    "arch": Knob("EVOXMI_ARCH", "gfx950", str, "offload architecture the HIP extension is compiled for"),
    "check_replicas_every": Knob("EVOXMI_CHECK_REPLICAS_EVERY", 0, int, "distributed: checksum the replicated state across ranks every k generations (0 = off)"),
    "heartbeat_interval": Knob("EVOXMI_HEARTBEAT_INTERVAL", 5.0, float, "seconds between rank heartbeats written to the TCPStore"),
    "heartbeat_timeout": Knob("EVOXMI_HEARTBEAT_TIMEOUT", 60.0, float, "a rank whose heartbeat is older than this is reported dead"),
}

_overrides: Dict[str, Any] = {}


def get(name: str) -> Any:
    if name in _overrides:
        return _overrides[name]
    k = KNOBS[name]
    raw = os.environ.get(k.env)
    return k.default if raw is None else k.parse(raw)


def set(name: str, value: Any) -> None:  # noqa: A001 - mirrors get()
    if name not in KNOBS:
        raise KeyError(f"unknown evoxmi knob {name!r}; known: {sorted(KNOBS)}")
    _overrides[name] = value


def reset(name: str = None) -> None:
    if name is None:
        _overrides.clear()
    else:
        _overrides.pop(name, None)


@contextlib.contextmanager
def override(**kw):
    saved = {k: _overrides[k] for k in kw if k in _overrides}
    try:
        for k, v in kw.items():
            set(k, v)
        yield
    finally:
        for k in kw:
            _overrides.pop(k, None)
        _overrides.update(saved)


def describe() -> str:
    """Table of every knob, its environment variable and its current value."""
    rows = [f"{n:22s} {k.env:30s} {get(n)!r:>10}  {k.doc}" for n, k in KNOBS.items()]
    return "\n".join(rows)
