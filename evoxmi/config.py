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
    "sbr_block": Knob("EVOXMI_SBR_BLOCK", 32, int, "sbr: near-pair block size — 32 or 16 (blocks in a shifted sorted order, eigh_sbr16.hip; 32 converges in fewer iterations on the bench matrices) or 64 (eigh_sbr.hip)"),
    "sbr_mode": Knob("EVOXMI_SBR_MODE", "device", str, "sbr: 'device' — fixed device-controlled iteration schedule inside the generation's graph (ops/sbr_device.py, no host read); 'host' — host-driven iterations with planned solves as a host phase between graph segments (ops/sbr.py)"),
    "sbr_device_iters": Knob("EVOXMI_SBR_DEVICE_ITERS", 7, int, "device eigensolver: refinement slots of the warm schedule (the tuned constants of the three schedules are in ops/sbr_device.py) (kernels of iterations past convergence return at once; round 5: 8 → 7 slots, 1.644-1.656 → 1.630 ms at 20 steps — warm solves at d ≤ 1000 take at most 6 iterations on F1 / F4 / F6 / F12 over 200 generations, and a capped solve escalates the schedule)"),
    "sbr_cold_iters": Knob("EVOXMI_SBR_COLD_ITERS", 16, int, "CMA-ES device eigensolver: refinement slots of the cold-start schedule (every run starts on it; CMAES moves down to the warm / late schedules after consecutive solves that fit them with a slot to spare)"),
    "sbr_late_iters": Knob("EVOXMI_SBR_LATE_ITERS", 5, int, "refinement slots of the late (settled) eigensolver schedule (settled solves take 4; a capped or slow solve moves the run back up two generations later — round 5: 6 → 5 slots, 1.439 → 1.424 ms over 50 steps)"),
    "sbr_corr_prec": Knob("EVOXMI_SBR_CORR_PREC", "x3late", str, "device eigensolver: precision of the correction products — 'x3': the Taylor terms of exp(αX) − I (X², X³, the Vᵀ GEMM) as bf16x3 (≈1e-5 of the correction's own size; the basis update Bq + Bq·(V − I), Newton–Schulz and the residual products Bᵀ C B, TᵀT stay bf16x6); 'x3late' (default): as 'x3', plus the basis update and Newton–Schulz correction at bf16x3 in the late (settled) schedule level only (50 steps 1.345 vs 1.363 ms; the eigensolver GPU tests pass unchanged); 'x3all': the basis update and Newton–Schulz's T·(TᵀT − I) at every level (2 % faster; trajectory parity over 15 seeds as good as x6, but one fallback in the degenerate-spectrum stress test tests/test_sbr_device_gpu.py::test_sim8_trajectory_recovers_from_divergence); 'x6': every product f32-accurate (the round-5 solver)"),
    "cma_fused": Knob("EVOXMI_CMA_FUSED", 1, int, "CMA-ES tell epilogue as the fused cmaes.hip kernels (0: reference-shaped torch ops)"),
    "cec_stack": Knob("EVOXMI_CEC_STACK", 1, int, "CEC'22 compositions (F9–F12) on the device: every rotated component from ONE GEMM over the stacked rotations with per-block exact shifts (1) or one GEMM per component (0)"),
    "cec_compose_fused": Knob("EVOXMI_CEC_COMPOSE_FUSED", 1, int, "CEC'22 compositions on the device: every component's basic function, the distances and the weighted sum in one kernel after the stacked GEMM (cec2022.hip: cec_compose_kernel) (1) or per-component launches (0)"),
    "cec_fused": Knob("EVOXMI_CEC_FUSED", 0, int, "CEC'22 F1 / F4 on the device: 1 = row terms from the rotation GEMM's epilogue (rotated population never written), 0 = GEMM + basic-function kernel (default: the fused epilogue measured 7 µs slower at pop 10 000 × d 1000, profiles/r3_cec_fused_epilogue.txt)"),
    "cec_rowterms_h3": Knob("EVOXMI_CEC_ROWTERMS_H3", 1, int, "CEC'22 F1 / F4 on the device with the f16x3 rotation: the basic function's row terms reduced in the GEMM epilogue (1; the rotated population is never written) or the GEMM + basic-function kernel (0)"),
    "gemm_prec": Knob("EVOXMI_GEMM_PREC", "x6", str, "framework f32 GEMMs (gemm_ks.hip): 'x6' — each f32 operand split exactly into three bf16 parts, six bf16 MFMA products (f32-accurate, 3/8 of the f32 MFMA time) — or 'f32' (v_mfma_f32_16x16x4_f32)"),
    "gemm_nw8_tiles": Knob("EVOXMI_GEMM_NW8_TILES", 384, int, "gemm_ks: grids of at most this many 64×64 (or smaller) tiles with K ≥ 3072 run 8-wave workgroups (K split 8 ways, two waves per SIMD: one wave's loads overlap the other's MFMAs; the rank-μ product 55.8 → 47.8 µs); 0 = always 4 waves"),
    "gemm_tall": Knob("EVOXMI_GEMM_TALL", "h3", str, "tall f32 NT products that fill the chip with 320×128 tiles (CMA-ES sampling 10 000×1000×1000, the CEC'22 rotation): 'h3' — operands split once into per-row-scaled f16 pairs (h + m, |x − h − m| ≤ 2⁻²²|x|) and multiplied by the LDS-staged gemm_blk.hip kernel as three f16 MFMA products (hh + hm + mh; ≤ 3·2⁻²²|ab| per product, inside the 2e-6·Σ|ab| bound of tests/test_gemm_blk.py; 73 µs vs 174-200 µs for gemm_ks at 10 000×1000×1000, profiles/r5_gemm_tall.jsonl) — or 'ks' (gemm_ks bf16x6)"),
    "plain_gemm": Knob("EVOXMI_PLAIN_GEMM", "evoxmi", str, "flagship GEMMs: 'evoxmi' (framework MFMA kernels, csrc/kernels/gemm_ks.hip) or 'blas' (hipBLASLt via torch, an A/B baseline only)"),
    "jacobi_sweeps": Knob("EVOXMI_JACOBI_SWEEPS", 2, int, "maximum warm-started Jacobi sweeps per decomposition (stops early once converged)"),
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
