"""Dense linear algebra on the matrix cores.

``gemm`` is the framework's one general f32 GEMM (``csrc/kernels/gemm_f32.hip``,
``v_mfma_f32_32x32x2_f32``) with fused operand prologues and a fused epilogue:

    C = alpha·(*alpha_ptr)·Ã B̃ + bias_n[None, :] + beta·Cin
    Ã[m, k] = (A[m, k] − sub[m|k]) · kscale[k] · kw[k] · sscale

Operands are described by :class:`Operand`; ``rc=False`` means the tensor is
(rows, K) with K contiguous, ``rc=True`` means (K, rows) with rows contiguous
(optionally with K-row indirection ``gather``).  ``splits>1`` returns the
``(splits, M, N)`` split-K partial slabs (deterministic, no atomics).

The CPU branch materialises Ã and B̃ with torch and is the numerics oracle of
the GPU tests.

``mm`` is the flagship's product (``csrc/kernels/gemm_ks.hip``: the four waves of a
workgroup split K, operand fragments go global → registers with no LDS staging and no
barrier in the main loop, ``v_mfma_f32_16x16x4_f32``), with symmetric / skew-symmetric
output modes that compute only the upper tiles, a fused bias / Cin epilogue, a device
scale and a device ``skip`` word (device-side control of fixed iteration schedules).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Optional

import torch

from . import _ext


@dataclass
class Operand:
    t: torch.Tensor
    rc: bool = False
    gather: Optional[torch.Tensor] = None
    sub: Optional[torch.Tensor] = None
    sub_on_k: bool = False
    kscale: Optional[torch.Tensor] = None
    kw: Optional[torch.Tensor] = None
    sscale: Optional[torch.Tensor] = None
    sscale_inv: bool = False

    def materialise(self, rows: int, K: int) -> torch.Tensor:
        """Ã as a dense (rows, K) tensor (CPU reference)."""
        t = self.t
        if self.rc:
            src = t.index_select(0, self.gather.long()) if self.gather is not None else t[:K]
            X = src[:K, :rows].T
        else:
            X = t[:rows, :K]
        X = X.to(torch.float32)
        if self.sub is not None:
            X = X - (self.sub[:K][None, :] if self.sub_on_k else self.sub[:rows][:, None])
        if self.kscale is not None:
            X = X * self.kscale[:K][None, :]
        if self.kw is not None:
            X = X * self.kw[:K][None, :]
        if self.sscale is not None:
            s = self.sscale.reshape(())
            X = X / s if self.sscale_inv else X * s
        return X


def _c(x):
    return None if x is None else x.contiguous()


def gemm(a: Operand, b: Operand, M: int, N: int, K: int, alpha: float = 1.0, alpha_ptr=None, bias_n=None, beta: float = 0.0,
         Cin=None, splits: int = 1) -> torch.Tensor:
    if a.t.is_cuda:
        g = None if a.gather is None else a.gather.to(torch.int32).contiguous()
        gb = None if b.gather is None else b.gather.to(torch.int32).contiguous()
        return _ext.ops().gemm_f32(
            a.t, int(a.rc), g, _c(a.sub), int(a.sub_on_k), _c(a.kscale), _c(a.kw), _c(a.sscale), int(a.sscale_inv),
            b.t, int(b.rc), gb, _c(b.sub), int(b.sub_on_k), _c(b.kscale), _c(b.kw), _c(b.sscale), int(b.sscale_inv),
            _c(alpha_ptr), _c(bias_n), float(beta), Cin, int(M), int(N), int(K), int(splits), float(alpha),
        )
    A = a.materialise(M, K)
    B = b.materialise(N, K)
    s = alpha * (alpha_ptr.reshape(()) if alpha_ptr is not None else 1.0)
    if splits > 1:
        # same slab semantics as the kernel: slice z covers K range [z*kps, (z+1)*kps)
        kps = -(-K // splits)
        kps = -(-kps // 64) * 64
        sl = []
        for z in range(-(-K // kps)):
            k0, k1 = z * kps, min(K, (z + 1) * kps)
            sl.append(s * (A[:, k0:k1] @ B[:, k0:k1].T))
        out = torch.stack(sl)
        if bias_n is not None:
            out = out + bias_n[None, None, :N]
        return out
    C = s * (A @ B.T)
    if bias_n is not None:
        C = C + bias_n[None, :N]
    if Cin is not None:
        C = C + beta * Cin[:M, :N]
    return C


def matmul_nt(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """A @ B.T on the matrix cores (A: (M, K), B: (N, K))."""
    return gemm(Operand(A), Operand(B), A.shape[0], B.shape[0], A.shape[1])


def matmul(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """A @ B (A: (M, K) K-contiguous; B: (K, N) N-contiguous)."""
    return gemm(Operand(A), Operand(B, rc=True), A.shape[0], B.shape[1], A.shape[1])


def matmul_tn(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """A.T @ B (A: (K, M), B: (K, N), both row-major)."""
    return gemm(Operand(A, rc=True), Operand(B, rc=True), A.shape[1], B.shape[1], A.shape[0])


def plain_nt(A: torch.Tensor, B: torch.Tensor, alpha: float = 1.0, bias_n: Optional[torch.Tensor] = None,
             a_sub_k: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``alpha·(A − a_sub_k)·Bᵀ (+ bias_n)`` for plain row-major operands: the framework GEMM
    (:func:`mm`).  ``EVOXMI_PLAIN_GEMM=blas`` routes it to the vendor GEMM instead (hipBLASLt
    via ``torch.addmm``) — an A/B baseline, never the default."""
    from .. import config

    if A.is_cuda and config.get("plain_gemm") == "blas":
        if a_sub_k is not None:
            A = A - a_sub_k
        bias = bias_n if bias_n is not None else A.new_zeros(())
        return torch.addmm(bias, A, B.t(), beta=1.0 if bias_n is not None else 0.0, alpha=alpha)
    return mm(A, B, tb=True, alpha=alpha, bias_n=bias_n, a_sub_k=a_sub_k)


_PREC = {"x6": 1, "x6w": 2, "f32": 0}
_prec_set = [None, None]


def _sync_prec():
    """Push the ``gemm_prec`` knob to the kernel launcher (read at launch / capture time)."""
    from .. import config

    p = config.get("gemm_prec")
    if p != _prec_set[0]:
        if p not in _PREC:
            raise ValueError(f"EVOXMI_GEMM_PREC must be one of {sorted(_PREC)}, got {p!r}")
        _ext.ops().gemm_ks_set_prec(_PREC[p])
        _prec_set[0] = p
    t = config.get("gemm_nw8_tiles")
    if t != _prec_set[1]:
        _ext.ops().gemm_ks_set_nw8(int(t))
        _prec_set[1] = t


def mm(A: torch.Tensor, B: torch.Tensor, *, ta: bool = False, tb: bool = False, mode: int = 0, alpha: float = 1.0,
       alpha_ptr: Optional[torch.Tensor] = None, bias_n: Optional[torch.Tensor] = None, beta: float = 0.0,
       Cin: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
       skip: Optional[torch.Tensor] = None, a_sub_k: Optional[torch.Tensor] = None, sel: Optional[torch.Tensor] = None,
       A2: Optional[torch.Tensor] = None, alpha2: Optional[float] = None, C2: Optional[torch.Tensor] = None,
       stat_part: Optional[torch.Tensor] = None, stat_diag_only: bool = False, prec: Optional[str] = None,
       diag_add: float = 0.0) -> torch.Tensor:
    """``alpha·(*alpha_ptr)·op(A)·op(B) (+ bias_n) (+ beta·Cin)`` with ``op(X) = Xᵀ`` when
    ``ta`` / ``tb`` (transposes are layouts, never copies).  ``mode`` 1 / 2: the result is
    symmetric / skew-symmetric by construction of the caller (Bᵀ C B, X·X for skew X, …);
    only tiles with tm ≤ tn are computed and the rest mirrored.  ``out``: written in place.
    ``skip``: int32 device word — the kernel does nothing while it is non-zero.
    ``a_sub_k``: op(A)(m, k) − a_sub_k[k] (fused shift, ``op(A) = A`` only).
    ``sel`` (device only, with ``out``): int32 device word; while non-zero the kernel uses
    ``A2`` / ``alpha2`` / ``C2`` (when given; ``alpha2`` defaults to ``alpha``) instead of
    ``A`` / ``alpha`` / ``out``.
    ``stat_part`` (mode 1): float64 partials of [Σ offdiag², Σ diag², min diag, max diag] per
    workgroup (``sbr_stats_final`` layout; length ``4·gemm_ks_grid``); ``stat_diag_only``: the
    diagonal's terms only (Σ offdiag² left 0 — the cheaper epilogue of the eigensolver's X²).
    ``prec="x3"`` (device, with ``out``): bf16x3 products (≈1e-5 relative per product) for
    results that are a small correction of something held exactly (the eigensolver's
    exp(αX) − I terms); default: the process-wide f32-accurate precision.  ``diag_add``: added
    to the result's diagonal (``out=`` only; Bᵀ B − I).

    On a GPU this is always the framework kernel (no vendor GEMM); shapes the kernel does
    not take (K % 4 ≠ 0 with a K-contiguous operand) go to :func:`gemm`."""
    M = A.shape[1] if ta else A.shape[0]
    K = A.shape[0] if ta else A.shape[1]
    N = B.shape[0] if tb else B.shape[1]
    if A.is_cuda:
        a_kc, b_kc = not ta, tb
        ok = (K % 4 == 0) or not (a_kc or b_kc)
        A_ = A if A.stride(-1) == 1 else A.contiguous()
        B_ = B if B.stride(-1) == 1 else B.contiguous()
        sub_ok = a_sub_k is None or (a_kc and a_sub_k.is_contiguous() and a_sub_k.data_ptr() % 16 == 0)
        if ok and sub_ok and A_.data_ptr() % 16 == 0 and B_.data_ptr() % 16 == 0:
            _sync_prec()
            args = (A_, int(a_kc), B_, int(b_kc), int(M), int(N), int(K), int(mode), float(alpha), alpha_ptr, bias_n,
                    float(beta), Cin)
            if out is not None:
                a2 = float(alpha if alpha2 is None else alpha2)
                _ext.ops().gemm_ks_out(*args, out, skip, a_sub_k, sel, A2, a2, C2, stat_part, int(stat_diag_only),
                                       3 if prec == "x3" else 0, float(diag_add))
                return out
            if sel is not None or stat_part is not None or prec is not None or diag_add:
                raise ValueError("mm: sel / stat_part / prec / diag_add need out=")
            return _ext.ops().gemm_ks(*args, skip, a_sub_k)
        if skip is not None or sel is not None or stat_part is not None:
            raise ValueError("mm: skip / sel / stat_part need a shape the gemm_ks kernel takes")
        Ao = Operand(A_, rc=ta, sub=a_sub_k, sub_on_k=a_sub_k is not None)
        C = gemm(Ao, Operand(B_, rc=not tb), M, N, K, alpha=alpha, alpha_ptr=alpha_ptr, bias_n=bias_n, beta=beta, Cin=Cin)
        if out is not None:
            out.copy_(C)
            return out
        return C
    Am = A.t() if ta else A
    Bm = B.t() if tb else B
    s = alpha * (alpha_ptr.reshape(()) if alpha_ptr is not None else 1.0)
    Am = Am[:M, :K].to(torch.float32)
    if a_sub_k is not None:
        Am = Am - a_sub_k[None, :K]
    C = s * (Am @ Bm[:K, :N].to(torch.float32))
    if bias_n is not None:
        C = C + bias_n[None, :N]
    if Cin is not None:
        C = C + beta * Cin[:M, :N]
    if diag_add:
        C = C + diag_add * torch.eye(M, N, dtype=C.dtype)
    if skip is not None and int(skip.reshape(-1)[0]) != 0:
        return out if out is not None else torch.zeros(M, N, dtype=torch.float32)
    if out is not None:
        out.copy_(C)
        return out
    return C


def mm_nt(A, B, *, alpha: float = 1.0, alpha_ptr: Optional[torch.Tensor] = None, bias_n: Optional[torch.Tensor] = None,
          out: Optional[torch.Tensor] = None, a_sub_k: Optional[torch.Tensor] = None, sub_cols: int = 0) -> torch.Tensor:
    """``alpha·(*alpha_ptr)·(A − a_sub_k)·Bᵀ (+ bias_n)`` for f32 A (M × K) and B (N × K).

    ``sub_cols > 0``: ``a_sub_k`` is a (blocks, K) matrix and output columns
    [c·sub_cols, (c+1)·sub_cols) use shift row c — several shifted products that share A (the
    CEC'22 composition rotations) in ONE launch that reads A's row panels once per tile."""
    if sub_cols:
        if not A.is_cuda:
            blocks = [((A - a_sub_k[c][None, :]) @ B[c * sub_cols : (c + 1) * sub_cols].T) for c in range(a_sub_k.shape[0])]
            C = alpha * torch.cat(blocks, 1)[:, : B.shape[0]]
            return C if alpha_ptr is None else C * alpha_ptr.reshape(())
        return _ext.ops().gemm_ks_pl(A, None, B, None, int(A.shape[0]), int(B.shape[0]), int(A.shape[1]), float(alpha), alpha_ptr, bias_n,
                                     out, a_sub_k.contiguous(), int(sub_cols), int(a_sub_k.stride(0)))
    return mm(A, B, tb=True, alpha=alpha, alpha_ptr=alpha_ptr, bias_n=bias_n, out=out, a_sub_k=a_sub_k)


# ---------------------------------------------------------------------------- blocked planes
class BlkPlanes:
    """An f32 matrix (rows × K) pre-split for the LDS-staged bf16x6 GEMM (``gemm_blk.hip``):
    bf16 [ceil(K/16)][Rp][3][16] — per 16-k block and row the high / middle / low bf16 parts
    of its 16 values in one 96-byte record, so a GEMM stage of BM rows is one contiguous copy.
    Built by :func:`blk_planes` (split pass, optional fused shift / column scale) or
    :func:`normal_blk_planes` (Philox noise generated straight into planes).  On the CPU the
    object holds the (shifted, scaled) f32 matrix itself."""

    __slots__ = ("t", "rows", "K")

    def __init__(self, t: torch.Tensor, rows: int, K: int):
        self.t, self.rows, self.K = t, int(rows), int(K)

    @property
    def is_cuda(self) -> bool:
        return self.t.is_cuda


def blk_planes(X: torch.Tensor, sub_k: Optional[torch.Tensor] = None, colscale: Optional[torch.Tensor] = None,
               out: Optional[torch.Tensor] = None) -> BlkPlanes:
    """Blocked planes of ``(X − sub_k[None, :])·diag(colscale)`` (shift and scale fused into the
    split pass; ``out``: a buffer from a previous call of the same shape, reused)."""
    rows, K = X.shape
    if X.is_cuda:
        X_ = X if X.stride(-1) == 1 else X.contiguous()
        return BlkPlanes(_ext.ops().blk_split(X_, _c(sub_k), _c(colscale), out), rows, K)
    Y = X.to(torch.float32)
    if sub_k is not None:
        Y = Y - sub_k[None, :K]
    if colscale is not None:
        Y = Y * colscale[None, :K]
    return BlkPlanes(Y, rows, K)


def normal_blk_planes(key: torch.Tensor, rows: int, d: int, row0: int = 0, out: Optional[torch.Tensor] = None) -> BlkPlanes:
    """Blocked planes of rows [row0, row0 + rows) of ``random.normal(key, (·, d))``, generated in
    place (the f32 noise is never written); d % 4 == 0 on the device."""
    if key.is_cuda and d % 4 == 0:
        return BlkPlanes(_ext.ops().blk_philox_normal(key.contiguous(), int(rows), int(d), int(row0), out), rows, d)
    from . import random as rnd

    return BlkPlanes(rnd.normal(key, (rows, d), offset=row0 * d).to(key.device), rows, d)


def blk_tile() -> tuple:
    """(BM, BN) output tile of the blocked-planes GEMM."""
    return int(_ext.ops().gemm_blk_tile(0)), int(_ext.ops().gemm_blk_tile(1))


def blk_worthwhile(M: int, N: int, n_cu: int = 256) -> bool:
    """True when the f16x3 tall launch fills the chip: the 320 × 128-tile launch with ≥ ¾ of
    the CUs busy in its last wave of tiles, or a population shard's product (M ≥ 1024 rows,
    N ≥ 512: ``evx_gemm_h3`` then takes the shortest of 64 / 128 / 192-row tiles whose tiles fit
    one wave of 256 — the sharded flagship's 5000 / 2500 / 1250 × 1000 × 1000 sampling and
    rotation products, which on the K-split ``gemm_ks`` ran at 100 / 37 µs each,
    profiles/r6_phase_table_sim.md).
    Smaller products stay on ``gemm_ks``."""
    tiles = -(-M // 320) * -(-N // 128)
    if M >= 1024 and N >= 512:
        return True
    if tiles < (3 * n_cu) // 4:
        return False
    rem = tiles % n_cu
    return rem == 0 or rem >= (3 * n_cu) // 4 or tiles >= 4 * n_cu


def mm_blk(A: BlkPlanes, B: BlkPlanes, *, alpha: float = 1.0, alpha_ptr: Optional[torch.Tensor] = None,
           bias_n: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
           skip: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``alpha·(*alpha_ptr)·A·Bᵀ (+ bias_n)`` for blocked-planes operands (A: M × K, B: N × K)."""
    if A.K != B.K:
        raise ValueError(f"mm_blk: K mismatch {A.K} vs {B.K}")
    if A.is_cuda:
        return _ext.ops().gemm_blk(A.t, A.rows, B.t, B.rows, A.K, float(alpha), _c(alpha_ptr), _c(bias_n), out, skip)
    C = alpha * (A.t @ B.t.T)
    if alpha_ptr is not None:
        C = C * alpha_ptr.reshape(())
    if bias_n is not None:
        C = C + bias_n[None, : B.rows]
    if skip is not None and int(skip.reshape(-1)[0]) != 0:
        return out if out is not None else torch.zeros_like(C)
    if out is not None:
        out.copy_(C)
        return out
    return C


# ---------------------------------------------------------------------------- f16x3 planes
class H3Planes:
    """An f32 matrix (rows × K) split for the f16x3 GEMM (``gemm_blk.hip: gemm_h3_kernel``):
    each row scaled by a power of two (largest |x| ≤ 2¹⁵), then split into two f16 parts
    h + m (RNE; |x − h − m| ≤ 2⁻²²|x|), stored as f16 [ceil(K/16)][Rp][2][16] 64-byte records
    with the row's inverse scale in ``rinv``.  The product keeps h·h + h·m + m·h (three
    v_mfma_f32_32x32x16_f16 per 32 × 32 block and 16-k block).  On the CPU ``t`` is the f32
    matrix (``ncomp`` × rows × K when stacked) and ``rinv`` is None.  ``ncomp`` > 1: one plane set
    per shift row (:func:`h3_planes` with a 2-D ``sub_k``), for :func:`mm_h3` ``sub_cols``."""

    __slots__ = ("t", "rinv", "rows", "K", "ncomp")

    def __init__(self, t: torch.Tensor, rinv: Optional[torch.Tensor], rows: int, K: int, ncomp: int = 1):
        self.t, self.rinv, self.rows, self.K, self.ncomp = t, rinv, int(rows), int(K), int(ncomp)

    @property
    def is_cuda(self) -> bool:
        return self.t.is_cuda


def h3_planes(X: torch.Tensor, sub_k: Optional[torch.Tensor] = None, colscale: Optional[torch.Tensor] = None,
              out: Optional[H3Planes] = None) -> H3Planes:
    """f16x3 planes of ``(X − sub_k[None, :])·diag(colscale)`` (shift and scale fused into the
    split pass; ``out``: planes of the same shape from an earlier call, overwritten).  A 2-D
    ``sub_k`` (ncomp × K) gives one plane set per shift row from one read of X."""
    rows, K = X.shape
    ncomp = sub_k.shape[0] if sub_k is not None and sub_k.dim() == 2 else 1
    if X.is_cuda:
        X_ = X if X.stride(-1) == 1 else X.contiguous()
        t, r = _ext.ops().h3_split(X_, _c(sub_k), _c(colscale), None if out is None else out.t, None if out is None else out.rinv)
        return H3Planes(t, r, rows, K, ncomp)
    Y = X.to(torch.float32)
    if sub_k is not None:
        Y = Y - (sub_k[None, :K] if sub_k.dim() == 1 else sub_k[:, None, :K])
    if colscale is not None:
        Y = Y * colscale[None, :K]
    return H3Planes(Y, None, rows, K, ncomp)


def normal_h3_planes(key: torch.Tensor, rows: int, d: int, row0: int = 0, out: Optional[H3Planes] = None) -> H3Planes:
    """f16x3 planes of rows [row0, row0 + rows) of ``random.normal(key, (·, d))`` generated in
    place (fixed scale 2¹³; the f32 noise is never written); d % 4 == 0 on the device."""
    if key.is_cuda and d % 4 == 0:
        t, r = _ext.ops().h3_philox_normal(key.contiguous(), int(rows), int(d), int(row0), None if out is None else out.t,
                                           None if out is None else out.rinv)
        return H3Planes(t, r, rows, d)
    from . import random as rnd

    return H3Planes(rnd.normal(key, (rows, d), offset=row0 * d).to(key.device), None, rows, d)


def mm_h3(A: H3Planes, B: H3Planes, *, alpha: float = 1.0, alpha_ptr: Optional[torch.Tensor] = None,
          bias_n: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
          skip: Optional[torch.Tensor] = None, sub_cols: int = 0) -> torch.Tensor:
    """``alpha·(*alpha_ptr)·A·Bᵀ (+ bias_n)`` for f16x3-planes operands (A: M × K, B: N × K).
    ``sub_cols`` > 0: A is stacked (``A.ncomp`` plane sets) and output columns
    [c·sub_cols, (c+1)·sub_cols) use set c — e.g. (x − o_c)·M_cᵀ for every component c of a
    composition function in one launch."""
    if A.K != B.K:
        raise ValueError(f"mm_h3: K mismatch {A.K} vs {B.K}")
    if sub_cols:
        if A.ncomp < -(-B.rows // sub_cols):
            raise ValueError(f"mm_h3: {B.rows} columns in blocks of {sub_cols} need {-(-B.rows // sub_cols)} plane sets, A has {A.ncomp}")
    elif A.ncomp != 1:
        raise ValueError("mm_h3: stacked A needs sub_cols")
    if A.is_cuda:
        return _ext.ops().gemm_h3(A.t, A.rinv, A.rows, B.t, B.rinv, B.rows, A.K, float(alpha), _c(alpha_ptr), _c(bias_n), out, skip,
                                  int(sub_cols))
    if sub_cols:
        C = alpha * torch.cat([A.t[c] @ B.t[c * sub_cols : (c + 1) * sub_cols].T for c in range(-(-B.rows // sub_cols))], 1)
    else:
        C = alpha * (A.t @ B.t.T)
    if alpha_ptr is not None:
        C = C * alpha_ptr.reshape(())
    if bias_n is not None:
        C = C + bias_n[None, : B.rows]
    if skip is not None and int(skip.reshape(-1)[0]) != 0:
        return out if out is not None else torch.zeros_like(C)
    if out is not None:
        out.copy_(C)
        return out
    return C


def tall_nt_ok(M: int, N: int, K: int, device) -> bool:
    """True when ``tall_nt`` takes the f16x3 LDS-staged path for an M × N × K NT product."""
    from .. import config

    return (device.type == "cuda" and config.get("gemm_tall") == "h3" and config.get("plain_gemm") == "evoxmi"
            and blk_worthwhile(M, N))


def tall_nt(A: torch.Tensor, B: torch.Tensor, *, alpha: float = 1.0, alpha_ptr: Optional[torch.Tensor] = None,
            bias_n: Optional[torch.Tensor] = None, a_sub_k: Optional[torch.Tensor] = None,
            b_colscale: Optional[torch.Tensor] = None, b_planes: Optional[H3Planes] = None,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``alpha·(*alpha_ptr)·(A − a_sub_k)·(B·diag(b_colscale))ᵀ (+ bias_n)`` for a tall product
    (A: M × K, B: N × K): the f16x3 path (:func:`mm_h3`) when :func:`tall_nt_ok`, otherwise
    the bf16x6 ``gemm_ks`` kernel.  ``b_planes``: B's planes already split (a constant operand
    cached by the caller); ``A`` may be an :class:`H3Planes` (a producer wrote them)."""
    M = A.rows if isinstance(A, H3Planes) else A.shape[0]
    K = A.K if isinstance(A, H3Planes) else A.shape[1]
    N = B.shape[0]
    dev = A.t.device if isinstance(A, H3Planes) else A.device
    if isinstance(A, H3Planes) or tall_nt_ok(M, N, K, dev):
        Ap = A if isinstance(A, H3Planes) else h3_planes(A, sub_k=a_sub_k)
        Bp = b_planes if b_planes is not None else h3_planes(B, colscale=b_colscale)
        return mm_h3(Ap, Bp, alpha=alpha, alpha_ptr=alpha_ptr, bias_n=bias_n, out=out)
    Bs = B if b_colscale is None else (B * b_colscale[None, :]).contiguous()
    return mm(A, Bs, tb=True, alpha=alpha, alpha_ptr=alpha_ptr, bias_n=bias_n, out=out, a_sub_k=a_sub_k)
