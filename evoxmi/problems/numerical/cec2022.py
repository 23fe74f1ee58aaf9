"""CEC 2022 single-objective bound-constrained suite, F1–F12.

Parity: reference ``src/evox/problems/numerical/cec2022_so.py`` (the fork's
addition): shift → scale → rotate → shuffle (``ssr_operat`` ``:109-119``), the 16
basic functions (``:139-345``), hybrid functions F6–F8 on shuffled segments, and
distance-weighted compositions F9–F12 (``compose_operat`` ``:121-135``).  Reference
quirks are kept: no CEC bias offsets, Levy uses ``1 + z/4``,
F3 evaluates Schaffer-F7 on the *unrotated* shifted vector, F7's Schaffer-F7
segment reads its ``y`` from the head of the shuffled vector, F12's sixth
component reuses the fifth shift/rotation, the ``f < 1e-8 → 0`` clamp.

Data: the official shift/rotation/shuffle files for D ∈ {2, 10, 20} ship in
``cec2022_input_data`` (benchmark data).  Any other D (e.g. the north-star
D = 1000) uses **synthetic** data generated deterministically from
``(func_num, D, seed)``: shifts ~ U(−80, 80), Haar-random orthogonal rotations
(QR of a Gaussian, sign-corrected, float64 → float32) and random shuffles — a
documented deviation, since the reference has no data beyond D = 20.

Execution (K6 of SURVEY §2.10): every rotation ``M (x − o)·s`` is one f32 MFMA
GEMM with the shift and scale fused into the A-operand prologue; the basic
functions, hybrid segments (with the shuffle applied as an index gather) and
composition distances are one wave-per-row HIP reduction kernel each
(``csrc/kernels/cec2022.hip``).  The torch code below is the CPU path and the
numerics oracle.
"""
from __future__ import annotations

import math
import os
from functools import lru_cache

import numpy as np
import torch

from ...core import Problem
from ...ops import linalg
from ...ops import _ext
from ...ops import numerical as nops

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "cec2022_input_data")
OFFICIAL_DIMS = (2, 10, 20)

# basic-function ids shared with the HIP kernel
ZAKHAROV, ROSENBROCK, SCHAFFERF7, RASTRIGIN, LEVY, BENTCIGAR, HGBAT, KATSUURA = range(8)
ACKLEY, SCHWEFEL, HAPPYCAT, ELLIPTIC, DISCUS, EXPSCHAFFER, EXPGRIEROSEN, GRIEWANK, SPHERE = range(8, 17)


# ------------------------------------------------------------------------- data
def _read_matrix(path):
    with open(path) as f:
        return np.array([[float(v) for v in line.split()] for line in f if line.strip()], dtype=np.float64)


def _read_vector(path):
    with open(path) as f:
        return np.array([float(v) for v in f.read().split()], dtype=np.float64)


def _haar(rng, d):
    a = rng.standard_normal((d, d))
    q, r = np.linalg.qr(a)
    return q * np.sign(np.diag(r))[None, :]


@lru_cache(maxsize=64)
def cec2022_data(func_num: int, D: int, seed: int = 2022):
    """(Os, M, S) as float64/int numpy arrays for function ``func_num`` at dimension ``D``."""
    comp = {9: 5, 10: 3, 11: 5, 12: 6}.get(func_num, 1)
    if D in OFFICIAL_DIMS:
        if func_num >= 9:
            Os = _read_matrix(os.path.join(_DATA, f"shift_data_{func_num}.txt"))[:, :D]
        else:
            Os = _read_vector(os.path.join(_DATA, f"shift_data_{func_num}.txt"))[:D]
        M = _read_matrix(os.path.join(_DATA, f"M_{func_num}_D{D}.txt"))
        S = None
        if func_num in (6, 7, 8) and D in (10, 20):
            S = _read_vector(os.path.join(_DATA, f"shuffle_data_{func_num}_D{D}.txt")).astype(np.int64)
        return Os, M, S
    rng = np.random.default_rng([seed, func_num, D])
    if func_num >= 9:
        Os = rng.uniform(-80.0, 80.0, size=(10, D))
        M = np.concatenate([_haar(rng, D) for _ in range(comp)], axis=0)
    else:
        Os = rng.uniform(-80.0, 80.0, size=(D,))
        M = _haar(rng, D)
    S = rng.permutation(D).astype(np.int64) + 1 if func_num in (6, 7, 8) else None
    return Os, M, S


def _group_ids(p, D):
    sizes = np.round(np.asarray(p) * D).astype(int)
    bounds = np.concatenate([[0], np.cumsum(sizes[:-1])])
    ends = np.concatenate([bounds[1:], [D]])
    return [(int(b), int(e - b)) for b, e in zip(bounds, ends)]


# ------------------------------------------------------------------------- torch basic functions
def _t_basic(fid, z, y=None):
    """Basic function ``fid`` on rows of z (N, L) → (N,). Mirrors cec2022_so.py:139-345."""
    L = z.shape[1]
    dev, dt = z.device, z.dtype
    if fid == ZAKHAROV:
        i = torch.arange(1, L + 1, device=dev, dtype=dt)
        t1 = (z * z).sum(1)
        t2 = (0.5 * i * z).sum(1)
        return t1 + t2**2 + t2**4
    if fid == ROSENBROCK:
        z = z + 1
        return 100 * ((z[:, :-1] ** 2 - z[:, 1:]) ** 2).sum(1) + ((1 - z[:, :-1]) ** 2).sum(1)
    if fid == SCHAFFERF7:
        nx = L
        s = torch.sqrt(y[:, : nx - 1] ** 2 + y[:, 1:nx] ** 2)
        tmp = torch.sin(50.0 * s**0.2)
        f = (s**0.5 + s**0.5 * tmp * tmp).sum(1)
        return f * f / (nx - 1) / (nx - 1)
    if fid == RASTRIGIN:
        z = z * 0.0512
        return (z * z - 10 * torch.cos(2 * math.pi * z) + 10).sum(1)
    if fid == LEVY:
        w = 1 + z / 4
        t1 = torch.sin(math.pi * w[:, 0]) ** 2
        w1 = w[:, :-1]
        t2 = (((w1 - 1) ** 2) * (1 + 10 * torch.sin(math.pi * w1 + 1) ** 2)).sum(1)
        wl = w[:, -1]
        t3 = ((wl - 1) ** 2) * (1 + torch.sin(2 * math.pi * wl) ** 2)
        return t1 + t2 + t3
    if fid == BENTCIGAR:
        return z[:, 0] ** 2 + 1e6 * (z[:, 1:] ** 2).sum(1)
    if fid == HGBAT:
        z = z * 0.05 - 1
        s2 = (z * z).sum(1)
        s1 = z.sum(1)
        return torch.abs(s2**2 - s1**2) ** 0.5 + (0.5 * s2 + s1) / L + 0.5
    if fid == KATSUURA:
        z = z * 0.05
        j = torch.arange(1, 33, device=dev, dtype=dt)
        p = 2.0**j
        t = (z[:, :, None] * p)
        temp = (torch.abs(t - torch.floor(t + 0.5)) / p).sum(2)
        i = torch.arange(1, L + 1, device=dev, dtype=dt)
        tmp3 = float(L) ** 1.2
        f = torch.prod((1.0 + i * temp) ** (10.0 / tmp3), dim=1)
        c = 10.0 / L / L
        return f * c - c
    if fid == ACKLEY:
        return -20 * torch.exp(-0.2 * torch.sqrt((z * z).sum(1) / L)) - torch.exp(torch.cos(2 * math.pi * z).sum(1) / L) + 20 + math.e
    if fid == SCHWEFEL:
        z = z * 10 + 4.209687462275036e002
        a = torch.fmod(z, 500.0)
        aa = torch.fmod(torch.abs(z), 500.0)
        big = -(500.0 - a) * torch.sin(torch.sqrt(500.0 - a)) + ((z - 500.0) / 100) ** 2 / L
        small = -(-500.0 + aa) * torch.sin(torch.sqrt(500.0 - aa)) + ((z + 500.0) / 100) ** 2 / L
        mid = -z * torch.sin(torch.sqrt(torch.abs(z)))
        term = torch.where(z > 500, big, torch.where(z < -500, small, mid))
        return term.sum(1) + 4.189828872724338e002 * L
    if fid == HAPPYCAT:
        z = z * 0.05 - 1
        s2 = (z * z).sum(1)
        s1 = z.sum(1)
        return torch.abs(s2 - L) ** 0.25 + (0.5 * s2 + s1) / L + 0.5
    if fid == ELLIPTIC:
        i = torch.arange(L, device=dev, dtype=dt)
        return ((10.0 ** (6 * i / (L - 1))) * z * z).sum(1)
    if fid == DISCUS:
        return 1e6 * z[:, 0] ** 2 + (z[:, 1:] ** 2).sum(1)
    if fid == EXPSCHAFFER:
        zr = torch.roll(z, 1, dims=1)
        sq = z * z + zr * zr
        return (0.5 + (torch.sin(torch.sqrt(sq)) ** 2 - 0.5) / (1 + 0.001 * sq) ** 2).sum(1)
    if fid == EXPGRIEROSEN:
        z = z * 0.05 + 1
        zn = torch.roll(z, -1, dims=1)
        t1 = z * z - zn
        t2 = z - 1.0
        temp = 100.0 * t1 * t1 + t2 * t2
        return (temp * temp / 4000.0 - torch.cos(temp) + 1.0).sum(1)
    if fid == GRIEWANK:
        i = torch.arange(1, L + 1, device=dev, dtype=dt)
        return (z * z).sum(1) / 4000 - torch.prod(torch.cos(z / torch.sqrt(i)), 1) + 1
    if fid == SPHERE:
        return (z * z).sum(1)
    raise ValueError(fid)


# ------------------------------------------------------------------------- problem classes
class _CEC2022(Problem):
    func_num = 0

    def __init__(self, dim: int = None, seed: int = 2022, device=None):
        super().__init__()
        self.dim = dim
        self.seed = seed
        self._cache = {}

    def _consts(self, D, device):
        key = (D, str(device))
        if key not in self._cache:
            Os, M, S = cec2022_data(self.func_num, D, self.seed)
            c = {
                "Os": torch.as_tensor(Os, dtype=torch.float32, device=device),
                "M": torch.as_tensor(M, dtype=torch.float32, device=device).contiguous(),
                "S": None if S is None else torch.as_tensor(S - 1, dtype=torch.int32, device=device),
            }
            self._cache[key] = c
        return self._cache[key]

    # ssr: z = M (x − o)·s.  The shift is applied to the operand before the products (exact
    # zero at the optimum, as in the reference): on the device it is the GEMM's fused A
    # prologue (no shifted copy of the population), the scale folds into the epilogue.
    def _ssr(self, X, o, M, s):
        N, D = X.shape
        if X.is_cuda:
            from ... import config

            if linalg.tall_nt_ok(N, M.shape[0], D, X.device):
                # tall rotation on the f16x3 LDS-staged GEMM: the population's planes with the
                # shift fused into the split pass; the constant rotation split once and cached
                key = ("h3", M.data_ptr(), M.shape)
                pl = self._cache.get(key)
                if pl is None:
                    pl = self._cache[key] = linalg.h3_planes(M)
                return linalg.tall_nt(X, M, alpha=float(s), a_sub_k=o.contiguous(), b_planes=pl)
            return linalg.plain_nt(X, M, alpha=float(s), a_sub_k=o.contiguous())
        return ((X - o) * s) @ M.T

    def _basic(self, Z, fid, perm=None, start=0, length=None, sub=None, scale=1.0, ysrc=None, ystart=0, clamp=None):
        """fid on z_eff[:, j] = (Z[:, idx_j] − sub[idx_j])·scale, idx_j = perm[start+j] (or start+j).
        ``clamp``: the f < clamp → 0 rule of the CEC'22 evaluation, fused into the device kernel."""
        N, D = Z.shape
        L = D - start if length is None else length
        if Z.is_cuda:
            return nops.cec_basic(Z, fid, perm, start, L, sub, scale, ysrc, ystart, clamp=clamp or 0.0)
        if clamp:
            return self._clamp(self._basic(Z, fid, perm, start, length, sub, scale, ysrc, ystart), clamp)
        idx = torch.arange(start, start + L, device=Z.device)
        if perm is not None:
            idx = perm.long()[idx]
        z = Z[:, idx]
        if sub is not None:
            z = z - sub[idx][None, :]
        z = z * scale
        y = None
        if fid == SCHAFFERF7:
            y = ysrc[:, ystart : ystart + L] if ysrc is not None else z
        return _t_basic(fid, z, y)

    @staticmethod
    def _clamp(f, thr=1e-8):
        return torch.where(f < thr, torch.zeros_like(f), f)

    def _compose(self, X, fs, Os, bias, sigma, lamb, d2=None):
        N, D = X.shape
        n = fs.shape[1]
        if d2 is None:
            d2 = torch.stack([self._basic(X, SPHERE, sub=Os[i]) for i in range(n)], 1)
        t1 = 1 / torch.sqrt(d2)
        t2 = torch.exp(-0.5 * d2 / (self._const_vec(sigma, X) ** 2 * D))
        W = t1 * t2
        # reference intent (cec2022_so.py:130-132): a zero distance selects that component;
        # 1/sqrt(0) is +inf (not NaN), so test finiteness instead of isnan
        nan = ~torch.isfinite(t1)
        any_nan = nan.any(1, keepdim=True)
        Wn = torch.where(any_nan, nan.to(X.dtype) / nan.sum(1, keepdim=True).clamp_min(1), W / W.sum(1, keepdim=True))
        return (Wn * (self._const_vec(lamb, X) * fs + self._const_vec(bias, X))).sum(1)

    _vecs = {}

    @classmethod
    def _const_vec(cls, vals, X):
        """Composition constants as device tensors, made once (the eager warm-up step) so a
        captured hipGraph never issues a host-to-device copy."""
        key = (tuple(float(v) for v in vals), str(X.device), X.dtype)
        t = cls._vecs.get(key)
        if t is None:
            t = cls._vecs[key] = torch.tensor(key[0], device=X.device, dtype=X.dtype)
        return t

    def evaluate(self, state, X):
        X = X.to(torch.float32).contiguous()
        c = self._consts(X.shape[1], X.device)
        return self._evaluate(X, c), state


def _rowterms(X, o, M, s, fid, cache=None):
    """K6 fused: f of every row of z = s·(X − o)·Mᵀ straight from the rotation GEMM's epilogue
    (per column tile additive terms + one finishing kernel) — the rotated population is never
    written.  None when the device path does not apply (CPU, odd shapes, a tile layout other
    than 64 columns wide)."""
    if not X.is_cuda or X.dtype != torch.float32:
        return None
    from ... import config

    N, D = X.shape
    ops = _ext.ops()
    if cache is not None and config.get("cec_rowterms_h3") and linalg.tall_nt_ok(N, D, D, X.device) and M.shape == (D, D):
        # f16x3 rotation with the terms reduced in the GEMM epilogue (gemm_blk.hip): the rotated
        # population is never written, no basic-function pass over it; the constant rotation's
        # planes are the problem's cached ones (the _ssr path's)
        key = ("h3", M.data_ptr(), M.shape)
        pl = cache.get(key)
        if pl is None:
            pl = cache[key] = linalg.h3_planes(M)
        Ap = linalg.h3_planes(X, sub_k=o.contiguous())
        return ops.gemm_h3_rowterms(Ap.t, Ap.rinv, N, pl.t, pl.rinv, D, D, float(s), int(fid))
    if config.get("plain_gemm") == "blas" or not config.get("cec_fused"):
        return None
    if D % 4 or int(ops.gemm_ks_tile(N, D, 0)) not in (4, 8) or X.stride(1) != 1 or X.stride(0) % 4 or X.data_ptr() % 16:
        return None
    o = o.contiguous()
    if o.data_ptr() % 16:
        return None
    return ops.cec_rotated_rowterms(X, M, o, float(s), int(fid))


class _RowSharded:
    """Decision-axis sharding (strategy P2, ``evoxmi.parallel.dim_sharded``) of a shifted-
    rotated function: the rotation mixes every column, so a rank does not take a column
    block of x but a block of z = M(x − o)·s — its rows of M against the replicated
    population (1/W of the rotation GEMM) — and returns per-row additive terms over its
    z indices (``dim_shard_full_rows``: ``partial_terms`` receives the full rows)."""

    dim_shard_full_rows = True
    dim_halo = 0
    ssr_scale = 1.0

    def _zblock(self, X, col0, d, own, halo=0):
        X = X.to(torch.float32).contiguous()
        c = self._consts(d, X.device)
        hi = min(col0 + own + halo, d)
        return self._ssr(X, c["Os"][:d], c["M"][col0:hi].contiguous(), self.ssr_scale)


class F1_CEC2022(_RowSharded, _CEC2022):
    """Shifted & rotated Zakharov."""
    func_num = 1

    def _evaluate(self, X, c):
        D = X.shape[1]
        f = _rowterms(X, c["Os"][:D], c["M"], 1.0, ZAKHAROV, self._cache)
        if f is not None:
            return f
        Z = self._ssr(X, c["Os"][:D], c["M"], 1.0)
        return self._basic(Z, ZAKHAROV, clamp=1e-8)

    def partial_terms(self, X, col0, d, own):
        z = self._zblock(X, col0, d, own)
        i = torch.arange(col0 + 1, col0 + own + 1, device=z.device, dtype=z.dtype)
        return torch.stack([(z * z).sum(1), (0.5 * i * z).sum(1)], 1)

    def combine_terms(self, T, d):
        return self._clamp(T[:, 0] + T[:, 1] ** 2 + T[:, 1] ** 4)


class F2_CEC2022(_RowSharded, _CEC2022):
    func_num = 2
    ssr_scale = 2.048 / 100.0

    def _evaluate(self, X, c):
        D = X.shape[1]
        Z = self._ssr(X, c["Os"][:D], c["M"], 2.048 / 100.0)
        return self._basic(Z, ROSENBROCK, clamp=1e-8)

    def partial_terms(self, X, col0, d, own):
        z = self._zblock(X, col0, d, own, halo=1) + 1  # pair terms whose left index is owned
        n = min(own, d - 1 - col0)
        if n <= 0:
            return z.new_zeros(z.shape[0], 1)
        a, b = z[:, :n], z[:, 1 : n + 1]
        return (100 * (a * a - b) ** 2 + (1 - a) ** 2).sum(1, keepdim=True)

    def combine_terms(self, T, d):
        return self._clamp(T[:, 0])


class F3_CEC2022(_CEC2022):
    """Schaffer F7 on y = x − o (the reference discards the rotation, kept for fidelity)."""
    func_num = 3
    dim_halo = 1  # pair terms (y_j, y_{j+1}): plain column blocks suffice (no rotation)

    def _evaluate(self, X, c):
        D = X.shape[1]
        o = c["Os"][:D]
        return self._basic(X, SCHAFFERF7, sub=o, clamp=1e-8)

    def partial_terms(self, Xb, col0, d, own):
        y = Xb.to(torch.float32) - self._consts(d, Xb.device)["Os"][col0 : col0 + Xb.shape[1]]
        n = min(own, d - 1 - col0)
        if n <= 0:
            return y.new_zeros(y.shape[0], 1)
        sq = torch.sqrt(y[:, :n] ** 2 + y[:, 1 : n + 1] ** 2)
        t = torch.sin(50.0 * sq**0.2)
        return (sq**0.5 + sq**0.5 * t * t).sum(1, keepdim=True)

    def combine_terms(self, T, d):
        f = T[:, 0]
        return self._clamp(f * f / (d - 1) / (d - 1))


class F4_CEC2022(_RowSharded, _CEC2022):
    func_num = 4

    def _evaluate(self, X, c):
        D = X.shape[1]
        f = _rowterms(X, c["Os"][:D], c["M"], 1.0, RASTRIGIN, self._cache)
        if f is not None:
            return f
        return self._basic(self._ssr(X, c["Os"][:D], c["M"], 1.0), RASTRIGIN, clamp=1e-8)

    def partial_terms(self, X, col0, d, own):
        z = self._zblock(X, col0, d, own) * 0.0512
        return (z * z - 10 * torch.cos(2 * math.pi * z) + 10).sum(1, keepdim=True)

    def combine_terms(self, T, d):
        return self._clamp(T[:, 0])


class F5_CEC2022(_RowSharded, _CEC2022):
    func_num = 5

    def _evaluate(self, X, c):
        D = X.shape[1]
        return self._basic(self._ssr(X, c["Os"][:D], c["M"], 1.0), LEVY, clamp=1e-8)

    def partial_terms(self, X, col0, d, own):
        w = 1 + self._zblock(X, col0, d, own) / 4
        j = torch.arange(col0, col0 + own, device=w.device)
        first = (j == 0).to(w.dtype)
        last = (j == d - 1).to(w.dtype)
        mid = 1 - last
        t1 = (first * torch.sin(math.pi * w) ** 2).sum(1)
        t2 = (mid * (w - 1) ** 2 * (1 + 10 * torch.sin(math.pi * w + 1) ** 2)).sum(1)
        t3 = (last * (w - 1) ** 2 * (1 + torch.sin(2 * math.pi * w) ** 2)).sum(1)
        return (t1 + t2 + t3)[:, None]

    def combine_terms(self, T, d):
        return self._clamp(T[:, 0])


class _Hybrid(_RowSharded, _CEC2022):
    """Hybrid functions: z = M(x − o), shuffled, cut into groups with different basic
    functions (reference ``cec2022_so.py:545-608``).  Decision-axis sharding: a rank rotates
    its block of z (rows of M); the blocks are all-gathered (``"cat"`` terms) because the
    shuffle mixes every coordinate into the groups."""

    p = ()
    funcs = ()

    def partial_terms(self, X, col0, d, own):
        return {"cat": self._zblock(X, col0, d, own)}

    def combine_terms(self, T, d):
        Z = T["cat"]
        return self._from_z(Z, self._consts(d, Z.device))

    def _evaluate(self, X, c):
        D = X.shape[1]
        return self._from_z(self._ssr(X, c["Os"][:D], c["M"], 1.0), c)

    def _from_z(self, Z, c):
        D = Z.shape[1]
        X = Z
        perm = c["S"] if c["S"] is not None else torch.arange(D, dtype=torch.int32, device=X.device)
        groups = _group_ids(self.p, D)
        f = 0
        for fid, (s, L) in zip(self.funcs, groups):
            if fid == SCHAFFERF7:
                # y = head of the shuffled vector (cec2022_so.py:552-561)
                if Z.is_cuda:
                    f = f + nops.cec_basic(Z, SCHAFFERF7, perm, s, L, None, 1.0, None, 0, yperm=True)
                else:
                    zs = Z[:, perm.long()]
                    f = f + _t_basic(SCHAFFERF7, zs[:, s : s + L], zs[:, :L])
            else:
                f = f + self._basic(Z, fid, perm=perm, start=s, length=L)
        return self._clamp(f)


class F6_CEC2022(_Hybrid):
    func_num = 6
    p = (0.4, 0.4, 0.2)
    funcs = (BENTCIGAR, HGBAT, RASTRIGIN)


class F7_CEC2022(_Hybrid):
    func_num = 7
    p = (0.1, 0.2, 0.2, 0.2, 0.1, 0.2)
    funcs = (HGBAT, KATSUURA, ACKLEY, RASTRIGIN, SCHWEFEL, SCHAFFERF7)


class F8_CEC2022(_Hybrid):
    func_num = 8
    p = (0.3, 0.2, 0.2, 0.1, 0.2)
    funcs = (KATSUURA, HAPPYCAT, EXPGRIEROSEN, SCHWEFEL, ACKLEY)


class _Composition(_CEC2022):
    """Composition functions (reference ``cec2022_so.py:121-135,610-738``).  Decision-axis
    sharding: a rank computes its block of every component's rotated z (rows of each M_c) and
    its columns' share of every ‖x − o_c‖² (additive ``"sum"`` terms); the z blocks are
    all-gathered (``"cat"``) and every rank finishes the weighted composition."""

    bias = ()
    lamb = ()
    sigma = ()
    # (fid, component index of shift/rotation, scale, rotate?)
    parts = ()
    threshold = 1e-8
    dim_shard_full_rows = True
    dim_halo = 0

    def partial_terms(self, X, col0, d, own):
        X = X.to(torch.float32).contiguous()
        c = self._consts(d, X.device)
        Os, M = c["Os"][:, :d], c["M"]
        cols = slice(col0, col0 + own)
        blocks = []
        for fid, comp, scale, rotate in self.parts:
            o = Os[comp]
            if rotate:
                blocks.append(self._ssr(X, o, M[comp * d + col0 : comp * d + col0 + own].contiguous(), scale))
            else:
                blocks.append((X[:, cols] - o[cols]).contiguous())
        d2 = torch.stack([((X[:, cols] - Os[i, cols]) ** 2).sum(1) for i in range(len(self.parts))], 1)
        return {"cat": blocks, "sum": d2}

    def combine_terms(self, T, d):
        Zs = T["cat"]
        c = self._consts(d, Zs[0].device)
        Os = c["Os"][:, :d]
        fs = torch.stack([self._basic(z, fid) for (fid, comp, scale, rotate), z in zip(self.parts, Zs)], 1)
        f = self._compose(Zs[0], fs, Os[: len(self.parts)], self.bias, self.sigma, self.lamb, d2=T["sum"])
        return self._clamp(f, self._thr(d))

    STACK = 1024  # column block of one component in the stacked rotation GEMM (multiple of every tile width)

    def _stacked(self, X, c):
        """Every rotated component's M_c·(x − o_c) from ONE GEMM over the stacked rotations
        (output column block c·STACK uses shift row c: the shift stays exact, applied to the
        operand before the products as in the reference ``cec2022_so.py:109-119,121-135``).
        None when the device path does not apply."""
        from ... import config

        D = X.shape[1]
        if not X.is_cuda or not config.get("cec_stack") or D % 4 or D > self.STACK or config.get("plain_gemm") != "evoxmi":
            return None
        key = ("stack", D, str(X.device))
        st = self._cache.get(key)
        if st is None:
            # one block per distinct (shift, rotation) component — F12's last two parts share one
            comps = sorted({comp for fid, comp, scale, rotate in self.parts if rotate})
            Ms = torch.zeros(len(comps) * self.STACK, D, device=X.device)
            Osh = torch.zeros(len(comps), D, device=X.device)
            for j, comp in enumerate(comps):
                Ms[j * self.STACK : j * self.STACK + D] = c["M"][comp * D : (comp + 1) * D]
                Osh[j] = c["Os"][comp, :D]
            slot = {i: comps.index(comp) for i, (fid, comp, scale, rotate) in enumerate(self.parts) if rotate}
            st = self._cache[key] = (Ms, Osh, slot)
        Ms, Osh, slot = st
        if linalg.tall_nt_ok(X.shape[0], Ms.shape[0], D, X.device):
            # f16x3 LDS-staged GEMM: X read once into one (x − o_c) plane set per component,
            # the stacked rotations split once (cached), one launch over every component
            bkey = ("stack_h3", D, str(X.device))
            Bp = self._cache.get(bkey)
            if Bp is None:
                Bp = self._cache[bkey] = linalg.h3_planes(Ms)
            Z = linalg.mm_h3(linalg.h3_planes(X, sub_k=Osh), Bp, sub_cols=self.STACK)
        else:
            Z = linalg.mm_nt(X, Ms, a_sub_k=Osh, sub_cols=self.STACK)
        return Z, slot

    def _evaluate(self, X, c):
        D = X.shape[1]
        Os = c["Os"][:, :D]
        M = c["M"]
        fs = []
        stacked = self._stacked(X, c)
        from ... import config

        if stacked is not None and config.get("cec_compose_fused"):
            # every component's basic function, distances and the weighted sum in one kernel
            Z, slot = stacked
            p = self.parts
            return _ext.ops().cec_compose(
                Z, X, c["Os"], [fid for fid, _, _, _ in p], [slot[i] * self.STACK if rot else -1 for i, (_, _, _, rot) in enumerate(p)],
                [comp for _, comp, _, _ in p], [float(sc) for _, _, sc, _ in p], [float(v) for v in self.sigma],
                [float(v) for v in self.lamb], [float(v) for v in self.bias], float(self._thr(D)))
        for i, (fid, comp, scale, rotate) in enumerate(self.parts):
            o = Os[comp]
            if rotate and stacked is not None:
                Z, slot = stacked
                fs.append(self._basic(Z, fid, start=slot[i] * self.STACK, length=D, scale=scale))
            elif rotate:
                Z = self._ssr(X, o, M[comp * D : (comp + 1) * D], scale)
                fs.append(self._basic(Z, fid))
            else:
                fs.append(self._basic(X, fid, sub=o))
        fs = torch.stack(fs, 1)
        f = self._compose(X, fs, Os[: len(self.parts)], self.bias, self.sigma, self.lamb)
        return self._clamp(f, self._thr(D))

    def _thr(self, D):
        return self.threshold


class F9_CEC2022(_Composition):
    func_num = 9
    bias = (0, 200, 300, 100, 400)
    lamb = (1, 1e-6, 1e-26, 1e-6, 1e-6)
    sigma = (10, 20, 30, 40, 50)
    parts = ((ROSENBROCK, 0, 2.048 / 100.0, True), (ELLIPTIC, 1, 1.0, True), (BENTCIGAR, 2, 1.0, True), (DISCUS, 3, 1.0, True), (ELLIPTIC, 4, 1.0, False))


class F10_CEC2022(_Composition):
    func_num = 10
    bias = (0, 200, 100)
    lamb = (1, 1, 1)
    sigma = (20, 10, 10)
    parts = ((SCHWEFEL, 0, 1.0, False), (RASTRIGIN, 1, 1.0, True), (HGBAT, 2, 1.0, True))


class F11_CEC2022(_Composition):
    func_num = 11
    bias = (0, 200, 300, 400, 200)
    lamb = (5e-4, 1, 10, 1, 10)
    sigma = (20, 20, 30, 30, 20)
    parts = ((EXPSCHAFFER, 0, 1.0, True), (SCHWEFEL, 1, 1.0, True), (GRIEWANK, 2, 6.0, True), (ROSENBROCK, 3, 2.048 / 100.0, True), (RASTRIGIN, 4, 1.0, True))

    def _thr(self, D):
        return 5.07e-6 if D == 10 else 1.46e-5


class F12_CEC2022(_Composition):
    func_num = 12
    bias = (0, 300, 500, 100, 400, 200)
    lamb = (10, 10, 2.5, 1e-26, 1e-6, 5e-4)
    sigma = (10, 20, 30, 40, 50, 60)
    parts = ((HGBAT, 0, 1.0, True), (RASTRIGIN, 1, 1.0, True), (SCHWEFEL, 2, 1.0, True), (BENTCIGAR, 3, 1.0, True), (ELLIPTIC, 4, 1.0, True), (EXPSCHAFFER, 4, 1.0, True))


class CEC2022TestSuit:
    """``CEC2022TestSuit.create(n)`` (reference ``cec2022_so.py:740-764``)."""

    func_num2class = {
        1: F1_CEC2022, 2: F2_CEC2022, 3: F3_CEC2022, 4: F4_CEC2022, 5: F5_CEC2022, 6: F6_CEC2022,
        7: F7_CEC2022, 8: F8_CEC2022, 9: F9_CEC2022, 10: F10_CEC2022, 11: F11_CEC2022, 12: F12_CEC2022,
    }

    @staticmethod
    def create(func_num: int, **kwargs):
        return CEC2022TestSuit.func_num2class[func_num](**kwargs)


CEC2022TestSuite = CEC2022TestSuit
