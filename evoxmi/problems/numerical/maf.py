"""MaF1–MaF15 many-objective suite (reference ``problems/numerical/maf.py:1-1165``).

Cheng et al., "A benchmark test suite for evolutionary many-objective optimization",
Complex & Intelligent Systems 3(1), 2017.  Every ``evaluate`` is batched over the
population with whole-tensor torch ops (it runs on whatever device X lives on); the
reference's per-row ``fori_loop`` constructions (MaF2/10/11 PF, MaF12's pairwise
non-separable reduction) are re-expressed as vectorised forms with the same values:

* MaF12 ``Σ_{i<j}|t_i − t_j|`` is computed from the sorted row in O(L log L)
  (``Σ_k t_(k)·(2k − L + 1)``) instead of the reference's O(L²) double loop.
* the ``K/(M−1)``-wide group reductions of MaF10/11/12 are width-1 (K = M−1 always),
  so they reduce to the identity on those columns exactly as in the reference.

Reference quirks kept on purpose (documented in tests/test_maf.py):
* MaF10's distance term indexes ``x[:, M]`` which JAX clamps to ``x[:, M−1]``;
* MaF13's ``m = max(m, 3)`` is overwritten by the base constructor, so default
  ``d = m + 9`` and m is not clamped;
* MaF6's PF divides every column by ``√2^(m−2)`` (not the per-column DTLZ5 form).
"""
from __future__ import annotations

import math

import torch

from ...core import Problem, State
from ...operators.sampling import UniformSampling
from .classic import griewank_func, sphere_func

PI = math.pi


def inside(x, a, b):
    """a ≤ x < b with the bounds in either order (reference maf.py:13-17)."""
    x, a, b = (torch.as_tensor(v, dtype=torch.float32) for v in (x, a, b))
    return (torch.minimum(a, b) <= x) & (x < torch.maximum(a, b))


def ray_intersect_segment(point, seg_init, seg_term):
    """Whether the horizontal ray cast right from ``point`` crosses the segment (maf.py:20-38).

    Broadcasts over leading dims of all three arguments (last dim = 2).
    """
    point, seg_init, seg_term = (torch.as_tensor(v, dtype=torch.float32) for v in (point, seg_init, seg_term))
    y_dist = seg_term[..., 1] - seg_init[..., 1]
    judge_1 = (point[..., 1] == seg_init[..., 1]) & inside(point[..., 0], seg_init[..., 0], seg_term[..., 0])
    lhs = seg_init[..., 0] * y_dist + (point[..., 1] - seg_init[..., 1]) * (seg_term[..., 0] - seg_init[..., 0])
    rhs = point[..., 0] * y_dist
    judge_2 = ((y_dist > 0) & (lhs >= rhs)) | ((y_dist < 0) & (lhs <= rhs))
    judge_3 = inside(point[..., 1], seg_init[..., 1], seg_term[..., 1])
    return ((y_dist == 0) & judge_1) | ((y_dist != 0) & judge_2 & judge_3)


def point_in_polygon(polygon, point):
    """Ray-casting point-in-polygon test (maf.py:41-58); ``point`` may be (2,) or (P, 2)."""
    polygon = torch.as_tensor(polygon, dtype=torch.float32)
    point = torch.as_tensor(point, dtype=torch.float32)
    single = point.dim() == 1
    P = point.reshape(-1, 1, 2)
    seg_term = torch.roll(polygon, 1, 0)
    hits = ray_intersect_segment(P, polygon[None], seg_term[None]).sum(1)
    is_vertex = (polygon[None] == P).all(-1).any(1)
    r = (hits % 2 == 1) | is_vertex
    return r[0] if single else r


def _front(h: torch.Tensor, t: torch.Tensor) -> torch.Tensor:
    """fliplr(cumprod([1, h])) · [1, fliplr(t)] for (n, m−1) factor matrices."""
    ones = torch.ones((h.shape[0], 1), dtype=h.dtype, device=h.device)
    return torch.flip(torch.cumprod(torch.cat([ones, h], 1), 1), [1]) * torch.cat([ones, torch.flip(t, [1])], 1)


def _sphere_front(X, m):
    return _front(torch.cos(X[:, : m - 1] * PI / 2), torch.sin(X[:, : m - 1] * PI / 2))


def _normalise_rows(R):
    return R / torch.sqrt((R * R).sum(1, keepdim=True))


def _pow2(exps, like):
    return torch.pow(2.0, exps.to(like.dtype)).to(like.device)


class _PositionDistance:
    """Decision-axis sharding (P2, ``evoxmi/parallel/dim_sharded.py``) for the MaF problems of
    DTLZ form: the first ``n_pos`` (position) variables travel as terms from the rank owning
    each column, and the distance part is ``n_sums`` additive per-row sums over the remaining
    columns (``_sums(Y, gcol0, d)``, Y = this rank's distance columns starting at global column
    gcol0).  ``_finish(Xp, S, d)`` forms the objectives; ``evaluate`` is the same formula on the
    whole row (the reference's ``maf.py`` evaluates rows whole under GSPMD)."""

    dim_halo = 0
    n_sums = 1

    def _n_pos(self):
        return self.m - 1

    def partial_terms(self, Xb, col0, d, own):
        k = self._n_pos()
        Xo = Xb[:, :own]
        T = torch.zeros((Xb.shape[0], k + self.n_sums), dtype=Xb.dtype, device=Xb.device)
        hi = min(col0 + own, k)
        if hi > col0:
            T[:, col0:hi] = Xo[:, : hi - col0]
        s = max(k - col0, 0)
        if s < own and self.n_sums:
            T[:, k:] = self._sums(Xo[:, s:], col0 + s, d)
        return T

    def combine_terms(self, T, d):
        k = self._n_pos()
        return self._finish(T[:, :k], T[:, k:], d)

    def evaluate(self, state, X):
        k = self._n_pos()
        d = X.shape[1]
        return self._finish(X[:, :k], self._sums(X[:, k:], k, d) if self.n_sums else X[:, :0], d), state


def _sq_half(Y, gcol0, d):
    return ((Y - 0.5) ** 2).sum(1, keepdim=True)


def _rastrigin_sum(Y, gcol0, d):
    Y = Y - 0.5
    return (Y * Y - torch.cos(20 * PI * Y)).sum(1, keepdim=True)


class MaF(Problem):
    def __init__(self, d=None, m=None, ref_num=1000):
        super().__init__()
        self.m = 3 if m is None else m
        self.d = self.m + 9 if d is None else d
        self.ref_num = ref_num

    def setup(self, key):
        return State(key=key)

    def _uniform(self, m=None):
        return UniformSampling(self.ref_num * self.m, self.m if m is None else m)()[0]

    def pf(self):
        return 1 - self._uniform()


class MaF1(_PositionDistance, MaF):
    """Inverted linear front (maf.py:98-130)."""

    _sums = staticmethod(_sq_half)

    def _finish(self, Xp, g, d):
        return (1 + g) - (1 + g) * _front(Xp, 1 - Xp)


class MaF2(_PositionDistance, MaF):
    """DTLZ2BZ: per-objective distance groups (maf.py:133-218)."""

    @property
    def n_sums(self):
        return self.m

    def _sums(self, Y, gcol0, d):
        # group i of objective i: columns [m − 1 + i·interval, m − 1 + (i + 1)·interval), the last to d
        m = self.m
        interval = int((d - m + 1) / m)
        c = torch.arange(gcol0, gcol0 + Y.shape[1], device=Y.device) - (m - 1)
        grp = torch.clamp(c // interval, max=m - 1) if interval > 0 else torch.full_like(c, m - 1)
        Z = (Y / 2 + 0.25 - 0.5) ** 2
        return torch.zeros((Y.shape[0], m), dtype=Y.dtype, device=Y.device).index_add_(1, grp, Z)

    def _finish(self, Xp, g, d):
        Y = Xp / 2 + 0.25
        return (1 + g) * _front(torch.cos(Y * PI / 2), torch.sin(Y * PI / 2))

    def pf(self):
        m = self.m
        r = self._uniform()
        c = torch.zeros((r.shape[0], m - 1), dtype=r.dtype)
        for j in range(2, m + 1):
            temp = r[:, j - 1] / r[:, 0] * torch.prod(c[:, m - j + 1 : m - 1], 1)
            c[:, m - j] = torch.sqrt(1 / (1 + temp * temp))
        lo, hi = math.cos(3 * PI / 8), math.cos(PI / 8)
        if m > 5:
            c = c * (hi - lo) + lo
        else:
            c = c[((c >= lo) & (c <= hi)).all(1)]
        return _front(c[:, : m - 1], torch.sqrt(1 - c[:, : m - 1] ** 2))


class MaF3(_PositionDistance, MaF):
    """Convex DTLZ3 (maf.py:221-259)."""

    _sums = staticmethod(_rastrigin_sum)

    def _finish(self, Xp, S, d):
        m = self.m
        f1 = (1 + 100 * (d - m + 1 + S)) * _sphere_front(Xp, m)
        return torch.cat([f1[:, : m - 1] ** 4, f1[:, m - 1 :] ** 2], 1)

    def pf(self):
        r = self._uniform() ** 2
        temp = (torch.sqrt(r[:, :-1]).sum(1) + r[:, -1])[:, None]
        return r / torch.cat([(temp * temp).expand(-1, r.shape[1] - 1), temp], 1)


class MaF4(_PositionDistance, MaF):
    """Inverted, badly-scaled DTLZ3 (maf.py:262-299)."""

    _sums = staticmethod(_rastrigin_sum)

    def _finish(self, Xp, S, d):
        m = self.m
        g1 = 1 + 100 * (d - m + 1 + S)
        f1 = g1 - g1 * _sphere_front(Xp, m)
        return f1 * _pow2(torch.arange(1, m + 1), Xp)[None]

    def pf(self):
        r1 = _normalise_rows(self._uniform())
        return (1 - r1) * _pow2(torch.arange(1, self.m + 1), r1)[None]


class MaF5(_PositionDistance, MaF):
    """Concave, badly-scaled DTLZ4 (maf.py:302-338)."""

    _sums = staticmethod(_sq_half)

    def _finish(self, Xp, g, d):
        m = self.m
        return (1 + g) * _sphere_front(Xp**100, m) * _pow2(torch.arange(m, 0, -1), Xp)[None]

    def pf(self):
        r1 = _normalise_rows(self._uniform())
        return r1 * _pow2(torch.arange(self.m, 0, -1), r1)[None]


class MaF6(_PositionDistance, MaF):
    """Degenerate DTLZ5 with I = 2 (maf.py:341-386)."""

    _sums = staticmethod(_sq_half)

    def _finish(self, Xp, g, d):
        m, i = self.m, 2
        mid = (1 + 2 * g * Xp[:, i - 1 : m - 1]) / (2 + 2 * g)
        return (1 + 100 * g) * _sphere_front(torch.cat([Xp[:, : i - 1], mid], 1), m)

    def pf(self):
        i, m = 2, self.m
        r = self._uniform(i)
        r1 = _normalise_rows(r)
        if r1.shape[1] < m:
            r1 = torch.cat([r1[:, [0] * (m - r1.shape[1])], r1], 1)
        return r1 / math.sqrt(2) ** max(m - i, 0)


class MaF7(_PositionDistance, MaF):
    """Disconnected DTLZ7 front (maf.py:389-443)."""

    _sums = staticmethod(lambda Y, gcol0, d: Y.sum(1, keepdim=True))

    def _finish(self, fm, S, d):
        m = self.m
        g = 1 + 9 * S / (d - m + 1)
        last = (1 + g) * (m - (fm / (1 + g) * (1 + torch.sin(3 * PI * fm))).sum(1, keepdim=True))
        return torch.cat([fm, last], 1)

    @staticmethod
    def _grid(N, M):
        gap = torch.linspace(0, 1, int(math.ceil(N ** (1 / M))))
        c = torch.meshgrid(*([gap] * M), indexing="xy")
        return torch.stack([x.reshape(-1) for x in c], 1)

    def pf(self):
        m = self.m
        iv = torch.tensor([0, 0.251412, 0.631627, 0.859401])
        median = (iv[1] - iv[0]) / (iv[3] - iv[2] + iv[1] - iv[0])
        X = self._grid(self.ref_num * m, m - 1)
        X = torch.where(X <= median, X * (iv[1] - iv[0]) / median + iv[0], X)
        X = torch.where(X > median, (X - median) * (iv[3] - iv[2]) / (1 - median) + iv[2], X)
        last = 2 * (m - (X / 2 * (1 + torch.sin(3 * PI * X))).sum(1, keepdim=True))
        return torch.cat([X, last], 1)


class _Polygon(MaF):
    def _points(self, device=None):
        theta = math.atan2(1.0, 0.0)
        t = torch.arange(1, self.m + 1, dtype=torch.float32)
        ang = theta - t * 2 * PI / self.m
        return torch.stack([torch.cos(ang), torch.sin(ang)], 1).to(device)

    def _pf_grid(self, order):
        n = self.ref_num * self.m
        temp = torch.linspace(-1, 1, int(math.ceil(math.sqrt(n))))
        # meshgrid 'xy': y[i, j] = temp[j], x[i, j] = temp[i]
        xi, yj = torch.meshgrid(temp, temp, indexing="ij")
        if order == "F":
            x, y = xi.T.reshape(-1), yj.T.reshape(-1)
        else:
            x, y = xi.reshape(-1), yj.reshape(-1)
        pts = torch.stack([x, y], 1)
        return pts[point_in_polygon(self._points(), pts)]


class MaF8(_PositionDistance, _Polygon):
    """Multi-point distance minimisation, 2-D decision space (maf.py:449-500); under
    decision-axis sharding the two used columns travel as terms."""

    n_sums = 0
    _n_pos = staticmethod(lambda: 2)

    def _finish(self, X2, S, d):
        return torch.cdist(X2, self._points(X2.device).to(X2.dtype))

    def __init__(self, d=None, m=None, ref_num=1000):
        super().__init__(2, m, ref_num)

    def pf(self):
        pts = self._pf_grid("F")
        return torch.cdist(pts, self._points())


class MaF9(_PositionDistance, _Polygon):
    """Multi-line distance minimisation (maf.py:503-560); the two used columns travel as
    terms under decision-axis sharding."""

    n_sums = 0
    _n_pos = staticmethod(lambda: 2)

    def _finish(self, X2, S, d):
        return self._eval(X2)

    def _eval(self, X):
        P = self._points(X.device).to(X.dtype)
        A, B = P, torch.roll(P, -1, 0)  # line i through points i and (i+1) mod m
        num = torch.abs((A[None, :, 0] - X[:, None, 0]) * (B[None, :, 1] - X[:, None, 1])
                        - (B[None, :, 0] - X[:, None, 0]) * (A[None, :, 1] - X[:, None, 1]))
        return num / torch.sqrt((A[:, 0] - B[:, 0]) ** 2 + (A[:, 1] - B[:, 1]) ** 2)[None]

    def pf(self):
        return self._eval(self._pf_grid("C"))


def _s_linear(y, A):
    return torch.abs(y - A) / torch.abs(torch.floor(A - y) + A)


def _wfg_shape_x(t_first, t_last):
    """x_i = max(t_M, 1)·(t_i − 0.5) + 0.5 for i < M, x_M = t_M."""
    return torch.cat([torch.clamp(t_last, min=1.0) * (t_first - 0.5) + 0.5, t_last], 1)


def _convex(x):
    return _front(1 - torch.cos(x[:, :-1] * PI / 2), 1 - torch.sin(x[:, :-1] * PI / 2))


def _concave(x):
    return _front(torch.sin(x[:, :-1] * PI / 2), torch.cos(x[:, :-1] * PI / 2))


def _wfg_pf_c(R, M):
    c = torch.ones((R.shape[0], M), dtype=R.dtype)
    for j in range(1, M):
        temp = R[:, j] / R[:, 0] * torch.prod(1 - c[:, M - j : M - 1], 1)
        c[:, M - j - 1] = (temp * temp - temp + torch.sqrt(2 * temp)) / (temp * temp + 1)
    return c


def _wfg_pf_x0(x, R, M, kind):
    temp = (1 - torch.sin(PI / 2 * x[:, 1])) * R[:, M - 1] / R[:, M - 2]
    a = torch.arange(0, 1.0001, 0.0001, dtype=torch.float32)[None]
    if kind == "mixed":
        E = torch.abs(temp[:, None] * (1 - torch.cos(PI / 2 * a)) - 1 + (a + torch.cos(10 * PI * a + PI / 2) / 10 / PI))
    else:
        E = torch.abs(temp[:, None] * (1 - torch.cos(PI / 2 * a)) - 1 + a * torch.cos(5 * PI * a) ** 2)
    first = torch.argsort(E, dim=1, stable=True)[:, :10].min(1).values
    x = x.clone()
    x[:, 0] = a[0, first]
    return x


class MaF10(MaF):
    """WFG1 (maf.py:563-684)."""

    def evaluate(self, state, X):
        n, d = X.shape
        M = self.m
        K = M - 1
        S = torch.arange(2, 2 * M + 1, 2, dtype=X.dtype, device=X.device)
        z01 = X / torch.arange(2, 2 * d + 1, 2, dtype=X.dtype, device=X.device)
        t1 = torch.cat([z01[:, :K], _s_linear(z01[:, K:], 0.35)], 1)
        y = t1[:, K:]
        A, B, C = 0.8, 0.75, 0.85
        bf = A + torch.clamp(torch.floor(y - B), max=0) * A * (B - y) / B \
            - torch.clamp(torch.floor(C - y), max=0) * (1 - A) * (y - C) / (1 - C)
        bf = torch.round(bf * 1e4) / 1e4
        t3 = torch.cat([t1[:, :K], bf], 1) ** 0.02
        w = torch.arange(2 * (K + 1), 2 * d + 1, 2, dtype=X.dtype, device=X.device)
        tM = (t3[:, K:] * w).sum(1, keepdim=True) / w.sum()
        x = _wfg_shape_x(t3[:, :K], tM)
        h = _convex(x)
        h[:, M - 1] = 1 - x[:, 0] - torch.cos(10 * PI * x[:, 0] + PI / 2) / 10 / PI
        return x[:, M - 1 : M] + S * h, state

    def pf(self):
        M = self.m
        R = self._uniform()
        x = torch.arccos(_wfg_pf_c(R, M)) * 2 / PI
        x = _wfg_pf_x0(x, R, M, "mixed")
        f = _convex(x)
        f[:, M - 1] = 1 - x[:, 0] - torch.cos(10 * PI * x[:, 0] + PI / 2) / 10 / PI
        return f * torch.arange(2, 2 * M + 1, 2, dtype=f.dtype)[None]


class MaF11(MaF):
    """WFG2 (maf.py:687-800); d is rounded so that the distance block has even size."""

    def __init__(self, d=None, m=None, ref_num=1000):
        super().__init__(d, m, ref_num)
        self.d = int(math.ceil((self.d - self.m + 1) / 2) * 2 + self.m - 1)

    def evaluate(self, state, X):
        n, d = X.shape
        M = self.m
        K = M - 1
        L = d - K
        S = torch.arange(2, 2 * M + 1, 2, dtype=X.dtype, device=X.device)
        z01 = X / torch.arange(2, 2 * d + 1, 2, dtype=X.dtype, device=X.device)
        t1 = torch.cat([z01[:, :K], _s_linear(z01[:, K:], 0.35)], 1)
        a, b = t1[:, K::2][:, : L // 2], t1[:, K + 1 :: 2][:, : L // 2]
        t2 = torch.cat([t1[:, :K], (a + b + 2 * torch.abs(a - b)) / 3], 1)
        tM = t2[:, K : K + L // 2].mean(1, keepdim=True)
        x = _wfg_shape_x(t2[:, :K], tM)
        h = _convex(x)
        h[:, M - 1] = 1 - x[:, 0] * torch.cos(5 * PI * x[:, 0]) ** 2
        return x[:, M - 1 : M] + S * h, state

    def pf(self):
        from ...operators.selection import non_dominated_sort

        M = self.m
        R = self._uniform()
        x = torch.arccos(_wfg_pf_c(R, M)) * 2 / PI
        x = _wfg_pf_x0(x, R, M, "disc")
        R = _convex(x)
        R[:, M - 1] = 1 - x[:, 0] * torch.cos(5 * PI * x[:, 0]) ** 2
        f = R[non_dominated_sort(R) == 0]
        return f * torch.arange(2, 2 * M + 1, 2, dtype=f.dtype)[None]


def _pairwise_abs_sum(t):
    """Σ_{i<j} |t_i − t_j| per row via the sorted-order identity."""
    L = t.shape[1]
    s = torch.sort(t, 1).values
    coef = 2 * torch.arange(L, dtype=t.dtype, device=t.device) - (L - 1)
    return (s * coef).sum(1)


class MaF12(MaF):
    """WFG9 (maf.py:803-924)."""

    def evaluate(self, state, X):
        n, d = X.shape
        M = self.m
        K = M - 1
        L = d - K
        S = torch.arange(2, 2 * M + 1, 2, dtype=X.dtype, device=X.device)
        z01 = X / torch.arange(2, 2 * d + 1, 2, dtype=X.dtype, device=X.device)
        # mean of the variables to the right of each position (last column unused)
        Y = (torch.flip(torch.cumsum(torch.flip(z01, [1]), 1), [1]) - z01)[:, :-1] / torch.arange(
            d - 1, 0, -1, dtype=X.dtype, device=X.device)
        r = 0.98 / 49.98
        e = 0.02 + (50 - 0.02) * (r - (1 - 2 * Y) * torch.abs(torch.floor(0.5 - Y) + r))
        t1 = torch.cat([z01[:, :-1] ** e, z01[:, -1:]], 1)
        y = t1[:, :K]
        A, B, C = 0.35, 0.001, 0.05
        dec = 1 + (torch.abs(y - A) - B) * (torch.floor(y - A + B) * (1 - C + (A - B) / B) / (A - B)
                                            + torch.floor(A + B - y) * (1 - C + (1 - A - B) / B) / (1 - A - B) + 1 / B)
        y = t1[:, K:]
        A, B, C = 30, 95, 0.35
        q = torch.abs(y - C) / 2 / (torch.floor(C - y) + C)
        mul = (1 + torch.cos((4 * A + 2) * PI * (0.5 - q)) + 4 * B * q * q) / (B + 2)
        t2 = torch.cat([dec, mul], 1)
        tail = t2[:, K:]
        cl = math.ceil(L / 2)
        tM = ((tail.sum(1) + 2 * _pairwise_abs_sum(tail)) / cl / (1 + 2 * L - 2 * cl))[:, None]
        x = _wfg_shape_x(t2[:, :K], tM)
        return x[:, M - 1 : M] + S * _concave(x), state

    def pf(self):
        R = _normalise_rows(self._uniform())
        return torch.arange(2, 2 * self.m + 1, 2, dtype=R.dtype)[None] * R


class MaF13(MaF):
    """PF7: degenerate front with coupled variables (maf.py:927-990)."""

    def evaluate(self, state, X):
        N, D = X.shape
        m = self.m
        j = torch.arange(1, D + 1, dtype=X.dtype, device=X.device)
        Y = X - 2 * X[:, 1:2] * torch.sin(2 * PI * X[:, 0:1] + j * PI / D)
        c0, s0 = torch.cos(X[:, 0] * PI / 2), torch.sin(X[:, 0] * PI / 2)
        c1, s1 = torch.cos(X[:, 1] * PI / 2), torch.sin(X[:, 1] * PI / 2)
        f0 = s0 + 2 * (Y[:, 3:D:3] ** 2).mean(1)
        f1 = c0 * s1 + 2 * (Y[:, 4:D:3] ** 2).mean(1)
        f2 = c0 * c1 + 2 * (Y[:, 2:D:3] ** 2).mean(1)
        rest = (f0 ** 2 + f1 ** 10 + f2 ** 10 + 2 * (Y[:, 3:D] ** 2).mean(1))[:, None].expand(-1, m - 3)
        return torch.cat([f0[:, None], f1[:, None], f2[:, None], rest], 1), state

    def pf(self):
        R = _normalise_rows(UniformSampling(self.ref_num * self.m, 3)()[0])
        extra = (R[:, 0] ** 2 + R[:, 1] ** 10 + R[:, 2] ** 10)[:, None].expand(-1, self.m - 3)
        return torch.cat([R, extra], 1)


class _LargeScale(MaF):
    """Shared variable grouping of MaF14/15 (maf.py:993-1015): a chaotic logistic map
    sizes the nk = 2 groups of distance variables per objective."""

    nk = 2

    def __init__(self, d=None, m=None, ref_num=1000):
        super().__init__(d, m, ref_num)
        self.d = 20 * self.m if d is None else d
        c = [3.8 * 0.1 * (1 - 0.1)]
        for _ in range(1, self.m):
            c.append(3.8 * c[-1] * (1 - c[-1]))
        c = torch.tensor(c, dtype=torch.float32)
        sub = torch.floor(c / c.sum() * (self.d - self.m + 1) / self.nk).to(torch.int64)
        self.sublen = tuple(int(v) for v in sub)
        self.len = tuple(int(v) for v in torch.cat([torch.zeros(1, dtype=torch.int64), torch.cumsum(sub * self.nk, 0)]))

    def _groups(self, X, fn_even, fn_odd):
        N = X.shape[0]
        cols = []
        for i in range(self.m):
            fn = fn_even if i % 2 == 0 else fn_odd
            acc = torch.zeros(N, dtype=X.dtype, device=X.device)
            for j in range(self.nk):
                start = self.len[i] + self.m - 1 + j * self.sublen[i]
                seg = X[:, start : start + self.sublen[i]]
                if seg.shape[1] > 0:
                    acc = acc + fn(seg)
            cols.append(acc)
        G = torch.stack(cols, 1)
        return G / (torch.tensor(self.sublen, dtype=X.dtype, device=X.device) * self.nk)[None]


def _rastrigin(x):
    return (x * x - 10 * torch.cos(2 * PI * x) + 10).sum(1)


def _rosenbrock(x):
    return (100 * (x[:, :-1] ** 2 - x[:, 1:]) ** 2 + (x[:, :-1] - 1) ** 2).sum(1)


class MaF14(_LargeScale):
    """LSMOP3-style large-scale problem (maf.py:993-1060)."""

    def evaluate(self, state, X):
        N, D = X.shape
        M = self.m
        j = torch.arange(M, D + 1, dtype=X.dtype, device=X.device)
        X = torch.cat([X[:, : M - 1], (1 + j / D) * X[:, M - 1 :] - X[:, 0:1] * 10], 1)
        G = self._groups(X, _rastrigin, _rosenbrock)
        return (1 + G) * _front(X[:, : M - 1], 1 - X[:, : M - 1]), state

    def pf(self):
        return self._uniform()


class MaF15(_LargeScale):
    """Inverted LSMOP8-style large-scale problem (maf.py:1063-1165)."""

    def evaluate(self, state, X):
        N, D = X.shape
        M = self.m
        j = torch.arange(M, D + 1, dtype=X.dtype, device=X.device)
        X = torch.cat([X[:, : M - 1], (1 + torch.cos(j / D * PI / 2)) * X[:, M - 1 :] - X[:, 0:1] * 10], 1)
        G = self._groups(X, lambda s: griewank_func(s.contiguous()), lambda s: sphere_func(s.contiguous()))
        Gs = torch.cat([G[:, 1:], torch.zeros((N, 1), dtype=X.dtype, device=X.device)], 1)
        return (1 + G + Gs) * (1 - _sphere_front(X, M)), state

    def pf(self):
        return 1 - _normalise_rows(self._uniform())
