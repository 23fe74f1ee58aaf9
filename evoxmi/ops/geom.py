"""k-nearest rows (K17) and Monte-Carlo hypervolume dominance counts (K18).

Device path: ``csrc/kernels/mo_geom.hip`` (fused distance + register top-T, no N×M
matrix; tiled sample×point dominance tests with a deterministic per-point reduction).
The CPU branches below are the numerics oracles the GPU tests compare against.
"""
from __future__ import annotations

import torch

from . import _ext

KNN_MAX_T, KNN_MAX_M, HV_MAX_M = 32, 64, 16


def _sqdist_rows(X, Y, chunk=512):
    out = []
    for s in range(0, X.shape[0], chunk):
        blk = X[s : s + chunk]
        out.append(((blk[:, None, :] - Y[None, :, :]) ** 2).sum(-1))
    return torch.cat(out, 0) if out else X.new_zeros((0, Y.shape[0]))


def knn(X: torch.Tensor, Y: torch.Tensor, T: int):
    """(distances (N, T), indices (N, T) int64) of the T nearest rows of ``Y`` for every
    row of ``X``, ascending by (squared euclidean distance, index) — a stable argsort of
    the direct-form distance row, as the reference's ``argsort(pairwise_euclidean_dist)``.
    NaN distances rank first (reported as NaN); inf distances are ordinary candidates."""
    X = X.to(torch.float32).contiguous()
    Y = Y.to(torch.float32).contiguous()
    T = int(T)
    if X.is_cuda and T <= KNN_MAX_T and X.shape[1] <= KNN_MAX_M:
        d, i = _ext.ops().knn(X, Y, T)
        return d, i.long()
    out_d, out_i = [], []
    for s in range(0, X.shape[0], 512):
        d2 = _sqdist_rows(X[s : s + 512], Y, 512)
        # a NaN distance ranks first so the nearest distance propagates it (as
        # torch.cdist(..).min() and the reference's min do); the kernel uses the same order
        key = torch.where(torch.isnan(d2), torch.full_like(d2, float("-inf")), d2)
        i = torch.argsort(key, dim=1, stable=True)[:, :T]
        out_d.append(torch.sqrt(torch.gather(d2, 1, i)))
        out_i.append(i)
    return torch.cat(out_d), torch.cat(out_i)


def min_dist(X: torch.Tensor, Y: torch.Tensor) -> torch.Tensor:
    """Distance from every row of ``X`` to its nearest row of ``Y`` (IGD / GD)."""
    return knn(X, Y, 1)[0][:, 0]


def hv_count(samples: torch.Tensor, points: torch.Tensor, strict: bool) -> torch.Tensor:
    """For each sample, the number of points dominating it: ``sample < point`` in every
    objective (strict, the HV metric on |objs − ref|) or ``point ≤ sample`` (HypE)."""
    samples = samples.to(torch.float32).contiguous()
    points = points.to(torch.float32).contiguous()
    if samples.is_cuda and samples.shape[1] <= HV_MAX_M:
        return _ext.ops().hv_count(samples, points, int(bool(strict))).long()
    out = []
    step = max(1, (1 << 22) // max(points.shape[0], 1))
    for s0 in range(0, samples.shape[0], step):
        s = samples[s0 : s0 + step]
        dom = (s[:, None, :] < points[None, :, :]) if strict else (points[None, :, :] <= s[:, None, :])
        out.append(dom.all(-1).sum(1))
    return torch.cat(out) if out else torch.zeros(0, dtype=torch.int64, device=samples.device)


def hv_contrib(samples: torch.Tensor, points: torch.Tensor, count: torch.Tensor, alpha: torch.Tensor) -> torch.Tensor:
    """HypE: f_i = Σ_s [point_i ≤ sample_s] · α[count_s − 1]."""
    samples = samples.to(torch.float32).contiguous()
    points = points.to(torch.float32).contiguous()
    alpha = alpha.to(torch.float32).contiguous()
    if samples.is_cuda and samples.shape[1] <= HV_MAX_M:
        return _ext.ops().hv_contrib(samples, points, count.to(torch.int32).contiguous(), alpha)
    f = torch.zeros(points.shape[0], device=points.device)
    w = torch.where(count > 0, alpha[(count - 1).clamp(min=0)], torch.zeros((), device=alpha.device))
    for s0 in range(0, samples.shape[0], 2048):
        s = samples[s0 : s0 + 2048]
        dom = (points[:, None, :] <= s[None, :, :]).all(-1)
        f = f + torch.where(dom, w[s0 : s0 + 2048][None, :], torch.zeros((), device=f.device)).sum(1)
    return f
