"""Hypervolume (reference ``metrics/hypervolume.py:7-96``).

* ``bounding_cube_monte_carlo_hv`` — uniform samples in the box spanned by |objs − ref|;
  fraction dominated × box volume;
* ``each_cube_monte_carlo_hv`` — per-point boxes, each sample weighted by
  1/(number of points dominating it) (the reference's bincount form);
* ``exact_hv`` — exact value by slicing (HSO) for any m, O(n^{m−1} log n), meant for
  fronts of moderate size / validation of the estimators.

Both estimators reduce to per-sample dominator counts (samples × points × m comparisons):
one tiled HIP kernel on the GPU (``ops.geom.hv_count``), chunked torch on the CPU.  Like the reference, points are measured as |objs − ref|
so either optimisation direction works.
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import geom
from ..ops import random as rnd

def _dominated_counts(samples, points):
    """For each sample, how many points strictly dominate it (sample < point in all m);
    one tiled kernel on the GPU (``ops.geom.hv_count``, K18)."""
    return geom.hv_count(samples, points, strict=True)


def bounding_cube_monte_carlo_hv(key, objs, ref, num_sample):
    points = torch.abs(objs - ref).to(torch.float32)
    m = points.shape[1]
    bound = points.max(0).values
    samples = rnd.uniform(key, (num_sample, m)).to(points.device) * bound
    inside = (_dominated_counts(samples, points) > 0).sum()
    return inside / num_sample * torch.prod(bound)


def each_cube_monte_carlo_hv(key, objs, ref, num_sample):
    points = torch.abs(objs - ref).to(torch.float32)
    n, m = points.shape
    per = num_sample // n
    u = rnd.uniform(key, (n, per, m)).to(points.device) * points[:, None, :]
    cnt = _dominated_counts(u.reshape(-1, m), points).reshape(n, per)
    contrib = (1.0 / cnt.clamp(min=1).to(torch.float32)) * (cnt > 0)
    return (torch.prod(points, 1) * contrib.sum(1) / per).sum()


def _hso(pts: np.ndarray) -> float:
    """Exact dominated volume of ``pts`` w.r.t. the origin for maximisation-style
    boxes [0, p] (pts ≥ 0), by slicing along the last objective."""
    n, m = pts.shape
    if n == 0:
        return 0.0
    if m == 1:
        return float(pts[:, 0].max())
    if m == 2:
        order = np.argsort(-pts[:, 0])
        vol, ymax = 0.0, 0.0
        for i in order:
            x, y = pts[i]
            if y > ymax:
                vol += x * (y - ymax)
                ymax = y
        return vol
    order = np.argsort(-pts[:, -1])
    p = pts[order]
    vol = 0.0
    for k in range(n):
        h = p[k, -1] - (p[k + 1, -1] if k + 1 < n else 0.0)
        if h > 0:
            vol += h * _hso(p[: k + 1, :-1])
    return vol


def exact_hv(objs, ref) -> float:
    pts = torch.abs(torch.as_tensor(objs, dtype=torch.float64) - torch.as_tensor(ref, dtype=torch.float64)).cpu().numpy()
    return _hso(pts)


class HV:
    def __init__(self, ref, num_sample=100_000, sample_method="bounding_cube"):
        self.ref = ref
        self.num_sample = num_sample
        if sample_method == "bounding_cube":
            self.hv_impl = bounding_cube_monte_carlo_hv
        elif sample_method == "each_cube":
            self.hv_impl = each_cube_monte_carlo_hv
        elif sample_method == "exact":
            self.hv_impl = lambda key, objs, ref, n: torch.tensor(exact_hv(objs, ref))
        else:
            raise ValueError(f"sample_method should be 'bounding_cube' or 'each_cube', got '{sample_method}'.")

    def __call__(self, key, objs):
        ref = torch.as_tensor(self.ref, dtype=torch.float32, device=objs.device)
        return self.hv_impl(key, objs.to(torch.float32), ref, self.num_sample)
