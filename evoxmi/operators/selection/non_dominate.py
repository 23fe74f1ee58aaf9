"""Non-dominated sorting and crowding distance (K9/K10 of SURVEY §2.10).

Reference: ``operators/selection/non_dominate.py``.  ``non_dominated_sort`` peels
fronts of the dominance matrix; on a GPU it runs the HIP path
(``csrc/kernels/nds.hip``): a bit-packed dominance matrix built by a tiled
compare kernel and a single-workgroup front-peeling kernel that keeps the whole
loop on the device (no host round trip per front).  ``method="host"`` is the
reference's numpy path (whose missing ``numpy`` import is fixed here).
"""
from __future__ import annotations

import numpy as np
import torch

from ...utils.common import dominate_relation


def _peel(dom: torch.Tensor, count: torch.Tensor) -> torch.Tensor:
    n = dom.shape[0]
    rank = torch.full((n,), -1, dtype=torch.int32, device=dom.device)
    count = count.clone()
    current = 0
    front = count == 0
    while bool(front.any()):
        rank = torch.where(front, torch.full_like(rank, current), rank)
        count = count - dom[front].sum(0).to(count.dtype) - front.to(count.dtype)
        current += 1
        front = count == 0
    return rank


def host_rank_from_domination_matrix(dominate_mat, dominate_count):
    dominate_mat = np.asarray(dominate_mat)
    dominate_count = np.array(dominate_count, copy=True)
    n = dominate_mat.shape[0]
    rank = np.empty((n,), dtype=np.int32)
    cur = 0
    front = dominate_count == 0
    while front.any():
        rank[front] = cur
        dominate_count -= dominate_mat[front, :].sum(axis=0)
        dominate_count -= front
        cur += 1
        front = dominate_count == 0
    return rank


def non_dominated_sort(x: torch.Tensor, method: str = "auto", until: int = 0) -> torch.Tensor:
    """Pareto rank of every row of ``x`` (n, m); 0 = first front (minimisation).

    ``until`` > 0 (GPU path) stops peeling once at least ``until`` rows are ranked;
    the remaining rows get rank ``n``.  Selection that keeps the best ``k`` rows only
    needs ``until = k`` (or ``k + 1`` to also read the rank just past the cut)."""
    assert method in ("auto", "scan", "full map-reduce", "host")
    if x.is_cuda and method in ("auto", "full map-reduce"):
        from ...ops import nds

        return nds.non_dominated_sort(x, until)
    dom = dominate_relation(x, x)
    count = dom.sum(0).to(torch.int32)
    if method == "host":
        r = host_rank_from_domination_matrix(dom.cpu().numpy(), count.cpu().numpy())
        return torch.as_tensor(r, device=x.device)
    return _peel(dom, count)


def crowding_distance(costs: torch.Tensor, mask: torch.Tensor = None) -> torch.Tensor:
    """NSGA-II crowding distance (reference ``non_dominate.py:116-156``).

    Extremes of every objective get +inf, masked-out rows −inf.
    """
    n, m = costs.shape
    dev = costs.device
    if mask is None:
        mask = torch.ones(n, dtype=torch.bool, device=dev)
    nvalid = int(mask.sum()) if not costs.is_cuda else None
    if costs.is_cuda:
        from ...ops import nds

        return nds.crowding_distance(costs, mask)
    dist = torch.zeros(n, dtype=costs.dtype, device=dev)
    if nvalid == 0:
        return torch.where(mask, dist, torch.full_like(dist, -float("inf")))
    for k in range(m):
        c = costs[:, k]
        # lexsort((cost, ~mask)): valid first, then by cost
        key = torch.where(mask, c, torch.full_like(c, float("inf")))
        order = torch.argsort(key, stable=True)
        sc = c[order]
        rng = sc[nvalid - 1] - sc[0]
        d = torch.empty(n, dtype=costs.dtype, device=dev)
        if n > 2:
            d[order[1:-1]] = (sc[2:] - sc[:-2]) / rng
        d[order[0]] = float("inf")
        d[order[nvalid - 1]] = float("inf")
        dist = dist + d
    return torch.where(mask, dist, torch.full_like(dist, -float("inf")))


def crowding_distance_sort(x: torch.Tensor, mask: torch.Tensor = None) -> torch.Tensor:
    return torch.argsort(crowding_distance(x, mask), stable=True)


def lexsort(keys):
    """numpy-style lexsort: the LAST key is primary."""
    order = torch.arange(keys[0].shape[0], device=keys[0].device)
    for k in keys:
        order = order[torch.argsort(k[order], stable=True)]
    return order


def non_dominate(population, fitness, topk: int):
    """NSGA-II environmental selection: rank, then crowding on the worst kept front.

    The reference passes ``crowding_distance_sort`` (an argsort *order*) as the
    tie-break key (``non_dominate.py:195-197``); the intent — larger crowding
    distance first — is implemented here.
    """
    rank = non_dominated_sort(fitness, until=topk)
    worst_rank = torch.sort(rank).values[topk - 1]
    mask = rank == worst_rank
    cd = crowding_distance(fitness, mask)
    combined = lexsort([-cd, rank.to(cd.dtype)])[:topk]
    return population[combined], fitness[combined]


class NonDominate:
    def __init__(self, topk):
        self.topk = topk

    def __call__(self, population, fitness):
        return non_dominate(population, fitness, self.topk)
