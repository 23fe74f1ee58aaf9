"""Device non-dominated sort (``nds.hip``) and crowding distance."""
from __future__ import annotations

import torch

from . import _ext
from .. import config


def non_dominated_sort(f: torch.Tensor, until: int = 0) -> torch.Tensor:
    """Pareto ranks; with ``until`` > 0 fronts are peeled only until ≥ ``until`` rows are
    ranked and the remaining rows get rank ``n`` (larger than every real rank)."""
    f = f.to(torch.float32).contiguous()
    if f.shape[0] <= 65536 and f.shape[1] <= 8:
        try:
            rank = _ext.ops().nds(f, int(until), _ext.error_flag(f.device))
        except RuntimeError as e:
            if "co-resident" not in str(e):
                raise
        else:
            if config.get("debug") and not torch.cuda.is_current_stream_capturing():
                _ext.check_kernel_errors()
            return rank
    from ..operators.selection.non_dominate import _peel
    from ..utils.common import dominate_relation

    dom = dominate_relation(f, f)
    return _peel(dom, dom.sum(0).to(torch.int32))


def crowding_distance(costs: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """Vectorised over objectives: one batched sort of the (m, n) masked keys."""
    n, m = costs.shape
    inf = torch.full((), float("inf"), device=costs.device, dtype=costs.dtype)  # fill kernel, not an H2D copy (capturable)
    nvalid = mask.sum()
    key = torch.where(mask[:, None], costs, inf).T  # (m, n)
    order = torch.argsort(key, dim=1, stable=True)
    sc = torch.gather(costs.T, 1, order)
    last = (nvalid - 1).clamp_min(0)
    rng = sc.gather(1, last.expand(m, 1)) - sc[:, :1]
    d = torch.empty((m, n), dtype=costs.dtype, device=costs.device)
    if n > 2:
        d.scatter_(1, order[:, 1:-1], (sc[:, 2:] - sc[:, :-2]) / rng)
    d.scatter_(1, order[:, :1], inf.expand(m, 1))
    d.scatter_(1, order.gather(1, last.expand(m, 1)), inf.expand(m, 1))
    dist = d.sum(0)
    return torch.where(mask, dist, -inf)


def nsga2_survivors(f: torch.Tensor, N: int, mask_pos: int, until: int = 0) -> torch.Tensor:
    """Indices of the N survivors of NSGA-II environmental selection (rank, then crowding
    distance on the front ``rank == sorted(rank)[mask_pos]``, lexsort order) — the fused
    ``nsga_select.hip`` kernel after the device non-dominated sort (n ≤ 8192)."""
    f = f.to(torch.float32).contiguous()
    rank = non_dominated_sort(f, until)
    return _ext.ops().nsga_select(rank, f, int(N), int(mask_pos))
