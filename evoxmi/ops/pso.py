"""Fused PSO tell (K7).  CPU path = torch reference; GPU path = one HIP kernel
that regenerates ``rp``/``rg`` from Philox counters in-register (never stored)."""
from __future__ import annotations

import torch

from . import _ext
from . import random as rnd


def pso_update(pop, vel, lbl, lbf, fit, gbl, rp_key, rg_key, w, phi_p, phi_g, lb, ub, col0: int = 0, d_total: int = None):
    """``pop`` may be the column block [col0, col0 + d) of a ``d_total``-dimensional swarm
    (decision-axis state sharding): rp / rg are then the same draws the unsharded swarm uses
    for those columns (Philox counter = row·d_total + column)."""
    n, d = pop.shape
    d_total = d if d_total is None else int(d_total)
    if pop.is_cuda:
        return _ext.ops().pso_update(pop.contiguous(), vel.contiguous(), lbl.contiguous(), lbf.contiguous(), fit.contiguous(),
                                     gbl.contiguous(), rp_key, rg_key, float(w), float(phi_p), float(phi_g),
                                     lb.contiguous(), ub.contiguous(), int(col0), int(d_total))
    rg = rnd.uniform(rg_key, (n, d_total))[:, col0 : col0 + d]
    rp = rnd.uniform(rp_key, (n, d_total))[:, col0 : col0 + d]
    compare = lbf > fit
    lbl = torch.where(compare[:, None], pop, lbl)
    lbf = torch.minimum(lbf, fit)
    vel = w * vel + phi_p * rp * (lbl - pop) + phi_g * rg * (gbl - pop)
    pop = torch.clamp(pop + vel, lb, ub)
    return pop, vel, lbl, lbf
