"""Fused PSO tell (K7).  CPU path = torch reference; GPU path = one HIP kernel
that regenerates ``rp``/``rg`` from Philox counters in-register (never stored)."""
from __future__ import annotations

import torch

from . import _ext
from . import random as rnd


def pso_update(pop, vel, lbl, lbf, fit, gbl, rp_key, rg_key, w, phi_p, phi_g, lb, ub):
    n, d = pop.shape
    if pop.is_cuda:
        return _ext.ops().pso_update(pop.contiguous(), vel.contiguous(), lbl.contiguous(), lbf.contiguous(), fit.contiguous(),
                                     gbl.contiguous(), rp_key, rg_key, float(w), float(phi_p), float(phi_g),
                                     lb.contiguous(), ub.contiguous())
    rg = rnd.uniform(rg_key, (n, d))
    rp = rnd.uniform(rp_key, (n, d))
    compare = lbf > fit
    lbl = torch.where(compare[:, None], pop, lbl)
    lbf = torch.minimum(lbf, fit)
    vel = w * vel + phi_p * rp * (lbl - pop) + phi_g * rg * (gbl - pop)
    pop = torch.clamp(pop + vel, lb, ub)
    return pop, vel, lbl, lbf
