"""Device launchers for the multi-objective selection kernels (``mo_scan.hip``),
with sequential CPU reference implementations (the numerics oracles)."""
from __future__ import annotations

import torch

from . import _ext

FUNCS = {"tchebycheff": 0, "pbi": 1, "weighted_sum": 2, "modified_tchebycheff": 3}


def _agg_cpu(func, f, w, z):
    if func == 2:
        return (f * w).sum(-1)
    if func == 1:
        nw = torch.linalg.norm(w, dim=-1)
        d1 = ((f - z) * w).sum(-1) / nw
        d2 = torch.linalg.norm(f - z - d1[..., None] * w / nw[..., None], dim=-1)
        return d1 + 5 * d2
    a = torch.abs(f - z)
    return (a / w if func == 3 else a * w).amax(-1)


def moead_scan(objs, off_objs, P, W, z, func="tchebycheff", nr=None, update_z=False):
    """Sequential neighbourhood replacement: for i = 0..R−1, (optionally z ← min(z, f_i)),
    slots P[i, t] with g(old) ≥ g(f_i) are taken over by offspring i, at most ``nr`` per
    offspring (first in P order).  Returns (owner (N,) int, new objs (N, M), z)."""
    fid = FUNCS[func] if isinstance(func, str) else int(func)
    T = P.shape[1]
    nr = T if nr is None else int(nr)
    if objs.is_cuda:
        owner, o, zz = _ext.ops().moead_scan(objs.to(torch.float32).contiguous(), off_objs.to(torch.float32).contiguous(),
                                            P.to(torch.int32).contiguous(), W.to(torch.float32).contiguous(),
                                            z.to(torch.float32).contiguous(), fid, nr, int(bool(update_z)))
        return owner.long(), o, zz
    o = objs.to(torch.float32).clone()
    zz = z.to(torch.float32).clone()
    owner = torch.full((objs.shape[0],), -1, dtype=torch.long)
    for i in range(off_objs.shape[0]):
        fo = off_objs[i].to(torch.float32)
        if update_z:
            zz = torch.minimum(zz, fo)
        p = P[i].long()
        ok = _agg_cpu(fid, o[p], W[p], zz) >= _agg_cpu(fid, fo[None].expand(len(p), -1), W[p], zz)
        sel = p[ok][:nr]
        o[sel] = fo
        owner[sel] = i
    return owner, o, zz
