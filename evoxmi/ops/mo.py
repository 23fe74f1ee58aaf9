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


# ---------------------------------------------------------------- MOEA/D generation (moead.hip)
MOEAD_FUNCS = {"tchebycheff": 0, "pbi": 1, "weighted_sum": 2, "modified_tchebycheff": 3, "tchebycheff_norm": 4}


def moead_parents(neighbors: torch.Tensor, key: torch.Tensor, row0: int = 0, rows: int = 0):
    """First two columns of a per-row random permutation of ``neighbors`` (N, T):
    the rows' two smallest ``uniform(key, (N, T))`` entries, ties by column index
    (= ``argsort(uniform, stable=True)[:, :2]``).  Returns int32 (p0, p1); ``rows > 0``:
    only rows row0 .. row0+rows−1 are drawn (the rest are 0)."""
    return _ext.ops().moead_parents(neighbors.to(torch.int64).contiguous(), key.contiguous(), int(row0), int(rows))


def moead_variation(pop, p0, p1, key_x, key_m, lb, ub, pro_c, dis_c, pro_m, dis_m, row0=0, rows=0, win=None, out=None):
    """clip(PM(SBX_type2(pop[p0], pop[p1]))) in one pass; ``key_x``/``key_m`` are the keys
    ``SimulatedBinary`` / ``Polynomial`` would receive (bit-identical results).

    ``rows > 0``: only offspring ``row0 .. row0+rows−1`` (a rank's slice); ``win``: output
    row s is offspring ``win[s]`` regenerated from ``pop`` (``pop[s]`` where ``win[s] < 0``)
    — the population-sharded MOEA/D's row update without moving offspring rows."""
    from . import random as rnd

    n, d = p0.numel(), pop.shape[1]
    nm = n if n == 1 else (n // 2) * 2
    lb = lb.to(device=pop.device, dtype=torch.float32).expand(d).contiguous()
    ub = ub.to(device=pop.device, dtype=torch.float32).expand(d).contiguous()
    w = win.to(torch.int32).contiguous() if win is not None else None
    return _ext.ops().moead_variation(pop.contiguous(), p0, p1, rnd.split(key_x, 2).contiguous(), rnd.split(key_m, 2).contiguous(),
                                      lb, ub, float(pro_c), float(dis_c), float(pro_m), float(dis_m), int(nm), int(row0), int(rows), w,
                                      out)


def moead_halo_replace(obj, off_obj, w, z, z_max, rowptr, owner, slots, func, win_h):
    """In place on ``obj``: the replacement of the slots in ``slots`` only (owner-computes
    MOEA/D: a rank keeps current just the rows its offspring can draw as parents)."""
    fid = MOEAD_FUNCS[func] if isinstance(func, str) else int(func)
    f32 = lambda t: t.to(torch.float32).contiguous()  # noqa: E731
    _ext.ops().moead_halo_replace(obj, f32(off_obj), f32(w), f32(z), f32(z_max), rowptr, owner, slots, fid, win_h)


def moead_halo_gather(pop, slots, win_h, peer, starts, first=None):
    """pop[slots[h]] ← offspring win_h[h] read from the generating rank's buffer (``peer``:
    int64 device pointers, IPC-mapped; ``starts``: first offspring index of every rank).
    ``first`` (int32[N] workspace): deduplicated — an offspring that wins several of this rank's
    slots is read over xGMI once (into its lowest halo slot, whose index ``first[w]`` holds
    afterwards) and copied locally to the others."""
    _ext.ops().moead_halo_gather(pop, slots, win_h, peer, starts, first)


def moead_replace(pop_obj, off_obj, w, z, z_max, rowptr, owner, func):
    """Winner offspring per slot (or −1) and the new objective matrix — the exact parallel
    form of the reference's sequential replacement scan (see algorithms/mo/moead.py)."""
    fid = MOEAD_FUNCS[func] if isinstance(func, str) else int(func)
    f32 = lambda t: t.to(torch.float32).contiguous()
    return _ext.ops().moead_replace(f32(pop_obj), f32(off_obj), f32(w), f32(z), f32(z_max), rowptr, owner, fid)


def moead_select_rows(pop, off, win):
    """pop'[s] = off[win[s]] if win[s] >= 0 else pop[s]."""
    return _ext.ops().moead_select_rows(pop.contiguous(), off.contiguous(), win.to(torch.int32).contiguous())


def moead_select_rows_(pop, off, win):
    """In place: pop[s] = off[win[s]] for every s with win[s] >= 0 (returns ``pop``)."""
    _ext.ops().moead_select_rows_(pop, off.contiguous(), win.to(torch.int32).contiguous())
    return pop
