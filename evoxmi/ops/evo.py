"""Device launchers of the fused variation operators (``evo_ops.hip``)."""
from __future__ import annotations


import torch

from . import _ext
from .. import config
from . import random as rnd


def sbx(key, x, pro_c, dis_c, type, cols=None):
    """``cols = (col0, d_total)``: x is that column block of a d_total-dim population."""
    keys = rnd.split(key, 2).contiguous()
    c0, dt = cols if cols is not None else (0, 0)
    return _ext.ops().sbx(x.contiguous(), keys, float(pro_c), float(dis_c), int(type), int(c0), int(dt))


def polynomial(key, x, lb, ub, pro_m, dis_m, cols=None):
    keys = rnd.split(key, 2).contiguous()
    c0, dt = cols if cols is not None else (0, 0)
    nm = x.shape[0] if x.shape[0] == 1 else (x.shape[0] // 2) * 2
    d = x.shape[1]
    lb = lb.to(device=x.device, dtype=torch.float32).expand(d).contiguous()
    ub = ub.to(device=x.device, dtype=torch.float32).expand(d).contiguous()
    return _ext.ops().pm(x.contiguous(), lb, ub, keys, float(pro_m), float(dis_m), int(nm), int(c0), int(dt))


_CROSS = {"bin": 0, "exp": 1, "arith": 2}
def _err_flag(dev):
    """Sticky device error word (``_ext.error_flag``); read with ``kernel_error_flags()``."""
    return _ext.error_flag(dev)


def kernel_error_flags(device="cuda") -> int:
    return _ext.kernel_error_flags()


_REPAIR = {"none": 0, "clip": 1, "midpoint": 2}


def de_trial(key, P, idx, coef, cur, mode, CR, jr, L, lb, ub, repair="clip", col0: int = 0, d_total: int = None):
    """Fused DE trial vectors (``evo_ops.hip: de_trial_kernel``).

    P: (rows, d) candidate matrix (population, or population ∪ archive);
    idx/coef: (R, K) gather rows and weights of the mutation vector;
    cur: (R,) target rows; mode: (R,) 0 = bin, 1 = exp, 2 = arith;
    CR: (R,) crossover rate (arith: recombination weight); jr: (R,) j_rand (bin) or
    window start (exp); L: (R,) exp window length; ``key`` seeds u(i, j) exactly as
    ``uniform(key, (R, d))``.  The CPU branch is the numerics oracle.
    ``col0`` / ``d_total``: ``P`` holds the column block [col0, col0 + d) of a d_total-dim
    population (decision-axis state sharding); draws, j_rand and windows use global columns.
    """
    R, K = idx.shape
    d = P.shape[1]
    rep = _REPAIR[repair] if isinstance(repair, str) else int(repair)
    dev = P.device
    lb = torch.as_tensor(lb, dtype=torch.float32, device=dev).expand(d).contiguous()
    ub = torch.as_tensor(ub, dtype=torch.float32, device=dev).expand(d).contiguous()
    if P.is_cuda:
        i32 = lambda t: t.to(device=dev, dtype=torch.int32).contiguous()
        f32 = lambda t: t.to(device=dev, dtype=torch.float32).contiguous()
        err = _err_flag(dev)
        out = _ext.ops().de_trial(P.contiguous(), i32(idx), f32(coef), i32(cur), i32(mode), f32(CR), i32(jr), i32(L),
                                  key.contiguous(), lb, ub, rep, err, int(col0), int(d if d_total is None else d_total))
        if config.get("debug") and not torch.cuda.is_current_stream_capturing():
            bad = int(err.item())
            if bad:
                raise RuntimeError(f"de_trial: out-of-range row index (flag {bad}); idx range "
                                   f"[{int(idx.min())}, {int(idx.max())}], cur range [{int(cur.min())}, {int(cur.max())}], rows {P.shape[0]}")
        return out
    m = torch.einsum("rk,rkd->rd", coef.to(P.dtype), P[idx.long()])
    x = P[cur.long()]
    dt = d if d_total is None else int(d_total)
    j = torch.arange(col0, col0 + d, device=dev)[None, :]
    u = rnd.uniform(key, (R, dt))[:, col0 : col0 + d]
    bin_mask = (u < CR[:, None]) | (j == jr[:, None])
    pos = (j - jr[:, None]) % dt
    exp_mask = pos < L[:, None]
    mode = mode[:, None]
    v = torch.where(mode == 0, torch.where(bin_mask, m, x),
                    torch.where(mode == 1, torch.where(exp_mask, m, x), x + CR[:, None] * (m - x)))
    if rep == 1:
        v = torch.minimum(torch.maximum(v, lb), ub)
    elif rep == 2:
        v = torch.where(v < lb, 0.5 * (x + lb), v)
        v = torch.where(v > ub, 0.5 * (x + ub), v)
    return v
