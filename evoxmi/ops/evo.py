"""Device launchers of the fused variation operators (``evo_ops.hip``)."""
from __future__ import annotations

import torch

from . import _ext
from . import random as rnd


def sbx(key, x, pro_c, dis_c, type):
    keys = rnd.split(key, 4).contiguous()
    return _ext.ops().sbx(x.contiguous(), keys, float(pro_c), float(dis_c), int(type))


def polynomial(key, x, lb, ub, pro_m, dis_m):
    keys = rnd.split(key, 2).contiguous()
    nm = x.shape[0] if x.shape[0] == 1 else (x.shape[0] // 2) * 2
    d = x.shape[1]
    lb = lb.to(device=x.device, dtype=torch.float32).expand(d).contiguous()
    ub = ub.to(device=x.device, dtype=torch.float32).expand(d).contiguous()
    return _ext.ops().pm(x.contiguous(), lb, ub, keys, float(pro_m), float(dis_m), int(nm))
