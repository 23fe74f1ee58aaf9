"""Simulated binary crossover, one-point and uniform crossover
(reference ``operators/crossover/{sbx,simulated_binary,one_point,uniform}.py``)."""
from __future__ import annotations

import torch

from ...ops import random as rnd


def simulated_binary(key, x, pro_c=1.0, dis_c=20.0, type=1, cols=None):
    """PlatEMO SBX: first half × second half; ``type=1`` → 2 children per pair
    (+ the odd last row passes through), ``type=2`` → 1 child per pair.

    Random streams (shared bit-for-bit with the HIP kernels): ``split(key, 2)`` →
    a per-gene word ``w`` whose top 24 bits give μ, bit 0 the sign of β and bit 1
    the 50 % "no crossover on this gene" coin; and a per-pair uniform compared with
    ``pro_c``.  One Philox word per gene instead of three.

    ``cols = (col0, d_total)``: ``x`` is the column block [col0, col0 + d) of a d_total-dim
    population (decision-axis state sharding); gene words are drawn at their global columns,
    so the block equals those columns of the unsharded offspring."""
    if x.is_cuda and x.dtype == torch.float32:
        from ...ops import evo as evo_ops

        return evo_ops.sbx(key, x, float(pro_c), float(dis_c), int(type), cols)
    gene_key, pair_key = rnd.split(key, 2)
    n, d = x.shape
    c0, dt = cols if cols is not None else (0, d)
    p1 = x[: n // 2]
    p2 = x[n // 2 : n // 2 * 2]
    n_p = p1.shape[0]
    dev = x.device
    w = rnd.bits(gene_key, (n_p, dt)).to(dev)[:, c0 : c0 + d]
    mu = rnd._u24(w)
    beta = torch.where(mu <= 0.5, (2 * mu) ** (1 / (dis_c + 1)), (2 - 2 * mu) ** (-1 / (dis_c + 1)))
    beta = torch.where((w & 1) == 1, -beta, beta)
    beta = torch.where(((w >> 1) & 1) == 1, torch.ones_like(beta), beta)
    beta = torch.where((rnd.uniform(pair_key, (n_p, 1)).to(dev) > pro_c).expand(n_p, d), torch.ones_like(beta), beta)
    beta = beta.to(x.dtype)
    mid, half = (p1 + p2) / 2, (p1 - p2) / 2
    if type == 1:
        off = torch.cat([mid + beta * half, mid - beta * half], 0)
        if n % 2 != 0:
            off = torch.cat([off, x[-1:]], 0)
        return off
    return mid + beta * half


class SimulatedBinary:
    column_blocks = True  # accepts cols= (decision-axis state sharding)

    def __init__(self, pro_c=1, dis_c=20, type=1):
        self.pro_c, self.dis_c, self.type = pro_c, dis_c, type

    def __call__(self, key, x, cols=None):
        return simulated_binary(key, x, self.pro_c, self.dis_c, self.type, cols)


def _random_pairing(key, x):
    b, d = x.shape
    x = rnd.permutation(key, x, axis=0)
    return x.reshape(b // 2, 2, d)


def sbx(key, x, distribution_factor):
    """Legacy SBX with random pairing and one β per pair-dimension vector (``simulated_binary.py``)."""
    kp, kc = rnd.split(key)
    paired = _random_pairing(kp, x)
    P, _, d = paired.shape
    u = rnd.uniform(kc, (P, d)).to(x.device)
    mu = distribution_factor
    all_low = (u <= 0.5).all(1, keepdim=True)
    beta = torch.where(all_low, (2 * u) ** (1 / (1 + mu)), (1 / (2 - 2 * u)) ** (1 / (1 + mu)))
    c1 = 0.5 * ((1 + beta) * paired[:, 0] + (1 - beta) * paired[:, 1])
    c2 = 0.5 * ((1 - beta) * paired[:, 0] + (1 + beta) * paired[:, 1])
    return torch.stack([c1, c2], 1).reshape(2 * P, d)


class SBXCrossover:
    def __init__(self, distribution_factor=1):
        self.distribution_factor = distribution_factor

    def __call__(self, key, x):
        return sbx(key, x, self.distribution_factor)


def one_point(key, x):
    kp, kc = rnd.split(key)
    paired = _random_pairing(kp, x)
    P, _, d = paired.shape
    point = rnd.randint(kc, (P, 1), 0, d).to(x.device) + 1
    mask = torch.arange(d, device=x.device)[None, :] < point
    c1 = torch.where(mask, paired[:, 0], paired[:, 1])
    c2 = torch.where(mask, paired[:, 1], paired[:, 0])
    return torch.stack([c1, c2], 1).reshape(2 * P, d)


class OnePoint:
    def __call__(self, key, x):
        return one_point(key, x)


def uniform_crossover(key, x):
    _, kp, kc = rnd.split(key, 3)
    paired = _random_pairing(kp, x)
    P, _, d = paired.shape
    mask = rnd.randint(kc, (P, d), 0, 2).to(x.device).bool()
    c1 = torch.where(mask, paired[:, 0], paired[:, 1])
    c2 = torch.where(mask, paired[:, 1], paired[:, 0])
    return torch.stack([c1, c2], 1).reshape(2 * P, d)


uniform_rand = uniform_crossover


class UniformRand:
    def __call__(self, key, x):
        return uniform_crossover(key, x)
