"""Counter-based random numbers with a JAX-like functional key API.

The reference draws every random number through ``jax.random`` (threefry keys,
e.g. ``cma_es.py:132``, ``pso.py:76-77``, ``de.py:76-97``).  evoxmi keeps the same
*functional* contract — a key is a value, ``split``/``fold_in`` derive new keys,
samplers never mutate global state — but uses **Philox4x32-10**, the
counter-based generator that maps cleanly onto CDNA4: one 64-lane wave computes
256 independent 32-bit words with integer-multiply-high instructions, no state
is carried between threads, and any shard can regenerate any element from its
global index (``counter = element // 4``).  That last property is what makes
population-sharded runs on 1/2/4/8 GPUs produce identical populations.

A key is an ``int64`` tensor of shape ``(2,)`` holding two 32-bit words.  The CPU
implementation below uses wrapping int64 arithmetic (exactly the low 64 bits of
the 32x32 product); the GPU path runs the same function in a HIP kernel
(``csrc/kernels/rng.hip``) and produces bit-identical words.
"""
from __future__ import annotations

import math
from typing import Sequence, Union

import torch

M0 = 0xD2511F53
M1 = 0xCD9E8D57
W0 = 0x9E3779B9
W1 = 0xBB67AE85
MASK32 = 0xFFFFFFFF

# domain separation for the fourth counter word
_DOMAIN_BITS = 0
_DOMAIN_SPLIT = 0x5EED5EED
_DOMAIN_FOLD = 0xF01DF01D


def _as_shape(shape) -> tuple:
    if isinstance(shape, int):
        return (shape,)
    return tuple(int(s) for s in shape)


def _numel(shape) -> int:
    n = 1
    for s in shape:
        n *= s
    return n


def PRNGKey(seed: int, device=None) -> torch.Tensor:
    """Key from an integer seed (reference: ``jax.random.PRNGKey``)."""
    seed = int(seed) & 0xFFFFFFFFFFFFFFFF
    return torch.tensor([(seed >> 32) & MASK32, seed & MASK32], dtype=torch.int64, device=device)


key = PRNGKey


def philox4x32(c0, c1, c2, c3, k0, k1, rounds: int = 10):
    """Vectorised Philox4x32 on int64 tensors holding uint32 values."""
    for _ in range(rounds):
        p0 = c0 * M0
        p1 = c2 * M1
        hi0 = (p0 >> 32) & MASK32
        lo0 = p0 & MASK32
        hi1 = (p1 >> 32) & MASK32
        lo1 = p1 & MASK32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0), lo1, (hi0 ^ c3 ^ k1), lo0
        k0 = (k0 + W0) & MASK32
        k1 = (k1 + W1) & MASK32
    return c0, c1, c2, c3


def _blocks(key: torch.Tensor, nblocks: int, domain: int, offset: int = 0):
    dev = key.device
    if key.is_cuda:
        # one HIP launch (rng.hip: philox_words) instead of ~80 int64 elementwise kernels
        w = _ext().ops().philox_words(key.contiguous(), int(nblocks), int(domain), int(offset))
        return w[:, 0], w[:, 1], w[:, 2], w[:, 3]
    idx = torch.arange(offset, offset + nblocks, dtype=torch.int64, device=dev)
    c0 = idx & MASK32
    c1 = (idx >> 32) & MASK32
    c2 = torch.zeros_like(idx)
    c3 = torch.full_like(idx, domain)
    k0 = key[0].expand_as(idx)
    k1 = key[1].expand_as(idx)
    return philox4x32(c0, c1, c2, c3, k0, k1)


def split(key: torch.Tensor, num: int = 2) -> torch.Tensor:
    """``num`` new keys, shape ``(num, 2)`` (reference ``jax.random.split``)."""
    _check_key(key)
    if key.is_cuda and key.dim() == 1:
        # the (num, 2) keys straight from one launch (no stacking copy)
        return _ext().ops().philox_words(key.contiguous(), int(num), int(_DOMAIN_SPLIT), 0, 2)
    w0, w1, _, _ = _blocks(key, num, _DOMAIN_SPLIT)
    return torch.stack([w0, w1], dim=1)


def fold_in(key: torch.Tensor, data: int) -> torch.Tensor:
    """Derive a key from ``key`` and an integer (reference ``jax.random.fold_in``)."""
    _check_key(key)
    w0, w1, _, _ = _blocks(key, 1, _DOMAIN_FOLD, offset=int(data) & 0xFFFFFFFFFFFF)
    return torch.stack([w0[0], w1[0]])


def _check_key(key):
    if not (isinstance(key, torch.Tensor) and key.dtype == torch.int64 and key.shape == (2,)):
        raise TypeError(f"expected a PRNG key (int64 tensor of shape (2,)), got {type(key)} {getattr(key, 'shape', '')}")


def bits(key: torch.Tensor, shape, offset: int = 0) -> torch.Tensor:
    """Raw uint32 words (as int64) — element ``i`` is word ``i % 4`` of block ``i // 4``.

    ``offset`` is an element offset (multiple of 4) so that a shard can generate
    rows ``[r0, r1)`` of a larger virtual tensor without producing the rest.
    """
    _check_key(key)
    shape = _as_shape(shape)
    n = _numel(shape)
    assert offset % 4 == 0
    nb = (n + 3) // 4
    w = _blocks(key, nb, _DOMAIN_BITS, offset=offset // 4)
    out = torch.stack(w, dim=1).reshape(-1)[:n]
    return out.reshape(shape)


def _u24(w: torch.Tensor) -> torch.Tensor:
    # strictly inside (0, 1): ((w >> 8) + 0.5) * 2^-24, exact in float32
    return ((w >> 8).to(torch.float32) + 0.5) * (1.0 / 16777216.0)


def _ext():
    from . import _ext as ext

    return ext


def uniform(key, shape=(), dtype=torch.float32, minval=0.0, maxval=1.0, offset: int = 0) -> torch.Tensor:
    """U(minval, maxval) samples (reference ``jax.random.uniform``)."""
    if offset & 3:
        return _aligned(lambda k, s, dtype, offset: uniform(k, s, dtype, 0.0, 1.0, offset), key, shape, dtype, offset) * (maxval - minval) + minval
    shape = _as_shape(shape)
    if key.is_cuda and _numel(shape) >= 4096:
        u = _ext().philox_fill(key, _numel(shape), 0, offset).reshape(shape)
    else:
        u = _u24(bits(key, shape, offset))
    u = u.to(dtype)
    if not (minval == 0.0 and maxval == 1.0):
        u = u * (maxval - minval) + minval
    return u


def _aligned(fn, key, shape, dtype, offset):
    """Support element offsets that are not a multiple of 4 (shard starts)."""
    shape = _as_shape(shape)
    lead = offset & 3
    n = _numel(shape)
    flat = fn(key, (n + lead,), dtype=dtype, offset=offset - lead)
    return flat[lead:].reshape(shape)


def normal(key, shape=(), dtype=torch.float32, offset: int = 0) -> torch.Tensor:
    """Standard normal samples via Box–Muller on word pairs (0,1) and (2,3).

    Element ``4b + j`` uses block ``b``: ``r = sqrt(-2 ln u_{2p})``, ``θ = 2π u_{2p+1}``
    with ``p = j // 2``; ``j`` even takes ``r cos θ``, odd ``r sin θ``.
    """
    if offset & 3:
        return _aligned(normal, key, shape, dtype, offset)
    shape = _as_shape(shape)
    n = _numel(shape)
    if key.is_cuda and n >= 4096:
        return _ext().philox_fill(key, n, 1, offset).reshape(shape).to(dtype)
    nb = (n + 3) // 4
    w0, w1, w2, w3 = _blocks(key, nb, _DOMAIN_BITS, offset=offset // 4)
    u0, u1, u2, u3 = _u24(w0), _u24(w1), _u24(w2), _u24(w3)
    r0 = torch.sqrt(-2.0 * torch.log(u0))
    r1 = torch.sqrt(-2.0 * torch.log(u2))
    t0 = (2.0 * math.pi) * u1
    t1 = (2.0 * math.pi) * u3
    z = torch.stack([r0 * torch.cos(t0), r0 * torch.sin(t0), r1 * torch.cos(t1), r1 * torch.sin(t1)], dim=1)
    return z.reshape(-1)[:n].reshape(shape).to(dtype)


def _window(key, rows, dtot, col0, own, row0, device, dist):
    dev = torch.device(device) if device is not None else key.device
    if dev.type == "cuda":
        return _ext().ops().philox_window(key.to(dev).contiguous(), int(rows), int(dtot), int(col0), int(own), int(row0), int(dist))
    fn = normal if dist else uniform
    if own == dtot and col0 == 0:
        return fn(key, (rows, dtot), offset=row0 * dtot).to(dev)
    if not rows:
        return torch.zeros(0, own, device=dev)
    return torch.stack([fn(key, (own,), offset=(row0 + r) * dtot + col0) for r in range(rows)]).to(dev)


def normal_window(key, rows: int, dtot: int, col0: int, own: int, row0: int = 0, device=None) -> torch.Tensor:
    """Columns [col0, col0 + own) of rows [row0, row0 + rows) of ``normal(key, (·, dtot))`` —
    the block a decision-axis-sharded rank owns, bitwise equal to slicing the full matrix.  On a
    GPU one kernel draws only the block (rng.hip: philox_window_kernel)."""
    return _window(key, rows, dtot, col0, own, row0, device, 1)


def uniform_window(key, rows: int, dtot: int, col0: int, own: int, row0: int = 0, device=None) -> torch.Tensor:
    """The same column window of ``uniform(key, (·, dtot))``."""
    return _window(key, rows, dtot, col0, own, row0, device, 0)


def randint(key, shape, minval: int, maxval: int, dtype=torch.int64) -> torch.Tensor:
    """Integers in ``[minval, maxval)`` (reference ``jax.random.randint``)."""
    shape = _as_shape(shape)
    span = int(maxval) - int(minval)
    assert span > 0
    w = bits(key, shape)
    # 32-bit multiply-shift (Lemire) for an unbiased-enough range reduction
    r = (w * span) >> 32
    return (r + int(minval)).to(dtype)


def bernoulli(key, p=0.5, shape=()) -> torch.Tensor:
    return uniform(key, shape) < p


def cauchy(key, shape=(), dtype=torch.float32) -> torch.Tensor:
    u = uniform(key, shape, dtype=torch.float32)
    return torch.tan(math.pi * (u - 0.5)).to(dtype)


def gumbel(key, shape=(), dtype=torch.float32) -> torch.Tensor:
    u = uniform(key, shape)
    return (-torch.log(-torch.log(u))).to(dtype)


def truncated_normal(key, lower, upper, shape=(), dtype=torch.float32) -> torch.Tensor:
    """Inverse-CDF truncated normal."""
    u = uniform(key, shape)
    sq2 = math.sqrt(2.0)
    lo = torch.as_tensor(lower, dtype=torch.float32, device=key.device)
    hi = torch.as_tensor(upper, dtype=torch.float32, device=key.device)
    a = torch.special.ndtr(lo)
    b = torch.special.ndtr(hi)
    return (sq2 * torch.erfinv(2 * (a + u * (b - a)) - 1)).clamp(lo, hi).to(dtype)


def permutation(key, x: Union[int, torch.Tensor], axis: int = 0) -> torch.Tensor:
    """Random permutation of ``range(x)`` or of ``x`` along ``axis`` (sort of random keys)."""
    if isinstance(x, int):
        n = x
        perm = torch.argsort(uniform(key, (n,)), stable=True)
        return perm
    n = x.shape[axis]
    perm = torch.argsort(uniform(key, (n,)), stable=True).to(x.device)
    return torch.index_select(x, axis, perm)


def batched_permutation(key, rows: int, n: int) -> torch.Tensor:
    """``rows`` independent permutations of ``range(n)``, shape ``(rows, n)``."""
    return torch.argsort(uniform(key, (rows, n)), dim=1, stable=True)


def _topk(x, k, dim=-1, largest=True):
    from .sort import topk

    return topk(x, k, dim, largest)


def choice(key, a: Union[int, torch.Tensor], shape=(), replace: bool = True, p=None, axis: int = 0) -> torch.Tensor:
    """Sample from ``a`` (int ⇒ ``range(a)``), optionally weighted by ``p``."""
    shape = _as_shape(shape)
    n = a if isinstance(a, int) else a.shape[axis]
    m = _numel(shape)
    dev = key.device
    if p is None:
        if replace:
            idx = randint(key, (m,), 0, n)
        else:
            assert m <= n, "cannot take a larger sample than population when replace=False"
            idx = torch.argsort(uniform(key, (n,)), stable=True)[:m]
    else:
        p = torch.as_tensor(p, dtype=torch.float32, device=dev)
        if replace:
            cdf = torch.cumsum(p, 0)
            cdf = cdf / cdf[-1]
            u = uniform(key, (m,))
            idx = torch.searchsorted(cdf, u).clamp_max(n - 1)
        else:
            g = gumbel(key, (n,)) + torch.log(p)
            idx = _topk(g, m)[1]
    idx = idx.reshape(shape)
    if isinstance(a, int):
        return idx
    return torch.index_select(a, axis, idx.reshape(-1).to(a.device)).reshape(shape + tuple(a.shape[axis + 1 :]))


def key_to_int(key: torch.Tensor) -> int:
    k = key.tolist()
    return (int(k[0]) << 32) | int(k[1])
