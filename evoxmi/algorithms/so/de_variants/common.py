"""Shared DE machinery: one batched trial generator for every variant of the zoo.

The reference builds each trial vector in a ``vmap``-ed ``_ask_one`` (e.g.
``de_variants/jade.py:89-125``, ``code.py:95-140``): pick a random base, the
best, a random p-best and the current vector, combine them with a
strategy code ``[base_prim, base_sec, n_diff, cross]``
(``0 = rand, 1 = best, 2 = pbest, 3 = current``; ``cross: 0 = bin, 1 = exp, 2 = arith``)

    base     = prim + F·(sec − prim)
    mutation = base + F·Σ_{k ≤ n_diff}(x_{2k−1} − x_{2k})

then cross it with the current vector and clip.  Here all N rows are produced at
once: the random index sets are drawn with batched, graph-capture-safe tensor ops
(no host synchronisation, dynamic population sizes are tensors), the mutation is
expressed as a weighted gather ``Σ_k coef[i,k]·P[idx[i,k]]`` and the gather,
crossover and repair run as a single fused HIP kernel (``ops.evo.de_trial``).

Differences from the reference that are deliberate (documented per variant):
random streams are Philox (not threefry) and the per-row keys of the reference are
replaced by whole-population draws; indices equal to the target are remapped to
``pop_size_reduced − 1`` exactly as in ``operators/crossover/differential_evolution.py:80-82``.
"""
from __future__ import annotations

import math
from typing import Optional, Union

import torch

from evoxmi.ops.sort import topk as _topk

from ....core import State
from ....ops import evo as evo_ops
from ....ops import random as rnd

RAND, BEST, PBEST, CURRENT = 0, 1, 2, 3
BIN, EXP, ARITH = 0, 1, 2

# strategy codes (reference code.py:16-24, epsde.py:16-26)
rand_1_bin = (0, 0, 1, 0)
rand2best_2_bin = (0, 1, 2, 0)
rand_2_bin = (0, 0, 2, 0)
best_2_bin = (1, 1, 2, 0)
current2rand_1_bin = (3, 0, 1, 0)
current2rand_1 = (0, 0, 1, 2)  # ≡ rand/1/arith
current2pbest_1_bin = (3, 2, 1, 0)

IntLike = Union[int, torch.Tensor]

_CONST = {}


def dconst(value, device, dtype=torch.float32) -> torch.Tensor:
    """Device-resident constant, created once per (value, device, dtype).

    Host→device copies are not allowed while a hipGraph is being captured; the
    workflow's eager warm-up step creates every constant before capture starts.
    """
    if isinstance(value, torch.Tensor):
        if value.device == torch.device(device):
            return value if value.dtype == dtype else value.to(dtype)
        k = ("t", id(value), value.data_ptr(), str(device), dtype)
        if k not in _CONST:
            _CONST[k] = (value, value.to(device=device, dtype=dtype))  # keep the source alive so id() stays unique
        return _CONST[k][1]
    k = ("v", value if not isinstance(value, list) else tuple(value), str(device), dtype)
    if k not in _CONST:
        _CONST[k] = torch.as_tensor(value, dtype=dtype, device=device)
    return _CONST[k]


def _t(x, device, dtype=torch.float32):
    return x.to(dtype) if isinstance(x, torch.Tensor) else dconst(x, device, dtype)


def init_population(key, pop_size, lb, ub, mean=None, stdvar=None):
    """Uniform in the box, or N(mean, stdvar²) clipped (reference ``de.py:49-58``;
    the reference omits ``+ mean`` there — we add it so ``mean`` has its documented effect)."""
    d = lb.shape[0]
    if mean is not None and stdvar is not None:
        pop = mean + stdvar * rnd.normal(key, (pop_size, d)).to(lb.device)
        return torch.clamp(pop, lb, ub)
    return rnd.uniform(key, (pop_size, d)).to(lb.device) * (ub - lb) + lb


def sample_distinct(key, rows: int, k: int, n: int, upper: Optional[IntLike] = None, device=None) -> torch.Tensor:
    """``rows`` independent ordered samples of ``k`` distinct integers in ``[0, upper)``.

    ``upper`` (≤ n, may be a 0-d tensor) is honoured without host synchronisation.
    Small n: argsort of masked uniform keys (one kernel); large n: sequential
    selection with sorted-rank adjustment (O(rows·k²), independent of n).
    """
    upper = n if upper is None else upper
    if n <= 4096:
        u = rnd.uniform(key, (rows, n)).to(device)
        j = torch.arange(n, device=device)[None, :]
        u = torch.where(j < upper, u, u + 2.0)
        kk = min(k, n)
        out = torch.argsort(u, dim=1)[:, :kk]
        if kk < k:  # fewer candidates than requested: repeat the last (padding only)
            out = torch.cat([out, out[:, -1:].expand(-1, k - kk)], 1)
        return out
    u = rnd.uniform(key, (rows, k)).to(device)
    up = _t(upper, device)
    picks = []
    srt = torch.empty((rows, 0), dtype=torch.int64, device=device)
    for t in range(k):
        r = torch.floor(u[:, t] * torch.clamp(up - t, min=1)).to(torch.int64)
        for s in range(t):
            r = r + (r >= srt[:, s]).to(torch.int64)
        picks.append(r)
        srt = torch.sort(torch.cat([srt, r[:, None]], 1), dim=1).values
    return torch.stack(picks, 1)


def pbest_indices(key, rows: int, fitness: torch.Tensor, p) -> torch.Tensor:
    """A uniformly random member of the best ⌊N·p⌋ per row (reference
    ``find_pbest.py:12-25``; ⌊N·p⌋ = 0 degenerates to the whole population as there)."""
    N = fitness.shape[0]
    top = torch.floor(_t(p, fitness.device) * N).to(torch.int64)
    top = torch.where(top <= 0, torch.full_like(top, N), top)
    order = torch.argsort(fitness, stable=True)
    r = torch.floor(rnd.uniform(key, (rows,)).to(fitness.device) * top).to(torch.int64)
    return order[torch.clamp(r, max=N - 1)]


def _remap_self(choice, cur, reduced):
    red = _t(reduced, choice.device, choice.dtype)
    return torch.where(choice == cur[:, None], (red - 1).expand_as(choice), choice)


def diff_choices(key, cur, P: int, population, reduced=None, archive=None, rank_k=None, fitness=None):
    """Index sets of the difference members, (R, P), and the candidate matrix they index.

    * plain (reference ``de_diff_sum``): distinct indices in [0, reduced);
    * ``archive`` (``de_diff_sum_archive``): minuends from the population, subtrahends
      (positions 2, 4, …) from P ∪ A with NaN rows moved to the end, drawn from
      [0, 2·reduced);
    * ``rank_k`` (``de_diff_sum_rank``): weighted without replacement, weight
      ``k·(N − rank) + 1`` restricted to the best ``reduced`` ranks.
    """
    N, d = population.shape
    R = cur.shape[0]
    dev = population.device
    red = N if reduced is None else reduced
    if rank_k is not None:
        ranks = torch.argsort(torch.argsort(fitness, stable=True), stable=True)
        w = rank_k * (N - ranks).to(torch.float32) + 1
        kth = torch.clamp(N - _t(red, dev, torch.int64), 0, N - 1)
        nth = torch.sort(w).values.gather(0, kth.reshape(1))
        w = torch.where(w < nth, torch.zeros_like(w), w)
        logp = torch.log(w / w.sum())
        g = rnd.gumbel(key, (R, N)).to(dev) + logp[None, :]
        choice = _topk(g, min(P, N), dim=1)[1]
        return _remap_self(choice, cur, red), population
    if archive is None:
        choice = sample_distinct(key, R, P, N, red, dev)
        return _remap_self(choice, cur, red), population
    k1, k2 = rnd.split(key)
    pa = torch.cat([population, archive], 0)
    nan_rows = torch.isnan(pa.sum(1))
    order = torch.argsort(nan_rows.to(torch.int64), stable=True)
    moved = pa[order]
    base = sample_distinct(k1, R, P, N, red, dev)
    sub = sample_distinct(k2, R, P, pa.shape[0], 2 * red, dev)
    j = torch.arange(P, device=dev)
    even = (j >= 2) & (j % 2 == 0)
    ids = torch.where(even[None, :], sub, base)
    return _remap_self(ids, cur, red), moved


def as_strategy(strat, R, device):
    s = _t(strat if isinstance(strat, torch.Tensor) else tuple(strat), device, torch.int64)
    return s.expand(R, 4) if s.ndim == 1 else s


def generate_trials(key, population, fitness, best_index, cur, strategy, F, CR, diff_padding_num: int, lb, ub, *,
                    p=0.05, reduced=None, archive=None, rank_k=None, Fw=None, repair="clip", choices=None, cols=None):
    """Trial vectors for target rows ``cur`` (R,) under per-row strategies.

    Returns ``(trials (R, d), rand_idx (R,))``.  ``Fw`` scales the pbest term
    (jSO's F_w).  ``choices`` optionally provides pre-drawn difference indices into
    the population (plain DE / ODE path).  ``cols = (col0, d_total)``: ``population`` is this
    rank's column block of a d_total-dim population (decision-axis state sharding); every
    per-row draw is the unsharded one and the trial block equals those columns of the
    unsharded trials.
    """
    N, d = population.shape
    col0, d_tot = cols if cols is not None else (0, d)
    R = cur.shape[0]
    dev = population.device
    k_sel, k_pb, k_jr, k_u, k_exp = rnd.split(key, 5)
    if choices is None:
        choices, cand = diff_choices(k_sel, cur, diff_padding_num, population, reduced, archive, rank_k, fitness)
    else:
        cand = population
    P = choices.shape[1]
    strat = as_strategy(strategy, R, dev)
    F = _t(F, dev).expand(R)
    CR = _t(CR, dev).expand(R)
    off = cand.shape[0] if cand is not population else 0
    Pext = torch.cat([cand, population], 0) if off else population
    pb = pbest_indices(k_pb, R, fitness, p)
    best = _t(best_index, dev, torch.int64).expand(R)
    # columns: rand, best, pbest, current, diff members 1..P-1 (the rand member of the
    # archive path indexes the moved P ∪ A matrix, reference differential_evolution.py:139-141)
    base_idx = torch.stack([choices[:, 0], best + off, pb + off, cur + off], 1)
    idx = torch.cat([base_idx, choices[:, 1:]], 1)
    prim, sec, nd, cross = strat[:, 0], strat[:, 1], strat[:, 2], strat[:, 3]
    Fs = F if Fw is None else F * _t(Fw, dev)
    # out-of-place (one-hot sums, concatenation) so the same code runs under torch.func.vmap
    # (BatchedRuns: independent runs as one launch sequence)
    c4 = torch.arange(4, device=dev)[None, :]
    base_coef = (c4 == prim[:, None]).to(torch.float32) * (1 - Fs)[:, None] + (c4 == sec[:, None]).to(torch.float32) * Fs[:, None]
    j = torch.arange(1, P, device=dev)[None, :]
    keep = (j < 2 * nd[:, None] + 1).to(torch.float32)
    sign = torch.where(j % 2 == 1, 1.0, -1.0)
    coef = torch.cat([base_coef, F[:, None] * keep * sign], 1)
    jr = rnd.randint(k_jr, (R,), 0, d_tot).to(dev)
    # exponential crossover: window length min(Geometric(CR), d) − 1 from a random start
    u = rnd.uniform(k_exp, (R,)).to(dev)
    geo = torch.where(CR >= 1, torch.ones_like(u), torch.ceil(torch.log(u) / torch.log1p(-CR.clamp(max=1 - 1e-7))))
    L = (torch.minimum(geo, torch.full_like(geo, d_tot)) - 1).to(torch.int32)
    trials = evo_ops.de_trial(k_u, Pext, idx, coef, cur + off, cross, CR, jr, L, lb, ub, repair, col0=col0, d_total=d_tot)
    return trials, choices[:, 0]


def greedy_replace(population, fitness, trials, trial_fitness, cur=None, strict=True):
    """One-to-one replacement (``<`` when strict, else ``<=``) of rows ``cur``."""
    if cur is None:
        better = trial_fitness < fitness if strict else trial_fitness <= fitness
        return torch.where(better[:, None], trials, population), torch.where(better, trial_fitness, fitness), better
    old_f = fitness[cur]
    better = trial_fitness < old_f if strict else trial_fitness <= old_f
    pop = population.index_copy(0, cur, torch.where(better[:, None], trials, population[cur]))
    fit = fitness.index_copy(0, cur, torch.where(better, trial_fitness, old_f))
    return pop, fit, better


def lehmer_update(values_ok: torch.Tensor, vals: torch.Tensor, weights: Optional[torch.Tensor] = None):
    """Weighted Lehmer mean Σw v² / Σw v over successful entries (NaN if none)."""
    nan = torch.full_like(vals, float("nan"))
    v = torch.where(values_ok, vals, nan)
    w = torch.ones_like(vals) if weights is None else weights
    w = torch.where(values_ok, w, nan)
    return torch.nansum(w * v * v) / torch.nansum(w * v)


def roll_in(memory: torch.Tensor, value: torch.Tensor) -> torch.Tensor:
    """roll(memory, 1) with ``value`` at slot 0, unless value is NaN."""
    upd = torch.cat([value.reshape(1).to(memory.dtype), memory[:-1]])
    return torch.where(torch.isnan(value), memory, upd)


def scalar(x, device, dtype=torch.float32):
    return torch.as_tensor(x, dtype=dtype, device=device).clone()


def base_state(key, population, **extra):
    dev = population.device
    return State(
        population=population,
        fitness=torch.full((population.shape[0],), float("inf"), device=dev),
        best_index=scalar(0, dev, torch.int64),
        key=key,
        **extra,
    )


def move_n_small(a: torch.Tensor, n: IntLike):
    """Graph-safe ``move_n_small_numbers`` (reference ``differential_evolution.py:49-60``):
    a stable partition putting the ``n`` smallest entries (first in stable sort order)
    in front, keeping the original relative order on both sides.  Returns the indices."""
    N = a.shape[0]
    rank = torch.argsort(torch.argsort(a, stable=True), stable=True)  # inverse permutation, out of place
    small = rank < _t(n, a.device, torch.int64)
    key = (~small).to(torch.int64) * N + torch.arange(N, device=a.device)
    return torch.argsort(key)


def choice_p(key, p: torch.Tensor, shape) -> torch.Tensor:
    """Categorical draws with probabilities ``p`` (inverse CDF, graph-safe)."""
    c = torch.cumsum(p, 0)
    u = rnd.uniform(key, shape).to(p.device) * c[-1]
    return torch.clamp(torch.searchsorted(c, u.reshape(-1), right=True).reshape(u.shape), max=p.shape[0] - 1)


def progress_of(state, device):
    return _t(state.progress, device)
