"""Cooperative co-evolution containers (reference ``containers/coevolution.py:15-257``).

The decision vector is split into ``num_subpops`` equal blocks (optionally under a
fixed random permutation); sub-algorithm k optimises block k, and its candidates are
evaluated inside the current best full solution (the "context vector").

* ``VectorizedCoevolution`` advances every sub-population each generation
  (num_subpops × subpop_size evaluations);
* ``Coevolution`` advances one sub-population per generation, round-robin.

The sub-algorithms' states are stacked (``StackedModules``) and addressed with
``use_state(fn, index=k)``; the reference's ``vmap`` over them becomes a loop over
k (few, device-resident sub-generations — our algorithms run fused HIP kernels that
are not vmappable).
"""
from __future__ import annotations

import torch

from ...core import Algorithm, State, StackedModules, use_state
from ...ops import random as rnd


def _as_stack(algos):
    return algos if isinstance(algos, StackedModules) else StackedModules(list(algos))


class _CoevolutionBase(Algorithm):
    def __init__(self, base_algorithms, dim, num_subpops, random_subpop=False, dtype=torch.float32):
        super().__init__()
        self.base_algorithms = _as_stack(base_algorithms)
        assert len(self.base_algorithms) == num_subpops and dim % num_subpops == 0
        self.dim, self.num_subpops, self.random_subpop, self.dtype = dim, num_subpops, random_subpop, dtype
        self.sub_dim = dim // num_subpops

    def setup(self, key):
        perm = rnd.permutation(rnd.split(key)[1], self.dim) if self.random_subpop else None
        dev = key.device
        return State(coop_pops=None, best_dec=torch.zeros(self.dim, dtype=self.dtype, device=dev),
                     best_fit=torch.full((self.num_subpops,), float("inf"), device=dev), permutation=perm)

    def _scatter_perm(self, pop, state):
        if not self.random_subpop:
            return pop
        out = torch.empty_like(pop)
        out[:, state.permutation.to(pop.device)] = pop
        return out

    def _gather_perm(self, x, state):
        return x[..., state.permutation.to(x.device)] if self.random_subpop else x

    def _each(self, method, state, *args):
        outs = []
        for k, alg in enumerate(self.base_algorithms):
            res = use_state(getattr(alg, method), k)(state, *[a[k] if isinstance(a, list) else a for a in args])
            if isinstance(res, tuple):
                outs.append(res[0])
                state = res[-1]
            else:
                state = res
        return outs, state

    def init_ask(self, state):
        subs, state = self._each("init_ask", state)
        init = torch.stack(subs).transpose(0, 1).reshape(-1, self.dim)  # member i = concat of the k-th subpops' row i
        init = self._scatter_perm(init, state)
        return init, state.update(coop_pops=init)

    def ask(self, state):
        subs, state = self._each("ask", state)
        K = self.num_subpops
        P = subs[0].shape[0]
        best = state.best_dec.to(subs[0].device)
        coop = best.expand(K, P, self.dim).clone()
        for k in range(K):
            coop[k, :, k * self.sub_dim : (k + 1) * self.sub_dim] = subs[k]
        coop = self._scatter_perm(coop.reshape(K * P, self.dim), state)
        return coop, state.update(coop_pops=coop)

    def init_tell(self, state, fitness):
        _, state = self._each("init_tell", state, fitness)
        i = torch.argmin(fitness)
        best_dec = self._gather_perm(state.coop_pops[i], state)
        return state.update(best_fit=fitness.min().expand(self.num_subpops).clone(), best_dec=best_dec, coop_pops=None)

    def tell(self, state, fitness):
        K = self.num_subpops
        fit = fitness.reshape(K, -1)
        _, state = self._each("tell", state, [fit[k] for k in range(K)])
        mins, arg = fit.min(1)
        coop = state.coop_pops.reshape(K, fit.shape[1], self.dim)
        best_this = self._gather_perm(coop[torch.arange(K, device=coop.device), arg], state)  # (K, dim)
        blocks = best_this.reshape(K, K, self.sub_dim)[torch.arange(K), torch.arange(K)]  # block k of subpop k's best
        old = state.best_dec.to(blocks.device).reshape(K, self.sub_dim)
        bf = state.best_fit.to(mins.device)
        best_dec = torch.where((bf > mins)[:, None], blocks, old).reshape(self.dim)
        return state.update(best_dec=best_dec, best_fit=torch.minimum(bf, mins), coop_pops=None)


class VectorizedCoevolution(_CoevolutionBase):
    """Every sub-population advances each generation.  Multi-GPU (the
    reference's vmap over sub-algorithms mapped onto devices): under
    ``StdWorkflow.enable_distributed`` rank r owns sub-populations
    [r·K/W, (r+1)·K/W) — it runs only their ask/tell and evaluates only their cooperative
    rows; the objectives are all-gathered by the workflow and the K best blocks by one
    all-gather of K × dim/K floats, so the context vector stays replicated.  Sub-states of
    the other ranks' sub-populations are not advanced locally (rank-owned state)."""

    pop_size = None  # rows per generation depend on the sub-algorithms (CSO asks P/2): dynamic all-gather

    def _owned(self, dist):
        K, W = self.num_subpops, dist.world_size
        if K % W:
            raise ValueError(f"VectorizedCoevolution on {W} ranks needs num_subpops divisible by the world size (got {K})")
        per = K // W
        return list(range(dist.rank * per, (dist.rank + 1) * per))

    def init_ask_sharded(self, state, dist):
        # every rank initialises every sub-algorithm (replicated, as the states are at this
        # point); each owned sub-population scores the shared initial rows, so the global
        # batch keeps the K·P shape of the later generations
        init, state = self.init_ask(state)
        local = init.repeat(len(self._owned(dist)), 1)
        return local, state.update(coop_pops=init)

    def init_tell_sharded(self, state, fitness, dist):
        P = fitness.shape[0] // self.num_subpops
        return self.init_tell(state, fitness[:P])  # the K copies are identical

    def ask_sharded(self, state, dist):
        ks = self._owned(dist)
        subs = []
        for k in ks:
            sub, state = use_state(self.base_algorithms[k].ask, k)(state)
            subs.append(sub)
        P = subs[0].shape[0]
        coop = state.best_dec.to(subs[0].device).expand(len(ks), P, self.dim).clone()
        for i, k in enumerate(ks):
            coop[i, :, k * self.sub_dim : (k + 1) * self.sub_dim] = subs[i]
        coop = self._scatter_perm(coop.reshape(len(ks) * P, self.dim), state)
        return coop, state.update(coop_pops=coop)

    def tell_sharded(self, state, fitness, dist):
        K = self.num_subpops
        ks = self._owned(dist)
        fit = fitness.reshape(K, -1)  # ranks own equal numbers of equal-size sub-populations
        for k in ks:
            state = use_state(self.base_algorithms[k].tell, k)(state, fit[k])
        mins, arg = fit.min(1)
        P = fit.shape[1]
        loc = torch.arange(len(ks), device=fit.device)
        kt = torch.tensor(ks, device=fit.device)
        coop = state.coop_pops.reshape(len(ks), P, self.dim)
        best_loc = self._gather_perm(coop[loc, arg[kt]], state)  # (|ks|, dim)
        blocks = best_loc.reshape(len(ks), K, self.sub_dim)[loc, kt]  # block k of owned sub-population k's best
        blocks = dist.all_gather_rows(blocks.contiguous(), K)  # (K, sub_dim), sub-population order
        old = state.best_dec.to(blocks.device).reshape(K, self.sub_dim)
        bf = state.best_fit.to(mins.device)
        best_dec = torch.where((bf > mins)[:, None], blocks, old).reshape(self.dim)
        return state.update(best_dec=best_dec, best_fit=torch.minimum(bf, mins), coop_pops=None)


class Coevolution(_CoevolutionBase):
    def setup(self, key):
        return super().setup(key).update(iter_counter=0)

    def ask(self, state):
        k = state.iter_counter % self.num_subpops
        sub, state = use_state(self.base_algorithms[k].ask, k)(state)
        coop = state.best_dec.to(sub.device).expand(sub.shape[0], self.dim).clone()
        coop[:, k * self.sub_dim : (k + 1) * self.sub_dim] = sub
        coop = self._scatter_perm(coop, state)
        return coop, state.update(coop_pops=coop)

    def tell(self, state, fitness):
        k = state.iter_counter % self.num_subpops
        state = use_state(self.base_algorithms[k].tell, k)(state, fitness)
        m = fitness.min()
        best_this = self._gather_perm(state.coop_pops[torch.argmin(fitness)], state)
        bf = state.best_fit.to(fitness.device)
        better = bf[k] > m
        best_dec = torch.where(better, best_this, state.best_dec.to(best_this.device))
        bf = bf.clone()
        bf[k] = torch.minimum(bf[k], m)
        return state.update(best_dec=best_dec, best_fit=bf, iter_counter=state.iter_counter + 1, coop_pops=None)
