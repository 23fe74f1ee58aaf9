"""SaDE — strategy-adaptive DE (reference ``de_variants/sade.py:44-276``).

Four strategies {rand/1/bin, rand-to-best/2/bin, rand/2/bin, current-to-rand/1}
are drawn with probabilities learned over a learning period LP from success /
failure memories; CR per strategy ~ N(CRm_k, 0.1) with CRm_k the median of the
remembered successful CRs.  The reference fills the success/failure counts and the
CR memory with sequential ``fori_loop``s over the population (``:16-40, 251-266``);
here they are exact parallel equivalents: counts are ``bincount``s, and the CR
memory column of strategy k becomes [successful CRs of k in reverse index order,
then the old column], truncated to LP — the same result the scan produces.
"""
from __future__ import annotations

import torch

from ....core import Algorithm
from ....ops import random as rnd
from . import common as C


class SaDE(Algorithm):
    def __init__(self, lb, ub, pop_size=100, diff_padding_num=9, LP=50):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub = lb, ub
        self.pop_size = pop_size
        self.batch_size = pop_size
        self.diff_padding_num = diff_padding_num
        self.LP = LP
        self.strategy_pool = torch.tensor([C.rand_1_bin, C.rand2best_2_bin, C.rand_2_bin, C.current2rand_1])

    def setup(self, key):
        state_key, init_key = rnd.split(key)
        pop = C.init_population(init_key, self.pop_size, self.lb, self.ub)
        dev = pop.device
        N = self.pop_size
        return C.base_state(
            state_key, pop,
            trial_vectors=torch.empty((N, self.dim), device=dev),
            success_memory=torch.zeros((self.LP, 4), dtype=torch.int64, device=dev),
            failure_memory=torch.zeros((self.LP, 4), dtype=torch.int64, device=dev),
            CR_memory=torch.full((self.LP, 4), float("nan"), device=dev),
            CRs=torch.zeros(N, device=dev),
            strategy_ids=torch.zeros(N, dtype=torch.int64, device=dev),
            iter=C.scalar(0, dev, torch.int64),
        )

    def ask(self, state):
        key, k_trial, k_strat, k_cr, k_cr2, k_f = rnd.split(state.key, 6)
        dev = state.population.device
        N = self.pop_size
        s_sum = state.success_memory.sum(0).to(torch.float32)
        f_sum = state.failure_memory.sum(0).to(torch.float32)
        S = s_sum / (s_sum + f_sum) + 0.01
        p = torch.where(state.iter >= self.LP, S / S.sum(), torch.full((4,), 0.25, device=dev))
        CRM = torch.where(state.iter > self.LP, torch.median(state.CR_memory, 0).values, torch.full((4,), 0.5, device=dev))
        sid = C.choice_p(k_strat, p, (N,))
        CRv = rnd.normal(k_cr, (N, 4)).to(dev) * 0.1 + CRM
        CRr = rnd.normal(k_cr2, (N, 4)).to(dev) * 0.1 + CRM
        CRv = torch.where((CRv < 0) | (CRv > 1), CRr, CRv)
        CR = CRv.gather(1, sid[:, None])[:, 0]
        F = rnd.normal(k_f, (N,)).to(dev) * 0.3 + 0.5
        strat = C.dconst(self.strategy_pool, dev, torch.int64)[sid]
        cur = torch.arange(N, device=dev)
        trials, _ = C.generate_trials(k_trial, state.population, state.fitness, state.best_index, cur, strat, F, CR,
                                      self.diff_padding_num, self.lb, self.ub)
        return trials, state.update(trial_vectors=trials, key=key, CRs=CR, strategy_ids=sid, iter=state.iter + 1)

    def tell(self, state, trial_fitness):
        pop, fit, ok = C.greedy_replace(state.population, state.fitness, state.trial_vectors, trial_fitness, strict=False)
        sid = state.strategy_ids
        succ = torch.zeros(4, dtype=torch.int64, device=sid.device).scatter_add(0, sid, ok.to(torch.int64))
        fail = torch.zeros(4, dtype=torch.int64, device=sid.device).scatter_add(0, sid, (~ok).to(torch.int64))
        sm = torch.cat([succ[None], state.success_memory[:-1]], 0)
        fm = torch.cat([fail[None], state.failure_memory[:-1]], 0)
        return state.update(population=pop, fitness=fit, best_index=torch.argmin(fit), success_memory=sm, failure_memory=fm,
                            CR_memory=_cr_memory_update(state.CR_memory, sid, ok, state.CRs))


def _cr_memory_update(mem, sid, ok, CRs):
    """Parallel form of the sequential per-success roll-in (reference ``sade.py:26-40``)."""
    LP, S = mem.shape
    N = sid.shape[0]
    dev = mem.device
    onehot = (sid[:, None] == torch.arange(S, device=dev)[None, :]) & ok[:, None]  # (N, S)
    cnt = onehot.sum(0)  # successes per strategy
    # position of each success within its strategy, counted from the last one (0 = most recent)
    order_from_end = torch.flip(torch.cumsum(torch.flip(onehot.to(torch.int64), [0]), 0), [0]) - 1  # (N, S)
    new = torch.full((LP, S), float("nan"), device=dev)
    r = torch.arange(LP, device=dev)[:, None]
    # rows r < cnt come from the successes; rows r ≥ cnt from the old column shifted by cnt
    src_old = (r - cnt[None, :]).clamp(min=0)
    shifted = mem.gather(0, src_old.clamp(max=LP - 1))
    new = torch.where(r >= cnt[None, :], shifted, new)
    pos = torch.where(onehot, order_from_end, torch.full_like(order_from_end, LP))  # (N, S)
    valid = pos < LP
    rows = torch.where(valid, pos, torch.zeros_like(pos))
    vals = CRs[:, None].expand(N, S)
    cols = torch.arange(S, device=dev)[None, :].expand(N, S)
    flat = torch.where(valid, rows * S + cols, torch.full_like(rows, LP * S)).reshape(-1)
    buf = torch.cat([new.reshape(-1), new.new_zeros(1)])
    buf = buf.scatter(0, flat, vals.reshape(-1))  # invalid entries land in the discarded slot LP·S
    return buf[: LP * S].reshape(LP, S)
