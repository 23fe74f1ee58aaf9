"""EVDE — ensemble of DE variants (Wu et al. 2018; reference ``de_variants/evde.py:30-398``).

The population is split into indicator sub-populations for JaDE (λ1), CoDE (λ2,
expanded ×3 trials) and EPSDE (λ3) plus a reward sub-population (λ4) that runs the
currently best variant (JaDE-style or EPSDE-style parameters).  Every ``ng``
generations the variant with the largest accumulated best-fitness improvement per
trial wins the reward sub-population.  One fused kernel generates all
λ1 + 3λ2 + λ3 + λ4 trials (per-row strategy code, F and CR).

Deliberate differences from the reference (its indexing mixes up sub-populations):
* every trial targets the row of its own sub-population — the reference indexes
  ``population[arange(pop_size_expanded)]`` (clamped past N), so CoDE's second and
  third trial blocks and the EPSDE/reward rows use other individuals as "current";
* EPSDE / reward success flags compare against their own rows;
* ``iter`` advances inside ``tell`` (the reference relies on the harness to inject it);
* the EPSDE parameter vectors in use are persisted in the state (the reference never
  stores them back, so successful rows fall back to their initial vectors).
"""
from __future__ import annotations

import torch

from ....core import Algorithm
from ....ops import random as rnd
from . import common as C
from .epsde import random_params

CODE_POOL = torch.tensor([[1, 0.1], [1, 0.9], [0.8, 0.2]], dtype=torch.float32)
CODE_STRATEGIES = torch.tensor([C.rand_1_bin, C.rand_2_bin, C.current2rand_1], dtype=torch.float32)
JADE_STRATEGY = torch.tensor(C.current2pbest_1_bin, dtype=torch.float32)


class EVDE(Algorithm):
    def __init__(self, lb, ub, pop_size=100, diff_padding_num=5, differential_weight=None, cross_probability=None, p=0.05,
                 c=0.1, ng=20, lambda_1=0.1, lambda_2=0.1, lambda_3=0.1, lambda_4=0.7):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub = lb, ub
        self.pop_size = pop_size
        self.diff_padding_num = diff_padding_num
        self.p, self.c, self.ng = p, c, ng
        self.n1 = round(lambda_1 * pop_size)
        self.n2 = round(lambda_2 * pop_size)
        self.n3 = round(lambda_3 * pop_size)
        self.n4 = pop_size - self.n1 - self.n2 - self.n3
        self.n_expanded = self.n1 + 3 * self.n2 + self.n3 + self.n4

    def setup(self, key):
        state_key, init_key, k1, k2, k3, k4, k5, k6 = rnd.split(key, 8)
        pop = C.init_population(init_key, self.pop_size, self.lb, self.ub)
        dev = pop.device
        e = random_params(k1, k2, k3, self.n3, dev)
        r = random_params(k4, k5, k6, self.n4, dev)
        z = lambda: C.scalar(0.0, dev)
        return C.base_state(
            state_key, pop, trial_vectors=torch.zeros((self.n_expanded, self.dim), device=dev),
            param_vect_expanded=torch.zeros((self.n_expanded, 6), device=dev),
            F_u=C.scalar(0.5, dev), CR_u=C.scalar(0.5, dev),
            EPSDE_param_vect=e, EPSDE_S_param_vect=e.clone(), EPSDE_compare=torch.ones(self.n3, dtype=torch.bool, device=dev),
            reward_EPSDE_param_vect=r, reward_EPSDE_S_param_vect=r.clone(),
            reward_EPSDE_compare=torch.ones(self.n4, dtype=torch.bool, device=dev),
            iter=C.scalar(0, dev, torch.int64), JaDE_delta_sum=z(), CoDE_delta_sum=z(), EPSDE_delta_sum=z(),
            best_alg_ng=z(), reward_alg_id=C.scalar(0, dev, torch.int64),
        )

    def _jade_params(self, kf, kc, n, state, dev):
        F = torch.clamp(rnd.cauchy(kf, (n,)).to(dev) * 0.1 + state.F_u, 0, 1)
        CR = torch.clamp(rnd.normal(kc, (n,)).to(dev) * 0.1 + state.CR_u, 0, 1)
        return torch.cat([C.dconst(JADE_STRATEGY, dev).expand(n, 4), F[:, None], CR[:, None]], 1)

    def _epsde_params(self, keys, n, S, prev, compare, dev):
        ks, kf, kc, kr = keys
        rand_pv = random_params(ks, kf, kc, n, dev)
        renew = rnd.randint(kr, (n,), 0, 2).to(dev).bool()
        return torch.where(compare[:, None], prev, torch.where(renew[:, None], S, rand_pv))

    def _targets(self, dev):
        n1, n2, n3, n4 = self.n1, self.n2, self.n3, self.n4
        a = torch.arange(self.pop_size, device=dev)
        return torch.cat([a[:n1], a[n1:n1 + n2].repeat(3), a[n1 + n2:]])

    def ask(self, state):
        key, k_trial, k_code, *ks = rnd.split(state.key, 15)
        dev = state.population.device
        n1, n2, n3, n4 = self.n1, self.n2, self.n3, self.n4
        jade = self._jade_params(ks[0], ks[1], n1, state, dev)
        fcr = C.dconst(CODE_POOL, dev)[rnd.randint(k_code, (3 * n2,), 0, 3).to(dev)]
        code = torch.cat([C.dconst(CODE_STRATEGIES, dev).repeat_interleave(n2, 0), fcr], 1)
        eps = self._epsde_params(ks[2:6], n3, state.EPSDE_S_param_vect, state.EPSDE_param_vect, state.EPSDE_compare, dev)
        rj = self._jade_params(ks[6], ks[7], n4, state, dev)
        re = self._epsde_params(ks[8:12], n4, state.reward_EPSDE_S_param_vect, state.reward_EPSDE_param_vect,
                                state.reward_EPSDE_compare, dev)
        reward = torch.where(state.reward_alg_id == 0, rj, re)
        pv = torch.cat([jade, code, eps, reward], 0)
        strat = pv[:, :4].to(torch.int64)
        trials, _ = C.generate_trials(k_trial, state.population, state.fitness, state.best_index, self._targets(dev), strat,
                                      pv[:, 4], pv[:, 5], self.diff_padding_num, self.lb, self.ub, p=self.p)
        return trials, state.update(trial_vectors=trials, key=key, param_vect_expanded=pv,
                                    EPSDE_param_vect=eps, reward_EPSDE_param_vect=torch.where(state.reward_alg_id == 0, state.reward_EPSDE_param_vect, re))

    def tell(self, state, trial_fitness):
        n1, n2, n3, n4 = self.n1, self.n2, self.n3, self.n4
        dev = trial_fitness.device
        o2, o3 = n1, n1 + 3 * n2
        code_f = trial_fitness[o2:o3].reshape(3, n2)
        pick = torch.argmin(code_f, 0) * n2 + torch.arange(n2, device=dev) + o2
        sel = torch.cat([torch.arange(n1, device=dev), pick, torch.arange(o3, self.n_expanded, device=dev)])
        tf, tv = trial_fitness[sel], state.trial_vectors[sel]
        pop, fit, ok = C.greedy_replace(state.population, state.fitness, tv, tf, strict=False)
        strict_ok = tf < state.fitness
        pv = state.param_vect_expanded
        # JaDE adaptation on the λ1 rows
        jok = strict_ok[:n1]
        Fl = C.lehmer_update(jok, pv[:n1, 4])
        CRm = torch.nanmean(torch.where(jok, pv[:n1, 5], torch.full_like(pv[:n1, 5], float("nan"))))
        anyj = jok.any()
        F_u = torch.where(anyj, (1 - self.c) * state.F_u + self.c * Fl, state.F_u)
        CR_u = torch.where(anyj, (1 - self.c) * state.CR_u + self.c * CRm, state.CR_u)
        # EPSDE memories
        s3, s4 = n1 + n2, n1 + n2 + n3
        eok = strict_ok[s3:s4]
        E_S = torch.where(eok[:, None], pv[o3:o3 + n3], state.EPSDE_S_param_vect)
        rok = strict_ok[s4:]
        R_S = torch.where(rok[:, None], pv[o3 + n3:], state.reward_EPSDE_S_param_vect)
        # reward assignment by accumulated best-fitness improvement per trial
        def delta(a, b):
            return state.fitness[a:b].min() - fit[a:b].min()
        J = state.JaDE_delta_sum + delta(0, n1)
        Co = state.CoDE_delta_sum + delta(n1, n1 + n2)
        Ep = state.EPSDE_delta_sum + delta(s3, s4)
        check = (state.iter % self.ng) == 0
        best = torch.argmax(torch.stack([J / n1, Co / (3 * n2), Ep / n3]))
        reward_alg_id = torch.where(check, torch.where(best == 0, 0, 2), state.reward_alg_id)
        zero = torch.zeros_like(J)
        return state.update(
            population=pop, fitness=fit, best_index=torch.argmin(fit), F_u=F_u, CR_u=CR_u,
            EPSDE_S_param_vect=E_S, EPSDE_compare=eok, reward_EPSDE_S_param_vect=R_S, reward_EPSDE_compare=rok,
            JaDE_delta_sum=torch.where(check, zero, J), CoDE_delta_sum=torch.where(check, zero, Co),
            EPSDE_delta_sum=torch.where(check, zero, Ep),
            best_alg_ng=torch.where(check, best.to(J.dtype), torch.full_like(J, float("nan"))),
            reward_alg_id=reward_alg_id, iter=state.iter + 1,
        )
