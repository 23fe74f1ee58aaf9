"""L-SHADE family: LSHADE, ILSHADE, JSO, LSHADE_RSP
(reference ``de_variants/lshade.py:21-256``, ``ilshade.py:21-286``, ``jso.py:21-274``,
``lshade_rsp.py:20-263``).

Shared skeleton (one class, per-variant schedule hooks):

* H-slot success-history memories, F ~ Cauchy(M_F, 0.1), CR ~ N(M_CR, 0.1);
* current-to-pbest/1/bin over a *linearly shrinking* population: the population
  array keeps its static shape N; rows ≥ ``pop_size_reduced`` are NaN-padded with
  fitness +inf and receive the current worst solution as their "trial", exactly like
  the reference (``lshade.py:190-203, 241-243``) — and, unlike a host-side resize,
  this keeps the whole generation capturable in one hipGraph;
* bound repair by midpoint with the parent;
* ``state.progress`` ∈ [0, 1] is injected by the harness (``run/run_de.py:90-94``)
  and drives the size reduction and the schedules.

Variant hooks: LSHADE adds the CR cut-off; iL-SHADE caps F by progress stages,
floors CR, averages memory updates with the old slot and pins slot H−1 to 0.9;
jSO additionally weights the p-best term by F_w ∈ {0.7, 0.8, 1.2}; LSHADE-RSP uses
rank-based selective pressure for the difference members.
"""
from __future__ import annotations

import torch

from ....parallel.dim_sharded import ColumnSeparable
from ....core import Algorithm
from ....ops import random as rnd
from . import common as C


class LSHADE(ColumnSeparable, Algorithm):
    # decision-axis state sharding (P2) for the whole family (iL-SHADE, jSO, LSHADE-RSP only
    # override hooks): trials per global column, the shrinking population's row moves and the
    # memories from the replicated fitness
    column_separable = True
    dim_fields = ("population", "trial_vectors", "archive", "worst_solution")

    memory_F_init = 0.5
    memory_CR_init = 0.5

    def __init__(self, lb, ub, pop_size=100, diff_padding_num=3, with_archive=1, pop_size_min=4):
        super().__init__()
        self.dim = lb.shape[0]
        self.lb, self.ub = lb, ub
        self.pop_size = pop_size
        self.diff_padding_num = diff_padding_num
        self.H = 5
        self.p = 0.1
        self.with_archive = with_archive
        self.pop_size_min = pop_size_min

    # ----------------------------------------------------------- variant hooks
    def _p0(self):
        return self.p

    def _adjust_F(self, F, progress):
        return F

    def _adjust_CR(self, CR, state, progress):
        return torch.where(state.CR_cutoff > 0, torch.zeros_like(CR), CR)

    def _Fw(self, progress):
        return None

    def _memory_value(self, lehmer, old_slot0):
        return lehmer

    def _pin(self, mem):
        return mem

    def _p_next(self, progress):
        return torch.full_like(progress, self.p)

    def _reduced_next(self, progress):
        t = (self.pop_size - (self.pop_size - self.pop_size_min) * progress).to(torch.int64)
        return torch.where(t < self.pop_size_min, torch.full_like(t, self.pop_size_min), t)

    def _diff_mode(self, state):
        return dict(archive=state.archive if self.with_archive else None)

    # ----------------------------------------------------------- protocol
    def setup(self, key):
        state_key, init_key = rnd.split(key)
        return self._setup_state(state_key, C.init_population(init_key, self.pop_size, self.lb, self.ub))

    def _setup_state(self, state_key, pop):
        dev = pop.device
        N = self.pop_size
        st = C.base_state(state_key, pop)
        return st.update(
            best_index=C.scalar(1, dev, torch.int64),
            trial_vectors=torch.zeros_like(pop),
            Memory_F=torch.full((self.H,), self.memory_F_init, device=dev),
            Memory_CR=torch.full((self.H,), self.memory_CR_init, device=dev),
            F_vect=torch.zeros(N, device=dev), CR_vect=torch.zeros(N, device=dev),
            archive=pop.clone(),
            CR_cutoff=C.scalar(0, dev, torch.int64),
            pop_size_reduced=C.scalar(N, dev, torch.int64),
            worst_solution=pop[0].clone(),
            progress=C.scalar(0.0, dev),
            p=C.scalar(self._p0(), dev),
        )

    def ask(self, state):
        key, k_trial, k_choice, k_f, k_cr = rnd.split(state.key, 5)
        dev = state.population.device
        N = self.pop_size
        prog = C.progress_of(state, dev)
        ids = rnd.randint(k_choice, (N,), 0, self.H).to(dev)
        F = torch.clamp(rnd.cauchy(k_f, (N,)).to(dev) * 0.1 + state.Memory_F[ids], 0, 1)
        F = self._adjust_F(F, prog)
        CR = torch.clamp(rnd.normal(k_cr, (N,)).to(dev) * 0.1 + state.Memory_CR[ids], 0, 1)
        CR = self._adjust_CR(CR, state, prog)
        cur = torch.arange(N, device=dev)
        red = state.pop_size_reduced
        c0, own, d = self.cols()
        trials, _ = C.generate_trials(k_trial, state.population, state.fitness, state.best_index, cur, C.current2pbest_1_bin, F,
                                      CR, self.diff_padding_num, self.col_vec(self.lb), self.col_vec(self.ub), p=state.p, reduced=red,
                                      Fw=self._Fw(prog), repair="midpoint", cols=(c0, d), **self._diff_mode(state))
        live = cur < red
        trials = torch.where(live[:, None], trials, state.worst_solution)
        return trials, state.update(trial_vectors=trials, key=key, F_vect=F, CR_vect=CR)

    def tell(self, state, trial_fitness):
        N = self.pop_size
        dev = trial_fitness.device
        prog = C.progress_of(state, dev)
        red = state.pop_size_reduced
        live = torch.arange(N, device=dev) < red
        tfit = torch.where(live, trial_fitness, torch.full_like(trial_fitness, float("inf")))
        pop, fit, _ = C.greedy_replace(state.population, state.fitness, state.trial_vectors, tfit, strict=False)
        best_index = torch.argmin(fit)
        # shrink: the `red` best rows move to the front (stable), the rest become padding
        mv = C.move_n_small(fit, red)
        moved_fit = torch.where(live, fit[mv], torch.full_like(fit, float("inf")))
        moved_pop = torch.where(live[:, None], pop[mv], torch.full_like(pop, float("nan")))
        worst = pop.index_select(0, torch.argmax(torch.where(torch.isnan(fit), torch.full_like(fit, -float("inf")), fit)).reshape(1))[0]
        # success-history memories
        ok = tfit < state.fitness
        nan = torch.full_like(tfit, float("nan"))
        S_CR = torch.where(ok, state.CR_vect, nan)
        S_delta = torch.where(ok, state.fitness - tfit, nan)
        cr_max = torch.where(ok, state.CR_vect, torch.full_like(tfit, -float("inf"))).max()
        CR_cutoff = torch.where(ok.any() & (cr_max <= 0), torch.ones_like(state.CR_cutoff), state.CR_cutoff)
        w = S_delta / torch.nansum(S_delta)
        M_CR = self._memory_value(torch.nansum(w * S_CR * S_CR) / torch.nansum(w * S_CR), state.Memory_CR[0])
        M_F = self._memory_value(C.lehmer_update(ok, state.F_vect, w), state.Memory_F[0])
        Memory_F = self._pin(C.roll_in(state.Memory_F, M_F))
        Memory_CR = self._pin(C.roll_in(state.Memory_CR, M_CR))
        archive = torch.where(ok[:, None], state.population, state.archive)
        return state.update(population=moved_pop, fitness=moved_fit, best_index=best_index, Memory_F=Memory_F,
                            Memory_CR=Memory_CR, archive=archive, CR_cutoff=CR_cutoff,
                            pop_size_reduced=self._reduced_next(prog), worst_solution=worst, p=self._p_next(prog))


def _stage(progress, edges, values):
    """values[k] for the first edge with progress <= edge (last value otherwise)."""
    out = torch.full_like(progress, values[-1])
    for e, v in reversed(list(zip(edges, values[:-1]))):
        out = torch.where(progress <= e, torch.full_like(progress, v), out)
    return out


class ILSHADE(LSHADE):
    memory_CR_init = 0.8

    def __init__(self, lb, ub, pop_size=100, diff_padding_num=3, with_archive=1, pop_size_min=4, p_max=0.2, p_min=0.1):
        super().__init__(lb, ub, pop_size, diff_padding_num, with_archive, pop_size_min)
        self.p_min, self.p_max = p_min, p_max

    def _p0(self):
        return self.p_min

    def _adjust_F(self, F, progress):
        return torch.minimum(F, _stage(progress, (0.25, 0.5, 0.75), (0.7, 0.8, 0.9, 1.0)))

    def _adjust_CR(self, CR, state, progress):
        return torch.maximum(CR, _stage(progress, (0.25, 0.5), (0.5, 0.25, 0.0)))

    def _memory_value(self, lehmer, old_slot0):
        return (lehmer + old_slot0) / 2

    def _pin(self, mem):
        return torch.cat([mem[: self.H - 1], torch.full_like(mem[:1], 0.9)])

    def _p_next(self, progress):
        return self.p_min + (self.p_max - self.p_min) * progress

    def _reduced_next(self, progress):
        return (self.pop_size - (self.pop_size - self.pop_size_min) * progress).to(torch.int64)


class JSO(ILSHADE):
    def _adjust_F(self, F, progress):
        return torch.where(progress < 0.6, torch.minimum(F, torch.full_like(F, 0.7)), F)

    def _adjust_CR(self, CR, state, progress):
        # jnp.select over (≤.25, (.25,.5], >.5) → (0.7, 0.6, 0.0)
        return torch.maximum(CR, _stage(progress, (0.25, 0.5), (0.7, 0.6, 0.0)))

    def _Fw(self, progress):
        return _stage(progress, (0.2, 0.4), (0.7, 0.8, 1.2))


class LSHADE_RSP(JSO):
    memory_F_init = 0.3

    def __init__(self, lb, ub, pop_size=100, diff_padding_num=3, pop_size_min=4, p_const=0.085, k_factor=3):
        super().__init__(lb, ub, pop_size, diff_padding_num, 1, pop_size_min)
        self.p_const = p_const
        self.k_factor = k_factor

    def _p0(self):
        return self.p_const

    def _p_next(self, progress):
        return self.p_const + self.p_const * progress

    def _diff_mode(self, state):
        return dict(rank_k=self.k_factor)
