"""BCE-IBEA — bi-criterion evolution with IBEA (Li, Yang & Liu 2016; reference ``algorithms/mo/bce_ibea.py:174-332``).

Two cooperating populations: the Pareto-criterion population PC (non-dominated,
niche-truncated to N) and the IBEA non-Pareto-criterion population NPC.  Generations
alternate: odd ones explore around under-populated PC members, even ones run IBEA
variation on NPC; NPC is always updated by IBEA environmental selection and PC by
the PC selection over everything evaluated.  The reference mixes up the objective
arrays between the two populations in its odd/even tells (e.g. ``fitness=npc_obj``
in ``_tell_odd``); here each population keeps its own objectives.
"""
from __future__ import annotations

import torch

from ...core import State
from ...operators import crossover, selection
from ...operators.selection.non_dominate import non_dominated_sort
from ...ops import random as rnd
from .common import MOAlgorithm
from .ibea import cal_fitness, ibea_truncate


def exploration(pc_obj, npc_obj, n_nd, n):
    f_max, f_min = pc_obj.max(0).values, pc_obj.min(0).values
    span = (f_max - f_min).clamp(min=1e-12)
    npc_n = (npc_obj - f_min) / span
    pc_n = (pc_obj - f_min) / span
    d = torch.cdist(pc_n, pc_n).masked_fill(torch.eye(pc_n.shape[0], dtype=torch.bool, device=pc_obj.device), float("inf"))
    d = torch.nan_to_num(d, nan=float("inf"))
    sd = torch.sort(d, 1).values
    r0 = sd[:, min(2, sd.shape[1] - 1)].mean()
    r = n_nd / n * r0
    return (torch.cdist(pc_n, npc_n) <= r).sum(1) <= 1


def pc_selection(pc, pc_obj, n):
    rank = non_dominated_sort(pc_obj)
    mask = rank == 0
    n_nd = int(mask.sum())
    if n_nd > n:
        f = pc_obj[mask]
        f_max, f_min = f.max(0).values, f.min(0).values
        norm = (f - f_min) / (f_max - f_min).clamp(min=1e-12)
        d = torch.cdist(norm, norm).masked_fill(torch.eye(n_nd, dtype=torch.bool, device=pc_obj.device), float("inf"))
        sd = torch.sort(d, 1).values
        r = sd[:, min(2, n_nd - 1)].sum() / n_nd
        R = torch.clamp(d / r, max=1)
        keep = torch.ones(n_nd, dtype=torch.bool, device=pc_obj.device)
        for _ in range(n_nd - n):
            score = torch.where(keep, 1 - torch.prod(R, 0), torch.full((n_nd,), -1.0, device=R.device))
            i = int(torch.argmax(score))
            keep[i] = False
            R[i, :] = 1
            R[:, i] = 1
        idx = torch.nonzero(mask).flatten()[keep]
    else:
        idx = torch.nonzero(mask).flatten()
        idx = torch.cat([idx, idx[:1].expand(n - idx.shape[0])])  # pad with the first member
    return pc[idx], pc_obj[idx], n_nd


def ibea_selection(pop, obj, n, kappa):
    f, I, C = cal_fitness(obj, kappa)
    keep = ibea_truncate(f, I, C, kappa, obj.shape[0] - n)
    idx = torch.argsort((~keep).to(torch.int64), stable=True)[:n]
    return pop[idx], obj[idx]


class BCEIBEA(MOAlgorithm):
    def __init__(self, lb, ub, n_objs, pop_size, kappa=0.05, selection_op=None, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.kappa = kappa
        self.selection = selection.Tournament(n_round=pop_size)
        self.crossover_odd = crossover.SimulatedBinary(type=2)

    def setup(self, key):
        st = super().setup(key)
        z = torch.zeros((self.pop_size, self.n_objs), device=st.population.device)
        return st.update(npc=st.population.clone(), npc_obj=z, n_nd=0, counter=1)

    def init_tell(self, state, fitness):
        pc, pc_obj, n_nd = pc_selection(state.population, fitness, self.pop_size)
        return state.update(population=pc, fitness=pc_obj, npc=state.population, npc_obj=fitness, n_nd=n_nd)

    def ask(self, state):
        key, k1, x_key, mut_key = rnd.split(state.key, 4)
        N = self.pop_size
        if state.counter % 2 == 0:  # IBEA variation on NPC
            fit = -cal_fitness(state.npc_obj, self.kappa)[0]
            selected, _ = self.selection(k1, state.npc, fit)
            off = self.mutation(mut_key, self.crossover(x_key, selected))
        else:  # PC exploration
            s = exploration(state.fitness, state.npc_obj, state.n_nd, N)
            if bool(s.any()):
                cand = torch.nonzero(s).flatten()
                mate = rnd.randint(k1, (N,), 0, N).to(cand.device)
                first = cand[torch.arange(N, device=cand.device) % cand.shape[0]]
                parents = torch.cat([state.population[first], state.population[mate]])
                off = self.mutation(mut_key, self.crossover_odd(x_key, parents))
            else:
                off = state.population.clone()
        off = torch.clamp(off, self.lb, self.ub)
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        N = self.pop_size
        npc, npc_obj = ibea_selection(torch.cat([state.npc, state.next_generation]), torch.cat([state.npc_obj, fitness]), N, self.kappa)
        pc, pc_obj, n_nd = pc_selection(torch.cat([state.population, state.next_generation]), torch.cat([state.fitness, fitness]), N)
        return state.update(population=pc, fitness=pc_obj, npc=npc, npc_obj=npc_obj, n_nd=n_nd, counter=state.counter + 1)
