"""KnEA — knee-point-driven EA (Zhang, Tian & Jin 2015; reference ``algorithms/mo/knea.py:39-221``).

Mating: binary tournament by (front rank, knee flag, weighted distance DW).
Environmental selection: non-dominated fronts up to the critical one; in every front
the knee points are found by scanning the members in order of their distance to the
extreme hyperplane and suppressing neighbours within the adaptive radius R (a
sequential scan, on the host); the last front is completed / trimmed by hyperplane
distance.
"""
from __future__ import annotations

import torch

from ...core import State
from ...operators.selection.misc import tournament_multi_fit
from ...operators.selection.non_dominate import non_dominated_sort
from ...ops import random as rnd
from .common import MOAlgorithm


def calc_DW(fit, k):
    dis = torch.cdist(fit, fit)
    nb = torch.sort(dis, 1).values[:, 1 : k + 1]
    avg = nb.mean(1, keepdim=True)
    r = 1 / torch.abs(nb - avg).clamp(min=1e-12)
    w = r / r.sum(1, keepdim=True)
    return (nb * w).sum(1)


def _plane(points, m):
    sol, info = torch.linalg.solve_ex(points, torch.ones(m, 1, device=points.device))
    if int(info) == 0 and bool(torch.isfinite(sol).all()):
        return sol[:, 0]
    return 1.0 / torch.clamp(torch.diagonal(points), min=1e-6)


class KnEA(MOAlgorithm):
    def __init__(self, lb, ub, n_objs, pop_size, knee_rate=0.5, k_neighbors=3, mutation_op=None, crossover_op=None):
        super().__init__(lb, ub, n_objs, pop_size, mutation_op, crossover_op)
        self.knee_rate, self.k_neighbors = knee_rate, k_neighbors

    def setup(self, key):
        st = super().setup(key)
        return st.update(knee=torch.zeros(self.pop_size, dtype=torch.bool, device=st.population.device), r=1.0, t=0.0)

    def ask(self, state):
        k0, k1, k2, k3 = rnd.split(state.key, 4)
        rank = non_dominated_sort(state.fitness).to(torch.float32)
        DW = calc_DW(state.fitness, self.k_neighbors)
        keys = torch.stack([rank, (~state.knee).to(torch.float32), -DW], 1)
        selected, _ = tournament_multi_fit(k1, state.population, keys, self.pop_size)
        off = self._variation(k2, k3, selected)
        return off, state.update(next_generation=off, key=k0)

    def tell(self, state, fitness):
        N, m = self.pop_size, self.n_objs
        pop = torch.cat([state.population, state.next_generation])
        obj = torch.cat([state.fitness, fitness])
        rank = non_dominated_sort(obj)
        order = torch.argsort(rank, stable=True)
        rank, pop, obj = rank[order], pop[order], obj[order]
        last = int(rank[N])
        n = obj.shape[0]
        knee = torch.zeros(n, dtype=torch.bool, device=obj.device)
        r, t = float(state.r), float(state.t)
        plane = torch.ones(m, device=obj.device)
        for i in range(last + 1):
            idx = torch.nonzero(rank == i).flatten()
            f = obj[idx]
            mx, mn = f.max(0).values, f.min(0).values
            plane = _plane(f[torch.argmax(f, 0)], m)
            dist_order = idx[torch.argsort(f @ plane, stable=True)]
            r = r * float(torch.exp(torch.tensor(-(1 - t / self.knee_rate) / m)))
            R = (mx - mn) * r
            cand = torch.ones(n, dtype=torch.bool, device=obj.device)
            cand[idx] = True
            front_knee = torch.zeros(n, dtype=torch.bool, device=obj.device)
            front_knee[idx] = True
            for p in dist_order.tolist():
                if bool(front_knee[p]):
                    nb = (torch.abs(obj[idx] - obj[p]) < R).all(1)
                    nb_idx = idx[nb]
                    front_knee[nb_idx] = False
                    front_knee[p] = True
            knee |= front_knee
            t = float((front_knee[idx]).sum()) / idx.shape[0]
        knee &= rank <= last
        selected = (rank < last) | knee
        dif = int(selected.sum()) - N
        last_mask = rank == last
        if dif > 0:
            cand = torch.nonzero(knee & last_mask).flatten()
            far = cand[torch.argsort(-(obj[cand] @ plane), stable=True)][:dif]
            selected[far] = False
        elif dif < 0:
            cand = torch.nonzero(~knee & last_mask).flatten()
            near = cand[torch.argsort(obj[cand] @ plane, stable=True)][:-dif]
            selected[near] = True
        idx = torch.nonzero(selected).flatten()[:N]
        return state.update(population=pop[idx], fitness=obj[idx], knee=knee[idx], r=r, t=t)
