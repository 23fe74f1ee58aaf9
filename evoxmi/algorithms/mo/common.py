"""Shared skeleton of the multi-objective algorithms: random initial population in
the box, ``init_ask``/``init_tell`` evaluation of it, SBX + polynomial-mutation
variation (fused HIP kernels on a GPU), NSGA-II-style environmental selection."""
from __future__ import annotations

import torch

from ...core import Algorithm, State
from ...operators import crossover, mutation
from ...parallel.dim_sharded import ColumnSeparable
from ...operators.selection.non_dominate import crowding_distance, lexsort, non_dominated_sort
from ...ops import random as rnd


class ColumnVariation(ColumnSeparable):
    """SBX + polynomial mutation on this rank's column block (decision-axis state sharding,
    the reference's GSPMD dim sharding ``std_workflow.py:253-270``): the operators draw every
    gene at its global column (``cols=``), the bounds are the block's, and the survivor
    selection only gathers rows by indices computed from the replicated fitness — so a subclass
    whose ``ask`` / ``tell`` use nothing else of the decision vectors declares
    ``column_separable = True`` and keeps only its column block of the population."""

    dim_fields = ("population", "next_generation")

    def dim_shard(self, state, col0: int, own: int):
        for op in (self.crossover, self.mutation):
            if not getattr(op, "column_blocks", False):
                raise ValueError(f"{type(op).__name__} does not draw per global column (no cols=): the state cannot be column-sharded")
        return super().dim_shard(state, col0, own)

    def _vary(self, x_key, mut_key, parents, clip=True):
        c0, own, d = self.cols()
        if own == d:
            off = self.mutation(mut_key, self.crossover(x_key, parents))
            return torch.clamp(off, self.lb, self.ub) if clip else off
        lb, ub = self.col_vec(self.lb), self.col_vec(self.ub)
        cols = (c0, d)
        off = self.mutation(mut_key, self.crossover(x_key, parents, cols=cols), cols=cols, boundary=(lb, ub))
        return torch.clamp(off, lb, ub) if clip else off


class MOAlgorithm(ColumnVariation, Algorithm):
    def __init__(self, lb, ub, n_objs, pop_size, mutation_op=None, crossover_op=None):
        super().__init__()
        self.lb, self.ub = lb, ub
        self.n_objs = n_objs
        self.dim = lb.shape[0]
        self.pop_size = pop_size
        self.mutation = mutation_op if mutation_op is not None else mutation.Polynomial((lb, ub))
        self.crossover = crossover_op if crossover_op is not None else crossover.SimulatedBinary()

    def _init_pop(self, key):
        return rnd.uniform(key, (self.pop_size, self.dim)).to(self.lb.device) * (self.ub - self.lb) + self.lb

    def setup(self, key):
        key, sub = rnd.split(key)
        pop = self._init_pop(sub)
        return State(population=pop, fitness=torch.zeros((self.pop_size, self.n_objs), device=pop.device), next_generation=pop, key=key)

    def init_ask(self, state):
        return state.population, state

    def init_tell(self, state, fitness):
        return state.update(fitness=fitness)

    def _variation(self, x_key, mut_key, parents, clip=True):
        return self._vary(x_key, mut_key, parents, clip)


def nsga2_select(fitness, n):
    """Indices of the n survivors by (rank, −crowding) (reference ``eagmoead.py:22-30``)."""
    if fitness.is_cuda and fitness.shape[0] <= 8192:
        from ...ops import nds

        return nds.nsga2_survivors(fitness, n, n - 1, until=n)
    rank = non_dominated_sort(fitness, until=n)
    worst = torch.sort(rank).values[n - 1]  # 0-d view: no host sync (capturable)
    cd = crowding_distance(fitness, rank == worst)
    return lexsort([-cd, rank.to(cd.dtype)])[:n]


def weights_and_neighbours(w, T):
    d = torch.cdist(w, w)
    return torch.argsort(d, dim=1, stable=True)[:, :T]
