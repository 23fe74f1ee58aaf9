"""NSGA-II (reference ``algorithms/mo/nsga2.py:22-100``).

``ask``: SBX (type 1) + polynomial mutation over the whole population, clipped
(the reference's mating selection is commented out, ``nsga2.py:78``).
``tell``: merge parents and offspring (2N), non-dominated sort, crowding distance
on the worst kept front, lexsort by (rank, −crowding) and keep N.  On a GPU the
sort is the bit-matrix HIP kernel and SBX/PM are fused elementwise kernels.
"""
from __future__ import annotations

import torch

from ...core import Algorithm, State
from ...operators import crossover, mutation, selection
from .common import ColumnVariation
from ...operators.selection.non_dominate import crowding_distance, lexsort, non_dominated_sort
from ...ops import random as rnd


class NSGA2(ColumnVariation, Algorithm):
    # SBX / PM per global column and row selection from the replicated fitness: the state can
    # be column-sharded (StdWorkflow.enable_multi_devices(shard_state=True))
    column_separable = True

    def __init__(self, lb, ub, n_objs, pop_size, selection_op=None, mutation_op=None, crossover_op=None):
        super().__init__()
        self.lb, self.ub = lb, ub
        self.n_objs = n_objs
        self.dim = lb.shape[0]
        self.pop_size = pop_size
        self.selection = selection_op if selection_op is not None else selection.UniformRand(1)
        self.mutation = mutation_op if mutation_op is not None else mutation.Polynomial((lb, ub))
        self.crossover = crossover_op if crossover_op is not None else crossover.SimulatedBinary()

    def setup(self, key):
        key, sub = rnd.split(key)
        dev = self.lb.device
        pop = rnd.uniform(sub, (self.pop_size, self.dim)).to(dev) * (self.ub - self.lb) + self.lb
        return State(population=pop, fitness=torch.zeros((self.pop_size, self.n_objs), device=dev), next_generation=pop, key=key)

    def init_ask(self, state):
        return state.population, state

    def init_tell(self, state, fitness):
        return state.update(fitness=fitness)

    def ask(self, state):
        key, _sel, x_key, mut_key = rnd.split(state.key, 4)
        off = self._vary(x_key, mut_key, state.population)
        return off, state.update(next_generation=off, key=key)

    def tell(self, state, fitness):
        merged_pop = torch.cat([state.population, state.next_generation], 0)
        merged_fit = torch.cat([state.fitness, fitness], 0)
        if merged_fit.is_cuda and merged_fit.shape[0] <= 8192:
            # fused selection kernel: same ranks/crowding/lexsort semantics as below
            from ...ops import nds

            keep = nds.nsga2_survivors(merged_fit, self.pop_size, self.pop_size, until=self.pop_size + 1)
            return state.update(population=merged_pop[keep], fitness=merged_fit[keep])
        rank = non_dominated_sort(merged_fit, until=self.pop_size + 1)
        # the (pop_size)-th smallest rank, read as a 0-d view (no host sync: graph-capturable)
        worst = torch.sort(rank).values[self.pop_size]
        mask = rank == worst
        cd = crowding_distance(merged_fit, mask)
        keep = lexsort([-cd, rank.to(cd.dtype)])[: self.pop_size]
        return state.update(population=merged_pop[keep], fitness=merged_fit[keep])
