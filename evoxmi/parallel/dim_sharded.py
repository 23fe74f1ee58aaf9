"""Decision-variable (column) sharding of the evaluation — strategy P2.

Reference: ``std_workflow.py:253-309`` (``enable_multi_devices``) shards every
``(pop, dim)`` array along the dim axis with GSPMD and lets XLA insert the
all-reduce wherever a row reduction crosses the sharded axis.  With one process
per GPU the same data flow is explicit: every rank evaluates only its balanced
column block of the (replicated) population into per-row *additive* terms, one
``all_reduce(SUM)`` of the small ``(N, k)`` term matrix crosses xGMI, and the
problem's ``combine_terms`` finishes the fitness identically on every rank.

The wrapped problem implements the protocol documented in
``evoxmi/problems/numerical/classic.py`` (``partial_terms``, ``combine_terms``,
``dim_halo``).  Traffic per evaluation is ``N·k·4`` bytes (e.g. 40 KB for
Ackley at N = 10 000 — latency-bound, so one collective per evaluation), while the
``N·d`` elementwise work is split ``world_size`` ways.
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..core import Problem, State, use_state
from .context import balanced_slices


def supports_dim_sharding(problem) -> bool:
    return all(hasattr(problem, a) for a in ("partial_terms", "combine_terms", "dim_halo"))


def dim_sharded_fitness(problem, X: torch.Tensor, group=None) -> torch.Tensor:
    """Fitness of the replicated population ``X`` with the column work split over
    the ranks of ``group`` (whole evaluation when no process group exists)."""
    if dist.is_available() and dist.is_initialized():
        rank, world = dist.get_rank(group), dist.get_world_size(group)
    else:
        rank, world = 0, 1
    d = X.shape[1]
    col0, own = balanced_slices(d, world)[rank]
    hi = min(col0 + own + problem.dim_halo, d)
    # shifted-rotated problems shard the rotated coordinates: they take the full rows
    Xb = X if getattr(problem, "dim_shard_full_rows", False) else X[:, col0:hi]
    T = problem.partial_terms(Xb, col0, d, own)
    if isinstance(T, tuple):  # (sum terms, max terms), e.g. LSMOP's Schwefel groups
        Ts, Tm = T[0].contiguous(), T[1].contiguous()
        if world > 1:
            dist.all_reduce(Ts, op=dist.ReduceOp.SUM, group=group)
            dist.all_reduce(Tm, op=dist.ReduceOp.MAX, group=group)
        return problem.combine_terms((Ts, Tm), d)
    T = T.contiguous()
    if world > 1:
        dist.all_reduce(T, op=dist.ReduceOp.SUM, group=group)
    return problem.combine_terms(T, d)


def dim_sharded_fitness_local(problem, Xloc: torch.Tensor, col0: int, d: int, group=None) -> torch.Tensor:
    """Fitness when the population itself is column-sharded (``Xloc`` = this rank's columns
    [col0, col0 + own) of every row; problems with ``dim_halo == 0`` that take column blocks)."""
    own = Xloc.shape[1]
    T = problem.partial_terms(Xloc, col0, d, own)
    if isinstance(T, tuple):
        Ts, Tm = T[0].contiguous(), T[1].contiguous()
        if dist.is_available() and dist.is_initialized():
            dist.all_reduce(Ts, op=dist.ReduceOp.SUM, group=group)
            dist.all_reduce(Tm, op=dist.ReduceOp.MAX, group=group)
        return problem.combine_terms((Ts, Tm), d)
    T = T.contiguous()
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(T, op=dist.ReduceOp.SUM, group=group)
    return problem.combine_terms(T, d)


def supports_state_sharding(algorithm, problem) -> bool:
    """Full P2 (state and evaluation column-sharded): the algorithm can slice its state into
    column blocks and the problem's terms need no halo and no full rows."""
    return (hasattr(algorithm, "dim_shard") and supports_dim_sharding(problem) and getattr(problem, "dim_halo", 1) == 0
            and not getattr(problem, "dim_shard_full_rows", False))


class DimShardedProblem(Problem):
    def __init__(self, problem: Problem, group=None):
        super().__init__()
        if not supports_dim_sharding(problem):
            raise TypeError(f"{type(problem).__name__} does not implement the dim-sharding protocol "
                            "(partial_terms / combine_terms / dim_halo)")
        self.problem = problem
        self.group = group

    def setup(self, key):
        return State()

    def evaluate(self, state, X):
        return dim_sharded_fitness(self.problem, X, self.group), state
