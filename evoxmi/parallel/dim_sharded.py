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
    """The problem returns per-rank partial terms (``partial_terms`` / ``combine_terms`` /
    ``dim_halo``).  Problems without them are still evaluated under decision-axis sharding,
    by the generic column all-gather (:func:`dim_sharded_fitness_local`)."""
    return all(hasattr(problem, a) for a in ("partial_terms", "combine_terms", "dim_halo"))


def _world(group):
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


def _gather_cols(block: torch.Tensor, d: int, group) -> torch.Tensor:
    """All-gather per-rank column blocks (balanced slices of ``d``; trailing dims on the
    last axis) into the full (…, d) matrix on every rank."""
    rank, world = _world(group)
    if world == 1:
        return block
    sl = balanced_slices(d, world)
    w = max(o for _, o in sl)
    pad = block.new_zeros(*block.shape[:-1], w)
    pad[..., : block.shape[-1]] = block
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad.contiguous(), group=group)
    return torch.cat([p[..., :o] for p, (_, o) in zip(parts, sl)], -1)


def _reduce_terms(T, d: int, group):
    """The collective of one partial-terms result.  ``T`` is a tensor (SUM-reduced), a
    ``(sum, max)`` tuple, or a dict with any of ``"sum"`` / ``"max"`` (reduced) and ``"cat"``
    (a (…, own) block or a list of them, all-gathered along the decision axis — for
    functions whose value needs every coordinate of a sharded intermediate, e.g. the rotated
    z of the CEC'22 hybrids; GSPMD inserts the same all-gather)."""
    _, world = _world(group)
    if isinstance(T, dict):
        out = {}
        for k, op in (("sum", dist.ReduceOp.SUM), ("max", dist.ReduceOp.MAX)):
            if k in T:
                v = T[k].contiguous()
                if world > 1:
                    dist.all_reduce(v, op=op, group=group)
                out[k] = v
        if "cat" in T:
            c = T["cat"]
            out["cat"] = [_gather_cols(x, d, group) for x in c] if isinstance(c, (list, tuple)) else _gather_cols(c, d, group)
        return out
    if isinstance(T, tuple):  # (sum terms, max terms), e.g. LSMOP's Schwefel groups
        Ts, Tm = T[0].contiguous(), T[1].contiguous()
        if world > 1:
            dist.all_reduce(Ts, op=dist.ReduceOp.SUM, group=group)
            dist.all_reduce(Tm, op=dist.ReduceOp.MAX, group=group)
        return (Ts, Tm)
    T = T.contiguous()
    if world > 1:
        dist.all_reduce(T, op=dist.ReduceOp.SUM, group=group)
    return T


def dim_sharded_fitness(problem, X: torch.Tensor, group=None) -> torch.Tensor:
    """Fitness of the replicated population ``X`` with the column work split over
    the ranks of ``group`` (whole evaluation when no process group exists, or when the
    problem has no partial terms: the rows are replicated, so it evaluates them itself)."""
    if not supports_dim_sharding(problem):
        return problem.evaluate(None, X)[0]
    rank, world = _world(group)
    d = X.shape[1]
    col0, own = balanced_slices(d, world)[rank]
    hi = min(col0 + own + problem.dim_halo, d)
    # shifted-rotated problems shard the rotated coordinates: they take the full rows
    Xb = X if getattr(problem, "dim_shard_full_rows", False) else X[:, col0:hi]
    return problem.combine_terms(_reduce_terms(problem.partial_terms(Xb, col0, d, own), d, group), d)


def dim_sharded_fitness_local(problem, Xloc: torch.Tensor, col0: int, d: int, group=None) -> torch.Tensor:
    """Fitness when the population itself is column-sharded (``Xloc`` = this rank's columns
    [col0, col0 + own) of every row).  Problems whose partial terms need no halo and no full
    rows reduce their terms; every other problem is evaluated on the all-gathered rows (the
    generic rule: the state stays column-sharded, the evaluation replicated)."""
    own = Xloc.shape[1]
    if supports_dim_sharding(problem) and getattr(problem, "dim_halo", 1) == 0 and not getattr(problem, "dim_shard_full_rows", False):
        return problem.combine_terms(_reduce_terms(problem.partial_terms(Xloc, col0, d, own), d, group), d)
    X = _gather_cols(Xloc, d, group)
    return dim_sharded_fitness(problem, X, group)


def algorithm_column_separable(algorithm) -> bool:
    """The class that implements the algorithm's ``ask`` / ``tell`` (the first in the MRO to
    define either) declares ``column_separable = True`` itself or is a subclass of one that
    does and adds no ``ask`` / ``tell`` of its own — a subclass that inherits ``dim_shard`` but
    overrides ``ask`` / ``tell`` (e.g. ODE over DE) is not assumed to handle column blocks."""
    if not hasattr(algorithm, "dim_shard"):
        return False
    mro = type(algorithm).__mro__
    impl = next((i for i, c in enumerate(mro) if "ask" in vars(c) or "tell" in vars(c)), None)
    flag = next((i for i, c in enumerate(mro) if "column_separable" in vars(c)), None)
    return impl is not None and flag is not None and flag <= impl and bool(vars(mro[flag])["column_separable"])


class ColumnSeparable:
    """Decision-axis (column) state sharding for algorithms whose ``ask`` / ``tell`` act on each
    column independently given replicated per-row quantities (fitness, row draws) — the
    reference's GSPMD ``_auto_shard`` (``std_workflow.py:253-270``) shards every (pop, dim) and
    (dim,) array of such a state along dim.  A subclass lists those fields in ``dim_fields``
    and sets ``column_separable = True`` in the class that defines its ``ask`` / ``tell``;
    per-column constants (bounds) are read through :meth:`cols` / :meth:`col_vec`, and its
    random draws must be indexed by global column (Philox counters) so that every split
    reproduces the single-process run."""

    dim_fields: tuple = ()
    # child-module state fields with a trailing decision axis (tensors, or tuples of them such
    # as an optimiser's (t, m, v): elements whose last dimension is d are sliced)
    dim_child_fields: dict = {}
    _cols = None

    @staticmethod
    def _map_d(x, d, fn):
        if isinstance(x, (tuple, list)):
            return type(x)(ColumnSeparable._map_d(v, d, fn) for v in x)
        if torch.is_tensor(x) and x.dim() >= 1 and x.shape[-1] == d:
            return fn(x)
        return x

    def dim_shard(self, state, col0: int, own: int):
        d = int(self.dim)
        self._cols = (int(col0), int(own), d)
        state = state.update(**{f: state[f][..., col0 : col0 + own].contiguous() for f in self.dim_fields})
        for child, fields in self.dim_child_fields.items():
            cs = state.get_child_state(child)
            cs = cs.update(**{f: self._map_d(cs[f], d, lambda x: x[..., col0 : col0 + own].contiguous()) for f in fields})
            state = state.update_child(child, cs)
        return state

    def cols(self):
        """(first column, columns owned, total columns) of this rank's block."""
        return self._cols if self._cols is not None else (0, int(self.dim), int(self.dim))

    def col_vec(self, v):
        """This rank's block of a per-column vector (bounds, means)."""
        c0, own, _ = self.cols()
        return v[..., c0 : c0 + own]

    def normal_cols(self, key, rows: int, device, row0: int = 0):
        """This rank's columns of rows [row0, row0 + rows) of ``normal(key, (·, dim))`` — the
        full matrix when the state is not sharded (every split draws the same numbers)."""
        from ..ops import random as rnd

        c0, own, d = self.cols()
        if own == d and torch.device(device).type != "cuda":
            return rnd.normal(key, (rows, d), offset=row0 * d).to(device)
        # on a GPU every split (one rank included) draws through the same window kernel: bitwise
        # equal blocks for any world size
        return rnd.normal_window(key, rows, d, c0, own, row0, device)

    def uniform_cols(self, key, rows: int, device, row0: int = 0):
        """This rank's columns of ``uniform(key, (rows, dim))`` (see :meth:`normal_cols`)."""
        from ..ops import random as rnd

        c0, own, d = self.cols()
        if own == d and torch.device(device).type != "cuda":
            return rnd.uniform(key, (rows, d), offset=row0 * d).to(device)
        # on a GPU every split (one rank included) draws through the same window kernel: bitwise
        # equal blocks for any world size
        return rnd.uniform_window(key, rows, d, c0, own, row0, device)

    def col_sum(self, x: torch.Tensor) -> torch.Tensor:
        """``x`` summed over the ranks of the decision-axis shard group (identity when the state
        is not sharded): the per-column partial of a reduction over all decision variables,
        e.g. ‖p_σ‖² — GSPMD inserts the same all-reduce for a sum over a sharded axis."""
        if self._cols is None or self._cols[1] == self._cols[2] or not (dist.is_available() and dist.is_initialized()):
            return x
        x = x.contiguous().clone()
        dist.all_reduce(x, group=getattr(self, "_dim_group", None))
        return x

    def dim_gather(self, state, group=None):
        """The state with every ``dim_fields`` array reassembled to full width on every rank
        (one all-gather per field; for checkpoints, monitors and final results)."""
        if self._cols is None or not (dist.is_available() and dist.is_initialized()):
            return state
        d = self._cols[2]
        own = self._cols[1]
        state = state.update(**{f: _gather_cols(state[f], d, group) for f in self.dim_fields})
        for child, fields in self.dim_child_fields.items():
            cs = state.get_child_state(child)
            cs = cs.update(**{f: self._map_d(cs[f], own, lambda x: _gather_cols(x, d, group)) for f in fields})
            state = state.update_child(child, cs)
        return state


def supports_state_sharding(algorithm, problem) -> bool:
    """Full P2 (state column-sharded): the algorithm can slice its state into column blocks.
    Any problem then works — halo-free partial terms reduce per-row terms, every other problem
    sees the all-gathered rows (:func:`dim_sharded_fitness_local`)."""
    return algorithm_column_separable(algorithm)


class DimShardedProblem(Problem):
    def __init__(self, problem: Problem, group=None):
        super().__init__()
        self.problem = problem
        self.group = group

    def setup(self, key):
        return State()

    def evaluate(self, state, X):
        return dim_sharded_fitness(self.problem, X, self.group), state
