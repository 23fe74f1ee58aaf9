"""The standard single-/multi-GPU workflow.

Parity: reference ``src/evox/workflows/std_workflow.py`` — one generation per
``step`` with the hook order

``pre_step → pre_ask → ask|init_ask → post_ask → sol_transforms → pre_eval →
evaluate → ×opt_direction → post_eval → fit_transforms → pre_tell →
tell|init_tell → post_tell → generation += 1 → post_step``

(``std_workflow.py:129-199``); ``init_ask``/``init_tell`` are used at generation 0
when the algorithm overrides them (``:203-213``).

MI355X-first execution model (replaces ``jax.jit`` / ``pmap``):

* ``graph=True`` captures one full generation (ask, evaluation, tell — every HIP
  kernel and, in distributed mode, the RCCL collectives) into a **hipGraph** via
  ``torch.cuda.CUDAGraph`` on a side stream and replays it, so a generation costs
  one graph launch instead of dozens of host-side kernel launches.  The state
  returned in graph mode aliases the workflow's static buffers (clone to keep a
  snapshot).  Monitor hooks that consume the step's tensors are replayed on the
  host after each graph launch with the graph's static output buffers, so
  monitors need not be capture-safe.  ``graph="auto"`` tries the capture once and
  falls back to eager steps (with a warning) if the step is not capturable.
  Steps that need host decisions mid-generation call
  :func:`evoxmi.runtime.host_phase`; the capture is then split into graph segments
  with that host phase replayed eagerly between them
  (:class:`evoxmi.runtime.SegmentedGraph`).
* ``enable_distributed(state)`` turns the workflow into an SPMD program with one
  process per GPU (``torch.distributed``; backend ``nccl`` = RCCL over xGMI on
  MI355X, ``gloo`` on CPU).  The algorithm state is replicated; every rank
  evaluates a balanced slice of the population and the fitness slices are
  all-gathered (reference ``std_workflow.py:311-345``, without its dropped
  remainder rows).  Algorithms that implement the sharded protocol
  (``ask_sharded``/``tell_sharded``, e.g. :class:`~evoxmi.algorithms.CMAES`)
  generate only their own rows and all-reduce partial statistics instead.
"""
from __future__ import annotations

import contextlib
import warnings
from typing import Callable, List, Optional, Union

import torch

from ..core import capture_warmup, Algorithm, Monitor, Problem, State, Workflow, use_state
from ..core.algorithm import algorithm_has_init_ask
from ..core.state import tree_flatten, tree_map
from .. import config
from ..utils.common import parse_opt_direction
from ..utils.profiling import trace_range
from ..runtime.graph import SegmentedGraph, copy_into

HOOKS = ("pre_step", "pre_ask", "post_ask", "pre_eval", "post_eval", "pre_tell", "post_tell", "post_step")


class StdWorkflow(Workflow):
    def __init__(
        self,
        algorithm: Algorithm,
        problem: Union[Problem, List[Problem]],
        monitors: List[Monitor] = (),
        opt_direction: Union[str, List[str]] = "min",
        sol_transforms: List[Callable] = (),
        fit_transforms: List[Callable] = (),
        pop_transform: Optional[Callable] = None,
        jit_problem: bool = True,
        num_objectives: Optional[int] = None,
        monitor=None,
        graph: Union[bool, str] = False,
        nan_policy: str = "keep",
        phase_timer=None,
    ):
        super().__init__()
        self.algorithm = algorithm
        self.problem = problem
        self.monitors = list(monitors)
        if monitor is not None:
            warnings.warn("`monitor` is deprecated, use `monitors=[...]`", DeprecationWarning)
            self.monitors = [monitor]
        self.registered_hooks = {h: [] for h in HOOKS}
        for m in self.monitors:
            for h in m.hooks():
                self.registered_hooks[h].append(m)
        self.opt_direction = parse_opt_direction(opt_direction)
        for m in self.monitors:
            m.set_opt_direction(self.opt_direction)
        self.sol_transforms = list(sol_transforms)
        if pop_transform is not None:
            warnings.warn("`pop_transform` is deprecated, use `sol_transforms`", DeprecationWarning)
            self.sol_transforms = [pop_transform]
        self.fit_transforms = list(fit_transforms)
        self.jit_problem = jit_problem
        self.num_objectives = num_objectives
        if jit_problem is False and num_objectives is None:
            warnings.warn("Using external problem but num_objectives isn't set, assuming to be 1.")
            self.num_objectives = 1
        assert nan_policy in ("keep", "inf"), "nan_policy must be 'keep' or 'inf'"
        self.nan_policy = nan_policy
        self.graph = graph
        # optional evoxmi.utils.profiling.PhaseTimer (per-phase hipEvent timing, eager steps;
        # in graph mode the whole replay is one "graph_replay" phase)
        self.phase_timer = phase_timer
        self._has_init_ask = algorithm_has_init_ask(algorithm)
        # distributed context
        self.distributed_step = False
        self._dist = None
        self._dim_shard_group = None  # set by enable_multi_devices (decision-axis sharding)
        # graph-mode bookkeeping
        self._graph = None
        self._graphs = {}  # graph variant (Algorithm.graph_variant) → (graph, hook record)
        self._graph_failed = False
        self._static = None
        self._static_out = None
        self._hook_args = None

    # ------------------------------------------------------------------ state
    def setup(self, key):
        return State(generation=0)

    # ------------------------------------------------------------------ core
    def _opt_dir(self, fitness):
        od = self.opt_direction
        if isinstance(od, torch.Tensor):
            od = od.to(fitness.device)
            return fitness * od
        return fitness if od == 1 else fitness * od

    def _evaluate(self, state, transformed):
        if self._dim_shard_group is not None:
            from ..parallel.dim_sharded import _gather_cols, dim_sharded_fitness, dim_sharded_fitness_local, supports_dim_sharding

            if not torch.is_tensor(transformed):
                raise TypeError("decision-axis sharding evaluates a (pop, dim) tensor; got " + type(transformed).__name__)
            grp = self._dim_shard_group[0]
            if not supports_dim_sharding(self.problem):
                # no partial terms: the problem evaluates the replicated full rows through its own
                # state (Brax / EnvPool keys, episode counters advance identically on every rank)
                X = _gather_cols(transformed, self._dim_shard_group[2], grp) if len(self._dim_shard_group) > 1 else transformed
                return use_state(self.problem.evaluate)(state, X)
            if len(self._dim_shard_group) > 1:  # state-sharded: `transformed` is this rank's column block
                _, col0, d = self._dim_shard_group
                return dim_sharded_fitness_local(self.problem, transformed, col0, d, grp), state
            return dim_sharded_fitness(self.problem, transformed, grp), state
        if self.jit_problem:
            return use_state(self.problem.evaluate)(state, transformed)
        fitness, state = use_state(self.problem.evaluate)(state, transformed)
        if not isinstance(fitness, torch.Tensor):
            fitness = torch.as_tensor(fitness)
        return fitness.to(torch.float32), state

    def _proto_step(self, is_init: bool, state: State, record=None):
        for m in self.registered_hooks["pre_ask"]:
            m.pre_ask(state)
        alg = self.algorithm
        sharded = self.distributed_step and self._dist.algorithm_sharded
        if is_init:
            ask, tell = alg.init_ask, alg.init_tell
        else:
            ask, tell = alg.ask, alg.tell
        with self._phase("ask"):
            if sharded:
                d = self._dist
                ask_s = alg.init_ask_sharded if is_init else alg.ask_sharded
                cand_sol, state = use_state(ask_s)(state, d)
            else:
                cand_sol, state = use_state(ask)(state)
        for m in self.registered_hooks["post_ask"]:
            m.post_ask(state, cand_sol)

        if self.distributed_step and not sharded:
            start, size = self._dist.slice_of(cand_sol.shape[0])
            local = cand_sol[start : start + size]
        else:
            local = cand_sol

        transformed = local
        for t in self.sol_transforms:
            transformed = t(transformed)
        for m in self.registered_hooks["pre_eval"]:
            m.pre_eval(state, local, transformed)

        with self._phase("evaluate"):
            fitness, state = self._evaluate(state, transformed)
        if self.nan_policy == "inf":
            fitness = torch.nan_to_num(fitness, nan=float("inf"))

        if self.distributed_step:
            with self._phase("all_gather"):
                fitness = self._dist.all_gather_rows(fitness, cand_sol.shape[0] if not sharded else self._dist.global_pop)

        fitness = self._opt_dir(fitness)
        for m in self.registered_hooks["post_eval"]:
            m.post_eval(state, local, transformed, fitness)
        tfit = fitness
        for t in self.fit_transforms:
            tfit = t(tfit)
        for m in self.registered_hooks["pre_tell"]:
            m.pre_tell(state, local, transformed, fitness, tfit)
        with self._phase("tell"):
            if sharded:
                tell_s = alg.init_tell_sharded if is_init else alg.tell_sharded
                state = use_state(tell_s)(state, tfit, self._dist)
            else:
                state = use_state(tell)(state, tfit)
        for m in self.registered_hooks["post_tell"]:
            m.post_tell(state)
        if record is not None:
            record.update(cand_sol=local, transformed=transformed, fitness=fitness, tfit=tfit)
        return state.update(generation=state.generation + 1)

    def _phase(self, name):
        """roctx range (EVOXMI_TRACE=1) and/or hipEvent timer around one phase;
        inert while a hipGraph is being captured."""
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            return contextlib.nullcontext()
        timer = self.phase_timer
        if timer is None and not config.get("trace"):
            return contextlib.nullcontext()
        stack = contextlib.ExitStack()
        stack.enter_context(trace_range(name))
        if timer is not None:
            stack.enter_context(timer.phase(name))
        return stack

    def _variant(self, state):
        gv = getattr(self.algorithm, "graph_variant", None)
        return gv(int(state.generation)) if gv is not None else None

    def _step_eager(self, state):
        from ..utils import profiling

        is_init = self._has_init_ask and state.generation == 0
        prev = profiling._ACTIVE_TIMER
        profiling._ACTIVE_TIMER = self.phase_timer
        variant = self._variant(state)
        ctx = self.algorithm.graph_variant_context(variant) if variant is not None else contextlib.nullcontext()
        try:
            with ctx:
                return self._proto_step(bool(is_init), state)
        finally:
            profiling._ACTIVE_TIMER = prev

    # ------------------------------------------------------------------ hipGraph path
    def _hooks_inside_step(self):
        return any(self.registered_hooks[h] for h in HOOKS[1:-1])

    def _capture(self, state, variant=None):
        """Capture one (non-init) generation into a hipGraph.

        ``variant``: the algorithm's graph variant for this generation
        (:meth:`evoxmi.core.Algorithm.graph_variant`, e.g. CMA-ES's longer cold-start
        eigensolver schedule).  Every variant is captured once, over the SAME static state
        buffers, and replayed by generation index from then on."""
        dev = None
        for x in tree_flatten(state)[0]:
            if isinstance(x, torch.Tensor) and x.is_cuda:
                dev = x.device
                break
        if dev is None:
            raise RuntimeError("graph=True requires the state to live on a GPU")
        static = self._static if self._static is not None else tree_map(lambda x: x.clone() if isinstance(x, torch.Tensor) else x, state)
        if self._static is not None and state is not static and state is not self._static_out:
            self._load_static(static, state)
        ctx = self.algorithm.graph_variant_context(variant) if variant is not None else contextlib.nullcontext()
        # warm-up on a side stream (allocator / lazy init), as required for capture
        s = torch.cuda.Stream(device=dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        saved_hooks = self.registered_hooks
        self.registered_hooks = {h: [] for h in HOOKS}
        try:
            ctx.__enter__()
            with torch.cuda.stream(s), capture_warmup():
                self._proto_step(False, tree_map(lambda x: x.clone() if isinstance(x, torch.Tensor) else x, static))
            torch.cuda.current_stream(dev).wait_stream(s)
            torch.cuda.synchronize(dev)
            # segmented capture: steps that need host decisions mid-generation (e.g. the
            # CMA-ES eigensolver's convergence checks) split the graph at host phases
            g = SegmentedGraph()
            record = {}
            counters = getattr(self._dist, "counters", None) if self._dist is not None else None
            if counters is not None and hasattr(counters, "begin_capture"):
                counters.begin_capture(variant)  # this variant's wire counters (all its segments)

            def body():
                out = self._proto_step(False, static, record=record)
                in_leaves, in_spec = tree_flatten(static)
                out_leaves, out_spec = tree_flatten(out)
                if in_spec != out_spec:
                    raise RuntimeError("graph=True: the step changed the state structure; this algorithm is not graph-safe")
                groups = {}
                for a, b in zip(in_leaves, out_leaves):
                    if isinstance(a, torch.Tensor):
                        if a.shape != b.shape or a.dtype != b.dtype:
                            raise RuntimeError("graph=True: a state tensor changed shape/dtype across a step")
                        if a.data_ptr() != b.data_ptr():
                            groups.setdefault(a.device, ([], []))
                            groups[a.device][0].append(a)
                            groups[a.device][1].append(b)
                # write the new state into the static buffers with one multi-tensor copy per
                # device (a dozen small leaves of mixed dtypes would otherwise be a dozen copy
                # launches per replay; copy_into moves them as 32-bit words)
                for dst, src in groups.values():
                    copy_into(dst, src)
                return in_leaves, out_leaves

            in_leaves, out_leaves = g.capture(body, s)
        finally:
            ctx.__exit__(None, None, None)
            self.registered_hooks = saved_hooks
        # python (non-tensor) leaves must be step-invariant, except the generation counter
        py_changed = [
            (a, b)
            for a, b in zip(in_leaves, out_leaves)
            if not isinstance(a, torch.Tensor) and a != b
        ]
        if len(py_changed) > 1:
            raise RuntimeError(f"graph=True: host-side state fields change every step {py_changed}; not graph-safe")
        self._graph = g
        self._graphs[variant] = (g, record)
        self._static = static
        self._hook_args = record
        return static

    @staticmethod
    def _load_static(static, state):
        """A foreign state (e.g. a restored checkpoint) into the static buffers."""
        for a, b in zip(tree_flatten(static)[0], tree_flatten(state)[0]):
            if isinstance(a, torch.Tensor):
                if isinstance(b, torch.Tensor):
                    if b.data_ptr() != a.data_ptr():
                        a.copy_(b)
                else:  # e.g. a harness writing progress=0.3 into a tensor field
                    a.fill_(b)

    def _step_graph(self, state):
        variant = self._variant(state)
        if variant not in self._graphs:
            static = self._capture(state, variant)
        else:
            self._graph, self._hook_args = self._graphs[variant]
            static = self._static
            if state is not static and state is not self._static_out:
                self._load_static(static, state)
        with self._phase("graph_replay"):
            self._graph.replay()
        counters = getattr(self._dist, "counters", None) if self._dist is not None else None
        if counters is not None and hasattr(counters, "note_replay"):
            counters.note_replay(variant)
        gen = state.generation + 1
        out = static.update(generation=gen)
        self._static = out
        self._static_out = out
        # post-hoc monitor hooks on the graph's static buffers
        r = self._hook_args
        for m in self.registered_hooks["post_ask"]:
            m.post_ask(out, r["cand_sol"])
        for m in self.registered_hooks["pre_eval"]:
            m.pre_eval(out, r["cand_sol"], r["transformed"])
        for m in self.registered_hooks["post_eval"]:
            m.post_eval(out, r["cand_sol"], r["transformed"], r["fitness"])
        for m in self.registered_hooks["pre_tell"]:
            m.pre_tell(out, r["cand_sol"], r["transformed"], r["fitness"], r["tfit"])
        for m in self.registered_hooks["post_tell"]:
            m.post_tell(out)
        return out

    # ------------------------------------------------------------------ public
    def prepare_graphs(self, state: State, horizon: int) -> State:
        """Capture, ahead of time, the hipGraph of every algorithm graph variant that the next
        ``horizon`` generations will replay (e.g. CMA-ES's late eigensolver schedule), so that
        no capture happens later inside a timed loop.  The state is not advanced (capture
        records; its warm-up runs on a copy of the state)."""
        if not self.graph or self._graph_failed or state.generation == 0 and self._has_init_ask:
            return state
        g0 = int(state.generation)
        gv = getattr(self.algorithm, "graph_variant", None)
        variants = []
        for k in range(horizon):
            v = gv(g0 + k) if gv is not None else None
            if v not in variants:
                variants.append(v)
        vs = getattr(self.algorithm, "graph_variant_set", None)
        for v in (vs() if vs is not None else ()):
            if v not in variants:
                variants.append(v)
        for v in variants:
            if v not in self._graphs:
                if self.graph == "auto":
                    try:
                        self._capture(state, v)
                    except (RuntimeError, torch.AcceleratorError) as e:
                        self._give_up_graphs(e)
                        return state
                else:
                    self._capture(state, v)
        return state

    def _give_up_graphs(self, e):
        """graph='auto': a capture failed (host sync / H2D copy / data-dependent shape) — the
        input state is untouched; every generation runs eagerly from now on."""
        self._graph_failed = True
        self._graph = None
        self._graphs = {}
        self._static = None
        torch.cuda.synchronize()
        warnings.warn(f"graph='auto': {type(self.algorithm).__name__} step is not capturable ({str(e).splitlines()[0]}); running eagerly")

    def step(self, state: State) -> State:
        for m in self.registered_hooks["pre_step"]:
            m.pre_step(state)
        if self.graph and not self._graph_failed and not (self._has_init_ask and state.generation == 0):
            if self.graph == "auto" and (self._graph is None or self._variant(state) not in self._graphs):
                # a capture is due (the first one, or a graph variant not captured yet — e.g.
                # CMA-ES's late eigensolver schedule): a capture-unsafe step falls back to eager
                try:
                    state = self._step_graph(state)
                except (RuntimeError, torch.AcceleratorError) as e:
                    self._give_up_graphs(e)
                    state = self._step_eager(state)
            else:
                state = self._step_graph(state)
        else:
            state = self._step_eager(state)
        hook = getattr(self.algorithm, "after_step", None)
        if hook is not None:
            hook(int(state.generation))
        for m in self.registered_hooks["post_step"]:
            m.post_step(state)
        k = config.get("check_replicas_every")
        if self.distributed_step and k and int(state.generation) % k == 0:
            # race/divergence detector: replicas must stay bit-identical
            chk = state
            local = getattr(self.algorithm, "rank_local_fields", ()) if self._dist.algorithm_sharded else ()
            # fields an owner-computes algorithm keeps current only where a rank needs them
            local = tuple(local) + tuple(getattr(self.algorithm, "rank_divergent_fields", ()) if self._dist.algorithm_sharded else ())
            if local:
                alg = state.get_child_state("algorithm")
                chk = state.update_child("algorithm", alg.replace(**{f: torch.zeros(0) for f in local}))
            if not self._dist.check_replicas(chk):
                raise RuntimeError(f"replicated algorithm state diverged across ranks at generation {int(state.generation)}")
        return state

    def valid(self, state: State, metric: str = "loss"):
        """Evaluate the current proposal in the problem's validation mode (``std_workflow.py:218-234``)."""
        new_state = use_state(self.problem.valid)(state, metric=metric)
        pop, new_state = use_state(self.algorithm.ask)(new_state)
        if self.distributed_step and not self._dist.algorithm_sharded:
            start, size = self._dist.slice_of(pop.shape[0])
            pop = pop[start : start + size]
        for t in self.sol_transforms:
            pop = t(pop)
        fitness, _ = use_state(self.problem.evaluate)(new_state, pop)
        if self.distributed_step:
            fitness = self._dist.all_gather_rows(fitness, None)
        return fitness, state

    def enable_distributed(self, state: State, group=None, context=None) -> State:
        """Population-shard this workflow across the ranks of ``torch.distributed``.

        Every rank must call this with an identical state (same key ⇒ identical
        replicas).  The state is broadcast from rank 0 to make that explicit.
        ``context``: a ready context instead of one over the default process group (e.g.
        :class:`evoxmi.parallel.context.SimulatedDistContext` for one rank's share of an
        N-GPU step on one device).
        """
        from ..parallel.context import DistContext

        self._dist = context if context is not None else DistContext(group=group, algorithm=self.algorithm)
        self.distributed_step = True
        for m in self.monitors:  # monitors that track sharded rows (EvalMonitor best solution)
            if hasattr(m, "set_dist"):
                m.set_dist(self._dist)
        state = self._dist.broadcast_state(state)
        if self._dist.algorithm_sharded:
            # None: the algorithm's per-step row count varies (e.g. co-evolution containers
            # of CSO sub-swarms) — the fitness all-gather then exchanges the sizes
            pop_size = getattr(self.algorithm, "pop_size", None)
            self._dist.set_global_pop(pop_size)
            # rank-local fields (e.g. the sampled rows) hold only this rank's slice from the
            # start, so every step keeps the same shapes (required for hipGraph capture)
            local = getattr(self.algorithm, "rank_local_fields", ())
            if local and pop_size is not None:
                start, size = self._dist.slice_of(pop_size)
                alg = state.get_child_state("algorithm")
                state = state.update_child("algorithm", alg.update(**{f: alg[f][start : start + size].clone() for f in local}))
        return state

    def enable_multi_devices(self, state: State, devices=None, shard_state: bool = False) -> State:
        """Shard the evaluation along the decision axis (reference
        ``std_workflow.py:272-309``, GSPMD over ``PositionalSharding(devices)``).

        One process per GPU: if the problem implements the dim-sharding protocol
        (:func:`evoxmi.parallel.supports_dim_sharding`), each rank evaluates its
        column block and the per-row partial terms are all-reduced
        (:class:`evoxmi.parallel.DimShardedProblem`); the algorithm stays replicated
        (same key on every rank).  A problem without the protocol falls back to population
        sharding (:meth:`enable_distributed`) with a warning.  The state structure is
        unchanged, so this may be called after ``init``.

        ``shard_state=True`` shards the algorithm state too, as GSPMD does for every (pop, dim)
        array: column-separable algorithms (:class:`evoxmi.parallel.ColumnSeparable` — PSO, DE,
        ODE, …) keep only their column block of every ``dim_fields`` array on each rank; problems
        with halo-free terms evaluate that block (the only traffic is the (N, k) term all-reduce),
        every other problem evaluates the all-gathered rows (GSPMD's all-gather of a sharded
        operand).  An algorithm that is not column-separable (CMA-ES and the other
        full-covariance ES) keeps its state replicated, with a warning — the same results as
        GSPMD's column-sharded matrices, which it would gather for every product.  The state then holds column blocks: :meth:`gather_state` reassembles the
        full arrays (the reference's sharded arrays stay logically global).  Default ``False``:
        a state read after the run has the reference's full shapes."""
        if not self.jit_problem:
            raise ValueError("multi-devices with non jit problem isn't currently supported")
        if not (torch.distributed.is_available() and torch.distributed.is_initialized()):
            return state
        from ..parallel.context import DistContext, balanced_slices
        from ..parallel.dim_sharded import supports_dim_sharding, supports_state_sharding

        if shard_state and not supports_state_sharding(self.algorithm, self.problem):
            # GSPMD would shard a full-covariance ES's d×d matrices by columns and gather them for
            # every product; its results equal the unsharded run's, which is what the replicated
            # state gives (at d ≤ 8192 the matrices are ≤ 256 MiB of a GPU's 288 GB, and the
            # column-distributed eigensolver does not pay at d = 1000 — profiles/NOTES.md, round 6)
            warnings.warn(f"enable_multi_devices(shard_state=True): {type(self.algorithm).__name__} is not column-separable "
                          "(parallel.ColumnSeparable); its state stays replicated on every rank and only the "
                          "evaluation is sharded")
            shard_state = False
        if not supports_dim_sharding(self.problem) and not shard_state:
            warnings.warn(f"enable_multi_devices: {type(self.problem).__name__} has no dim-sharding terms "
                          "(partial_terms / combine_terms / dim_halo); sharding the population instead "
                          "(shard_state=True keeps the decision axis sharded and all-gathers the rows to evaluate)")
            return self.enable_distributed(state)
        if shard_state and self.sol_transforms:
            # a solution transform maps whole decision vectors; under state sharding it would see
            # this rank's column block
            raise ValueError("enable_multi_devices(shard_state=True): sol_transforms act on whole decision vectors; "
                             "use shard_state=False (the population stays replicated) or enable_distributed")
        ctx = DistContext(group=devices if isinstance(devices, torch.distributed.ProcessGroup) else None)
        state = ctx.broadcast_state(state)
        if shard_state:
            d = int(self.algorithm.dim)
            rank, world = torch.distributed.get_rank(ctx.group), torch.distributed.get_world_size(ctx.group)
            col0, own = balanced_slices(d, world)[rank]
            alg = state.get_child_state("algorithm")
            state = state.update_child("algorithm", self.algorithm.dim_shard(alg, col0, own))
            self.algorithm._dim_group = ctx.group
            self._dim_shard_group = (ctx.group, col0, d)
        else:
            self._dim_shard_group = (ctx.group,)
        return state

    def gather_state(self, state: State) -> State:
        """The state with a decision-axis-sharded algorithm state reassembled to full-width
        arrays on every rank (identity otherwise)."""
        grp = getattr(self, "_dim_shard_group", None)
        if grp is None or len(grp) < 3:
            return state
        alg = state.get_child_state("algorithm")
        return state.update_child("algorithm", self.algorithm.dim_gather(alg, grp[0]))
