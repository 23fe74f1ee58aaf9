"""Decision-axis (column) sharding of the evaluation — strategy P2 (reference
``std_workflow.py:253-309``): per-block additive terms must reproduce the full
evaluation for every split, and a gloo world-size-2 run through
``enable_multi_devices`` must follow the single-process trajectory."""
import math
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

from evoxmi import random as rnd
from evoxmi.algorithms import PSO
from evoxmi.parallel import balanced_slices, supports_dim_sharding
from evoxmi.problems.numerical import Ackley, Ellipsoid, Griewank, Rastrigin, Rosenbrock, Schwefel, Sphere
from evoxmi.workflows import StdWorkflow

PROBLEMS = [Sphere, Ackley, Rastrigin, Rosenbrock, Griewank, Schwefel, Ellipsoid]


@pytest.mark.parametrize("cls", PROBLEMS)
@pytest.mark.parametrize("world", [1, 2, 3, 7])
def test_partial_terms_reproduce_full_evaluation(cls, world):
    p = cls()
    assert supports_dim_sharding(p)
    torch.manual_seed(0)
    d = 23
    X = torch.randn(11, d, dtype=torch.float64) * 3
    full, _ = p.evaluate(None, X)
    T = 0
    for col0, own in balanced_slices(d, world):
        hi = min(col0 + own + p.dim_halo, d)
        T = T + p.partial_terms(X[:, col0:hi], col0, d, own)
    assert torch.allclose(p.combine_terms(T, d), full, rtol=1e-10, atol=1e-9)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _make():
    lb, ub = torch.full((30,), -32.0), torch.full((30,), 32.0)
    return StdWorkflow(PSO(lb=lb, ub=ub, pop_size=40), Ackley())


def _worker(rank, world, port, out, shard_state=False):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from evoxmi.parallel import destroy, init_distributed

    init_distributed(backend="gloo")
    wf = _make()
    st = wf.init(rnd.PRNGKey(3))
    st = wf.enable_multi_devices(st, shard_state=shard_state)
    for _ in range(20):
        st = wf.step(st)
    a = st.get_child_state("algorithm")
    out[rank] = (a.global_best_fitness.clone(), a.population.clone(), a.global_best_location.clone())
    destroy()


def test_enable_multi_devices_gloo_matches_single_process():
    wf = _make()
    st = wf.init(rnd.PRNGKey(3))
    for _ in range(20):
        st = wf.step(st)
    ref = st.get_child_state("algorithm")
    if st.has_child("problem") and "count" in st.get_child_state("problem").keys():
        ref = {**{k: ref[k] for k in ref.keys()}, "problem_count": st.get_child_state("problem")["count"]}
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    g0, p0, _ = out[0]
    g1, p1, _ = out[1]
    assert torch.equal(p0, p1)  # replicas stay identical: every rank combines the same all-reduced terms
    assert torch.allclose(g0, ref.global_best_fitness, rtol=1e-4, atol=1e-4)
    assert torch.allclose(p0, ref.population, rtol=1e-3, atol=1e-3)


def _de_worker(rank, world, port, out, cls="DE", prob="Rastrigin"):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from evoxmi.parallel import destroy, init_distributed

    init_distributed(backend="gloo")
    wf = _make_de(cls, prob)
    st = wf.init(rnd.PRNGKey(4))
    st = wf.enable_multi_devices(st, shard_state=True)
    for _ in range(15):
        st = wf.step(st)
    a = st.get_child_state("algorithm")
    full = wf.gather_state(st).get_child_state("algorithm")
    out[rank] = (a.fitness.clone(), a.population.clone(), full.population.clone())
    destroy()


def _make_de(cls="DE", prob="Rastrigin"):
    import evoxmi.algorithms as A
    import evoxmi.problems.numerical as P

    lb, ub = torch.full((30,), -5.0), torch.full((30,), 5.0)
    return StdWorkflow(getattr(A, cls)(lb, ub, 40), getattr(P, prob)())


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("cls", ["DE", "ODE"])
def test_state_sharded_de_gloo_matches_single_process(world, cls):
    """Full P2 for DE and ODE: mutation, binomial crossover (global j_rand and Philox words),
    the opposite points lb + ub − x and the greedy replacement run on each rank's column
    block; the blocks reassemble the single-process population, and ``gather_state`` returns
    it whole on every rank."""
    wf = _make_de(cls)
    st = wf.init(rnd.PRNGKey(4))
    for _ in range(15):
        st = wf.step(st)
    ref = st.get_child_state("algorithm")
    if st.has_child("problem") and "count" in st.get_child_state("problem").keys():
        ref = {**{k: ref[k] for k in ref.keys()}, "problem_count": st.get_child_state("problem")["count"]}
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_de_worker, args=(world, _free_port(), out, cls), nprocs=world, join=True)
    blocks = [out[r] for r in range(world)]
    assert all(torch.equal(b[0], blocks[0][0]) for b in blocks)
    assert [b[1].shape[1] for b in blocks] == [own for _, own in balanced_slices(30, world)]
    assert torch.allclose(blocks[0][0], ref.fitness, rtol=1e-4, atol=1e-3)
    cat = torch.cat([b[1] for b in blocks], 1)
    assert torch.allclose(cat, ref.population, rtol=1e-4, atol=1e-4)
    assert all(torch.equal(b[2], cat) for b in blocks)


def test_column_separable_needs_the_implementing_class_to_opt_in():
    """A subclass that inherits dim_shard but brings its own ask / tell is not state-sharded."""
    from evoxmi.algorithms import DE, ODE, PSO
    from evoxmi.parallel.dim_sharded import algorithm_column_separable

    lb, ub = torch.zeros(4), torch.ones(4)

    class MyDE(DE):
        def ask(self, state):
            return super().ask(state)

    assert algorithm_column_separable(DE(lb, ub, 8)) and algorithm_column_separable(ODE(lb, ub, 8))
    assert algorithm_column_separable(PSO(lb, ub, 8))
    assert not algorithm_column_separable(MyDE(lb, ub, 8))


@pytest.mark.parametrize("world", [2, 3])
def test_state_sharded_pso_gloo_matches_single_process(world):
    """Full P2: every rank keeps only its column block of the swarm (population, velocity,
    personal / global best locations) and draws the same Philox words for it as the unsharded
    swarm; the concatenated blocks follow the single-process trajectory and the replicated
    scalars agree bitwise across ranks."""
    wf = _make()
    st = wf.init(rnd.PRNGKey(3))
    for _ in range(20):
        st = wf.step(st)
    ref = st.get_child_state("algorithm")
    if st.has_child("problem") and "count" in st.get_child_state("problem").keys():
        ref = {**{k: ref[k] for k in ref.keys()}, "problem_count": st.get_child_state("problem")["count"]}
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out, True), nprocs=world, join=True)
    blocks = [out[r] for r in range(world)]
    assert all(torch.equal(b[0], blocks[0][0]) for b in blocks)  # global best fitness replicated
    widths = [b[1].shape[1] for b in blocks]
    assert widths == [own for _, own in balanced_slices(30, world)]
    pop = torch.cat([b[1] for b in blocks], 1)
    gbl = torch.cat([b[2] for b in blocks], 0)
    assert torch.allclose(blocks[0][0], ref.global_best_fitness, rtol=1e-4, atol=1e-4)
    assert torch.allclose(pop, ref.population, rtol=1e-3, atol=1e-3)
    assert torch.allclose(gbl, ref.global_best_location, rtol=1e-3, atol=1e-3)


def _reduce_blocks(terms):
    """What dim_sharded._reduce_terms does across ranks, for per-rank results in rank order:
    tensors / "sum" add, "max" maximise, "cat" blocks concatenate along the decision axis."""
    if isinstance(terms[0], dict):
        out = {}
        if "sum" in terms[0]:
            out["sum"] = sum(t["sum"] for t in terms)
        if "max" in terms[0]:
            out["max"] = torch.stack([t["max"] for t in terms]).max(0).values
        if "cat" in terms[0]:
            c0 = terms[0]["cat"]
            if isinstance(c0, (list, tuple)):
                out["cat"] = [torch.cat([t["cat"][i] for t in terms], -1) for i in range(len(c0))]
            else:
                out["cat"] = torch.cat([t["cat"] for t in terms], -1)
        return out
    return sum(terms)


@pytest.mark.parametrize("fn", range(1, 13))
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_cec2022_partial_terms_reproduce_full_evaluation(fn, world):
    """Shifted-rotated CEC'22 functions shard the rotated coordinates (their rows of M);
    F3 (no rotation) takes plain column blocks with a halo of one; the hybrids (F6–F8) and
    compositions (F9–F12) all-gather their rotated blocks ("cat" terms) and sum the
    composition distances."""
    from evoxmi.problems.numerical import CEC2022TestSuit

    p = CEC2022TestSuit.create(fn)
    assert supports_dim_sharding(p)
    d = 20
    X = (torch.rand(13, d, generator=torch.Generator().manual_seed(fn)) * 20 - 10)
    full, _ = p.evaluate(None, X)
    Ts = []
    for col0, own in balanced_slices(d, world):
        hi = min(col0 + own + p.dim_halo, d)
        Xb = X if getattr(p, "dim_shard_full_rows", False) else X[:, col0:hi]
        Ts.append(p.partial_terms(Xb, col0, d, own))
    assert torch.allclose(p.combine_terms(_reduce_blocks(Ts), d), full, rtol=2e-5, atol=1e-4)


@pytest.mark.parametrize("fn", range(1, 10))
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_lsmop_partial_terms_reproduce_full_evaluation(fn, world):
    """LSMOP (config 5's problem, the d ≥ 10⁴ use case): every rank reduces the parts of the
    m·nk variable groups inside its column block (sum terms; the Schwefel groups by max,
    the Griewank products through log|cos| + sign counts)."""
    import evoxmi.problems.numerical as P

    p = getattr(P, f"LSMOP{fn}")(d=120, m=3)
    assert supports_dim_sharding(p)
    X = torch.rand(9, 120, generator=torch.Generator().manual_seed(fn), dtype=torch.float64)
    X[:, 2:] = X[:, 2:] * 10
    full, _ = p.evaluate(None, X)
    Ts = Tm = 0
    for col0, own in balanced_slices(120, world):
        ts, tm = p.partial_terms(X, col0, 120, own)
        Ts = Ts + ts
        Tm = torch.maximum(Tm, tm) if torch.is_tensor(Tm) else tm
    assert torch.allclose(p.combine_terms((Ts, Tm), 120), full, rtol=1e-9, atol=1e-9)


@pytest.mark.parametrize("name", ["DTLZ1", "DTLZ2", "DTLZ3", "DTLZ4", "DTLZ5", "DTLZ6", "DTLZ7", "ZDT1", "ZDT2", "ZDT3", "ZDT4", "ZDT6"])
@pytest.mark.parametrize("world", [1, 2, 3, 7])
def test_dtlz_zdt_partial_terms_reproduce_full_evaluation(name, world):
    """Multi-objective suites: position variables travel as terms from their owners, the
    distance function g as an additive partial sum (m = 4, so position columns straddle the
    first blocks' boundaries)."""
    from evoxmi.problems import numerical as N

    d = 23
    p = getattr(N, name)(d=d, m=4) if name.startswith("DTLZ") else getattr(N, name)(n=d)
    assert supports_dim_sharding(p)
    X = torch.rand(11, d, dtype=torch.float64, generator=torch.Generator().manual_seed(world))
    full, _ = p.evaluate(None, X)
    T = 0
    for col0, own in balanced_slices(d, world):
        T = T + p.partial_terms(X[:, col0 : col0 + own], col0, d, own)
    torch.testing.assert_close(p.combine_terms(T, d), full, rtol=1e-10, atol=1e-10)


def _make_coupled():
    """A non-separable problem with no partial terms: f(x) = (Σ x)² + Σ x² (the generic
    decision-axis path all-gathers the rows)."""
    from evoxmi.core import Problem

    class Coupled(Problem):
        def evaluate(self, state, X):
            return X.sum(1) ** 2 + (X * X).sum(1), state

    return Coupled()


def _make_counting():
    """A stateful problem without partial terms: its state counts evaluations and its fitness
    depends on that count (state must be threaded through the decision-axis evaluation)."""
    from evoxmi.core import Problem, State

    class Counting(Problem):
        def setup(self, key):
            return State(count=torch.zeros((), dtype=torch.int64))

        def evaluate(self, state, X):
            return (X * X).sum(1) + 0.01 * state.count.to(X.dtype), state.update(count=state.count + 1)

    return Counting()


def _generic_worker(rank, world, port, out, algo):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from evoxmi.parallel import destroy, init_distributed

    init_distributed(backend="gloo")
    wf = _make_generic(algo)
    st = wf.init(rnd.PRNGKey(5))
    st = wf.enable_multi_devices(st, shard_state=True)
    for _ in range(8):
        st = wf.step(st)
    full = wf.gather_state(st).get_child_state("algorithm")
    out[rank] = {k: full[k].clone() for k in ("population", "center", "mean", "sigma", "stdev", "C", "velocity", "pbest_position", "fitness") if k in full.keys()}
    if st.has_child("problem") and "count" in st.get_child_state("problem").keys():
        out[rank] = {**out[rank], "problem_count": st.get_child_state("problem")["count"].clone()}
    destroy()


def _make_generic(algo):
    import evoxmi.algorithms as A
    from evoxmi.problems.numerical import Sphere

    d = 24
    if algo in ("nsga2", "nsga3", "ibea", "hype", "rvea", "spea2", "tdea"):
        from evoxmi.problems.numerical import DTLZ2

        cls = {"nsga2": A.NSGA2, "nsga3": A.NSGA3, "ibea": A.IBEA, "hype": A.HypE, "rvea": A.RVEA, "spea2": A.SPEA2, "tdea": A.TDEA}[algo]
        kw = {"n_sample": 500} if algo == "hype" else {}
        return StdWorkflow(cls(torch.zeros(d), torch.ones(d), 3, 32, **kw), DTLZ2(d=d, m=3))
    lb, ub = torch.full((d,), -5.0), torch.full((d,), 5.0)
    if algo == "de":
        return StdWorkflow(A.DE(lb, ub, 32), _make_coupled())
    if algo in ("jade", "shade", "lshade", "jso"):
        cls = {"jade": A.JaDE, "shade": A.SHADE, "lshade": A.LSHADE, "jso": A.JSO}[algo]
        return StdWorkflow(cls(lb, ub, 32), _make_coupled())
    if algo == "cso":
        return StdWorkflow(A.CSO(lb, ub, 32, phi=0.1), _make_coupled())
    if algo == "clpso":
        return StdWorkflow(A.CLPSO(lb, ub, 32, 0.5, 1.5, 0.3), _make_coupled())
    if algo in ("pgpe", "pgpe_adam"):
        return StdWorkflow(A.PGPE(32, torch.full((d,), 2.0), "clipup" if algo == "pgpe" else "adam"), Sphere())
    if algo == "ars":
        return StdWorkflow(A.ARS(32, torch.full((d,), 2.0)), Sphere())
    if algo == "des":
        return StdWorkflow(A.DES(32, torch.full((d,), 2.0)), Sphere())
    if algo == "snes":
        return StdWorkflow(A.SNES(32, torch.full((d,), 2.0), sigma=0.5), Sphere())
    if algo == "sepcmaes":
        return StdWorkflow(A.SepCMAES(torch.full((d,), 2.0), 0.5, pop_size=32), _make_coupled())
    if algo == "openes_stateful":
        return StdWorkflow(A.OpenES(torch.full((d,), 2.0), 32, 0.05, 0.1), _make_counting())
    opt = "adam" if algo == "openes_adam" else None
    return StdWorkflow(A.OpenES(torch.full((d,), 2.0), 32, 0.05, 0.1, optimizer=opt), Sphere())


@pytest.mark.parametrize("algo", ["de", "jade", "shade", "lshade", "jso", "openes", "openes_adam", "openes_stateful", "snes",
                                  "pgpe", "pgpe_adam", "ars", "des", "cso", "clpso", "sepcmaes", "nsga2",
                                  "nsga3", "ibea", "hype", "rvea", "spea2", "tdea"])
@pytest.mark.parametrize("world", [2, 3])
def test_state_sharded_generic_gloo_matches_single_process(algo, world):
    """Generic decision-axis state sharding: the DE family (JaDE / SHADE / L-SHADE / jSO:
    trials drawn per global column, the archive as column blocks) on a problem without partial
    terms (rows all-gathered for the evaluation), OpenES (SGD and Adam: centre, population and
    the optimiser's moments as column blocks), SNES, PGPE (ClipUp's norms all-reduced), ARS and
    DES on Sphere's terms, CSO / CLPSO (coefficients drawn per global column), Sep-CMA-ES (‖p_σ‖
    all-reduced), the SBX + PM MOEAs (operators drawn per global column, selection from the
    replicated objectives) on DTLZ2's terms (whose state carries a key), and a stateful problem
    without terms (its state advances through the all-gathered evaluation) — worlds 2 and 3
    reproduce one process."""
    wf = _make_generic(algo)
    st = wf.init(rnd.PRNGKey(5))
    for _ in range(8):
        st = wf.step(st)
    ref = st.get_child_state("algorithm")
    if st.has_child("problem") and "count" in st.get_child_state("problem").keys():
        ref = {**{k: ref[k] for k in ref.keys()}, "problem_count": st.get_child_state("problem")["count"]}
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_generic_worker, args=(world, _free_port(), out, algo), nprocs=world, join=True)
    assert set(out[0].keys()) <= set(ref.keys())
    for k, v in out[0].items():
        assert torch.allclose(v.double(), ref[k].double(), rtol=1e-4, atol=1e-4, equal_nan=True), k
        assert all(torch.equal(out[r][k].nan_to_num(1e30), v.nan_to_num(1e30)) for r in range(world))


def test_mo_column_sharding_rejects_operators_without_column_blocks():
    import evoxmi.algorithms as A

    class RowOnly:
        def __call__(self, key, x):
            return x

    algo = A.NSGA2(torch.zeros(8), torch.ones(8), 2, 16, crossover_op=RowOnly())
    st = algo.setup(rnd.PRNGKey(0))
    with pytest.raises(ValueError, match="column"):
        algo.dim_shard(st, 0, 4)


@pytest.mark.parametrize("world", [2, 3])
def test_sbx_pm_column_blocks_equal_full_columns(world):
    """The operators' cols= draws: every column block equals those columns of the full result."""
    from evoxmi.operators import crossover, mutation

    d = 30
    x = torch.rand(20, d, generator=torch.Generator().manual_seed(1))
    lb, ub = torch.zeros(d), torch.ones(d)
    key = rnd.PRNGKey(3)
    full_x = crossover.simulated_binary(key, x)
    full_m = mutation.polynomial(key, full_x, (lb, ub))
    for c0, own in balanced_slices(d, world):
        blk = crossover.simulated_binary(key, x[:, c0 : c0 + own], cols=(c0, d))
        assert torch.equal(blk, full_x[:, c0 : c0 + own])
        mb = mutation.polynomial(key, blk, (lb[c0 : c0 + own], ub[c0 : c0 + own]), cols=(c0, d))
        assert torch.equal(mb, full_m[:, c0 : c0 + own])


@pytest.mark.parametrize("name", [f"MaF{i}" for i in range(1, 10)])
@pytest.mark.parametrize("world", [1, 2, 3, 7])
def test_maf_partial_terms_reproduce_full_evaluation(name, world):
    """MaF1-MaF9: position variables (MaF8/9: the two used columns) as terms from their owners,
    the distance sums (MaF2: one per objective group, by global column) additive."""
    from evoxmi.problems import numerical as N

    p = getattr(N, name)(d=23, m=4)
    d = p.d
    assert supports_dim_sharding(p)
    X = torch.rand(11, d, dtype=torch.float64, generator=torch.Generator().manual_seed(world))
    full, _ = p.evaluate(None, X)
    T = 0
    for col0, own in balanced_slices(d, min(world, d)):
        T = T + p.partial_terms(X[:, col0 : col0 + own], col0, d, own)
    torch.testing.assert_close(p.combine_terms(T, d), full, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
@pytest.mark.parametrize("rows,d,c0,own,row0", [(37, 1000, 0, 334, 0), (37, 1000, 334, 333, 5), (64, 24, 8, 8, 3), (9, 30, 7, 11, 2),
                                                (5, 7, 3, 1, 0)])
def test_philox_windows_equal_full_matrix_columns(device, rows, d, c0, own, row0):
    """normal_window / uniform_window (GPU: rng.hip philox_window_kernel, 4-aligned and ragged
    windows) are bitwise the columns of the full matrix drawn at the same row offset."""
    key = rnd.PRNGKey(17, device=device)
    for win, full in ((rnd.normal_window, rnd.normal), (rnd.uniform_window, rnd.uniform)):
        F = full(key, (rows, d), offset=row0 * d)
        W = win(key, rows, d, c0, own, row0, device)
        assert W.shape == (rows, own) and W.device.type == device
        if device == "cuda" and rows * d < 4096 and win is rnd.normal_window:
            # small GPU draws of rnd.normal take the torch Box–Muller (its own sin / cos): ulps
            assert torch.allclose(W, F[:, c0 : c0 + own], rtol=1e-6, atol=1e-6)
        else:
            assert torch.equal(W, F[:, c0 : c0 + own]), (win.__name__, float((W - F[:, c0 : c0 + own]).abs().max()))


def _make_cmaes():
    from evoxmi.algorithms import CMAES

    return StdWorkflow(CMAES(center_init=torch.full((16,), 3.0), init_stdev=1.0, pop_size=24), Ellipsoid())


def _cmaes_worker(rank, world, port, out):
    import warnings

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from evoxmi.parallel import destroy, init_distributed

    init_distributed(backend="gloo")
    wf = _make_cmaes()
    st = wf.init(rnd.PRNGKey(5))
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        st = wf.enable_multi_devices(st, shard_state=True)
    for _ in range(30):
        st = wf.step(st)
    a = st.get_child_state("algorithm")
    out[rank] = (a.mean.clone(), a.C.clone(), a.sigma.clone(), [str(x.message) for x in w])
    destroy()


def test_full_covariance_es_under_state_sharding_keeps_replicated_state():
    """CMA-ES is not column-separable: enable_multi_devices(shard_state=True) keeps its d×d state
    replicated (warning) and shards the evaluation — the run equals the single-process one, as the
    reference's GSPMD column-sharded matrices do (std_workflow.py:253-270)."""
    wf = _make_cmaes()
    st = wf.init(rnd.PRNGKey(5))
    for _ in range(30):
        st = wf.step(st)
    ref = st.get_child_state("algorithm")
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_cmaes_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    m0, C0, s0, msgs = out[0]
    m1, C1, s1, _ = out[1]
    assert any("not column-separable" in m for m in msgs), msgs
    assert torch.equal(m0, m1) and torch.equal(C0, C1) and torch.equal(s0, s1)
    assert C0.shape == (16, 16)
    assert torch.allclose(m0, ref.mean, rtol=1e-3, atol=1e-3)
    assert torch.allclose(C0, ref.C, rtol=1e-3, atol=1e-4)
