"""BatchedRuns: n independent runs of a DE variant as one vmapped computation must equal
the runs executed one at a time from the same per-run keys (the fork's 32-run protocol,
reference run/run_de.py:54-114), including the injected ``progress`` schedule."""
import pytest
import torch

from evoxmi import random as rnd
from evoxmi.algorithms import de_variants
from evoxmi.algorithms.containers.batched import BatchedRuns
from evoxmi.problems.numerical import CEC2022TestSuit

D, POP, RUNS, GENS = 10, 40, 3, 8
ALGOS = ["DE", "ODE", "CoDE", "JaDE", "SaDE", "SHADE", "LSHADE", "ILSHADE", "JSO", "LSHADE_RSP", "EPSDE", "EVDE"]


def _make(name, dev):
    lb, ub = torch.full((D,), -100.0, device=dev), torch.full((D,), 100.0, device=dev)
    cls = getattr(de_variants, name)
    return cls(lb, ub, pop_size=POP)


def run_single(algo, key, prob, pst):
    st = algo.init(key)
    from evoxmi.core import Algorithm

    pop, st2 = algo.init_ask(st) if type(algo).init_ask is not Algorithm.init_ask else (None, st)
    if pop is not None:
        f, _ = prob.evaluate(pst, pop)
        st = algo.init_tell(st2, f)
    for g in range(GENS):
        pop, st = algo.ask(st)
        f, _ = prob.evaluate(pst, pop)
        st = algo.tell(st, f)
        if "progress" in st._state_dict:
            st = st.update(progress=torch.tensor((g + 1) / GENS, dtype=st.progress.dtype, device=st.progress.device))
    return st


def _eval_blocks(prob, pst, pop, n):
    # evaluate each run's block on its own: the CEC rotation is a GEMM whose rounding can
    # depend on the row count (library blocking), which is a property of the problem, not of
    # the batched algorithm this test pins
    return torch.cat([prob.evaluate(pst, blk)[0] for blk in pop.chunk(n)])


def run_batched(b, key, prob, pst):
    st = b.init(key)
    pop, st2 = b.init_ask(st)
    if pop is not None:
        f = _eval_blocks(prob, pst, pop, b.n_runs)
        st = b.init_tell(st2, f)
    for g in range(GENS):
        pop, st = b.ask(st)
        f = _eval_blocks(prob, pst, pop, b.n_runs)
        st = b.tell(st, f)
        if "progress" in st.runs._state_dict:
            st = b.set_field(st, progress=(g + 1) / GENS)
    return st


def _same(a, b):
    return a.shape == b.shape and bool((torch.eq(a, b) | (torch.isnan(a) & torch.isnan(b))).all())


def _check(name, dev):
    prob = CEC2022TestSuit.create(1)
    pst = prob.init(rnd.PRNGKey(1, device=dev))
    key = rnd.PRNGKey(11, device=dev)
    b = BatchedRuns(_make(name, dev), RUNS)
    bst = run_batched(b, key, prob, pst)
    for r, k in enumerate(b.run_keys(key)):
        sst = run_single(_make(name, dev), k, prob, pst)
        # LSHADE-family padding rows are NaN: compare bitwise with NaN == NaN
        assert _same(bst.runs.population[r], sst.population), f"{name} run {r}: population differs"
        assert _same(bst.runs.fitness[r], sst.fitness), f"{name} run {r}: fitness differs"


@pytest.mark.parametrize("name", ALGOS)
def test_batched_runs_equal_sequential_cpu(name):
    _check(name, "cpu")


@pytest.mark.gpu
@pytest.mark.parametrize("name", ALGOS)
def test_batched_runs_equal_sequential_gpu(name):
    _check(name, "cuda")


def _run_de(tmp_path, tag, extra):
    import importlib.util
    import os

    spec = importlib.util.spec_from_file_location("run_de", os.path.join(os.path.dirname(__file__), "..", "run", "run_de.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    argv = ["--funcs", "1-3", "--dim", "20", "--pop", "100", "--runs", "4", "--max-steps", "12", "--progress", "steps",
            "--max-time", "1e9", "--out", str(tmp_path / tag)] + extra
    return mod.main(argv)


@pytest.mark.parametrize("algo", ["LSHADE", "EVDE"])
def test_run_de_batched_harness_cpu(tmp_path, algo):
    """``run/run_de.py --batched`` runs the same per-run keys and progress schedule as the
    sequential harness; on CPU the (runs·pop)-row CEC rotation GEMM may round differently
    from the pop-row one (library blocking depends on the row count), so the bests agree to
    rtol 1e-3 here; the GPU variant below checks bit equality."""
    seq = _run_de(tmp_path, "seq", ["--algo", algo, "--device", "cpu"])
    bat = _run_de(tmp_path, "bat", ["--algo", algo, "--device", "cpu", "--batched"])
    for fn in seq:
        a, b = torch.tensor(seq[fn]["best"]), torch.tensor(bat[fn]["best"])
        assert seq[fn]["steps"] == bat[fn]["steps"]
        assert torch.allclose(a, b, rtol=1e-3), (fn, a, b)


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["LSHADE", "EVDE"])
def test_run_de_batched_harness_identical_gpu(tmp_path, algo):
    """On the GPU the batched harness (one vmapped hipGraph per generation) reproduces the
    sequential one run by run, bit for bit."""
    seq = _run_de(tmp_path, "seq", ["--algo", algo])
    bat = _run_de(tmp_path, "bat", ["--algo", algo, "--batched"])
    for fn in seq:
        assert seq[fn]["best"] == bat[fn]["best"], (fn, seq[fn]["best"], bat[fn]["best"])
