"""hipGraph capture of whole generations for the multi-objective zoo (MI355X, marked gpu).

A generation captured with ``StdWorkflow(graph=True)`` must replay to the same
state as eager execution.  Algorithms whose step is data-dependent in shape
(host-side loops over fronts, Gaussian-process fits) are listed in ``EAGER_ONLY``
and checked to fall back cleanly under ``graph="auto"``.
"""
import warnings

import pytest
import torch

import evoxmi.algorithms as A
from evoxmi import random as rnd
from evoxmi.problems.numerical import DTLZ2, LSMOP1
from evoxmi.workflows import StdWorkflow

pytestmark = pytest.mark.gpu

D, M, N = 12, 3, 100


def _mk(name):
    lb, ub = torch.zeros(D, device="cuda"), torch.ones(D, device="cuda")
    return {
        "NSGA2": lambda: A.NSGA2(lb, ub, M, N), "MOEAD": lambda: A.MOEAD(lb, ub, M, N),
        "NSGA3": lambda: A.NSGA3(lb, ub, M, N), "RVEA": lambda: A.RVEA(lb, ub, M, N),
        "IBEA": lambda: A.IBEA(lb, ub, M, N), "HypE": lambda: A.HypE(lb, ub, M, N),
        "SPEA2": lambda: A.SPEA2(lb, ub, M, N), "GDE3": lambda: A.GDE3(lb, ub, M, N),
        "MOEADDRA": lambda: A.MOEADDRA(lb, ub, M, N), "EAGMOEAD": lambda: A.EAGMOEAD(lb, ub, M, N),
        "BiGE": lambda: A.BiGE(lb, ub, M, N), "KnEA": lambda: A.KnEA(lb, ub, M, N),
        "TDEA": lambda: A.TDEA(lb, ub, M, N), "LMOCSO": lambda: A.LMOCSO(M, lb, ub, N),
        "RVEAa": lambda: A.RVEAa(lb, ub, M, N), "BCEIBEA": lambda: A.BCEIBEA(lb, ub, M, N),
        "MOEADM2M": lambda: A.MOEADM2M(lb, ub, M, N), "SRA": lambda: A.SRA(lb, ub, M, N),
    }[name]()


GRAPH_SAFE = ["NSGA2", "MOEAD", "RVEA", "IBEA", "HypE", "SPEA2", "GDE3", "MOEADDRA", "EAGMOEAD", "TDEA", "LMOCSO", "BiGE"]
EAGER_ONLY = ["NSGA3", "KnEA", "RVEAa", "BCEIBEA", "MOEADM2M", "SRA"]


def _run(name, graph, gens=5, problem=None):
    wf = StdWorkflow(_mk(name), problem if problem is not None else DTLZ2(d=D, m=M), graph=graph)
    st = wf.init(rnd.PRNGKey(11, device="cuda"))
    for _ in range(gens):
        st = wf.step(st)
    torch.cuda.synchronize()
    return wf, st.get_child_state("algorithm")


@pytest.mark.parametrize("name", GRAPH_SAFE)
def test_moea_graph_matches_eager(name):
    _, a = _run(name, False)
    wf, b = _run(name, True)
    assert wf._graph is not None
    fa, fb = a.fitness, b.fitness
    fin = torch.isfinite(fa)
    assert torch.equal(fin, torch.isfinite(fb))
    assert torch.allclose(fa[fin], fb[fin], rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("name", EAGER_ONLY)
def test_moea_graph_auto_falls_back(name):
    _, a = _run(name, False)
    with warnings.catch_warnings():
        warnings.simplefilter("ignore")
        wf, b = _run(name, "auto")
    fa, fb = a.fitness, b.fitness
    fin = torch.isfinite(fa)
    assert torch.equal(fin, torch.isfinite(fb))
    assert torch.allclose(fa[fin], fb[fin], rtol=1e-5, atol=1e-5)


def test_lsmop1_moead_graph():
    """North-star config 5 shape family (reduced): MOEA/D + LSMOP1 under capture."""
    lb = torch.zeros(600, device="cuda")
    ub = torch.cat([torch.ones(2, device="cuda"), 10 * torch.ones(598, device="cuda")])
    outs = []
    for graph in (False, True):
        wf = StdWorkflow(A.MOEAD(lb, ub, M, 300, func_name="tchebycheff"), LSMOP1(d=600, m=M), graph=graph)
        st = wf.init(rnd.PRNGKey(5, device="cuda"))
        for _ in range(4):
            st = wf.step(st)
        outs.append(st.get_child_state("algorithm").fitness.clone())
    assert torch.allclose(outs[0], outs[1], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("func", list(range(1, 13)))
def test_cec2022_generation_captures_and_replays(func):
    """Every CEC'22 function (hybrid F6-F8 and composition F9-F12 included) evaluates inside a
    captured CMA-ES generation: no host-to-device copies during capture, same state as eager."""
    from evoxmi.algorithms import CMAES
    from evoxmi.problems.numerical import CEC2022TestSuit

    def run(graph):
        wf = StdWorkflow(CMAES(torch.zeros(20, device="cuda"), 10.0, pop_size=32), CEC2022TestSuit.create(func), graph=graph)
        st = wf.init(rnd.PRNGKey(5, device="cuda"))
        for _ in range(4):
            st = wf.step(st)
        torch.cuda.synchronize()
        return st.get_child_state("algorithm")

    a, b = run(True), run(False)
    assert torch.allclose(a.mean, b.mean, rtol=1e-4, atol=1e-4)


def test_graph_auto_falls_back_when_a_later_variant_is_not_capturable():
    """graph='auto': a graph variant first needed after the first capture (CMA-ES's late
    eigensolver schedule is one) whose step cannot be captured falls back to eager too, with
    the same result as an eager run, instead of raising to the caller."""
    from evoxmi.problems.numerical import Sphere

    class LateHostSync(A.PSO):
        late = False

        def graph_variant(self, generation):
            self.late = generation >= 3
            return "late" if self.late else None

        def tell(self, state, fitness):
            if self.late:
                fitness.sum().item()  # a host read: not capturable
            return super().tell(state, fitness)

    def run(graph):
        lb, ub = -torch.ones(8, device="cuda"), torch.ones(8, device="cuda")
        wf = StdWorkflow(LateHostSync(lb, ub, 64), Sphere(), graph=graph)
        st = wf.init(rnd.PRNGKey(4, device="cuda"))
        for _ in range(6):
            st = wf.step(st)
        torch.cuda.synchronize()
        return wf, st.get_child_state("algorithm")

    _, a = run(False)
    with pytest.warns(UserWarning, match="not capturable"):
        wf, b = run("auto")
    assert wf._graph_failed
    assert torch.allclose(a.population, b.population, rtol=1e-6, atol=1e-6)
