"""Port of the reference's tests/test_multi_objective_algorithms.py: every MOEA runs 10
generations on DTLZ1 (m = 3, d = 12, N = 100) through StdWorkflow; the reference only
checks that it runs — here the final front must also be finite with a finite IGD."""
import pytest
import torch

import evoxmi.algorithms as A
from evoxmi import random as rnd
from evoxmi.metrics import IGD
from evoxmi.monitors import EvalMonitor
from evoxmi.problems.numerical import DTLZ1, DTLZ2
from evoxmi.workflows import StdWorkflow

N, M, POP_SIZE, ITER = 12, 3, 100, 10
LB, UB = torch.zeros(N), torch.ones(N)


def run_moea(algorithm, problem=None, iters=ITER):
    problem = problem if problem is not None else DTLZ1(m=M)
    wf = StdWorkflow(algorithm=algorithm, problem=problem)
    state = wf.init(rnd.PRNGKey(42))
    for _ in range(iters):
        state = wf.step(state)
    fit = state.get_child_state("algorithm").fitness
    fit = fit[~torch.isnan(fit).any(1)]
    assert fit.shape[0] > 0 and torch.isfinite(fit).all()
    return float(IGD(problem.pf())(fit))


ALGOS = {
    "IBEA": lambda: A.IBEA(LB, UB, M, POP_SIZE), "MOEAD": lambda: A.MOEAD(LB, UB, M, POP_SIZE),
    "NSGA2": lambda: A.NSGA2(LB, UB, M, POP_SIZE), "RVEA": lambda: A.RVEA(LB, UB, M, POP_SIZE),
    "NSGA3": lambda: A.NSGA3(LB, UB, M, POP_SIZE), "EAGMOEAD": lambda: A.EAGMOEAD(LB, UB, M, POP_SIZE),
    "HypE": lambda: A.HypE(LB, UB, M, POP_SIZE), "MOEADDRA": lambda: A.MOEADDRA(LB, UB, M, POP_SIZE),
    "SPEA2": lambda: A.SPEA2(LB, UB, M, POP_SIZE), "GDE3": lambda: A.GDE3(LB, UB, M, POP_SIZE),
    "BiGE": lambda: A.BiGE(LB, UB, M, POP_SIZE), "KnEA": lambda: A.KnEA(LB, UB, M, POP_SIZE),
    "SRA": lambda: A.SRA(LB, UB, M, POP_SIZE), "TDEA": lambda: A.TDEA(LB, UB, M, POP_SIZE),
    "LMOCSO": lambda: A.LMOCSO(M, LB, UB, POP_SIZE), "RVEAa": lambda: A.RVEAa(LB, UB, M, POP_SIZE),
    "BCEIBEA": lambda: A.BCEIBEA(LB, UB, M, POP_SIZE), "MOEADM2M": lambda: A.MOEADM2M(LB, UB, M, POP_SIZE),
    "IMMOEA": lambda: A.IMMOEA(LB, UB, M, 105),
}


@pytest.mark.parametrize("name", sorted(ALGOS))
def test_moea_runs(name):
    assert run_moea(ALGOS[name]()) < float("inf")


# IGD on DTLZ2 (m = 3, d = 12, N = 100) after 100 generations, seed 42 (measured:
# BCEIBEA .055, BiGE .071, EAGMOEAD .239, GDE3 .083, HypE .104, IBEA .079, IMMOEA .109,
# KnEA .061, LMOCSO .067, MOEAD .055, MOEADDRA .083, MOEADM2M .135, NSGA2 .075, NSGA3 .054,
# RVEA .055, RVEAa .065, SPEA2 .058, SRA .088, TDEA .054).  Bounds are 0.1 except where the
# algorithm's design limits it on this front: EAG-MOEA/D decomposes with a *weighted sum*
# (reference eagmoead.py:79), which cannot reach the concave parts of the DTLZ2 front;
# M2M splits N = 100 over regional subpopulations; HypE's Monte-Carlo HV and IM-MOEA's
# inverse models converge more slowly in 100 generations.
IGD_BOUND = {"EAGMOEAD": 0.3, "MOEADM2M": 0.2, "HypE": 0.15, "IMMOEA": 0.15}


@pytest.mark.parametrize("name", sorted(ALGOS))
def test_moea_converges_dtlz2(name):
    algo = ALGOS[name]()
    assert run_moea(algo, DTLZ2(d=N, m=M), iters=100) < IGD_BOUND.get(name, 0.1)


def test_moead_scan_gpu_semantics_cpu_oracle():
    from evoxmi.ops.mo import moead_scan

    g = torch.Generator().manual_seed(0)
    objs, off = torch.rand(20, 3, generator=g), torch.rand(20, 3, generator=g) * 0.8
    P = torch.randint(0, 20, (20, 4), generator=g)
    W = torch.rand(20, 3, generator=g) + 0.1
    owner, o, z = moead_scan(objs, off, P, W, torch.zeros(3), "tchebycheff", nr=2, update_z=True)
    assert (owner >= -1).all() and torch.equal(o[owner >= 0], off[owner[owner >= 0]])


def test_immoea_gp_fit_matches_gp_regression():
    """IM-MOEA's batched closed-form fit reproduces GPRegression(Linear) + Adam(1e-3) × 250
    (the reference's inverse-model fit, im_moea.py:310-314)."""
    from evoxmi.algorithms.mo.im_moea import linear_gp_fit
    from evoxmi.operators.gaussian_process import GPRegression
    from evoxmi.operators.gaussian_process.kernels import Linear
    from evoxmi.utils import optim

    sp = torch.nn.functional.softplus
    g = torch.Generator().manual_seed(0)
    stats, ref = [], []
    for slope, noise, n in ((0.7, 0.3, 40), (-1.5, 0.05, 12), (0.0, 2.0, 25)):
        f = torch.rand(n, generator=g, dtype=torch.float64) * 3
        x = slope * f + noise * torch.randn(n, generator=g, dtype=torch.float64)
        m = GPRegression(kernel=Linear()).fit(f[:, None], x, optimzer=optim.adam(1e-3))
        ref.append((float(sp(m._u["k_variance"])), float(sp(m._u["obs_stddev"])) ** 2))
        stats.append(((f * f).sum(), (f * x).sum(), (x * x).sum(), float(n)))
    a, b, c, n = (torch.tensor([s[i] for s in stats], dtype=torch.float64) for i in range(4))
    v, s2 = linear_gp_fit(a, b, c, n)
    for i, (rv, rs2) in enumerate(ref):
        assert abs(float(v[i]) - rv) < 1e-4 and abs(float(s2[i]) - rs2) < 1e-4
