"""Run-to-run bitwise reproducibility on the GPU as the race detector (GPU
sanitizers are unavailable on this pool).  A kernel with a data race, an uninitialised
read or order-dependent atomics shows up as two identical runs diverging; the replicated
state of the sharded paths relies on the same property across ranks."""
import pytest
import torch

from evoxmi import random as rnd

pytestmark = pytest.mark.gpu


def _twice(make, steps, read):
    outs = []
    for _ in range(2):
        wf = make()
        st = wf.init(rnd.PRNGKey(123, device="cuda"))
        for _ in range(steps):
            st = wf.step(st)
        torch.cuda.synchronize()
        outs.append([t.detach().clone() for t in read(st)])
    return outs


def _assert_same(outs):
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_cmaes_sbr_graph_runs_bit_identical():
    from evoxmi.algorithms import CMAES
    from evoxmi.problems.numerical import CEC2022TestSuit
    from evoxmi.workflows import StdWorkflow

    def make():
        return StdWorkflow(CMAES(torch.zeros(300, device="cuda") + 5, 10.0, pop_size=2000), CEC2022TestSuit.create(1), graph=True)

    _assert_same(_twice(make, 12, lambda st: (st.get_child_state("algorithm").mean, st.get_child_state("algorithm").B)))


def test_nsga2_and_moead_runs_bit_identical():
    from evoxmi.algorithms import MOEAD, NSGA2
    from evoxmi.problems.numerical import DTLZ2, LSMOP1
    from evoxmi.workflows import StdWorkflow

    lb, ub = torch.zeros(30, device="cuda"), torch.ones(30, device="cuda")
    _assert_same(_twice(lambda: StdWorkflow(NSGA2(lb, ub, 3, 1024), DTLZ2(d=30, m=3)), 8,
                        lambda st: (st.get_child_state("algorithm").population,)))
    d = 256
    lb2 = torch.zeros(d, device="cuda")
    ub2 = torch.cat([torch.ones(2, device="cuda"), 10 * torch.ones(d - 2, device="cuda")])
    _assert_same(_twice(lambda: StdWorkflow(MOEAD(lb2, ub2, 3, 300), LSMOP1(d=d, m=3)), 8,
                        lambda st: (st.get_child_state("algorithm").population,)))


def test_openes_ant_runs_bit_identical():
    from evoxmi.algorithms import OpenES
    from evoxmi.models import MLPPolicy
    from evoxmi.problems.neuroevolution import Brax
    from evoxmi.utils import TreeAndVector
    from evoxmi.workflows import StdWorkflow

    policy = MLPPolicy([27, 64, 64, 8])
    params = policy.init(rnd.PRNGKey(1))
    tv = TreeAndVector(params)
    center = tv.to_vector(params).cuda()

    def make():
        return StdWorkflow(OpenES(center, 256, learning_rate=0.01, noise_stdev=0.05), Brax(policy, "ant", 100),
                           sol_transforms=[tv.batched_to_tree], opt_direction="max")

    _assert_same(_twice(make, 4, lambda st: (st.get_child_state("algorithm").center,)))
