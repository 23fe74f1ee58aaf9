"""Host-adapter problems whose external packages are not in this image (reference
``tests/test_evoxbench.py`` skips for the database download, ``tests/test_envpool.py``
needs envpool): EvoXBench is driven through a stand-in benchmark object with the same
interface, EnvPool through its native batched-environment backend."""
import numpy as np
import torch

from evoxmi import random as rnd


class _FakeBench:
    """EvoXBench interface: ``search_space.{lb,ub}``, ``evaluator.n_objs``, ``evaluate(X)``
    (numpy in/out; the real benchmark samples noise from the global numpy RNG)."""

    class search_space:
        lb = np.zeros(6)
        ub = np.array([3, 3, 3, 2, 2, 2])

    class evaluator:
        n_objs = 2

    def __init__(self):
        self.calls = []

    def evaluate(self, X):
        self.calls.append(X.shape)
        noise = np.random.rand(X.shape[0], 1) * 1e-3
        return np.stack([X.sum(1), (self.search_space.ub - X).sum(1)], 1) + noise


def test_evoxbench_problem_interface_and_seeding():
    from evoxmi.algorithms import NSGA2
    from evoxmi.problems.evoxbench import EvoXBenchProblem
    from evoxmi.workflows import StdWorkflow

    outs = []
    for _ in range(2):
        bench = _FakeBench()
        prob = EvoXBenchProblem(bench)
        assert prob.n_objs == 2 and prob.ub.tolist() == [3, 3, 3, 2, 2, 2]
        algo = NSGA2(prob.lb.float(), prob.ub.float(), 2, 16)
        wf = StdWorkflow(algo, prob, jit_problem=False, num_objectives=2)
        st = wf.init(rnd.PRNGKey(0))
        for _ in range(3):
            st = wf.step(st)
        assert bench.calls and all(c == (16, 6) for c in bench.calls)
        outs.append(st.get_child_state("algorithm").fitness.clone())
    assert torch.equal(outs[0], outs[1])  # the benchmark's numpy noise is seeded from the problem key


def test_envpool_cartpole_runs_on_native_batched_env():
    from evoxmi.algorithms import PGPE
    from evoxmi.models import MLPPolicy
    from evoxmi.problems.neuroevolution import EnvPool
    from evoxmi.utils import TreeAndVector
    from evoxmi.workflows import StdWorkflow

    policy = MLPPolicy([4, 8, 2])
    params = policy.init(rnd.PRNGKey(1))
    tv = TreeAndVector(params)
    results = []
    for _ in range(2):
        prob = EnvPool(policy, "CartPole-v1", num_envs=16, cap_episode_length=200)
        wf = StdWorkflow(PGPE(16, tv.to_vector(params), optimizer="adam"), prob, sol_transforms=[tv.batched_to_tree],
                         opt_direction="max")
        st = wf.init(rnd.PRNGKey(2))
        for _ in range(3):
            st = wf.step(st)
        results.append(st.get_child_state("algorithm").center.clone())
    assert torch.isfinite(results[0]).all() and torch.equal(results[0], results[1])


def test_envpool_loop_matches_manual_rollout():
    """The reference's EnvPool loop (seed, reset, vmapped policy, masked reward sum until all
    done) over the envpool-style batched API."""
    from evoxmi.models import MLPPolicy
    from evoxmi.problems.neuroevolution import EnvPool
    from evoxmi.problems.neuroevolution.reinforcement_learning.env_pool import make
    from evoxmi.utils import TreeAndVector

    policy = MLPPolicy([4, 8, 2])
    params = policy.init(rnd.PRNGKey(1))
    tv = TreeAndVector(params)
    pop = tv.to_vector(params) + 0.5 * torch.randn(8, tv.to_vector(params).numel(), generator=torch.Generator().manual_seed(0))
    tree = tv.batched_to_tree(pop)
    prob = EnvPool(policy, "CartPole-v1", num_envs=8, cap_episode_length=150)
    st = prob.init(rnd.PRNGKey(3))
    ret, _ = prob.evaluate(st, tree)
    # manual replay with the same seed
    _, sub = rnd.split(st.key)
    env = make("CartPole-v1", 8)
    env.seed(rnd.randint(sub, (1,), 0, 2**31 - 1))
    obs, _ = env.reset()
    done = torch.zeros(8, dtype=torch.bool)
    tot = torch.zeros(8)
    for _ in range(150):
        a = torch.stack([policy(torch.utils._pytree.tree_map(lambda x: x[i], tree), obs[i]) for i in range(8)])
        obs, r, term, trunc, _ = env.step(a)
        tot += (~done).float() * r
        done |= term | trunc
        if done.all():
            break
    assert torch.allclose(ret, tot) and float(ret.max()) >= 9
