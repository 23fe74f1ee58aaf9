"""Neuroevolution: ports of the reference's tests/test_neuroevolution.py (supervised
loss on a dataset — an in-memory synthetic Fashion-MNIST-shaped set replaces the
TFDS download) and tests/test_gym.py (CartPole through the Gym problem with CSO; the
reference's "== 40.0" value depends on flax initialisation and is parity-unpinned),
plus the Brax-style Ant: environment invariants, and OpenES improving the return."""
import math

import pytest
import torch

from evoxmi import random as rnd
from evoxmi.algorithms import CSO, PGPE, OpenES
from evoxmi.models import MLPPolicy
from evoxmi.monitors import EvalMonitor, StdSOMonitor
from evoxmi.problems.neuroevolution import Brax, Gym, TensorflowDataset, get_environment
from evoxmi.utils import TreeAndVector, rank_based_fitness
from evoxmi.workflows import StdWorkflow


def test_supervised_dataset_problem():
    g = torch.Generator().manual_seed(0)
    images = torch.randint(0, 256, (512, 28, 28, 1), generator=g).to(torch.uint8)
    labels = (images[:, ::4, ::4, 0].float().mean((1, 2)) > 127).long() * 9
    model = MLPPolicy([49, 16, 10], activation="relu", output_activation=None)
    params = model.init(rnd.PRNGKey(1))

    def loss_func(w, data):
        x = data["image"][:, ::4, ::4, 0].reshape(data["image"].shape[0], -1).float() / 255.0
        h = torch.relu(x @ w["layer0"]["w"] + w["layer0"]["b"])
        out = torch.softmax(h @ w["layer1"]["w"] + w["layer1"]["b"], -1)
        return ((out - torch.nn.functional.one_hot(data["label"], 10)) ** 2).mean()

    problem = TensorflowDataset({"image": images, "label": labels}, batch_size=8, loss_func=loss_func)
    adapter = TreeAndVector(params)
    mon = EvalMonitor()
    wf = StdWorkflow(PGPE(64, adapter.to_vector(params), optimizer="adam", stdev_init=0.1), problem,
                     sol_transforms=[adapter.batched_to_tree], fit_transforms=[rank_based_fitness], monitors=[mon])
    st = wf.init(rnd.PRNGKey(42))
    for _ in range(3):
        st = wf.step(st)
    best = float(mon.get_best_fitness())
    assert 0.0 < best < 0.1  # loss of a 10-way softmax against one-hot targets


@pytest.mark.parametrize("batch_policy", [True, False])
def test_cartpole(batch_policy):
    model = MLPPolicy([4, 32, 2], activation="sigmoid", output_activation=None)
    params = model.init(rnd.PRNGKey(0))
    adapter = TreeAndVector(params)
    center = adapter.to_vector(params)
    policy = model.apply if batch_policy else (lambda w, x: model.apply(torch.utils._pytree.tree_map(lambda t: t[None], w), x[None])[0])
    problem = Gym(env_name="CartPole-v1", policy=policy, num_workers=3, batch_policy=batch_policy, cap_episode=500)
    mon = StdSOMonitor()
    wf = StdWorkflow(CSO(lb=torch.full_like(center, -10.0), ub=torch.full_like(center, 10.0), mean=center, stdev=1.0, pop_size=16),
                     problem, monitors=[mon], jit_problem=False, num_objectives=1, sol_transforms=[adapter.batched_to_tree],
                     opt_direction="max")
    st = wf.init(rnd.PRNGKey(42))
    for _ in range(27):
        st = wf.step(st)
    assert float(mon.get_best_fitness()) >= 100.0  # the pole is balanced for 100+ steps


def test_ant_env_invariants():
    env = get_environment("ant")
    s, o = env.reset(rnd.PRNGKey(0), 3)
    assert o.shape == (3, 27) and torch.equal(o[0], o[1])  # same key ⇒ identical copies
    for _ in range(100):
        s, o, r, d = env.step(s, torch.zeros(3, 8))
    assert torch.isfinite(s).all() and not d.any()
    assert 0.3 < float(s[0, 2]) < 0.8  # stands on its legs with zero torque
    assert torch.allclose(s[:, 3:7].norm(dim=1), torch.ones(3), atol=1e-5)


def test_ant_mass_matrix_momenta_and_coriolis_match_autograd():
    """The closed-form generalized momenta π = M(q)u (torso and hinges) and the velocity-product
    terms ∂T/∂q of the articulated Ant equal autograd derivatives of the kinetic energy
    assembled independently from the link velocities."""
    from evoxmi.problems.neuroevolution.reinforcement_learning import envs

    env = envs.Ant()
    g = torch.Generator().manual_seed(0)
    f64 = dict(dtype=torch.float64)
    jq = (torch.tensor([0, 1, 0, -1, 0, -1, 0, 1.0], **f64) + 0.3 * torch.randn(5, 8, generator=g, **f64)).requires_grad_(True)
    vB, wB = torch.randn(5, 3, generator=g, **f64).requires_grad_(True), torch.randn(5, 3, generator=g, **f64).requires_grad_(True)
    phid, ad = torch.randn(5, 4, generator=g, **f64).requires_grad_(True), torch.randn(5, 4, generator=g, **f64).requires_grad_(True)
    T = env.kinetic_energy(jq, vB, wB, phid, ad)
    gq, gv, gw, gp, ga = torch.autograd.grad(T.sum(), [jq, vB, wB, phid, ad])
    k = env._kin(jq.detach())
    hB, pphi, pa = env._momenta(k, vB.detach(), wB.detach(), phid.detach(), ad.detach())
    torch.testing.assert_close(hB, torch.cat([gv, gw], -1), rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(pphi, gp, rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(pa, ga, rtol=1e-10, atol=1e-10)
    dphi, da = env._dTdq(k, vB.detach(), wB.detach(), phid.detach(), ad.detach())
    torch.testing.assert_close(dphi, gq[:, 0::2], rtol=1e-10, atol=1e-10)
    torch.testing.assert_close(da * k["sg"], gq[:, 1::2], rtol=1e-10, atol=1e-10)
    # M is symmetric positive definite: 2T = uᵀMu > 0
    assert bool((T > 0).all())


@pytest.mark.parametrize("dtype,tol", [(torch.float64, 1e-9), (torch.float32, 1e-4)])
def test_ant_momentum_conserved_without_external_forces(dtype, tol):
    """Zero gravity, no contacts, no body damping, random joint torques (joint damping and limit
    springs are internal): total linear momentum and angular momentum about the world origin are
    conserved over 200 control steps (1000 sub-steps), to rounding."""
    from evoxmi.problems.neuroevolution.reinforcement_learning import envs

    env = envs.Ant()
    env.P = dict(envs.ANT, gravity=0.0, ang_damp=0.0, lin_damp=0.0, k_contact=0.0, c_contact=0.0, z0=5.0)
    s, _ = env.reset(rnd.PRNGKey(0), 4)
    s = s.to(dtype)
    s[:, 7:13] += torch.randn(4, 6, generator=torch.Generator().manual_seed(1)).to(dtype)
    P0, L0 = env.momentum(s)
    g = torch.Generator().manual_seed(2)
    for _ in range(200):
        s, _, _, _ = env.step(s, (torch.rand(4, 8, generator=g) * 2 - 1).to(dtype))
    P1, L1 = env.momentum(s)
    assert torch.isfinite(s).all()
    assert float((P1 - P0).norm(dim=1).max()) <= tol * float(P0.norm(dim=1).max())
    assert float((L1 - L0).norm(dim=1).max()) <= tol * float(L0.norm(dim=1).max())
    assert float(s[:, 21:29].abs().max()) > 0.1  # the legs did move


def test_ant_joint_torques_react_on_the_torso():
    """In free fall at rest, driving every hip one way turns the legs that way and the torso the
    other way, with zero total angular momentum."""
    from evoxmi.problems.neuroevolution.reinforcement_learning import envs

    env = envs.Ant()
    env.P = dict(envs.ANT, gravity=0.0, ang_damp=0.0, lin_damp=0.0, joint_damping=0.0, z0=5.0)
    s, _ = env.reset(rnd.PRNGKey(0), 1)
    s = s.double()
    s[:, 7:] = 0.0  # at rest
    s[:, 13:21] = torch.tensor([0.0, 1.0, 0.0, -1.0, 0.0, -1.0, 0.0, 1.0], dtype=torch.float64)
    for _ in range(6):
        s, _, _, _ = env.step(s, torch.tensor([[0.2, 0.0] * 4], dtype=torch.float64))
    assert float(s[0, 21]) > 0 and float(s[0, 12]) < 0
    _, L = env.momentum(s)
    assert float(L.abs().max()) < 1e-9


def test_openes_ant_improves():
    """The centre policy's episode return (not the monotone best-so-far) must improve
    after OpenES generations on the native Ant."""
    policy = MLPPolicy([27, 16, 16, 8])
    params = policy.init(rnd.PRNGKey(1))
    adapter = TreeAndVector(params)
    problem = Brax(policy, "ant", cap_episode=60)
    algo = OpenES(adapter.to_vector(params), 64, learning_rate=0.01, noise_stdev=0.02, optimizer="adam")
    wf = StdWorkflow(algo, problem, sol_transforms=[adapter.batched_to_tree], fit_transforms=[rank_based_fitness], opt_direction="max")
    st = wf.init(rnd.PRNGKey(3))

    def centre_return(st):
        centre = st.get_child_state("algorithm").center
        ret, _ = problem.evaluate(st.get_child_state("problem"), adapter.batched_to_tree(centre[None, :]))
        return float(ret[0])

    before = centre_return(st)
    for _ in range(15):
        st = wf.step(st)
    after = centre_return(st)
    assert math.isfinite(before) and after > 1.5 * before, (before, after)


def test_normalizer_running_statistics():
    from evoxmi.problems.neuroevolution.reinforcement_learning import Normalizer

    n = Normalizer()
    st = n.init(rnd.PRNGKey(0))
    torch.manual_seed(0)
    a, b = torch.randn(50, 3) * 4 + 1, torch.randn(30, 3) * 4 + 1
    _, st = n.normalize_obvs(st, a)
    out, st = n.normalize_obvs(st, b)
    allx = torch.cat([a, b])
    ref = (b - allx.mean(0)) / allx.std(0, unbiased=False)
    assert torch.allclose(out, ref, atol=1e-4)


def test_gym_host_env_workers_match_sequential():
    """Host environments stepped by 3 worker processes (the reference's Ray actors) give the
    same returns as one worker; the policy runs batched in the controller."""
    from evoxmi.problems.neuroevolution.reinforcement_learning import Gym
    from evoxmi.problems.neuroevolution.reinforcement_learning.host_envs import PyCartPole

    torch.manual_seed(0)
    W = torch.randn(7, 4, 2)

    def policy(w, obs):
        return torch.einsum("no,noa->na", obs, w)

    out = []
    for nw in (1, 3):
        prob = Gym(policy, num_workers=nw, env_creator=PyCartPole, batch_policy=True, cap_episode=200)
        st = prob.init(rnd.PRNGKey(4))
        r, _ = prob.evaluate(st, W)
        out.append(r)
    assert torch.equal(out[0], out[1]) and float(out[0].max()) > 9
