"""Gym-style neuroevolution problem (reference ``reinforcement_learning/gym.py:284-426``).

The reference runs CPU gymnasium environments in Ray worker actors and evaluates
the policy in a controller actor.  Here:

* with an ``env_creator`` (or ``env_name`` when ``gymnasium`` is importable) the host
  environments are stepped in ``num_workers`` parallel worker processes
  (:class:`.host_envs.EnvWorkers`, the reference's Ray worker actors), the policy runs
  batched on the policy device (the controller);
* otherwise (this image) the native batched re-implementations of
  :mod:`.envs` are used (CartPole-v1 / Pendulum-v1 / MountainCarContinuous-v0 have
  the gymnasium dynamics), on whatever device the weights live on.

``policy(params, obs)``: with ``batch_policy=True`` it is called once with the whole
population's parameters (leading axis N); otherwise per individual.  Discrete
environments take ``argmax`` of the policy output, as the reference test's policy does.
Fitness = episode return (``mo_keys`` → several objectives from ``info``, host path).
"""
from __future__ import annotations

from typing import Callable, List, Optional

import torch

from ....core import Problem, State, Stateful
from .envs import get_environment

try:  # pragma: no cover - not installed in this image
    import gymnasium as _gym
except Exception:  # noqa: BLE001
    _gym = None


class Normalizer(Stateful):
    """Running observation normaliser (reference ``gym.py:21-56``, unused there).

    Keeps Σx, Σx² and the count in the state; ``std = sqrt(max(E[x²] − mean², 1e-2))``.
    The reference unpacks ``mean``/``std`` in the wrong order (``:33-34``) — here
    both methods return ``(value, state)`` consistently."""

    def setup(self, key):
        return State(sum=torch.zeros(()), sumOfSquares=torch.zeros(()), count=torch.zeros(()))

    def mean(self, state):
        return state.sum / state.count, state

    def std(self, state):
        m = state.sum / state.count
        return torch.sqrt(torch.clamp(state.sumOfSquares / state.count - m * m, min=1e-2)), state

    def normalize(self, state, x):
        state = state.update(count=state.count + 1, sum=state.sum + x, sumOfSquares=state.sumOfSquares + x * x)
        mean, state = self.mean(state)
        std, state = self.std(state)
        return (x - mean) / std, state

    def normalize_obvs(self, state, obvs):
        state = state.update(count=state.count + obvs.shape[0], sum=state.sum + obvs.sum(0),
                             sumOfSquares=state.sumOfSquares + (obvs * obvs).sum(0))
        mean, state = self.mean(state)
        std, state = self.std(state)
        return (obvs - mean) / std, state


class CapEpisode:
    """Adaptive episode cap (reference ``gym.py:267-282``)."""

    def __init__(self, init_cap=100):
        self.cap = init_cap

    def update(self, episode_lengths):
        self.cap = max(self.cap, int(2 * float(torch.as_tensor(episode_lengths, dtype=torch.float32).median())))
        return self.cap


class Gym(Problem):
    def __init__(self, policy: Callable, num_workers: int = 1, env_name: Optional[str] = None, env_options: dict = None,
                 env_creator: Optional[Callable] = None, mo_keys: List = (), controller_options: dict = None,
                 worker_options: dict = None, init_cap: Optional[int] = None, batch_policy: bool = False, cap_episode: int = 1000):
        super().__init__()
        self.policy, self.num_workers, self.env_name = policy, num_workers, env_name
        self.env_options = env_options or {}
        self.env_creator = env_creator
        self.mo_keys = list(mo_keys)
        self.batch_policy = batch_policy
        self.cap_episode = init_cap or cap_episode
        self.native = None
        if env_creator is None and (_gym is None or env_name is not None):
            try:
                self.native = get_environment(env_name)
            except ValueError:
                if _gym is None:
                    raise ImportError(f"gymnasium is not installed and {env_name!r} has no native implementation")

    def setup(self, key):
        return State(key=key)

    def _act(self, weights, obs, n):
        if self.batch_policy:
            return self.policy(weights, obs)
        outs = []
        for i in range(n):
            w = torch.utils._pytree.tree_map(lambda x: x[i], weights)
            outs.append(self.policy(w, obs[i]))
        return torch.stack(outs)

    def evaluate(self, state, weights):
        leaves = [x for x in torch.utils._pytree.tree_leaves(weights) if isinstance(x, torch.Tensor)]
        n, dev = leaves[0].shape[0], leaves[0].device
        if self.native is not None:
            env = self.native
            s, obs = env.reset(state.key.cpu(), n)
            s, obs = s.to(dev), obs.to(dev)
            total = torch.zeros(n, device=dev)
            alive = torch.ones(n, dtype=torch.bool, device=dev)
            for _ in range(self.cap_episode):
                out = self._act(weights, obs, n)
                if env.discrete and out.dim() == 1:
                    out = torch.nn.functional.one_hot(out.long(), env.act_dim).to(obs.dtype)
                s, obs, r, done = env.step(s, out)
                total = total + alive.to(total.dtype) * r  # the step that ends the episode still pays (gym semantics)
                alive = alive & ~done
                if not bool(alive.any()):
                    break
            return total, state
        return self._host_rollout(state, weights, n, dev)  # pragma: no cover

    def _host_rollout(self, state, weights, n, dev):
        from .host_envs import EnvWorkers

        creator = self.env_creator
        if creator is None:  # pragma: no cover - requires gymnasium
            name, opts = self.env_name, self.env_options
            creator = _GymCreator(name, opts)
        discrete = bool(getattr(creator, "discrete", True))
        workers = EnvWorkers(creator, n, self.num_workers, self.mo_keys, discrete=discrete)
        try:
            seed = int(state.key[1])
            obs = torch.as_tensor(workers.reset(seed)).to(dev)
            total = torch.zeros(n, len(self.mo_keys) or 1)
            alive = torch.ones(n, dtype=torch.bool)
            for _ in range(self.cap_episode):
                act = self._act(weights, obs, n).detach().cpu().numpy()
                o, r, done = workers.step(act)
                total += alive[:, None].to(total.dtype) * torch.as_tensor(r)
                alive &= ~torch.as_tensor(done)
                obs = torch.as_tensor(o).to(dev)
                if not bool(alive.any()):
                    break
        finally:
            workers.close()
        out = total.to(dev)
        return (out[:, 0] if not self.mo_keys else out), state


class _GymCreator:  # pragma: no cover - requires gymnasium
    def __init__(self, name, opts):
        self.name, self.opts = name, opts

    def __call__(self):
        return _gym.make(self.name, **self.opts)
