"""EnvPool problem (reference ``reinforcement_learning/env_pool.py:15-80``).

The reference drives ``envpool.make(env_name, num_envs, env_type="gymnasium")`` — one
C++-vectorised environment holding the whole population — through host callbacks: seed,
reset, then ``step`` with the vmapped policy's actions until every environment is done
(or the cap), accumulating rewards under the done mask.  envpool is not part of this
stack; :func:`make` returns :class:`NativeEnvPool`, the same batched API
(``seed`` / ``reset`` / ``step`` → ``(obs, reward, terminated, truncated, info)``) over
the native device-resident environments of :mod:`.envs`, so the loop below is the
reference's loop with no per-step host round trip.
"""
from __future__ import annotations

from typing import Callable, Optional

import torch

from ....core import Problem, State
from ....ops import random as rnd
from .envs import get_environment


class NativeEnvPool:
    """``num_envs`` copies of a native environment with the envpool/gymnasium batch API."""

    def __init__(self, env_name: str, num_envs: int, device=None, **env_options):
        self.env = get_environment(env_name, **env_options)
        self.num_envs = num_envs
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._seed = 0
        self._s = None

    def seed(self, seed):
        self._seed = int(torch.as_tensor(seed).reshape(-1)[0])

    def reset(self, env_ids=None):
        self._s, obs = self.env.reset(rnd.PRNGKey(self._seed), self.num_envs)
        self._s = self._s.to(self.device)
        return obs.to(self.device), {}

    def step(self, action):
        a = torch.as_tensor(action, device=self.device)
        if self.env.discrete and a.dim() == 1:
            a = torch.nn.functional.one_hot(a.long(), self.env.act_dim).to(torch.float32)
        self._s, obs, reward, done = self.env.step(self._s, a.to(torch.float32))
        return obs, reward, done, torch.zeros_like(done), {}


def make(env_name: str, num_envs: int, env_type: str = "gymnasium", device=None, **env_options) -> NativeEnvPool:
    """envpool.make stand-in (only the gymnasium-style batched API)."""
    if env_type not in ("gymnasium", "gym"):
        raise ValueError(f"env_type {env_type!r} is not supported")
    return NativeEnvPool(env_name, num_envs, device=device, **env_options)


class EnvPool(Problem):
    def __init__(self, policy: Callable, env_name: str, num_envs: int, env_options: dict = None,
                 cap_episode_length: Optional[int] = None, device=None):
        super().__init__()
        self.policy = policy
        self.batch_policy = torch.func.vmap(policy)  # the reference's jit(vmap(policy))
        self.num_envs = num_envs
        self.env = make(env_name, num_envs=num_envs, env_type="gymnasium", device=device, **(env_options or {}))
        self.cap_episode_length = cap_episode_length

    def setup(self, key):
        return State(key=key)

    def evaluate(self, state, pop):
        key, subkey = rnd.split(state.key)
        self.env.seed(rnd.randint(subkey, (1,), 0, 2**31 - 1))
        leaves = [x for x in torch.utils._pytree.tree_leaves(pop) if isinstance(x, torch.Tensor)]
        self.env.device = leaves[0].device
        obs, _ = self.env.reset(None)
        done = torch.zeros(self.num_envs, dtype=torch.bool, device=obs.device)
        total = torch.zeros(self.num_envs, device=obs.device)
        i = 0
        while (self.cap_episode_length is None or i < self.cap_episode_length) and not bool(done.all()):
            action = self.batch_policy(pop, obs)
            obs, reward, terminated, truncated, _ = self.env.step(action)
            total = total + (~done).to(total.dtype) * reward
            done = done | (terminated | truncated)
            i += 1
        return total, state.update(key=key)
