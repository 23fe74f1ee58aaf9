"""Brax-compatible neuroevolution problem (reference ``reinforcement_learning/brax.py:11-109``).

``Brax(policy, env_name, cap_episode)``: every individual's policy controls its own
copy of the environment, all copies reset from the same key (as the reference tiles
one key, ``brax.py:54``), and the fitness is the episode return.  Brax itself is not
part of this stack: ``env_name`` resolves to the native batched environments of
:mod:`.envs` (``"ant"`` is a Brax-style re-implementation, see there).

Execution paths:

* **fused** (``"ant"`` + :class:`~evoxmi.models.MLPPolicy` 27-h1-h2-8 tanh, on a GPU):
  one persistent HIP kernel runs whole episodes with each individual's weights held
  in LDS (``ops.neuro.ant_rollout``);
* **generic**: a device-resident loop of batched policy forward + batched env step;
  the all-done early exit is checked every ``check_every`` steps to avoid per-step
  host synchronisation.

Returns are accumulated as ``(1 − done) · reward`` with *sticky* termination (an
individual stops earning after its first terminal step; the reference keeps
stepping terminated Brax states and can re-admit rewards).
"""
from __future__ import annotations

from typing import Callable

import torch

from ....core import Problem, State
from ....models.mlp import MLPPolicy
from ....ops import neuro as neuro_ops
from .envs import Ant, get_environment


class Brax(Problem):
    def __init__(self, policy: Callable, env_name: str, cap_episode: int, backend: str = None, fused: bool = True, check_every: int = 16):
        super().__init__()
        self.policy = policy
        self.env_name = env_name
        self.backend = backend
        self.env = get_environment(env_name)
        self.cap_episode = cap_episode
        self.fused = fused
        self.check_every = check_every
        self._s0 = None

    def setup(self, key):
        return State(key=key)

    def _fused_ok(self, weights):
        return (self.fused and isinstance(self.env, Ant) and isinstance(self.policy, MLPPolicy) and len(self.policy.sizes) == 4
                and self.policy.sizes[0] == 27 and self.policy.sizes[-1] == 8 and self.policy.activation == "tanh"
                and self.policy.output_activation == "tanh" and isinstance(weights, dict)
                and next(iter(weights.values()))["w"].is_cuda)

    def _initial_state(self, key, device):
        """The reset state (one row; every individual starts from it).  The problem key
        never changes (reference ``brax.py:53-54`` resets from ``state.key`` and returns
        ``state`` unchanged), so the reset is computed once — the key is read on the
        host only then — and reused, including inside a captured hipGraph (whose
        warm-up step always runs eagerly on the same state first)."""
        c = self._s0
        if c is not None and (c[0] is key or (key.is_cuda and torch.cuda.is_current_stream_capturing())):
            return c[1]
        s0, _ = self.env.reset(key.cpu(), 1)
        s0 = s0[0].to(device)
        self._s0 = (key, s0)
        return s0

    def evaluate(self, state, weights):
        if self._fused_ok(weights):
            w = self.policy.flat(weights)
            s0 = self._initial_state(state.key, w.device)
            h1, h2 = self.policy.sizes[1], self.policy.sizes[2]
            ret, steps = neuro_ops.ant_rollout(w, h1, h2, s0, self.cap_episode)
            self.last_episode_lengths = steps  # diagnostics only (not part of the state)
            return ret, state
        leaves = [x for x in torch.utils._pytree.tree_leaves(weights) if isinstance(x, torch.Tensor)]
        n, dev = leaves[0].shape[0], leaves[0].device
        s, obs = self.env.reset(state.key.cpu(), n)
        s, obs = s.to(dev), obs.to(dev)
        total = torch.zeros(n, device=dev)
        alive = torch.ones(n, dtype=torch.bool, device=dev)
        for t in range(self.cap_episode):
            act = self.policy(weights, obs)
            s, obs, r, done = self.env.step(s, act)
            alive = alive & ~done
            total = total + alive.to(total.dtype) * r
            if (t + 1) % self.check_every == 0 and not bool(alive.any()):
                break
        return total, state

    def visualize(self, key, weights, output_type: str = "trajectory", respect_done=False, **kwargs):
        """Roll out one policy and return its state trajectory (list of (state_dim,)
        tensors); Brax's HTML renderer is not available here."""
        s, obs = self.env.reset(key.cpu(), 1)
        traj = [s[0].clone()]
        for _ in range(self.cap_episode):
            act = self.policy(torch.utils._pytree.tree_map(lambda x: x[None] if x.dim() < 3 else x, weights), obs)
            s, obs, _, done = self.env.step(s, act)
            traj.append(s[0].clone())
            if respect_done and bool(done[0]):
                break
        return traj
