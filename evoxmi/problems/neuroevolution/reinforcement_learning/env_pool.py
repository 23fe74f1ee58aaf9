"""EnvPool adapter (reference ``reinforcement_learning/env_pool.py:15-80``).

EnvPool is not part of this stack; with the same constructor the problem runs the
native batched environments (which is what EnvPool provides: one vectorised env
for the whole population), entirely on the device — no per-step host callback.
"""
from __future__ import annotations

from .gym import Gym


class EnvPool(Gym):
    def __init__(self, policy, env_name: str, env_options: dict = None, cap_episode: int = 1000, batch_policy: bool = True):
        super().__init__(policy, 1, env_name=env_name, env_options=env_options, batch_policy=batch_policy, cap_episode=cap_episode)
