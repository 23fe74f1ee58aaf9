"""Host-side (CPU, pure-Python) environments with the gymnasium API, and the worker pool
that steps them in parallel processes for :class:`.Gym` (reference ``gym.py:58-265``: Ray
worker actors own the environments, a controller evaluates the policy).

* :class:`PyCartPole` — gymnasium CartPole-v1 dynamics, ``reset(seed) -> (obs, info)``,
  ``step(a) -> (obs, reward, terminated, truncated, info)``; stands in for a gymnasium
  environment in this image (gymnasium is not installed) and in tests.
* :class:`EnvWorkers` — ``num_workers`` child processes (``spawn``: safe after the parent
  initialised the GPU — children start fresh interpreters, the parent is never replaced),
  each owning a contiguous slice of the population's environments.  Per control step
  the controller sends the slice's actions and receives observations, rewards (or the
  ``mo_keys`` info values) and done flags; finished environments are skipped.
"""
from __future__ import annotations

import math
import multiprocessing as mp
from typing import Callable, List, Sequence

import numpy as np


class PyCartPole:
    """gymnasium CartPole-v1 (Euler, τ = 0.02, ±12° / ±2.4 m, reward 1 per step)."""

    def __init__(self):
        self.state = None
        self.rng = np.random.default_rng(0)

    def reset(self, seed=None):
        if seed is not None:
            self.rng = np.random.default_rng(seed)
        self.state = self.rng.uniform(-0.05, 0.05, size=4)
        return self.state.astype(np.float32), {}

    def step(self, action):
        x, x_dot, th, th_dot = self.state
        force = 10.0 if int(action) == 1 else -10.0
        total_mass, pml = 1.1, 0.05
        ct, st = math.cos(th), math.sin(th)
        temp = (force + pml * th_dot**2 * st) / total_mass
        thacc = (9.8 * st - ct * temp) / (0.5 * (4.0 / 3.0 - 0.1 * ct**2 / total_mass))
        xacc = temp - pml * thacc * ct / total_mass
        x, x_dot = x + 0.02 * x_dot, x_dot + 0.02 * xacc
        th, th_dot = th + 0.02 * th_dot, th_dot + 0.02 * thacc
        self.state = np.array([x, x_dot, th, th_dot])
        term = bool(abs(x) > 2.4 or abs(th) > 12 * 2 * math.pi / 360)
        return self.state.astype(np.float32), 1.0, term, False, {"x": float(x)}


def _worker(conn, env_creator: Callable, n_envs: int, mo_keys: Sequence[str], discrete: bool):
    envs = [env_creator() for _ in range(n_envs)]
    alive = [True] * n_envs
    last = []
    while True:
        cmd, arg = conn.recv()
        if cmd == "reset":
            alive = [True] * n_envs
            last = [np.asarray(e.reset(seed=arg)[0], dtype=np.float32) for e in envs]
            conn.send(np.stack(last))
        elif cmd == "step":
            rew, done = [], []
            for i, e in enumerate(envs):
                if alive[i]:
                    a = arg[i]
                    o, r, term, trunc, info = e.step(int(np.argmax(a)) if discrete else a)
                    alive[i] = not (term or trunc)
                    last[i] = np.asarray(o, dtype=np.float32)
                    rew.append([float(info[k]) for k in mo_keys] if mo_keys else [float(r)])
                else:  # finished: its last observation, no reward
                    rew.append([0.0] * (len(mo_keys) or 1))
                done.append(not alive[i])
            conn.send((np.stack(last), np.asarray(rew, dtype=np.float32), np.asarray(done)))
        elif cmd == "close":
            conn.close()
            return


class EnvWorkers:
    def __init__(self, env_creator: Callable, n: int, num_workers: int, mo_keys: Sequence[str] = (), discrete: bool = True):
        ctx = mp.get_context("spawn")
        num_workers = max(1, min(num_workers, n))
        base, rem = divmod(n, num_workers)
        self.sizes: List[int] = [base + (i < rem) for i in range(num_workers)]
        self.conns, self.procs = [], []
        for sz in self.sizes:
            a, b = ctx.Pipe()
            p = ctx.Process(target=_worker, args=(b, env_creator, sz, tuple(mo_keys), discrete), daemon=True)
            p.start()
            self.conns.append(a)
            self.procs.append(p)

    def reset(self, seed: int) -> np.ndarray:
        for c in self.conns:
            c.send(("reset", seed))
        return np.concatenate([c.recv() for c in self.conns])

    def step(self, actions: np.ndarray):
        off = 0
        for c, sz in zip(self.conns, self.sizes):
            c.send(("step", actions[off : off + sz]))
            off += sz
        parts = [c.recv() for c in self.conns]
        return tuple(np.concatenate([p[j] for p in parts]) for j in range(3))

    def close(self):
        for c, p in zip(self.conns, self.procs):
            try:
                c.send(("close", None))
            except (BrokenPipeError, OSError):
                pass
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
