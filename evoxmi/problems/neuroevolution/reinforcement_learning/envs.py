"""Batched, device-resident control environments (the stand-in for Brax / gymnasium,
neither of which exists in this stack).

Every environment is a pure function of tensors with a leading batch dimension,
``reset(key, n) -> (state, obs)`` and ``step(state, action) -> (state, obs, reward,
done)``; the same code runs on the CPU (numerics oracle) and the GPU.  The Ant
additionally has a fused persistent HIP rollout kernel (``ops.neuro.ant_rollout``)
that keeps each individual's MLP weights in LDS for the whole episode.

* ``cartpole`` — gymnasium CartPole-v1 dynamics (Euler, τ = 0.02, ±12°/±2.4 m
  termination, reward 1 per step), discrete actions (argmax of 2 logits).
* ``pendulum`` — gymnasium Pendulum-v1 (max torque 2, reward −(θ² + 0.1θ̇² + 0.001u²)).
* ``mountain_car_continuous`` — gymnasium MountainCarContinuous-v0.
* ``ant`` — **Brax-style** quadruped (documented as such, not bit-compatible with
  Brax/MuJoCo): torso rigid body + 4 legs with hip and ankle joints, 8 actuators
  (gear 150 → joint torques on unit-inertia joints with damping and limits), feet by
  forward kinematics, penalty ground contacts with smooth Coulomb friction acting
  on the torso, 5 semi-implicit sub-steps of 10 ms per 50 ms control step.
  Observation (27) = torso z, orientation quaternion, 8 joint angles, torso linear
  and angular velocity, 8 joint velocities (Brax ``qpos[2:] ++ qvel``).  Reward =
  forward velocity + 1 (healthy) − 0.5‖a‖²; the episode ends when torso z leaves
  [0.2, 1.0].
"""
from __future__ import annotations

import math

import torch

from ....ops import random as rnd

ENVS = {}


def register(name):
    def deco(cls):
        ENVS[name] = cls
        return cls

    return deco


def get_environment(env_name: str, **kwargs):
    key = env_name.lower().replace("-v1", "").replace("-v0", "").replace("-v4", "").replace("-v5", "")
    aliases = {"cartpole": "cartpole", "pendulum": "pendulum", "mountaincarcontinuous": "mountain_car_continuous",
               "mountain_car_continuous": "mountain_car_continuous", "ant": "ant"}
    if key not in aliases:
        raise ValueError(f"unknown environment {env_name!r}; native environments: {sorted(ENVS)}")
    return ENVS[aliases[key]](**kwargs)


@register("cartpole")
class CartPole:
    obs_dim, act_dim, discrete = 4, 2, True
    gravity, masscart, masspole, length, force_mag, tau = 9.8, 1.0, 0.1, 0.5, 10.0, 0.02
    theta_threshold = 12 * 2 * math.pi / 360
    x_threshold = 2.4

    def reset(self, key, n):
        s = (rnd.uniform(key, (4,)) * 0.1 - 0.05).to(torch.float32)
        s = s.expand(n, 4).clone()
        return s, s.clone()

    def step(self, s, action):
        x, x_dot, th, th_dot = s.unbind(1)
        a = action.argmax(-1) if action.dim() > 1 else action
        force = torch.where(a == 1, self.force_mag, -self.force_mag)
        total_mass = self.masspole + self.masscart
        pml = self.masspole * self.length
        ct, st = torch.cos(th), torch.sin(th)
        temp = (force + pml * th_dot**2 * st) / total_mass
        thacc = (self.gravity * st - ct * temp) / (self.length * (4.0 / 3.0 - self.masspole * ct**2 / total_mass))
        xacc = temp - pml * thacc * ct / total_mass
        x = x + self.tau * x_dot
        x_dot = x_dot + self.tau * xacc
        th = th + self.tau * th_dot
        th_dot = th_dot + self.tau * thacc
        s = torch.stack([x, x_dot, th, th_dot], 1)
        done = (x < -self.x_threshold) | (x > self.x_threshold) | (th < -self.theta_threshold) | (th > self.theta_threshold)
        return s, s, torch.ones_like(x), done


@register("pendulum")
class Pendulum:
    obs_dim, act_dim, discrete = 3, 1, False
    max_speed, max_torque, dt, g, m, l = 8.0, 2.0, 0.05, 10.0, 1.0, 1.0

    def _obs(self, s):
        return torch.stack([torch.cos(s[:, 0]), torch.sin(s[:, 0]), s[:, 1]], 1)

    def reset(self, key, n):
        u = rnd.uniform(key, (2,)).to(torch.float32)
        s = torch.stack([u[0] * 2 * math.pi - math.pi, u[1] * 2 - 1]).expand(n, 2).clone()
        return s, self._obs(s)

    def step(self, s, action):
        th, thdot = s.unbind(1)
        u = torch.clamp(action.reshape(-1), -self.max_torque, self.max_torque)
        ang = ((th + math.pi) % (2 * math.pi)) - math.pi
        cost = ang**2 + 0.1 * thdot**2 + 0.001 * u**2
        thdot = torch.clamp(thdot + (3 * self.g / (2 * self.l) * torch.sin(th) + 3.0 / (self.m * self.l**2) * u) * self.dt, -self.max_speed, self.max_speed)
        th = th + thdot * self.dt
        s = torch.stack([th, thdot], 1)
        return s, self._obs(s), -cost, torch.zeros_like(th, dtype=torch.bool)


@register("mountain_car_continuous")
class MountainCarContinuous:
    obs_dim, act_dim, discrete = 2, 1, False

    def reset(self, key, n):
        p = rnd.uniform(key, ()).to(torch.float32) * 0.2 - 0.6
        s = torch.stack([p, torch.zeros_like(p)]).expand(n, 2).clone()
        return s, s.clone()

    def step(self, s, action):
        pos, vel = s.unbind(1)
        force = torch.clamp(action.reshape(-1), -1.0, 1.0)
        vel = torch.clamp(vel + force * 0.0015 - 0.0025 * torch.cos(3 * pos), -0.07, 0.07)
        pos = torch.clamp(pos + vel, -1.2, 0.6)
        vel = torch.where((pos <= -1.2) & (vel < 0), torch.zeros_like(vel), vel)
        done = (pos >= 0.45) & (vel >= 0)
        reward = torch.where(done, 100.0, 0.0) - 0.1 * force**2
        s = torch.stack([pos, vel], 1)
        return s, s, reward, done


# ------------------------------------------------------------------ Brax-style Ant
ANT = dict(
    dt=0.01, substeps=5, gear=150.0, joint_inertia=30.0, joint_damping=1.0, limit_k=500.0,
    hip_lo=-0.5236, hip_hi=0.5236, ank_lo=0.5236, ank_hi=1.2217,  # |ankle| range [30°, 70°]
    l1=0.2828, l2=0.5657, hip_r=0.2828, mass=10.0, inertia=1.0, ang_damp=0.5, lin_damp=0.05,
    k_contact=2000.0, c_contact=60.0, mu=1.0, eps_v=0.05, gravity=9.81, z0=0.75,
)
LEG_ANGLE = (0.7854, 2.3562, 3.9270, 5.4978)  # legs at 45°, 135°, 225°, 315°
ANKLE_SIGN = (1.0, -1.0, -1.0, 1.0)  # Brax init qpos: ankles 1, -1, -1, 1


def _quat_rotate(q, v):
    """Rotate v (…, 3) by unit quaternion q (…, 4) = (w, x, y, z)."""
    w, xyz = q[..., :1], q[..., 1:]
    t = 2 * torch.cross(xyz, v, dim=-1)
    return v + w * t + torch.cross(xyz, t, dim=-1)


@register("ant")
class Ant:
    """Brax-style Ant, torch reference implementation (see module docstring).

    State layout (N, 29): pos(3) quat(4) vel(3) angvel(3) joint q(8) joint qd(8)."""

    obs_dim, act_dim, discrete = 27, 8, False
    state_dim = 29
    P = ANT

    def reset(self, key, n):
        k1, k2 = rnd.split(key)
        q = torch.tensor([0, 0, self.P["z0"], 1, 0, 0, 0] + [0, 1, 0, -1, 0, -1, 0, 1], dtype=torch.float32)
        q = q + (rnd.uniform(k1, (15,)).to(torch.float32) * 0.2 - 0.1) * torch.tensor([1.0] * 3 + [0.0] * 4 + [1.0] * 8)
        qd = 0.1 * rnd.normal(k2, (14,)).to(torch.float32)
        s = torch.cat([q[:3], q[3:7] / q[3:7].norm(), qd[:6], q[7:], qd[6:]])
        s = s.expand(n, 29).clone()
        return s, self.obs(s)

    @staticmethod
    def obs(s):
        return torch.cat([s[:, 2:3], s[:, 3:7], s[:, 13:21], s[:, 7:13], s[:, 21:29]], 1)

    def _feet(self, s):
        """Foot positions relative to the torso centre in the torso frame, (N, 4, 3), and
        their time derivative due to joint motion."""
        P = self.P
        jq, jqd = s[:, 13:21], s[:, 21:29]
        hip, ank = jq[:, 0::2], jq[:, 1::2]
        hipd, ankd = jqd[:, 0::2], jqd[:, 1::2]
        base = torch.tensor(LEG_ANGLE, device=s.device)
        sgn = torch.tensor(ANKLE_SIGN, device=s.device)
        phi = base + hip
        a = ank * sgn  # positive = foot below the hip plane
        reach = P["hip_r"] + P["l1"] + P["l2"] * torch.cos(a)
        cphi, sphi = torch.cos(phi), torch.sin(phi)
        loc = torch.stack([reach * cphi, reach * sphi, -P["l2"] * torch.sin(a)], -1)
        dreach = -P["l2"] * torch.sin(a) * ankd * sgn
        dloc = torch.stack([dreach * cphi - reach * sphi * hipd, dreach * sphi + reach * cphi * hipd, -P["l2"] * torch.cos(a) * ankd * sgn], -1)
        return loc, dloc

    def _substep(self, s, tau):
        P = self.P
        dt = P["dt"]
        pos, quat, vel, avel, jq, jqd = s[:, 0:3], s[:, 3:7], s[:, 7:10], s[:, 10:13], s[:, 13:21], s[:, 21:29]
        # joints: torque − damping − limit penalty on unit-scaled inertia
        lo = torch.tensor([P["hip_lo"], P["ank_lo"]] * 4, device=s.device)
        hi = torch.tensor([P["hip_hi"], P["ank_hi"]] * 4, device=s.device)
        sg = torch.tensor([1.0, ANKLE_SIGN[0], 1.0, ANKLE_SIGN[1], 1.0, ANKLE_SIGN[2], 1.0, ANKLE_SIGN[3]], device=s.device)
        mag = jq * sg  # ankle limits apply to |angle| with the leg's sign
        viol = torch.clamp(lo - mag, min=0) - torch.clamp(mag - hi, min=0)
        jacc = (tau - P["joint_damping"] * jqd + P["limit_k"] * viol * sg) / P["joint_inertia"]
        jqd = jqd + dt * jacc
        jq = jq + dt * jqd
        s = torch.cat([pos, quat, vel, avel, jq, jqd], 1)
        # contacts at the feet
        loc, dloc = self._feet(s)
        r = _quat_rotate(quat[:, None, :].expand(-1, 4, -1), loc)  # world offset of each foot
        dr = _quat_rotate(quat[:, None, :].expand(-1, 4, -1), dloc)
        foot = pos[:, None, :] + r
        fvel = vel[:, None, :] + torch.cross(avel[:, None, :].expand(-1, 4, -1), r, dim=-1) + dr
        pen = torch.clamp(-foot[..., 2], min=0)
        fn = torch.clamp(P["k_contact"] * pen - P["c_contact"] * fvel[..., 2] * (pen > 0), min=0)
        vt = fvel[..., :2]
        vt_norm = torch.sqrt((vt * vt).sum(-1) + P["eps_v"] ** 2)
        ft = -P["mu"] * fn[..., None] * vt / vt_norm[..., None]
        F = torch.cat([ft, fn[..., None]], -1)  # (N, 4, 3)
        force = F.sum(1) + torch.tensor([0.0, 0.0, -P["mass"] * P["gravity"]], device=s.device) - P["lin_damp"] * vel
        torque = torch.cross(r, F, dim=-1).sum(1) - P["ang_damp"] * avel
        vel = vel + dt * force / P["mass"]
        avel = avel + dt * torque / P["inertia"]
        pos = pos + dt * vel
        w, x, y, z = quat.unbind(1)
        ox, oy, oz = avel.unbind(1)
        dq = 0.5 * torch.stack([-ox * x - oy * y - oz * z, ox * w + oy * z - oz * y, oy * w + oz * x - ox * z, oz * w + ox * y - oy * x], 1)
        quat = quat + dt * dq
        quat = quat / quat.norm(dim=1, keepdim=True)
        return torch.cat([pos, quat, vel, avel, jq, jqd], 1)

    def step(self, s, action):
        P = self.P
        a = torch.clamp(action, -1.0, 1.0)
        tau = P["gear"] * a
        x0 = s[:, 0]
        for _ in range(P["substeps"]):
            s = self._substep(s, tau)
        z = s[:, 2]
        healthy = (z >= 0.2) & (z <= 1.0)
        reward = (s[:, 0] - x0) / (P["dt"] * P["substeps"]) + healthy.to(s.dtype) - 0.5 * (a * a).sum(1)
        return s, self.obs(s), reward, ~healthy
