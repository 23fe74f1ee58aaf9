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
* ``ant`` — **articulated Brax-style** quadruped (documented as such, not bit-compatible
  with Brax/MuJoCo): a torso rigid body and 4 legs of two massive capsule links each
  (thigh on a hip yaw joint, shin on an ankle pitch joint), 8 actuators (gear 150) on a
  joint-space model with armature, damping and limit springs.  Per leg the 2×2 joint-space
  inertia (diagonal for this geometry) and its Coriolis/centrifugal terms come from the
  links' masses and inertias; gravity on the links and ground contacts enter as generalized
  forces through the leg Jacobian.  The torso is the base of a composite body: it moves
  under gravity on the total mass, the contact forces and the legs' momentum exchange —
  d/dt of the legs' relative linear and angular momentum (finite differences of the
  semi-implicit update) act on it, so joint torques react on the torso through the moving
  links.  Contacts: penalty spring-damper with smooth Coulomb friction at the end-cap
  spheres of each shin capsule (knee and foot).  5 semi-implicit sub-steps of 10 ms per
  50 ms control step.  Simplifications against a full articulated-body solver: the
  torso's rotation does not feed back into the joint equations (no base-acceleration
  coupling), and the composite rotational inertia is a constant scalar (nominal pose).
  Observation (27) = torso z, orientation quaternion, 8 joint angles, torso linear and
  angular velocity, 8 joint velocities (Brax ``qpos[2:] ++ qvel``).  Reward = forward
  velocity + 1 (healthy) − 0.5‖a‖²; the episode ends when torso z leaves [0.2, 1.0].
  Reference behaviour: ``src/evox/problems/neuroevolution/reinforcement_learning/brax.py:51-73``.
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


# ------------------------------------------------------------------ articulated Ant
ANT = dict(
    dt=0.01, substeps=5, gear=150.0, armature=30.0, joint_damping=1.0, limit_k=500.0,
    hip_lo=-0.5236, hip_hi=0.5236, ank_lo=0.5236, ank_hi=1.2217,  # |ankle| range [30°, 70°]
    l1=0.2828, l2=0.5657, hip_r=0.2828, m_torso=10.0, m_thigh=0.8, m_shin=1.2, i_torso=1.0,
    ang_damp=0.5, lin_damp=0.05, radius=0.08,
    k_contact=2000.0, c_contact=60.0, mu=1.0, eps_v=0.05, gravity=9.81, z0=0.75,
)
LEG_ANGLE = (0.7854, 2.3562, 3.9270, 5.4978)  # legs at 45°, 135°, 225°, 315°
ANKLE_SIGN = (1.0, -1.0, -1.0, 1.0)  # Brax init qpos: ankles 1, -1, -1, 1


def ant_derived(P=ANT):
    """Constants of the composite model (shared with csrc/kernels/neuro.hip): link inertias
    (thin rods about their centre), total mass and the scalar composite rotational inertia
    of the torso with the legs at the nominal pose (hip 0, |ankle| 1 rad)."""
    i1 = P["m_thigh"] * P["l1"] ** 2 / 12
    i2 = P["m_shin"] * P["l2"] ** 2 / 12
    m_tot = P["m_torso"] + 4 * (P["m_thigh"] + P["m_shin"])
    r1 = P["hip_r"] + 0.5 * P["l1"]
    r2 = P["hip_r"] + P["l1"] + 0.5 * P["l2"] * math.cos(1.0)
    z2 = 0.5 * P["l2"] * math.sin(1.0)
    i_c = P["i_torso"] + 4 * (P["m_thigh"] * r1 * r1 + i1 + P["m_shin"] * (r2 * r2 + z2 * z2) + i2)
    return dict(i1=i1, i2=i2, m_tot=m_tot, i_c=i_c)


def _quat_rotate(q, v):
    """Rotate v (…, 3) by unit quaternion q (…, 4) = (w, x, y, z)."""
    w, xyz = q[..., :1], q[..., 1:]
    t = 2 * torch.cross(xyz, v, dim=-1)
    return v + w * t + torch.cross(xyz, t, dim=-1)


def _quat_rotate_inv(q, v):
    return _quat_rotate(torch.cat([q[..., :1], -q[..., 1:]], -1), v)


@register("ant")
class Ant:
    """Articulated Brax-style Ant, torch reference implementation (see module docstring).

    State layout (N, 29): pos(3) quat(4) vel(3) angvel(3) joint q(8) joint qd(8) — the legs'
    relative momenta are functions of the joint state, so nothing else is carried."""

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

    def _leg_geometry(self, s):
        """Per leg (N, 4): yaw φ, pitch a = sign·ankle, their rates, and sign."""
        jq, jqd = s[:, 13:21], s[:, 21:29]
        base = torch.tensor(LEG_ANGLE, device=s.device)
        sg = torch.tensor(ANKLE_SIGN, device=s.device)
        return base + jq[:, 0::2], jq[:, 1::2] * sg, jqd[:, 0::2], jqd[:, 1::2] * sg, sg

    def _rel_momentum(self, phi, a, phid, ad):
        """Legs' linear / angular momentum relative to the torso frame (N, 4, 3) each,
        angular about the torso origin (links as rods: thigh radial, shin in the leg plane)."""
        P, D = self.P, ant_derived(self.P)
        cphi, sphi = torch.cos(phi), torch.sin(phi)
        ca, sa = torch.cos(a), torch.sin(a)
        z = torch.zeros_like(phi)
        er = torch.stack([cphi, sphi, z], -1)
        ep = torch.stack([-sphi, cphi, z], -1)
        ez = torch.stack([z, z, torch.ones_like(z)], -1)
        r1 = P["hip_r"] + 0.5 * P["l1"]
        r2 = P["hip_r"] + P["l1"] + 0.5 * P["l2"] * ca
        c1 = r1 * er
        c2 = r2[..., None] * er - (0.5 * P["l2"] * sa)[..., None] * ez
        v1 = (r1 * phid)[..., None] * ep
        v2 = (r2 * phid)[..., None] * ep - (0.5 * P["l2"] * sa * ad)[..., None] * er - (0.5 * P["l2"] * ca * ad)[..., None] * ez
        p = P["m_thigh"] * v1 + P["m_shin"] * v2
        L = (P["m_thigh"] * torch.cross(c1, v1, dim=-1) + P["m_shin"] * torch.cross(c2, v2, dim=-1)
             + ((D["i1"] + D["i2"] * ca * ca) * phid)[..., None] * ez + (D["i2"] * ad)[..., None] * ep)
        return p, L

    def _substep(self, s, tau):
        P, D = self.P, ant_derived(self.P)
        dt = P["dt"]
        pos, quat, vel, avel, jq, jqd = s[:, 0:3], s[:, 3:7], s[:, 7:10], s[:, 10:13], s[:, 13:21], s[:, 21:29]
        phi, a, phid, ad, sg = self._leg_geometry(s)
        cphi, sphi, ca, sa = torch.cos(phi), torch.sin(phi), torch.cos(a), torch.sin(a)
        z = torch.zeros_like(phi)
        er = torch.stack([cphi, sphi, z], -1)
        ep = torch.stack([-sphi, cphi, z], -1)
        ez = torch.stack([z, z, torch.ones_like(z)], -1)
        rk = P["hip_r"] + P["l1"]
        rf = rk + P["l2"] * ca
        # contact points (torso frame) and their joint-driven velocities: knee, foot
        xk = rk * er
        xf = rf[..., None] * er - (P["l2"] * sa)[..., None] * ez
        vk = (rk * phid)[..., None] * ep
        vf = (rf * phid)[..., None] * ep - (P["l2"] * sa * ad)[..., None] * er - (P["l2"] * ca * ad)[..., None] * ez
        qq = quat[:, None, :].expand(-1, 4, -1)
        F_t, F_w, T_w = [], torch.zeros_like(vel), torch.zeros_like(vel)
        for x, xd in ((xk, vk), (xf, vf)):
            r = _quat_rotate(qq, x)
            pt = pos[:, None, :] + r
            pv = vel[:, None, :] + torch.cross(avel[:, None, :].expand(-1, 4, -1), r, dim=-1) + _quat_rotate(qq, xd)
            pen = torch.clamp(P["radius"] - pt[..., 2], min=0)
            fn = torch.clamp(P["k_contact"] * pen - P["c_contact"] * pv[..., 2] * (pen > 0), min=0)
            vt = pv[..., :2]
            vt_norm = torch.sqrt((vt * vt).sum(-1) + P["eps_v"] ** 2)
            fw = torch.cat([-P["mu"] * fn[..., None] * vt / vt_norm[..., None], fn[..., None]], -1)
            F_w = F_w + fw.sum(1)
            T_w = T_w + torch.cross(r, fw, dim=-1).sum(1)
            F_t.append(_quat_rotate_inv(qq, fw))
        fk, ff = F_t
        g_w = torch.tensor([0.0, 0.0, -P["gravity"]], device=s.device)
        g_t = _quat_rotate_inv(quat, g_w.expand_as(vel))[:, None, :]
        # generalized forces (leg coordinates φ, a)
        r1 = P["hip_r"] + 0.5 * P["l1"]
        r2 = rk + 0.5 * P["l2"] * ca
        gp = (g_t * ep).sum(-1)
        gr = (g_t * er).sum(-1)
        gz = g_t[..., 2]
        Q_phi = (P["m_thigh"] * r1 + P["m_shin"] * r2) * gp + rk * (fk * ep).sum(-1) + rf * (ff * ep).sum(-1)
        Q_a = (P["m_shin"] * (-0.5 * P["l2"]) * (sa * gr + ca * gz)
               + P["l2"] * (-sa * (ff * er).sum(-1) - ca * ff[..., 2]))
        lo = torch.tensor([P["hip_lo"], P["ank_lo"]], device=s.device)
        hi = torch.tensor([P["hip_hi"], P["ank_hi"]], device=s.device)
        hip, ank, hipd, ankd = jq[:, 0::2], jq[:, 1::2], jqd[:, 0::2], jqd[:, 1::2]
        mag = ank * sg
        v_h = torch.clamp(lo[0] - hip, min=0) - torch.clamp(hip - hi[0], min=0)
        v_a = torch.clamp(lo[1] - mag, min=0) - torch.clamp(mag - hi[1], min=0)
        Qh = tau[:, 0::2] - P["joint_damping"] * hipd + P["limit_k"] * v_h + Q_phi
        Qa = tau[:, 1::2] - P["joint_damping"] * ankd + P["limit_k"] * v_a * sg + sg * Q_a
        H11 = P["armature"] + P["m_thigh"] * r1 * r1 + D["i1"] + P["m_shin"] * r2 * r2 + D["i2"] * ca * ca
        H22 = P["armature"] + P["m_shin"] * (0.5 * P["l2"]) ** 2 + D["i2"]
        dH = -P["m_shin"] * P["l2"] * r2 * sa - 2 * D["i2"] * ca * sa  # ∂H11/∂a
        hipdd = (Qh - dH * hipd * ad) / H11
        ankdd = (Qa + sg * 0.5 * dH * hipd * hipd) / H22
        p0, L0 = self._rel_momentum(phi, a, phid, ad)
        hipd = hipd + dt * hipdd
        ankd = ankd + dt * ankdd
        hip = hip + dt * hipd
        ank = ank + dt * ankd
        jq = torch.stack([hip, ank], -1).reshape(-1, 8)
        jqd = torch.stack([hipd, ankd], -1).reshape(-1, 8)
        base = torch.tensor(LEG_ANGLE, device=s.device)
        p1, L1 = self._rel_momentum(base + hip, ank * sg, hipd, ankd * sg)
        dp = _quat_rotate(quat, (p1 - p0).sum(1)) / dt
        dL = _quat_rotate(quat, (L1 - L0).sum(1)) / dt
        # gravity on the legs' links about the torso origin (world frame)
        c1 = r1 * er
        c2 = r2[..., None] * er - (0.5 * P["l2"] * sa)[..., None] * ez
        cg = _quat_rotate(qq, P["m_thigh"] * c1 + P["m_shin"] * c2).sum(1)
        force = F_w + D["m_tot"] * g_w - dp - P["lin_damp"] * vel
        torque = T_w + torch.cross(cg, g_w.expand_as(cg), dim=-1) - dL - P["ang_damp"] * avel
        vel = vel + dt * force / D["m_tot"]
        avel = avel + dt * torque / D["i_c"]
        pos = pos + dt * vel
        w, x, y, zq = quat.unbind(1)
        ox, oy, oz = avel.unbind(1)
        dq = 0.5 * torch.stack([-ox * x - oy * y - oz * zq, ox * w + oy * zq - oz * y, oy * w + oz * x - ox * zq, oz * w + ox * y - oy * x], 1)
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
