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
  (thigh on a hip yaw joint, shin on an ankle pitch joint), 8 actuators (gear 150) with
  armature, damping and limit springs; penalty spring-damper contacts with smooth Coulomb
  friction at the knee and foot end-cap spheres.  The exact equations of motion of the
  free-floating 14-DOF tree in momentum form (composite inertia of the current pose,
  base-acceleration coupling, closed-form Coriolis / centrifugal terms, a 6×6 Schur-complement
  solve per sub-step; see :class:`Ant`), 5 sub-steps of 10 ms per 50 ms control step; total
  momentum is conserved to rounding with no external forces.  The fused kernel integrates the
  same model on packed-f32 register pairs (``neuro.hip: art_substep_pk``).
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
    """Link inertias (solid capsule-radius cylinders: ``ip`` about axes perpendicular to the
    link through its centre, ``ia`` about the link axis) and the total mass; shared with
    csrc/kernels/neuro.hip."""
    r2 = P["radius"] ** 2
    return dict(ip1=P["m_thigh"] * (P["l1"] ** 2 / 12 + r2 / 4), ia1=P["m_thigh"] * r2 / 2,
                ip2=P["m_shin"] * (P["l2"] ** 2 / 12 + r2 / 4), ia2=P["m_shin"] * r2 / 2,
                m_tot=P["m_torso"] + 4 * (P["m_thigh"] + P["m_shin"]))


def _quat_rotate(q, v):
    """Rotate v (…, 3) by unit quaternion q (…, 4) = (w, x, y, z)."""
    w, xyz = q[..., :1], q[..., 1:]
    t = 2 * torch.cross(xyz, v, dim=-1)
    return v + w * t + torch.cross(xyz, t, dim=-1)


def _quat_rotate_inv(q, v):
    return _quat_rotate(torch.cat([q[..., :1], -q[..., 1:]], -1), v)


def _dot(a, b):
    return (a * b).sum(-1)


def _cross(a, b):
    return torch.cross(a, b, dim=-1)


def _skew(s):
    z = torch.zeros_like(s[..., 0])
    return torch.stack([torch.stack([z, -s[..., 2], s[..., 1]], -1), torch.stack([s[..., 2], z, -s[..., 0]], -1),
                        torch.stack([-s[..., 1], s[..., 0], z], -1)], -2)


@register("ant")
class Ant:
    """Articulated Brax-style Ant, torch reference implementation (the CPU numerics oracle of
    ``csrc/kernels/neuro.hip``; not bit-compatible with Brax/MuJoCo).

    Bodies: a torso (mass 10, isotropic inertia) and 4 legs of two capsule links each — a thigh
    on a hip yaw joint at ``hip_r`` from the torso centre and a shin on an ankle pitch joint at
    the knee — 14 degrees of freedom (free torso + 8 hinges), 8 actuators (gear 150) with
    armature, damping and limit springs; penalty spring-damper contacts with smooth Coulomb
    friction at the knee and foot end-cap spheres.

    Dynamics: the exact equations of motion of the free-floating tree in generalized coordinates,
    integrated in momentum form.  The generalized momentum is ``π = M(q) u`` with
    ``u = (v_B, ω_B, q̇)`` (torso velocities in the torso frame); for the torso it is the
    system's total linear / angular momentum, for a hinge the angular momentum of its subtree
    about the hinge axis.  One sub-step (symplectic Euler, positions first):

    1. ``q ← q + dt·u`` (quaternion for the torso);
    2. world momentum of the whole system += dt · external wrench (gravity, contacts, damping);
       hinge momenta += dt · (τ + generalized external forces + ∂T/∂q), with the velocity-product
       terms ∂T/∂q of every link in closed form;
    3. ``u = M(q)⁻¹ π`` by the Schur complement of the 14×14 mass matrix: each leg's 2×2 joint
       block is diagonal (hinge axes orthogonal), so the legs fold into a 6×6 system for the torso
       (composite inertia of the current pose, base-acceleration coupling included) and the hinge
       rates follow by back-substitution.

    With no external forces the total linear and angular momentum are conserved to rounding
    (``tests/test_neuroevolution.py``); the configuration-dependent composite inertia, the
    torso-rotation coupling and all Coriolis / centrifugal terms are part of the model.
    Observation (27) = torso z, orientation quaternion, 8 joint angles, torso linear and angular
    velocity (world), 8 joint velocities (Brax ``qpos[2:] ++ qvel``).  Reward = forward velocity
    + 1 (healthy) − 0.5‖a‖²; the episode ends when torso z leaves [0.2, 1.0].
    Reference behaviour: ``src/evox/problems/neuroevolution/reinforcement_learning/brax.py:51-73``.

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

    # -- kinematics and mass matrix of the current pose (torso frame) --------------------
    def _kin(self, jq):
        P, D = self.P, ant_derived(self.P)
        o = dict(dtype=jq.dtype, device=jq.device)
        base = torch.tensor(LEG_ANGLE, **o)
        sg = torch.tensor(ANKLE_SIGN, **o)
        phi, a = base + jq[:, 0::2], jq[:, 1::2] * sg
        cphi, sphi, ca, sa = torch.cos(phi), torch.sin(phi), torch.cos(a), torch.sin(a)
        z = torch.zeros_like(phi)
        k = dict(sg=sg, ca=ca, sa=sa)
        k["er"] = er = torch.stack([cphi, sphi, z], -1)
        k["ep"] = ep = torch.stack([-sphi, cphi, z], -1)
        k["ez"] = ez = torch.stack([z, z, torch.ones_like(z)], -1)
        k["h"] = h = (P["hip_r"] * torch.stack([torch.cos(base), torch.sin(base), torch.zeros_like(base)], -1)).expand_as(er)
        k["c1"] = h + 0.5 * P["l1"] * er
        k["K"] = K = h + P["l1"] * er
        k["d"] = d = ca[..., None] * er - sa[..., None] * ez  # shin axis
        k["dd"] = -(sa[..., None] * er + ca[..., None] * ez)  # ∂d/∂a
        k["c2"] = K + 0.5 * P["l2"] * d
        k["F"] = K + P["l2"] * d
        # CoM velocity per unit joint rate: thigh / shin per φ̇, shin per ȧ
        k["t1"] = t1 = 0.5 * P["l1"] * ep
        k["t2"] = t2 = (P["l1"] + 0.5 * P["l2"] * ca)[..., None] * ep
        k["s2"] = s2 = 0.5 * P["l2"] * k["dd"]
        m1, m2 = P["m_thigh"], P["m_shin"]
        I2ez = D["ip2"] * ez - ((D["ia2"] - D["ip2"]) * sa)[..., None] * d
        # columns of M_bj (linear; angular about the torso origin) and the diagonal joint block
        k["bphi"] = torch.cat([m1 * t1 + m2 * t2, m1 * _cross(k["c1"], t1) + m2 * _cross(k["c2"], t2) + D["ip1"] * ez + I2ez], -1)
        k["ba"] = torch.cat([m2 * s2, m2 * _cross(k["c2"], s2) + D["ip2"] * ep], -1)
        k["Hphi"] = m1 * _dot(t1, t1) + m2 * _dot(t2, t2) + D["ip1"] + D["ip2"] + (D["ia2"] - D["ip2"]) * sa * sa + P["armature"]
        k["Ha"] = m2 * _dot(s2, s2) + D["ip2"] + P["armature"]
        # composite rigid-body inertia of torso + legs about the torso origin
        E = torch.eye(3, **o)
        S1 = (m1 * k["c1"] + m2 * k["c2"]).sum(1)
        Io = P["i_torso"] * E
        for m, c, dv, ip, ia in ((m1, k["c1"], er, D["ip1"], D["ia1"]), (m2, k["c2"], d, D["ip2"], D["ia2"])):
            Io = Io + (ip * E + (ia - ip) * dv[..., :, None] * dv[..., None, :]
                       + m * (_dot(c, c)[..., None, None] * E - c[..., :, None] * c[..., None, :])).sum(1)
        top = torch.cat([D["m_tot"] * E.expand(jq.shape[0], 3, 3), -_skew(S1)], -1)
        k["Mbb"] = torch.cat([top, torch.cat([_skew(S1), Io], -1)], -2)
        return k

    def _link_vel(self, k, vB, wB, phid, ad):
        """CoM and angular velocities of thigh / shin (N, 4, 3), torso frame."""
        v, w = vB[:, None, :], wB[:, None, :]
        V1 = v + _cross(w.expand_as(k["c1"]), k["c1"]) + k["t1"] * phid[..., None]
        V2 = v + _cross(w.expand_as(k["c2"]), k["c2"]) + k["t2"] * phid[..., None] + k["s2"] * ad[..., None]
        O1 = w + k["ez"] * phid[..., None]
        O2 = O1 + k["ep"] * ad[..., None]
        return V1, V2, O1, O2

    def kinetic_energy(self, jq, vB, wB, phid, ad):
        """T of the whole system from the link velocities (independent of the mass-matrix
        assembly; used by the tests to check M, π and ∂T/∂q by autograd)."""
        P, D = self.P, ant_derived(self.P)
        k = self._kin(jq)
        V1, V2, O1, O2 = self._link_vel(k, vB, wB, phid, ad)

        def rot(O, dv, ip, ia):
            return ip * _dot(O, O) + (ia - ip) * _dot(O, dv) ** 2

        T = 0.5 * P["m_torso"] * _dot(vB, vB) + 0.5 * P["i_torso"] * _dot(wB, wB)
        T = T + 0.5 * (P["m_thigh"] * _dot(V1, V1) + P["m_shin"] * _dot(V2, V2) + rot(O1, k["er"], D["ip1"], D["ia1"])
                       + rot(O2, k["d"], D["ip2"], D["ia2"]) + P["armature"] * (phid * phid + ad * ad)).sum(1)
        return T

    def _momenta(self, k, vB, wB, phid, ad):
        """π = M(q) u: torso (6, torso frame, angular about the torso origin) and hinges."""
        ub = torch.cat([vB, wB], -1)
        hB = (k["Mbb"] @ ub[..., None])[..., 0] + (k["bphi"] * phid[..., None] + k["ba"] * ad[..., None]).sum(1)
        pphi = _dot(k["bphi"], ub[:, None, :]) + k["Hphi"] * phid
        pa = _dot(k["ba"], ub[:, None, :]) + k["Ha"] * ad
        return hB, pphi, pa

    def _dTdq(self, k, vB, wB, phid, ad):
        """∂T/∂φ and ∂T/∂a per leg at fixed u (velocity-product / Coriolis terms)."""
        P, D = self.P, ant_derived(self.P)
        m1, m2, l1, l2 = P["m_thigh"], P["m_shin"], P["l1"], P["l2"]
        V1, V2, O1, O2 = self._link_vel(k, vB, wB, phid, ad)
        w = wB[:, None, :].expand_as(V1)
        ez, ep, er, d, dd = k["ez"], k["ep"], k["er"], k["d"], k["dd"]
        IO1 = D["ip1"] * O1 + ((D["ia1"] - D["ip1"]) * _dot(er, O1))[..., None] * er
        IO2 = D["ip2"] * O2 + ((D["ia2"] - D["ip2"]) * _dot(d, O2))[..., None] * d
        wz = w[..., 2:3]
        r1, r2 = k["c1"] - k["h"], k["c2"] - k["h"]
        zc1 = -(0.5 * l1 * phid)[..., None] * er  # e_z × ċ1
        zc2 = -((l1 + 0.5 * l2 * k["ca"]) * phid)[..., None] * er - (0.5 * l2 * ad * k["sa"])[..., None] * ep
        dphi = (m1 * _dot(V1, ez * _dot(w, r1)[..., None] - r1 * wz + zc1) + m2 * _dot(V2, ez * _dot(w, r2)[..., None] - r2 * wz + zc2)
                - (w[..., 0] * (IO1 + IO2)[..., 1] - w[..., 1] * (IO1 + IO2)[..., 0]))
        dc2 = _cross(w, k["s2"]) + 0.5 * l2 * (-(phid * k["sa"])[..., None] * ep - ad[..., None] * d)
        da = m2 * _dot(V2, dc2) + (D["ia2"] - D["ip2"]) * _dot(O2, dd) * _dot(O2, d)
        return dphi, da

    def momentum(self, s):
        """Total linear momentum and angular momentum about the world origin (world frame)."""
        jq, jqd = s[:, 13:21], s[:, 21:29]
        k = self._kin(jq)
        quat, pos = s[:, 3:7], s[:, 0:3]
        vB, wB = _quat_rotate_inv(quat, s[:, 7:10]), _quat_rotate_inv(quat, s[:, 10:13])
        hB, _, _ = self._momenta(k, vB, wB, jqd[:, 0::2], jqd[:, 1::2] * k["sg"])
        PW = _quat_rotate(quat, hB[:, :3])
        return PW, _quat_rotate(quat, hB[:, 3:]) + _cross(pos, PW)

    def _substep(self, s, pi, tau):
        P, D = self.P, ant_derived(self.P)
        dt = P["dt"]
        pos, quat, vel, avel, jq, jqd = s[:, 0:3], s[:, 3:7], s[:, 7:10], s[:, 10:13], s[:, 13:21], s[:, 21:29]
        PW, LW, pi_h, pi_k = pi
        # 1. positions with the current velocities
        pos = pos + dt * vel
        w, x, y, zq = quat.unbind(1)
        ox, oy, oz = avel.unbind(1)
        dq = 0.5 * torch.stack([-ox * x - oy * y - oz * zq, ox * w + oy * zq - oz * y, oy * w + oz * x - ox * zq, oz * w + ox * y - oy * x], 1)
        quat = quat + dt * dq
        quat = quat / quat.norm(dim=1, keepdim=True)
        jq = jq + dt * jqd
        # 2. pose-dependent quantities, forces and velocity-product terms at the new pose
        k = self._kin(jq)
        sg = k["sg"]
        vB, wB = _quat_rotate_inv(quat, vel), _quat_rotate_inv(quat, avel)
        hipd, ankd = jqd[:, 0::2], jqd[:, 1::2]
        phid, ad = hipd, ankd * sg
        qq = quat[:, None, :].expand(-1, 4, -1)
        ep, dd = k["ep"], k["dd"]
        VK = vB[:, None, :] + _cross(wB[:, None, :].expand_as(ep), k["K"]) + (P["l1"] * phid)[..., None] * ep
        VF = (vB[:, None, :] + _cross(wB[:, None, :].expand_as(ep), k["F"]) + (P["l1"] * phid)[..., None] * ep
              + P["l2"] * ((phid * k["ca"])[..., None] * ep + ad[..., None] * dd))
        fB = []
        for xp, vp in ((k["K"], VK), (k["F"], VF)):
            pz = pos[:, None, 2] + _quat_rotate(qq, xp)[..., 2]
            vw = _quat_rotate(qq, vp)
            pen = torch.clamp(P["radius"] - pz, min=0)
            fn = torch.clamp(P["k_contact"] * pen - P["c_contact"] * vw[..., 2] * (pen > 0), min=0)
            vt_norm = torch.sqrt((vw[..., :2] ** 2).sum(-1) + P["eps_v"] ** 2)
            fw = torch.cat([-P["mu"] * fn[..., None] * vw[..., :2] / vt_norm[..., None], fn[..., None]], -1)
            fB.append(_quat_rotate_inv(qq, fw))
        fK, fF = fB
        gB = _quat_rotate_inv(quat, torch.tensor([0.0, 0.0, -P["gravity"]], dtype=s.dtype, device=s.device).expand_as(vel))[:, None, :]
        m1, m2 = P["m_thigh"], P["m_shin"]
        h, K, F, c1, c2 = k["h"], k["K"], k["F"], k["c1"], k["c2"]
        mom = _cross(c1 - h, m1 * gB) + _cross(c2 - h, m2 * gB) + _cross(K - h, fK) + _cross(F - h, fF)
        Q_phi = mom[..., 2]
        Q_a = _dot(ep, _cross(c2 - K, m2 * gB) + _cross(F - K, fF))
        dphi, da = self._dTdq(k, vB, wB, phid, ad)
        o = dict(dtype=s.dtype, device=s.device)
        lo = torch.tensor([P["hip_lo"], P["ank_lo"]], **o)
        hi = torch.tensor([P["hip_hi"], P["ank_hi"]], **o)
        hip, ank = jq[:, 0::2], jq[:, 1::2]
        mag = ank * sg
        v_h = torch.clamp(lo[0] - hip, min=0) - torch.clamp(hip - hi[0], min=0)
        v_a = torch.clamp(lo[1] - mag, min=0) - torch.clamp(mag - hi[1], min=0)
        pi_h = pi_h + dt * (tau[:, 0::2] - P["joint_damping"] * hipd + P["limit_k"] * v_h + Q_phi + dphi)
        pi_k = pi_k + dt * (tau[:, 1::2] - P["joint_damping"] * ankd + P["limit_k"] * v_a * sg + sg * (Q_a + da))
        # external wrench on the system (world; torque about the world origin)
        fsum = (fK + fF).sum(1)
        tsum = (_cross(K, fK) + _cross(F, fF) + _cross(c1, m1 * gB) + _cross(c2, m2 * gB)).sum(1)
        gW = torch.tensor([0.0, 0.0, -P["gravity"]], **o)
        FW = _quat_rotate(quat, fsum) + ant_derived(P)["m_tot"] * gW - P["lin_damp"] * vel
        TW = _cross(pos, FW) + _quat_rotate(quat, tsum) - P["ang_damp"] * avel
        PW = PW + dt * FW
        LW = LW + dt * TW
        # 3. velocities from the momenta at the new pose (Schur complement over the legs)
        hB = torch.cat([_quat_rotate_inv(quat, PW), _quat_rotate_inv(quat, LW - _cross(pos, PW))], -1)
        pphi, pa = pi_h, pi_k * sg
        bphi, ba, Hphi, Ha = k["bphi"], k["ba"], k["Hphi"], k["Ha"]
        Ks = k["Mbb"] - (bphi[..., :, None] * bphi[..., None, :] / Hphi[..., None, None]
                         + ba[..., :, None] * ba[..., None, :] / Ha[..., None, None]).sum(1)
        rhs = hB - (bphi * (pphi / Hphi)[..., None] + ba * (pa / Ha)[..., None]).sum(1)
        ub = torch.linalg.solve(Ks, rhs[..., None])[..., 0]
        phid = (pphi - _dot(bphi, ub[:, None, :])) / Hphi
        ad = (pa - _dot(ba, ub[:, None, :])) / Ha
        vel, avel = _quat_rotate(quat, ub[:, :3]), _quat_rotate(quat, ub[:, 3:])
        jqd = torch.stack([phid, ad * sg], -1).reshape(-1, 8)
        return torch.cat([pos, quat, vel, avel, jq, jqd], 1), (PW, LW, pi_h, pi_k)

    def initial_momenta(self, s):
        """Momenta (world P, L about the world origin, hinge π in raw joint coordinates) of a state."""
        k = self._kin(s[:, 13:21])
        quat, pos = s[:, 3:7], s[:, 0:3]
        vB, wB = _quat_rotate_inv(quat, s[:, 7:10]), _quat_rotate_inv(quat, s[:, 10:13])
        jqd = s[:, 21:29]
        hB, pphi, pa = self._momenta(k, vB, wB, jqd[:, 0::2], jqd[:, 1::2] * k["sg"])
        PW = _quat_rotate(quat, hB[:, :3])
        return PW, _quat_rotate(quat, hB[:, 3:]) + _cross(pos, PW), pphi, pa * k["sg"]

    def step(self, s, action):
        P = self.P
        a = torch.clamp(action, -1.0, 1.0)
        tau = P["gear"] * a
        x0 = s[:, 0]
        pi = self.initial_momenta(s)
        for _ in range(P["substeps"]):
            s, pi = self._substep(s, pi, tau)
        z = s[:, 2]
        healthy = (z >= 0.2) & (z <= 1.0)
        reward = (s[:, 0] - x0) / (P["dt"] * P["substeps"]) + healthy.to(s.dtype) - 0.5 * (a * a).sum(1)
        return s, self.obs(s), reward, ~healthy
