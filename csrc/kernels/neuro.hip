// Persistent neuroevolution rollout (K15): articulated Brax-style Ant + per-individual MLP policy.
//
// One wave64 owns one individual for the whole episode and its weights stay on-chip
// for every control step (no per-step weight traffic from HBM):
//  * ant_rollout_reg_kernel (h1, h2 <= 64): weights in VGPRs, lane j = hidden unit j;
//  * ant_rollout_kernel (larger layers): weights in LDS, lanes stride over units
//    ((in, out) row-major, so a row read is contiguous across lanes).
// Both integrate with the packed-f32 sub-step (art_substep_pk below); the scalar art_substep
// stays as its readable form and as the register kernel's EVOXMI_ANT_PACKED=0 A/B path.
//
// Physics (mirrors evoxmi/problems/neuroevolution/reinforcement_learning/envs.py:Ant, the CPU
// oracle; constants below must match ANT / ant_derived there): the free-floating 14-DOF tree
// (torso + 4 × thigh/shin) in generalized coordinates, integrated in momentum form.  The torso
// state and the system's world momentum (P, L about the world origin) are quad-uniform; lane
// quad position k owns leg k: its two hinges, their generalized momenta, and per 10 ms sub-step
//  1. positions from the current velocities,
//  2. knee/foot capsule-cap contacts, generalized forces, the closed-form velocity-product
//     terms ∂T/∂q of its two links, the hinge-momentum update,
//  3. its Schur-complement share of the 6×6 torso system (composite inertia of the pose minus
//     b bᵀ/H of its two hinge columns, 21 entries) and of the right-hand side (6), plus its
//     external wrench (6) — 33 quad sums (DPP) —
//  4. a lane-uniform 6×6 LDLᵀ solve for the torso velocity, then its hinge rates by
//     back-substitution.
// Waves leave the loop independently when their episode ends (sticky done), so there are no
// block barriers after the weight load.
#include "evoxmi_common.h"

#include <cstdlib>

namespace {

constexpr float DT = 0.01f, GEAR = 150.f, ARM = 30.f, JD = 1.f, LIMK = 500.f;
constexpr float HIP_LO = -0.5236f, HIP_HI = 0.5236f, ANK_LO = 0.5236f, ANK_HI = 1.2217f;
constexpr float L1 = 0.2828f, L2 = 0.5657f, HIPR = 0.2828f, ADAMP = 0.5f, LDAMP = 0.05f;
constexpr float M0 = 10.f, I0 = 1.f, M1 = 0.8f, M2 = 1.2f;  // torso, thigh, shin
constexpr float RAD = 0.08f, KC = 2000.f, CC = 60.f, MU = 1.f, EPSV = 0.05f, GRAV = 9.81f;
constexpr float IP1 = M1 * (L1 * L1 / 12.f + RAD * RAD / 4.f), IA1 = M1 * RAD * RAD / 2.f;
constexpr float IP2 = M2 * (L2 * L2 / 12.f + RAD * RAD / 4.f), IA2 = M2 * RAD * RAD / 2.f;
constexpr float MTOT = M0 + 4.f * (M1 + M2);
constexpr int SUB = 5;
__constant__ float LEG_ANG[4] = {0.7854f, 2.3562f, 3.9270f, 5.4978f};
__constant__ float ANK_SGN[4] = {1.f, -1.f, -1.f, 1.f};

struct AntBody {  // quad-uniform: torso pose / world velocities and the system's world momentum
  float p[3], q[4], v[3], w[3], P[3], L[3];
};
struct AntLeg {  // per lane: this lane's leg (raw joint coordinates)
  float hq, aq, hqd, aqd, pih, pik;
  float hx, hy, sg, base;
};

__device__ __forceinline__ void cross(const float* a, const float* b, float* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
__device__ __forceinline__ float dot3(const float* a, const float* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

__device__ __forceinline__ float quad_sum(float v) {
  // bound_ctrl DPP movs (no "old" operand to initialise): both stages fuse into v_add_f32_dpp
  v += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, true));  // xor 1
  v = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, true)) + v;  // xor 2
  return v;
}
// tanh via one v_exp and one v_rcp (|error| ~1e-7 near 0, saturates exactly)
__device__ __forceinline__ float fast_tanh(float x) {
  const float e = __expf(2.f * fminf(fmaxf(x, -15.f), 15.f));
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}
__device__ __forceinline__ float rl(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ float sel4(int k, float a, float b, float c, float d) {
  return k == 0 ? a : (k == 1 ? b : (k == 2 ? c : d));
}

// rotation matrix of a unit quaternion (row-major): R v and Rᵀ v then cost 9 FMAs each
__device__ __forceinline__ void quat_mat(const float* q, float* R) {
  const float w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1.f - 2.f * (y * y + z * z); R[1] = 2.f * (x * y - w * z); R[2] = 2.f * (x * z + w * y);
  R[3] = 2.f * (x * y + w * z); R[4] = 1.f - 2.f * (x * x + z * z); R[5] = 2.f * (y * z - w * x);
  R[6] = 2.f * (x * z - w * y); R[7] = 2.f * (y * z + w * x); R[8] = 1.f - 2.f * (x * x + y * y);
}
__device__ __forceinline__ void mrot(const float* R, const float* v, float* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = R[3 * i] * v[0] + R[3 * i + 1] * v[1] + R[3 * i + 2] * v[2];
}
__device__ __forceinline__ void mrot_t(const float* R, const float* v, float* o) {
#pragma unroll
  for (int i = 0; i < 3; ++i) o[i] = R[i] * v[0] + R[3 + i] * v[1] + R[6 + i] * v[2];
}

// pose of this lane's leg in the torso frame (Ant._kin in envs.py)
struct LegPose {
  float cphi, sphi, ca, sa;
  float er[3], ep[3], d[3], dd[3], c1[3], K[3], c2[3], F[3];
  float t1[3], t2[3], s2[3];
};
__device__ __forceinline__ void leg_pose(const AntLeg& g, LegPose& k) {
  const float phi = g.base + g.hq, a = g.aq * g.sg;
  k.cphi = __cosf(phi);
  k.sphi = __sinf(phi);
  k.ca = __cosf(a);
  k.sa = __sinf(a);
  const float er[3] = {k.cphi, k.sphi, 0.f}, ep[3] = {-k.sphi, k.cphi, 0.f};
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    k.er[i] = er[i];
    k.ep[i] = ep[i];
    k.d[i] = k.ca * er[i];
    k.dd[i] = -k.sa * er[i];
  }
  k.d[2] = -k.sa;
  k.dd[2] = -k.ca;
  const float h[3] = {g.hx, g.hy, 0.f};
  const float r2c = L1 + 0.5f * L2 * k.ca;
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    k.c1[i] = h[i] + 0.5f * L1 * er[i];
    k.K[i] = h[i] + L1 * er[i];
    k.c2[i] = k.K[i] + 0.5f * L2 * k.d[i];
    k.F[i] = k.K[i] + L2 * k.d[i];
    k.t1[i] = 0.5f * L1 * ep[i];
    k.t2[i] = r2c * ep[i];
    k.s2[i] = 0.5f * L2 * k.dd[i];
  }
}

// columns of M_bj for φ̇ and ȧ (linear | angular about the torso origin) and the joint diagonal
__device__ __forceinline__ void leg_columns(const LegPose& k, float* bphi, float* ba, float& Hphi, float& Ha) {
  float x1[3], x2[3], x3[3];
  cross(k.c1, k.t1, x1);
  cross(k.c2, k.t2, x2);
  cross(k.c2, k.s2, x3);
  const float cz = (IA2 - IP2) * k.sa;  // I2 e_z = IP2 e_z - (IA2 - IP2) sa d
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    bphi[i] = M1 * k.t1[i] + M2 * k.t2[i];
    bphi[3 + i] = M1 * x1[i] + M2 * x2[i] - cz * k.d[i];
    ba[i] = M2 * k.s2[i];
    ba[3 + i] = M2 * x3[i] + IP2 * k.ep[i];
  }
  bphi[5] += IP1 + IP2;
  Hphi = M1 * dot3(k.t1, k.t1) + M2 * dot3(k.t2, k.t2) + IP1 + IP2 + (IA2 - IP2) * k.sa * k.sa + ARM;
  Ha = M2 * dot3(k.s2, k.s2) + IP2 + ARM;
}

// link velocities (torso frame) and the rod-inertia angular momenta
__device__ __forceinline__ void leg_vel(const LegPose& k, const float* vB, const float* wB, float phid, float ad, float* V1, float* V2,
                                        float* O2, float* IO1, float* IO2) {
  float a1[3], a2[3];
  cross(wB, k.c1, a1);
  cross(wB, k.c2, a2);
  float O1[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    V1[i] = vB[i] + a1[i] + k.t1[i] * phid;
    V2[i] = vB[i] + a2[i] + k.t2[i] * phid + k.s2[i] * ad;
    O1[i] = wB[i];
    O2[i] = wB[i] + k.ep[i] * ad;
  }
  O1[2] += phid;
  O2[2] += phid;
  const float e1 = (IA1 - IP1) * dot3(k.er, O1), e2 = (IA2 - IP2) * dot3(k.d, O2);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    IO1[i] = IP1 * O1[i] + e1 * k.er[i];
    IO2[i] = IP2 * O2[i] + e2 * k.d[i];
  }
}

// penalty contact of a capsule end-cap sphere at torso-frame point x with torso-frame velocity
// vb: the contact force in the torso frame
__device__ __forceinline__ void cap_contact(const AntBody& s, const float* R, const float* x, const float* vb, float* fb) {
  float vw[3];
  mrot(R, vb, vw);
  const float pz = s.p[2] + R[6] * x[0] + R[7] * x[1] + R[8] * x[2];
  const float pen = fmaxf(RAD - pz, 0.f);
  const float fn = fmaxf(KC * pen - CC * vw[2] * (pen > 0.f ? 1.f : 0.f), 0.f);
  const float ivn = rsqrtf(vw[0] * vw[0] + vw[1] * vw[1] + EPSV * EPSV);
  const float f[3] = {-MU * fn * vw[0] * ivn, -MU * fn * vw[1] * ivn, fn};
  mrot_t(R, f, fb);
}

// 6×6 SPD solve A x = b (A symmetric, upper part used; fully unrolled, lane-uniform)
__device__ __forceinline__ void solve6(float (&A)[6][6], float (&b)[6], float (&x)[6]) {
  float inv[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    inv[k] = __builtin_amdgcn_rcpf(A[k][k]);
#pragma unroll
    for (int i = k + 1; i < 6; ++i) {
      const float f = A[k][i] * inv[k];
#pragma unroll
      for (int j = i; j < 6; ++j) A[i][j] -= f * A[k][j];
      b[i] -= f * b[k];
    }
  }
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    float r = b[k];
#pragma unroll
    for (int j = k + 1; j < 6; ++j) r -= A[k][j] * x[j];
    x[k] = r * inv[k];
  }
}

// velocities from the momenta at the current pose (Schur complement over the legs)
__device__ __forceinline__ void solve_velocities(AntBody& s, AntLeg& g, const LegPose& k, const float* R) {
  float bphi[6], ba[6], Hphi, Ha;
  leg_columns(k, bphi, ba, Hphi, Ha);
  const float iHp = __builtin_amdgcn_rcpf(Hphi), iHa = __builtin_amdgcn_rcpf(Ha);
  const float pphi = g.pih, pa = g.pik * g.sg;
  // this leg's composite inertia about the torso origin (thigh along er, shin along d)
  float S1[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) S1[i] = M1 * k.c1[i] + M2 * k.c2[i];
  const float n1 = M1 * dot3(k.c1, k.c1) + M2 * dot3(k.c2, k.c2) + IP1 + IP2;
  float sp[6], sa_[6];  // the hinge columns scaled by 1/H
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    sp[i] = bphi[i] * iHp;
    sa_[i] = ba[i] * iHa;
  }
  float A[6][6], b[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
#pragma unroll
    for (int j = i; j < 6; ++j) {
      float m = 0.f;
      if (i >= 3 && j >= 3) {
        const int r = i - 3, c = j - 3;
        m = (IA1 - IP1) * k.er[r] * k.er[c] + (IA2 - IP2) * k.d[r] * k.d[c] - M1 * k.c1[r] * k.c1[c] - M2 * k.c2[r] * k.c2[c];
        if (r == c) m += n1;
      } else if (i < 3 && j >= 3) {  // −[S1]×
        const int r = i, c = j - 3;
        if (r == 0 && c == 1) m = S1[2];
        if (r == 0 && c == 2) m = -S1[1];
        if (r == 1 && c == 0) m = -S1[2];
        if (r == 1 && c == 2) m = S1[0];
        if (r == 2 && c == 0) m = S1[1];
        if (r == 2 && c == 1) m = -S1[0];
      }
      A[i][j] = quad_sum(m - sp[i] * bphi[j] - sa_[i] * ba[j]);
    }
    b[i] = quad_sum(-sp[i] * pphi - sa_[i] * pa);
  }
  A[0][0] += MTOT; A[1][1] += MTOT; A[2][2] += MTOT;
  A[3][3] += I0; A[4][4] += I0; A[5][5] += I0;
  {
    float hP[3], pxP[3], Lo[3], hL[3];
    mrot_t(R, s.P, hP);
    cross(s.p, s.P, pxP);
#pragma unroll
    for (int i = 0; i < 3; ++i) Lo[i] = s.L[i] - pxP[i];
    mrot_t(R, Lo, hL);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      b[i] += hP[i];
      b[3 + i] += hL[i];
    }
  }
  float u[6];
  solve6(A, b, u);
  float bu = 0.f, au = 0.f;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    bu += bphi[i] * u[i];
    au += ba[i] * u[i];
  }
  g.hqd = (pphi - bu) * iHp;
  g.aqd = g.sg * (pa - au) * iHa;
  mrot(R, u, s.v);
  mrot(R, u + 3, s.w);
}

// momenta of the initial state (Ant.initial_momenta in envs.py)
__device__ __forceinline__ void init_momenta(AntBody& s, AntLeg& g) {
  float R[9];
  quat_mat(s.q, R);
  LegPose k;
  leg_pose(g, k);
  float vB[3], wB[3], V1[3], V2[3], O2[3], IO1[3], IO2[3];
  mrot_t(R, s.v, vB);
  mrot_t(R, s.w, wB);
  const float phid = g.hqd, ad = g.aqd * g.sg;
  leg_vel(k, vB, wB, phid, ad, V1, V2, O2, IO1, IO2);
  float x1[3], x2[3], PB[3], LB[3];
  cross(k.c1, V1, x1);
  cross(k.c2, V2, x2);
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    PB[i] = M0 * vB[i] + quad_sum(M1 * V1[i] + M2 * V2[i]);
    LB[i] = I0 * wB[i] + quad_sum(M1 * x1[i] + M2 * x2[i] + IO1[i] + IO2[i]);
  }
  mrot(R, PB, s.P);
  float Lw[3], pxP[3];
  mrot(R, LB, Lw);
  cross(s.p, s.P, pxP);
#pragma unroll
  for (int i = 0; i < 3; ++i) s.L[i] = Lw[i] + pxP[i];
  float bphi[6], ba[6], Hphi, Ha;
  leg_columns(k, bphi, ba, Hphi, Ha);
  const float ub[6] = {vB[0], vB[1], vB[2], wB[0], wB[1], wB[2]};
  float pphi = Hphi * phid, pa = Ha * ad;
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    pphi += bphi[i] * ub[i];
    pa += ba[i] * ub[i];
  }
  g.pih = pphi;
  g.pik = g.sg * pa;
}

// One 10 ms sub-step (Ant._substep in envs.py); th / ta: this lane's leg torques
__device__ __forceinline__ void art_substep(AntBody& s, AntLeg& g, float th, float ta) {
  // 1. positions with the current velocities
#pragma unroll
  for (int i = 0; i < 3; ++i) s.p[i] += DT * s.v[i];
  {
    const float w = s.q[0], x = s.q[1], y = s.q[2], z = s.q[3];
    const float ox = s.w[0], oy = s.w[1], oz = s.w[2];
    float nq[4] = {w + DT * 0.5f * (-ox * x - oy * y - oz * z), x + DT * 0.5f * (ox * w + oy * z - oz * y),
                   y + DT * 0.5f * (oy * w + oz * x - ox * z), z + DT * 0.5f * (oz * w + ox * y - oy * x)};
    const float in = rsqrtf(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
#pragma unroll
    for (int c = 0; c < 4; ++c) s.q[c] = nq[c] * in;
  }
  g.hq += DT * g.hqd;
  g.aq += DT * g.aqd;
  // 2. forces and velocity-product terms at the new pose, old velocities
  float R[9];
  quat_mat(s.q, R);
  LegPose k;
  leg_pose(g, k);
  float vB[3], wB[3];
  mrot_t(R, s.v, vB);
  mrot_t(R, s.w, wB);
  const float phid = g.hqd, ad = g.aqd * g.sg;
  float V1[3], V2[3], O2[3], IO1[3], IO2[3];
  leg_vel(k, vB, wB, phid, ad, V1, V2, O2, IO1, IO2);
  float fK[3], fF[3];
  {
    float a[3], vk[3], vf[3];
    cross(wB, k.K, a);
#pragma unroll
    for (int i = 0; i < 3; ++i) vk[i] = vB[i] + a[i] + L1 * phid * k.ep[i];
    cross(wB, k.F, a);
#pragma unroll
    for (int i = 0; i < 3; ++i) vf[i] = vB[i] + a[i] + L1 * phid * k.ep[i] + L2 * (phid * k.ca * k.ep[i] + ad * k.dd[i]);
    cap_contact(s, R, k.K, vk, fK);
    cap_contact(s, R, k.F, vf, fF);
  }
  const float gB[3] = {-GRAV * R[6], -GRAV * R[7], -GRAV * R[8]};
  // contact moments about the hip, the legs' first mass moment S1 = m1 c1 + m2 c2
  float Tk[3], S1[3], fs[3];
  {
    float kh[3] = {k.K[0] - g.hx, k.K[1] - g.hy, k.K[2]}, fh[3] = {k.F[0] - g.hx, k.F[1] - g.hy, k.F[2]}, a[3], b[3];
    cross(kh, fK, a);
    cross(fh, fF, b);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      Tk[i] = a[i] + b[i];
      S1[i] = M1 * k.c1[i] + M2 * k.c2[i];
      fs[i] = fK[i] + fF[i];
    }
  }
  // e_z · [(S1 − m_leg h) × g + Tk];  e_p · [(c2 − K) × m2 g + (F − K) × fF] = L2 δd · (½ m2 g + fF)
  const float Qphi = (S1[0] - (M1 + M2) * g.hx) * gB[1] - (S1[1] - (M1 + M2) * g.hy) * gB[0] + Tk[2];
  const float Qa = L2 * (k.dd[0] * (0.5f * M2 * gB[0] + fF[0]) + k.dd[1] * (0.5f * M2 * gB[1] + fF[1]) + k.dd[2] * (0.5f * M2 * gB[2] + fF[2]));
  float dphi, da;
  {
    float r1[3], r2[3], q1[3], q2[3];
    const float wz = wB[2];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      r1[i] = 0.5f * L1 * k.er[i];
      r2[i] = L1 * k.er[i] + 0.5f * L2 * k.d[i];
    }
    const float wr1 = dot3(wB, r1), wr2 = dot3(wB, r2);
    const float a2 = (L1 + 0.5f * L2 * k.ca) * phid, b2 = 0.5f * L2 * ad * k.sa;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      q1[i] = -r1[i] * wz - 0.5f * L1 * phid * k.er[i];
      q2[i] = -r2[i] * wz - a2 * k.er[i] - b2 * k.ep[i];
    }
    q1[2] += wr1;
    q2[2] += wr2;
    const float IOx = IO1[0] + IO2[0], IOy = IO1[1] + IO2[1];
    dphi = M1 * dot3(V1, q1) + M2 * dot3(V2, q2) - (wB[0] * IOy - wB[1] * IOx);
    float dc2[3];
    cross(wB, k.s2, dc2);
#pragma unroll
    for (int i = 0; i < 3; ++i) dc2[i] += 0.5f * L2 * (-phid * k.sa * k.ep[i] - ad * k.d[i]);
    da = M2 * dot3(V2, dc2) + (IA2 - IP2) * dot3(O2, k.dd) * dot3(O2, k.d);
  }
  const float mag = g.aq * g.sg;
  const float vh = fmaxf(HIP_LO - g.hq, 0.f) - fmaxf(g.hq - HIP_HI, 0.f);
  const float va = fmaxf(ANK_LO - mag, 0.f) - fmaxf(mag - ANK_HI, 0.f);
  g.pih += DT * (th - JD * g.hqd + LIMK * vh + Qphi + dphi);
  g.pik += DT * (ta - JD * g.aqd + LIMK * va * g.sg + g.sg * (Qa + da));
  // external wrench on the system: contacts and the legs' weight about the torso origin
  // (Tk + h × fs + S1 × g per leg)
  {
    float X[6], a[3], b[3];
    const float h[3] = {g.hx, g.hy, 0.f};
    cross(h, fs, a);
    cross(S1, gB, b);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      X[i] = quad_sum(fs[i]);
      X[3 + i] = quad_sum(Tk[i] + a[i] + b[i]);
    }
    float FW[3], TW[3], pxF[3];
    mrot(R, X, FW);
    FW[0] -= LDAMP * s.v[0];
    FW[1] -= LDAMP * s.v[1];
    FW[2] += -MTOT * GRAV - LDAMP * s.v[2];
    mrot(R, X + 3, TW);
    cross(s.p, FW, pxF);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      s.P[i] += DT * FW[i];
      s.L[i] += DT * (TW[i] + pxF[i] - ADAMP * s.w[i]);
    }
  }
  // 3. velocities from the momenta at the new pose
  solve_velocities(s, g, k, R);
}

__device__ __forceinline__ void load_body(AntBody& s, AntLeg& g, const float* __restrict__ init, int leg) {
  for (int i = 0; i < 3; ++i) s.p[i] = init[i];
  for (int i = 0; i < 4; ++i) s.q[i] = init[3 + i];
  for (int i = 0; i < 3; ++i) s.v[i] = init[7 + i];
  for (int i = 0; i < 3; ++i) s.w[i] = init[10 + i];
  g.hq = init[13 + 2 * leg];
  g.aq = init[14 + 2 * leg];
  g.hqd = init[21 + 2 * leg];
  g.aqd = init[22 + 2 * leg];
  g.base = LEG_ANG[leg];
  g.sg = ANK_SGN[leg];
  g.hx = HIPR * __cosf(g.base);
  g.hy = HIPR * __sinf(g.base);
  init_momenta(s, g);
}

// ---------------------------------------------------------------- packed-f32 sub-step
// The same sub-step written on register pairs for the lone-wave regime (pop ≤ #SIMDs: one wave
// owns its SIMD and the step is VALU-issue bound).  A v_pk_fma_f32 issues at about the cost of a
// v_fma_f32 (tools/probe_pk_f32.hip) but does two FMAs, so every 3-vector keeps (x, y) in an
// aligned pair and z apart, the two hinges of a leg share pairs (hip, signed ankle), and the
// rotation R is held both as column pairs (R v) and row pairs (Rᵀ v).  The compiler's SLP
// vectoriser found pairs too but paid ~400 v_mov for them (1139 vs 913 instructions, 9.8 vs
// 8.3 ms at pop 1024, profiles/r5_ant_packed.txt); the swizzles here ride on op_sel / neg
// modifiers of hand-written VOP3P instructions instead.  Signed ankle variables (a = sg·aq,
// its rate and momentum) make every leg's equations identical; sg appears only at the
// observation and the actuator.
// rsqrtf's subnormal guard (compare, two scalings, two selects) is 5 instructions around each
// v_rsq_f32: the arguments here (|q|² ≈ 1, |v|² + EPSV²) are never subnormal, so the bare
// instruction gives the same result.
typedef float f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f2 lo2(float s) {  // s in the low dword of a pair (the high dword unused)
  f2 r;
  r.x = s;
  return r;
}
// perp(a) = (−a.y, a.x) = e_z × a
__device__ __forceinline__ f2 perp_mul(f2 a, float s) {  // perp(a)·s
  f2 d;
  asm("v_pk_mul_f32 %0, %1, %2 op_sel:[1,0] op_sel_hi:[0,0] neg_lo:[1,0]" : "=v"(d) : "v"(a), "v"(lo2(s)));
  return d;
}
__device__ __forceinline__ f2 perp_fma(f2 a, float s, f2 c) {  // perp(a)·s + c
  f2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,0]" : "=v"(d) : "v"(a), "v"(lo2(s)), "v"(c));
  return d;
}
__device__ __forceinline__ f2 perp_fms(f2 a, float s, f2 c) {  // perp(a)·s − c
  f2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,1] neg_hi:[0,0,1]" : "=v"(d) : "v"(a), "v"(lo2(s)), "v"(c));
  return d;
}
__device__ __forceinline__ f2 negx_fma(f2 a, float s, f2 c) {  // (−a.x, a.y)·s + c
  f2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel_hi:[1,0,1] neg_lo:[1,0,0]" : "=v"(d) : "v"(a), "v"(lo2(s)), "v"(c));
  return d;
}
__device__ __forceinline__ f2 nswap_fma(f2 a, float s, f2 c) {  // −(a.y, a.x)·s + c
  f2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[0,0,1] neg_lo:[1,0,0] neg_hi:[1,0,0]" : "=v"(d) : "v"(a), "v"(lo2(s)), "v"(c));
  return d;
}
__device__ __forceinline__ f2 nperp_fma_hi(f2 a, f2 t, f2 c) {  // −perp(a)·t.y + c = (a.y, −a.x)·t.y + c
  f2 d;
  asm("v_pk_fma_f32 %0, %1, %2, %3 op_sel:[1,1,0] op_sel_hi:[0,1,1] neg_hi:[1,0,0]" : "=v"(d) : "v"(a), "v"(t), "v"(c));
  return d;
}
__device__ __forceinline__ float cross2(f2 a, f2 b) { return a.x * b.y - a.y * b.x; }
__device__ __forceinline__ float dot2(f2 a, f2 b) { return a.x * b.x + a.y * b.y; }

struct V3 {
  f2 xy;
  float z;
};
__device__ __forceinline__ V3 mk3(f2 xy, float z) {
  V3 r;
  r.xy = xy;
  r.z = z;
  return r;
}
// a × b = (a.z·perp(b) − b.z·perp(a), a.x b.y − a.y b.x)
__device__ __forceinline__ V3 crs(const V3& a, const V3& b) { return mk3(perp_fms(b.xy, a.z, perp_mul(a.xy, b.z)), cross2(a.xy, b.xy)); }
// a × b with b.z = 0
__device__ __forceinline__ V3 crs_b0(const V3& a, f2 b) { return mk3(perp_mul(b, a.z), cross2(a.xy, b)); }
__device__ __forceinline__ float dot3v(const V3& a, const V3& b) { return fmaf(a.z, b.z, dot2(a.xy, b.xy)); }

struct PkRot {  // R (row-major r0..r8) as column pairs (r0,r3) (r1,r4) (r2,r5) and row pairs (r0,r1) (r3,r4) (r6,r7)
  f2 c0, c1, c2, w0, w1, w2;
  float r2, r5, r6, r7, r8;
};
__device__ __forceinline__ PkRot pk_rot(f2 qwx, f2 qyz) {
  const float w = qwx.x, x = qwx.y, y = qyz.x, z = qyz.y;
  PkRot R;
  const float r0 = 1.f - 2.f * (y * y + z * z), r1 = 2.f * (x * y - w * z), r2 = 2.f * (x * z + w * y);
  const float r3 = 2.f * (x * y + w * z), r4 = 1.f - 2.f * (x * x + z * z), r5 = 2.f * (y * z - w * x);
  const float r6 = 2.f * (x * z - w * y), r7 = 2.f * (y * z + w * x), r8 = 1.f - 2.f * (x * x + y * y);
  R.c0 = f2{r0, r3};
  R.c1 = f2{r1, r4};
  R.c2 = f2{r2, r5};
  R.w0 = f2{r0, r1};
  R.w1 = f2{r3, r4};
  R.w2 = f2{r6, r7};
  R.r2 = r2;
  R.r5 = r5;
  R.r6 = r6;
  R.r7 = r7;
  R.r8 = r8;
  return R;
}
__device__ __forceinline__ V3 rmul(const PkRot& R, const V3& v) {  // R v
  return mk3(R.c0 * v.xy.x + R.c1 * v.xy.y + R.c2 * v.z, R.r6 * v.xy.x + R.r7 * v.xy.y + R.r8 * v.z);
}
__device__ __forceinline__ V3 rmul3(const PkRot& R, float x, float y, float z) {  // R (x, y, z)
  return mk3(R.c0 * x + R.c1 * y + R.c2 * z, R.r6 * x + R.r7 * y + R.r8 * z);
}
__device__ __forceinline__ V3 rtmul(const PkRot& R, const V3& v) {  // Rᵀ v
  return mk3(R.w0 * v.xy.x + R.w1 * v.xy.y + R.w2 * v.z, R.r2 * v.xy.x + R.r5 * v.xy.y + R.r8 * v.z);
}

struct PkBody {
  V3 p, v, w, P, L;
  f2 qwx, qyz;
};
struct PkLeg {
  f2 ang, rate, mom;  // (hip, signed ankle) angle, rate, momentum
  f2 h;          // hip position in the torso frame
  float sg, base;
};
__device__ __forceinline__ void pk_from(const AntBody& s, const AntLeg& g, PkBody& b, PkLeg& l) {
  b.p = mk3(f2{s.p[0], s.p[1]}, s.p[2]);
  b.v = mk3(f2{s.v[0], s.v[1]}, s.v[2]);
  b.w = mk3(f2{s.w[0], s.w[1]}, s.w[2]);
  b.P = mk3(f2{s.P[0], s.P[1]}, s.P[2]);
  b.L = mk3(f2{s.L[0], s.L[1]}, s.L[2]);
  b.qwx = f2{s.q[0], s.q[1]};
  b.qyz = f2{s.q[2], s.q[3]};
  l.ang = f2{g.hq, g.aq * g.sg};
  l.rate = f2{g.hqd, g.aqd * g.sg};
  l.mom = f2{g.pih, g.pik * g.sg};
  l.h = f2{g.hx, g.hy};
  l.sg = g.sg;
  l.base = g.base;
}

// cap_contact on pairs: contact force (torso frame) on a capsule end-cap at torso point x moving with vb
__device__ __forceinline__ V3 pk_contact(const PkBody& s, const PkRot& R, const V3& x, const V3& vb) {
  const V3 vw = rmul(R, vb);
  const float pz = s.p.z + R.r6 * x.xy.x + R.r7 * x.xy.y + R.r8 * x.z;
  const float pen = fmaxf(RAD - pz, 0.f);
  const float fn = fmaxf(KC * pen - CC * vw.z * (pen > 0.f ? 1.f : 0.f), 0.f);
  const float ivn = __builtin_amdgcn_rsqf(dot2(vw.xy, vw.xy) + EPSV * EPSV);
  return rtmul(R, mk3(vw.xy * (-MU * fn * ivn), fn));
}

// Ant._substep on pairs; tq = (hip torque, sg · ankle torque)
__device__ __forceinline__ void art_substep_pk(PkBody& s, PkLeg& g, f2 tq) {
  // 1. positions with the current velocities
  s.p.xy += DT * s.v.xy;
  s.p.z += DT * s.v.z;
  {
    // q += ½ dt · ω ⊗ q on the pairs (w, x), (y, z):
    // (w, x) += hox (−x, w) + hoy (−y, z) − hoz (z, y);  (y, z) += hox (−z, y) + w (hoy, hoz) + x (hoz, −hoy)
    const f2 ho = (DT * 0.5f) * s.w.xy;
    const float hoz = (DT * 0.5f) * s.w.z;
    const f2 n0 = nswap_fma(s.qyz, hoz, negx_fma(s.qyz, ho.y, perp_fma(s.qwx, ho.x, s.qwx)));
    const f2 hyz = f2{ho.y, hoz};
    const f2 n1 = nperp_fma_hi(hyz, s.qwx, hyz * s.qwx.x + perp_fma(s.qyz, ho.x, s.qyz));
    const float in = __builtin_amdgcn_rsqf(dot2(n0, n0) + dot2(n1, n1));
    s.qwx = n0 * in;
    s.qyz = n1 * in;
  }
  g.ang += DT * g.rate;
  // 2. forces and velocity-product terms at the new pose, old velocities
  const PkRot R = pk_rot(s.qwx, s.qyz);
  const V3 vB = rtmul(R, s.v), wB = rtmul(R, s.w);
  const float cphi = __cosf(g.base + g.ang.x), sphi = __sinf(g.base + g.ang.x), ca = __cosf(g.ang.y), sa = __sinf(g.ang.y);
  const f2 er = f2{cphi, sphi}, ep = f2{-sphi, cphi};
  const V3 d = mk3(er * ca, -sa), dd = mk3(er * (-sa), -ca);
  const f2 c1 = g.h + (0.5f * L1) * er, K = g.h + L1 * er;  // z = 0
  const V3 c2 = mk3(K + (0.5f * L2) * d.xy, -0.5f * L2 * sa), F = mk3(K + L2 * d.xy, -L2 * sa);
  const float r2c = L1 + 0.5f * L2 * ca;
  const f2 t1 = (0.5f * L1) * ep, t2 = r2c * ep;  // z = 0
  const V3 s2 = mk3((0.5f * L2) * dd.xy, -0.5f * L2 * ca);
  const float phid = g.rate.x, ad = g.rate.y;
  // link velocities and rod-inertia angular momenta (leg_vel)
  const V3 a1 = crs_b0(wB, c1), a2 = crs(wB, c2);
  const V3 V1 = mk3(vB.xy + a1.xy + t1 * phid, vB.z + a1.z);
  const V3 V2 = mk3(vB.xy + a2.xy + t2 * phid + s2.xy * ad, vB.z + a2.z + s2.z * ad);
  const float Oz = wB.z + phid;
  const V3 O2 = mk3(wB.xy + ep * ad, Oz);
  const float e1 = (IA1 - IP1) * dot2(er, wB.xy), e2 = (IA2 - IP2) * dot3v(d, O2);
  const V3 IO1 = mk3(IP1 * wB.xy + e1 * er, IP1 * Oz);
  const V3 IO2 = mk3(IP2 * O2.xy + e2 * d.xy, IP2 * Oz + e2 * d.z);
  // contacts at the knee (K) and the foot (F)
  const V3 wK = crs_b0(wB, K), wF = crs(wB, F);
  const f2 vlin = vB.xy + (L1 * phid) * ep;
  const V3 vk = mk3(vlin + wK.xy, vB.z + wK.z);
  const V3 vf = mk3(vlin + wF.xy + (L2 * phid * ca) * ep + (L2 * ad) * dd.xy, vB.z + wF.z + L2 * ad * dd.z);
  const V3 fK = pk_contact(s, R, mk3(K, 0.f), vk), fF = pk_contact(s, R, F, vf);
  const V3 gB = mk3(R.w2 * (-GRAV), -GRAV * R.r8);
  // contact moments about the hip, the legs' first mass moment S1 = m1 c1 + m2 c2
  const f2 kh = L1 * er;  // K − h (z = 0)
  const V3 fh = mk3(kh + L2 * d.xy, F.z);
  const V3 tka = mk3(perp_mul(kh, -fK.z), cross2(kh, fK.xy)), tkb = crs(fh, fF);
  const V3 Tk = mk3(tka.xy + tkb.xy, tka.z + tkb.z);
  const V3 S1 = mk3(M1 * c1 + M2 * c2.xy, M2 * c2.z);
  const V3 fs = mk3(fK.xy + fF.xy, fK.z + fF.z);
  const float Qphi = cross2(S1.xy - (M1 + M2) * g.h, gB.xy) + Tk.z;
  const V3 hg = mk3((0.5f * M2) * gB.xy + fF.xy, 0.5f * M2 * gB.z + fF.z);
  const float Qa = L2 * dot3v(dd, hg);
  float dphi, da;
  {
    const V3 r2 = mk3(L1 * er + (0.5f * L2) * d.xy, -0.5f * L2 * sa);
    const float wz = wB.z;
    const float wr1 = 0.5f * L1 * dot2(wB.xy, er), wr2 = dot3v(wB, r2);
    const float a2c = (L1 + 0.5f * L2 * ca) * phid, b2 = 0.5f * L2 * ad * sa;
    const V3 q1 = mk3(er * (-0.5f * L1 * (wz + phid)), wr1);
    const V3 q2 = mk3(r2.xy * (-wz) - a2c * er - b2 * ep, wr2 - r2.z * wz);
    const f2 IO = IO1.xy + IO2.xy;
    dphi = M1 * dot3v(V1, q1) + M2 * dot3v(V2, q2) - cross2(wB.xy, IO);
    const V3 ws2 = crs(wB, s2);
    const V3 dc2 = mk3(ws2.xy + (0.5f * L2) * (ep * (-phid * sa) - d.xy * ad), ws2.z - 0.5f * L2 * ad * d.z);
    da = M2 * dot3v(V2, dc2) + (IA2 - IP2) * dot3v(O2, dd) * dot3v(O2, d);
  }
  // limit springs: max(lo − q, 0) − max(q − hi, 0) = clamp(q, lo, hi) − q
  const f2 lim = f2{__builtin_amdgcn_fmed3f(g.ang.x, HIP_LO, HIP_HI), __builtin_amdgcn_fmed3f(g.ang.y, ANK_LO, ANK_HI)} - g.ang;
  g.mom += DT * (tq - JD * g.rate + LIMK * lim + f2{Qphi + dphi, Qa + da});
  // external wrench on the system: contacts and the legs' weight about the torso origin
  {
    const V3 hf = mk3(perp_mul(g.h, -fs.z), cross2(g.h, fs.xy));
    const V3 sg_ = crs(S1, gB);
    // quad sums stay scalars (a sum written into half of a pair does not fuse into v_add_f32_dpp)
    const f2 tx = Tk.xy + hf.xy + sg_.xy;
    V3 FW = rmul3(R, quad_sum(fs.xy.x), quad_sum(fs.xy.y), quad_sum(fs.z));
    FW.xy -= LDAMP * s.v.xy;
    FW.z += -MTOT * GRAV - LDAMP * s.v.z;
    const V3 TW = rmul3(R, quad_sum(tx.x), quad_sum(tx.y), quad_sum(Tk.z + hf.z + sg_.z)), pxF = crs(s.p, FW);
    s.P.xy += DT * FW.xy;
    s.P.z += DT * FW.z;
    s.L.xy += DT * (TW.xy + pxF.xy - ADAMP * s.w.xy);
    s.L.z += DT * (TW.z + pxF.z - ADAMP * s.w.z);
  }
  // 3. velocities from the momenta at the new pose (solve_velocities), in the permuted basis
  // (lin x, lin y | ang x, ang y | lin z, ang z) so that every pair of the 6-vectors and of the
  // Schur-complement rows is an (x, y) pair of the 3-vector algebra.
  // hinge columns of M_bj (leg_columns): bphi = (M1 t1 + M2 t2 | M1 c1×t1 + M2 c2×t2 − cz d + (IP1+IP2) e_z),
  // ba = (M2 s2 | M2 c2×s2 + IP2 ep)
  const float cz = (IA2 - IP2) * sa;
  const V3 x2 = crs_b0(c2, t2), x3 = crs(c2, s2);
  const float x1z = cross2(c1, t1);
  f2 Bp[3], Ba[3];
  Bp[0] = M1 * t1 + M2 * t2;
  Bp[1] = M2 * x2.xy - cz * d.xy;
  Bp[2] = f2{0.f, M1 * x1z + M2 * x2.z - cz * d.z + IP1 + IP2};  // lin z of bphi is 0
  Ba[0] = M2 * s2.xy;
  Ba[1] = M2 * x3.xy + IP2 * ep;
  Ba[2] = f2{M2 * s2.z, M2 * x3.z};
  const float Hphi = M1 * dot2(t1, t1) + M2 * dot2(t2, t2) + IP1 + IP2 + (IA2 - IP2) * sa * sa + ARM;
  const float Ha = M2 * dot3v(s2, s2) + IP2 + ARM;
  const f2 iH = f2{__builtin_amdgcn_rcpf(Hphi), __builtin_amdgcn_rcpf(Ha)};
  const float n1 = M1 * dot2(c1, c1) + M2 * dot3v(c2, c2) + IP1 + IP2;
  f2 Sp[3], Sq[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    Sp[q] = Bp[q] * iH.x;
    Sq[q] = Ba[q] * iH.y;
  }
  // composite-inertia block (ang, ang) rows x, y over columns (x, y): er_r ER + d_r DD − c1_r C1 − c2_r C2
  const f2 ER = (IA1 - IP1) * er, DD = (IA2 - IP2) * d.xy, C1 = M1 * c1, C2 = M2 * c2.xy;
  const float DDz = (IA2 - IP2) * d.z, C2z = M2 * c2.z;
  f2 M[6][3];  // the leg's m(i, pair) before the Schur terms; only pairs with 2·jp + 1 ≥ i are used
  // −[S1]× (lin rows, ang columns) and its transpose enter as scalar adds on single halves
  // (i, jp, half) → term; every index is a compile-time constant after unrolling
  auto sterm = [&](int i, int jp, int h, float v) -> float {
    if (i == 0 && jp == 1 && h == 1) return v + S1.z;
    if (i == 0 && jp == 2 && h == 1) return v - S1.xy.y;
    if (i == 1 && jp == 1 && h == 0) return v - S1.z;
    if (i == 1 && jp == 2 && h == 1) return v + S1.xy.x;
    if (i == 2 && jp == 2 && h == 0) return v + S1.xy.y;
    if (i == 3 && jp == 2 && h == 0) return v - S1.xy.x;
    return v;
  };
  M[2][1] = er.x * ER + d.xy.x * DD - c1.x * C1 - c2.xy.x * C2;
  M[2][1].x += n1;
  M[2][2] = f2{0.f, d.xy.x * DDz - c2.xy.x * C2z};
  M[3][1] = er.y * ER + d.xy.y * DD - c1.y * C1 - c2.xy.y * C2;
  M[3][1].y += n1;
  M[3][2] = f2{0.f, d.xy.y * DDz - c2.xy.y * C2z};
  M[5][2] = f2{0.f, d.z * DDz - c2.z * C2z + n1};
  f2 A2[6][3];
  float b[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) {
    const float spi = (i & 1) ? Sp[i / 2].y : Sp[i / 2].x, sqi = (i & 1) ? Sq[i / 2].y : Sq[i / 2].x;
#pragma unroll
    for (int jp = i / 2; jp < 3; ++jp) {
      const bool mz = i < 2 || i == 4;  // rows whose M pairs are zero
      const f2 e0 = mz ? -spi * Bp[jp] : M[i][jp] - spi * Bp[jp];
      const f2 e = e0 - sqi * Ba[jp];
      A2[i][jp].y = quad_sum(sterm(i, jp, 1, e.y));
      A2[i][jp].x = (2 * jp >= i) ? quad_sum(sterm(i, jp, 0, e.x)) : 0.f;  // the pair's lower entry is never read
    }
  }
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const f2 e = -Sp[q] * g.mom.x - Sq[q] * g.mom.y;
    b[2 * q] = quad_sum(e.x);
    b[2 * q + 1] = quad_sum(e.y);
  }
  A2[0][0].x += MTOT; A2[1][0].y += MTOT; A2[4][2].x += MTOT;
  A2[2][1].x += I0; A2[3][1].y += I0; A2[5][2].y += I0;
  {
    const V3 hP = rtmul(R, s.P);
    const V3 pxP = crs(s.p, s.P);
    const V3 hL = rtmul(R, mk3(s.L.xy - pxP.xy, s.L.z - pxP.z));
    b[0] += hP.xy.x; b[1] += hP.xy.y; b[2] += hL.xy.x;
    b[3] += hL.xy.y; b[4] += hP.z; b[5] += hL.z;
  }
  f2 bv[3] = {f2{b[0], b[1]}, f2{b[2], b[3]}, f2{b[4], b[5]}};
  // Gaussian elimination on the upper triangle (solve6), the row updates as pair FMAs
  float inv[6], u[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) {
    inv[k] = __builtin_amdgcn_rcpf((k & 1) ? A2[k][k / 2].y : A2[k][k / 2].x);
    f2 Fp[3];
#pragma unroll
    for (int jp = (k + 1) / 2; jp < 3; ++jp) Fp[jp] = A2[k][jp] * inv[k];
#pragma unroll
    for (int i = k + 1; i < 6; ++i) {
      const float f = (i & 1) ? Fp[i / 2].y : Fp[i / 2].x;
#pragma unroll
      for (int jp = i / 2; jp < 3; ++jp) A2[i][jp] -= f * A2[k][jp];
    }
    // b_i −= f_i b_k: whole pairs when both entries are below row k
    const float bk = (k & 1) ? bv[k / 2].y : bv[k / 2].x;
    if (!(k & 1)) bv[k / 2].y -= Fp[k / 2].y * bk;
#pragma unroll
    for (int jp = k / 2 + 1; jp < 3; ++jp) bv[jp] -= Fp[jp] * bk;
  }
#pragma unroll
  for (int k = 5; k >= 0; --k) {
    float r = (k & 1) ? bv[k / 2].y : bv[k / 2].x;
#pragma unroll
    for (int j = k + 1; j < 6; ++j) r -= ((j & 1) ? A2[k][j / 2].y : A2[k][j / 2].x) * u[j];
    u[k] = r * inv[k];
  }
  const f2 U0 = f2{u[0], u[1]}, U1 = f2{u[2], u[3]}, U2 = f2{u[4], u[5]};
  const f2 bu2 = Bp[0] * U0 + Bp[1] * U1 + Bp[2] * U2, au2 = Ba[0] * U0 + Ba[1] * U1 + Ba[2] * U2;
  g.rate = (g.mom - f2{bu2.x + bu2.y, au2.x + au2.y}) * iH;
  s.v = rmul(R, mk3(U0, u[4]));
  s.w = rmul(R, mk3(U1, u[5]));
}

// layer sizes: in = 27, hidden h1, h2 (any, ≤ 256), out = 8; tanh everywhere
__global__ void __launch_bounds__(256) ant_rollout_kernel(const float* __restrict__ W, int64_t P, int N, int h1, int h2,
                                                          const float* __restrict__ init, int cap, float* __restrict__ ret,
                                                          int* __restrict__ steps_out, int waves_per_block) {
  extern __shared__ float smem[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ind = blockIdx.x * waves_per_block + wv;
  // per-wave LDS: weights (P) | act0 (32) | act1 (h1) | act2 (h2)
  const int64_t per = P + 32 + h1 + h2 + 8;
  float* wl = smem + wv * per;
  float* a0 = wl + P;
  float* a1 = a0 + 32;
  float* a2 = a1 + h1;
  float* a3 = a2 + h2;
  if (ind >= N) return;
  const float* wg = W + (int64_t)ind * P;
  for (int64_t i = lane; i < P; i += 64) wl[i] = wg[i];
  const float* W1 = wl;
  const float* B1 = W1 + 27 * h1;
  const float* W2 = B1 + h1;
  const float* B2 = W2 + h1 * h2;
  const float* W3 = B2 + h2;
  const float* B3 = W3 + h2 * 8;
  AntBody s0;
  AntLeg g0;
  const int leg = lane & 3;
  load_body(s0, g0, init, leg);
  // the packed-f32 sub-step (art_substep_pk), as in the register-resident kernel
  PkBody s;
  PkLeg g;
  pk_from(s0, g0, s, g);
  float total = 0.f;
  int t = 0;
  for (; t < cap; ++t) {
    // observation → LDS (the joints come from the leg-owning lanes 0-3)
    float jq[8], jqd[8];
    const float aq = g.ang.y * g.sg, aqd = g.rate.y * g.sg;
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      jq[2 * l] = rl(g.ang.x, l);
      jq[2 * l + 1] = rl(aq, l);
      jqd[2 * l] = rl(g.rate.x, l);
      jqd[2 * l + 1] = rl(aqd, l);
    }
    if (lane == 0) {
      a0[0] = s.p.z;
      a0[1] = s.qwx.x;
      a0[2] = s.qwx.y;
      a0[3] = s.qyz.x;
      a0[4] = s.qyz.y;
#pragma unroll
      for (int i = 0; i < 8; ++i) a0[5 + i] = jq[i];
      a0[13] = s.v.xy.x;
      a0[14] = s.v.xy.y;
      a0[15] = s.v.z;
      a0[16] = s.w.xy.x;
      a0[17] = s.w.xy.y;
      a0[18] = s.w.z;
#pragma unroll
      for (int i = 0; i < 8; ++i) a0[19 + i] = jqd[i];
    }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    for (int j = lane; j < h1; j += 64) {
      float acc = B1[j];
      for (int i = 0; i < 27; ++i) acc = fmaf(a0[i], W1[i * h1 + j], acc);
      a1[j] = tanhf(acc);
    }
    __builtin_amdgcn_wave_barrier();
    for (int j = lane; j < h2; j += 64) {
      float acc = B2[j];
      for (int i = 0; i < h1; ++i) acc = fmaf(a1[i], W2[i * h2 + j], acc);
      a2[j] = tanhf(acc);
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < 8) {
      float acc = B3[lane];
      for (int i = 0; i < h2; ++i) acc = fmaf(a2[i], W3[i * 8 + lane], acc);
      a3[lane] = tanhf(acc);
    }
    __builtin_amdgcn_wave_barrier();
    float act[8], tau[8], csum = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      act[j] = fminf(fmaxf(a3[j], -1.f), 1.f);
      tau[j] = GEAR * act[j];
      csum += act[j] * act[j];
    }
    __builtin_amdgcn_wave_barrier();  // a0..a3 are rewritten next step
    const float x0 = s.p.xy.x;
    const float th = sel4(leg, tau[0], tau[2], tau[4], tau[6]), ta = sel4(leg, tau[1], tau[3], tau[5], tau[7]);
    const f2 tq = f2{th, ta * g.sg};
    for (int k = 0; k < SUB; ++k) art_substep_pk(s, g, tq);
    const bool healthy = (s.p.z >= 0.2f) && (s.p.z <= 1.0f);
    if (!healthy) break;  // sticky done: the terminating step earns nothing
    total += (s.p.xy.x - x0) * (1.f / (DT * SUB)) + 1.f - 0.5f * csum;
  }
  if (lane == 0) {
    ret[ind] = total;
    if (steps_out) steps_out[ind] = t;
  }
}

// Register-resident variant for h1, h2 <= 64 (the north-star 27-64-64-8 policy):
// lane j keeps column j of W1 / W2 and row j of W3 in VGPRs (≈100 registers), so
// the control step touches no memory.  The body part of the observation is lane-uniform
// (the body integration runs redundantly on every lane), the joints come from the
// leg-owning lanes by v_readlane, layer 2 broadcasts a1 through 256 B of LDS, and
// layer 3's eight 64-lane dot products are reduced by a transposing butterfly (4+2+1
// exchanges that halve the live values per stage, then 3 full stages: 10 lane
// exchanges instead of 48, all permlane-swap / DPP, none through the LDS permute
// unit).  Unused units are zero padded, which keeps their activations at tanh(0) = 0.
// cross-lane partners without the LDS permute unit (ds_bpermute costs an LDS round trip
// per exchange on the step's critical path): gfx950 permlane swaps for lane ^ 32 and
// lane ^ 16, DPP row rotate for lane ^ 8
__device__ __forceinline__ float xor32(float x, bool hi) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(hi ? r[0] : r[1]);
}
__device__ __forceinline__ float xor16(float x, bool hi) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(hi ? r[0] : r[1]);
}
__device__ __forceinline__ float xor8(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x128, 0xF, 0xF, false));  // row_ror:8
}

// Four individuals (waves) per workgroup: the waves of one workgroup go to the 4 SIMDs of a CU.
// Single-wave workgroups were placed by the dispatcher two to a SIMD on 6-7 % of the SIMDs
// whenever a streaming kernel ran just before the launch (profiles/r3_ant_wave_placement.log);
// two of these VALU-bound waves on one SIMD take 1.83x the cycles each, so the generation
// (= the slowest wave) took 16.3 instead of 8.9 ms at pop 1024.
constexpr int ANT_WAVES = 4;

typedef float ant_f4 __attribute__((ext_vector_type(4)));

// KM > 0: layer 2's first KM inputs go through the matrix cores while the VALU takes the rest, both
// issued from the same wave so the two pipes run concurrently.  v_mfma_f32_4x4x1_16b_f32 with
// A = the lane's weight (block b = output units 4b..4b+3) and B = a1[k] in all four columns: every
// block column holds the same four sums, so c[lane & 3] is unit `lane` whatever the column order.
// tools/k15_mfma_probe.hip measured the isolated 64x64 layer (one wave): VALU 1100 cycles, MFMA-only
// 4x4x1 1078, 16x16x4 with the vector padded to 16 columns 2755, split 16 / 48 907
// (profiles/r3_k15_mfma_probe.log).
template <int KM, bool PK>
__global__ void __launch_bounds__(64 * ANT_WAVES, 2) ant_rollout_reg_kernel(const float* __restrict__ W, int64_t P, int N, int h1, int h2,
                                                                          const float* __restrict__ init, int cap, float* __restrict__ ret,
                                                                          int* __restrict__ steps_out, int trace) {
  __shared__ float a1s_all[ANT_WAVES][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  float* a1s = a1s_all[wv];
  const unsigned long long t_start = trace ? __builtin_amdgcn_s_memtime() : 0ull;
  const int ind = blockIdx.x * ANT_WAVES + wv;  // waves never synchronise with each other
  if (ind >= N) return;
  const float* W1 = W + (int64_t)ind * P;
  const float* B1 = W1 + 27 * h1;
  const float* W2 = B1 + h1;
  const float* B2 = W2 + h1 * h2;
  const float* W3 = B2 + h2;
  const float* B3 = W3 + h2 * 8;
  const bool u1 = lane < h1, u2 = lane < h2;
  float w1[27], w2[64], w3[8], b3[8];
#pragma unroll
  for (int i = 0; i < 27; ++i) w1[i] = u1 ? W1[i * h1 + lane] : 0.f;
  const float b1 = u1 ? B1[lane] : 0.f;
#pragma unroll
  for (int i = 0; i < 64; ++i) w2[i] = (u2 && i < h1) ? W2[i * h2 + lane] : 0.f;
  const float b2 = u2 ? B2[lane] : 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    w3[k] = u2 ? W3[lane * 8 + k] : 0.f;
    b3[k] = B3[k];
  }
  const bool hb5 = lane & 32, hb4 = lane & 16, hb3 = lane & 8;
  const int leg = lane & 3;
  AntBody s;
  AntLeg g;
  load_body(s, g, init, leg);
  PkBody pb;
  PkLeg pl;
  if constexpr (PK) pk_from(s, g, pb, pl);
  float total = 0.f;
  int t = 0;
  for (; t < cap; ++t) {
    float o[27];
    if constexpr (PK) {
      o[0] = pb.p.z;
      o[1] = pb.qwx.x;
      o[2] = pb.qwx.y;
      o[3] = pb.qyz.x;
      o[4] = pb.qyz.y;
      const float aq = pl.ang.y * pl.sg, aqd = pl.rate.y * pl.sg;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        o[5 + 2 * l] = rl(pl.ang.x, l);
        o[6 + 2 * l] = rl(aq, l);
        o[19 + 2 * l] = rl(pl.rate.x, l);
        o[20 + 2 * l] = rl(aqd, l);
      }
      o[13] = pb.v.xy.x;
      o[14] = pb.v.xy.y;
      o[15] = pb.v.z;
      o[16] = pb.w.xy.x;
      o[17] = pb.w.xy.y;
      o[18] = pb.w.z;
    } else {
      o[0] = s.p[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) o[1 + i] = s.q[i];
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        o[5 + 2 * l] = rl(g.hq, l);
        o[6 + 2 * l] = rl(g.aq, l);
        o[19 + 2 * l] = rl(g.hqd, l);
        o[20 + 2 * l] = rl(g.aqd, l);
      }
#pragma unroll
      for (int i = 0; i < 3; ++i) o[13 + i] = s.v[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) o[16 + i] = s.w[i];
    }
    float acc = b1;
#pragma unroll
    for (int i = 0; i < 27; ++i) acc = fmaf(o[i], w1[i], acc);
    // layer 2: a1 is broadcast through 256 B of LDS (16 ds_read_b128 instead of 64
    // v_readlane + SGPR hazard nops)
    a1s[lane] = fast_tanh(acc);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float a2;
    if constexpr (KM == 0) {
      float c4[4] = {b2, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float4 a = reinterpret_cast<const float4*>(a1s)[i];
        c4[0] = fmaf(a.x, w2[4 * i], c4[0]);
        c4[1] = fmaf(a.y, w2[4 * i + 1], c4[1]);
        c4[2] = fmaf(a.z, w2[4 * i + 2], c4[2]);
        c4[3] = fmaf(a.w, w2[4 * i + 3], c4[3]);
      }
      a2 = fast_tanh((c4[0] + c4[1]) + (c4[2] + c4[3]));
    } else {
      ant_f4 m[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      float c2[2] = {b2, 0.f};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float4 a = reinterpret_cast<const float4*>(a1s)[i];
        const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = 4 * i + q;
          if (k < KM)
            m[q & 1] = __builtin_amdgcn_mfma_f32_4x4x1f32(w2[k], av[q], m[q & 1], 0, 0, 0);
          else
            c2[q & 1] = fmaf(av[q], w2[k], c2[q & 1]);
        }
      }
      const int r = lane & 3;
      a2 = fast_tanh((m[0][r] + m[1][r]) + (c2[0] + c2[1]));
    }
    // 8 partial products → transposing butterfly reduction
    float v4[4], v2[2], v1;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const float keep = hb5 ? a2 * w3[j + 4] : a2 * w3[j];
      const float send = hb5 ? a2 * w3[j] : a2 * w3[j + 4];
      v4[j] = keep + xor32(send, hb5);
    }
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const float keep = hb4 ? v4[j + 2] : v4[j];
      const float send = hb4 ? v4[j] : v4[j + 2];
      v2[j] = keep + xor16(send, hb4);
    }
    {
      const float keep = hb3 ? v2[1] : v2[0];
      const float send = hb3 ? v2[0] : v2[1];
      v1 = keep + xor8(send);
    }
    v1 = quad_sum(v1);  // lanes ^1, ^2
    v1 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v1), 0x141, 0xF, 0xF, false));  // row_half_mirror: the other quad
    float tau[8], csum = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      // output k lives in the lanes whose bits (5,4,3) spell k
      const float a = fminf(fmaxf(fast_tanh(rl(v1, ((k >> 2) & 1) * 32 + ((k >> 1) & 1) * 16 + (k & 1) * 8) + b3[k]), -1.f), 1.f);
      tau[k] = GEAR * a;
      csum += a * a;
    }
    const float th = sel4(leg, tau[0], tau[2], tau[4], tau[6]), ta = sel4(leg, tau[1], tau[3], tau[5], tau[7]);
    float x0, x1, z1;
    if constexpr (PK) {
      x0 = pb.p.xy.x;
      const f2 tq = f2{th, ta * pl.sg};
#pragma unroll 1
      for (int k = 0; k < SUB; ++k) art_substep_pk(pb, pl, tq);
      x1 = pb.p.xy.x;
      z1 = pb.p.z;
    } else {
      x0 = s.p[0];
#pragma unroll 1
      for (int k = 0; k < SUB; ++k) art_substep(s, g, th, ta);
      x1 = s.p[0];
      z1 = s.p[2];
    }
    const bool healthy = (z1 >= 0.2f) && (z1 <= 1.0f);
    if (!healthy) break;
    total += (x1 - x0) * (1.f / (DT * SUB)) + 1.f - 0.5f * csum;
  }
  if (lane == 0) {
    ret[ind] = total;
    if (steps_out) steps_out[ind] = t;
    if (trace) {  // diagnostics (EVOXMI_ANT_TRACE): shader cycles and the wave's hardware slot
      ret[ind] = (float)(__builtin_amdgcn_s_memtime() - t_start);
      steps_out[ind] = (int)((__builtin_amdgcn_s_getreg((31 << 11) | 4) & 0xFFFFu) | ((__builtin_amdgcn_s_getreg((3 << 11) | 20) & 0xFu) << 16));
    }
  }
}

}  // namespace

int64_t evx_ant_lds_bytes(int64_t P, int h1, int h2, int waves) { return (P + 32 + h1 + h2 + 8) * 4 * waves; }

void evx_ant_rollout(const float* W, int64_t P, int N, int h1, int h2, const float* init, int cap, float* ret, int* steps, hipStream_t s) {
  if (h1 <= 64 && h2 <= 64) {
    static const int trace = [] {
      const char* e = getenv("EVOXMI_ANT_TRACE");
      return e ? atoi(e) : 0;
    }();
    // EVOXMI_ANT_L2_MFMA: the first KM inputs of layer 2 on the matrix cores, concurrently with the
    // VALU on the rest (north-star K15: the policy's hidden layer on MFMA).  Default 16 — the split
    // that is fastest for the isolated layer (907 vs 1100 cycles, profiles/r3_k15_mfma_probe.log);
    // inside the rollout every setting is within noise (1000-step latency 8.63 ms at 0, 8.70 at 16,
    // 8.67 at 32; profiles/r3_k15_ant_l2_mfma_ab.txt) because layer 2 is ≈5 % of a control step.
    // 0 = VALU only.
    static const int km = [] {
      const char* e = getenv("EVOXMI_ANT_L2_MFMA");
      return e ? atoi(e) : 16;
    }();
    const dim3 grid((N + ANT_WAVES - 1) / ANT_WAVES), block(64 * ANT_WAVES);
    // EVOXMI_ANT_PACKED: the packed-f32 sub-step (art_substep_pk); 0 = the scalar one
    static const int pk = [] {
      const char* e = getenv("EVOXMI_ANT_PACKED");
      return e ? atoi(e) : 1;
    }();
    if (pk) {
      if (km >= 16)
        ant_rollout_reg_kernel<16, true><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
      else
        ant_rollout_reg_kernel<0, true><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
    } else if (km >= 32)
      ant_rollout_reg_kernel<32, false><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
    else if (km >= 16)
      ant_rollout_reg_kernel<16, false><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
    else if (km >= 8)
      ant_rollout_reg_kernel<8, false><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
    else
      ant_rollout_reg_kernel<0, false><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
    return;
  }
  const int64_t per = (P + 32 + h1 + h2 + 8) * 4;
  int waves = 4;
  while (waves > 1 && per * waves > 160 * 1024) --waves;
  const int blocks = (N + waves - 1) / waves;
  (void)hipFuncSetAttribute((const void*)ant_rollout_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(per * waves));
  ant_rollout_kernel<<<blocks, 64 * waves, per * waves, s>>>(W, P, N, h1, h2, init, cap, ret, steps, waves);
}
