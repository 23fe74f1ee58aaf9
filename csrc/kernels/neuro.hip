// Persistent neuroevolution rollout (K15): articulated Brax-style Ant + per-individual MLP policy.
//
// One wave64 owns one individual for the whole episode and its weights stay on-chip
// for every control step (no per-step weight traffic from HBM):
//  * ant_rollout_reg_kernel (h1, h2 <= 64): weights in VGPRs, lane j = hidden unit j;
//  * ant_rollout_kernel (larger layers): weights in LDS, lanes stride over units
//    ((in, out) row-major, so a row read is contiguous across lanes).
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
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));  // xor 1
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));  // xor 2
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
  AntBody s;
  AntLeg g;
  const int leg = lane & 3;
  load_body(s, g, init, leg);
  float total = 0.f;
  int t = 0;
  for (; t < cap; ++t) {
    // observation → LDS (the joints come from the leg-owning lanes 0-3)
    float jq[8], jqd[8];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      jq[2 * l] = rl(g.hq, l);
      jq[2 * l + 1] = rl(g.aq, l);
      jqd[2 * l] = rl(g.hqd, l);
      jqd[2 * l + 1] = rl(g.aqd, l);
    }
    if (lane == 0) {
      a0[0] = s.p[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a0[1 + i] = s.q[i];
#pragma unroll
      for (int i = 0; i < 8; ++i) a0[5 + i] = jq[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) a0[13 + i] = s.v[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) a0[16 + i] = s.w[i];
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
    const float x0 = s.p[0];
    const float th = sel4(leg, tau[0], tau[2], tau[4], tau[6]), ta = sel4(leg, tau[1], tau[3], tau[5], tau[7]);
    for (int k = 0; k < SUB; ++k) art_substep(s, g, th, ta);
    const bool healthy = (s.p[2] >= 0.2f) && (s.p[2] <= 1.0f);
    if (!healthy) break;  // sticky done: the terminating step earns nothing
    total += (s.p[0] - x0) * (1.f / (DT * SUB)) + 1.f - 0.5f * csum;
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
template <int KM>
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
  float total = 0.f;
  int t = 0;
  for (; t < cap; ++t) {
    float o[27];
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
    const float x0 = s.p[0];
    const float th = sel4(leg, tau[0], tau[2], tau[4], tau[6]), ta = sel4(leg, tau[1], tau[3], tau[5], tau[7]);
    #pragma unroll 1
    for (int k = 0; k < SUB; ++k) art_substep(s, g, th, ta);
    const bool healthy = (s.p[2] >= 0.2f) && (s.p[2] <= 1.0f);
    if (!healthy) break;
    total += (s.p[0] - x0) * (1.f / (DT * SUB)) + 1.f - 0.5f * csum;
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
    if (km >= 32)
      ant_rollout_reg_kernel<32><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
    else if (km >= 16)
      ant_rollout_reg_kernel<16><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
    else if (km >= 8)
      ant_rollout_reg_kernel<8><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
    else
      ant_rollout_reg_kernel<0><<<grid, block, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps, trace);
    return;
  }
  const int64_t per = (P + 32 + h1 + h2 + 8) * 4;
  int waves = 4;
  while (waves > 1 && per * waves > 160 * 1024) --waves;
  const int blocks = (N + waves - 1) / waves;
  (void)hipFuncSetAttribute((const void*)ant_rollout_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(per * waves));
  ant_rollout_kernel<<<blocks, 64 * waves, per * waves, s>>>(W, P, N, h1, h2, init, cap, ret, steps, waves);
}
