// Persistent neuroevolution rollout (K15): articulated Brax-style Ant + per-individual MLP policy.
//
// One wave64 owns one individual for the whole episode and its weights stay on-chip
// for every control step (no per-step weight traffic from HBM):
//  * ant_rollout_reg_kernel (h1, h2 <= 64): weights in VGPRs, lane j = hidden unit j;
//  * ant_rollout_kernel (larger layers): weights in LDS, lanes stride over units
//    ((in, out) row-major, so a row read is contiguous across lanes).
// The torso state is lane-uniform; lane quad position k owns leg k (its two joints and
// the leg's relative momentum).  Per 10 ms semi-implicit sub-step (5 per control step) a
// leg lane evaluates the knee/foot capsule-cap contacts, its joint-space dynamics (mass
// matrix, Coriolis, gravity and contact generalized forces), and the change of the leg's
// relative linear/angular momentum; the quad sums (DPP) drive the composite torso.  Waves leave
// the loop independently when their episode ends (sticky done), so there are no
// block barriers after the weight load.
//
// Semantics mirror evoxmi/problems/neuroevolution/reinforcement_learning/envs.py:Ant
// (the CPU reference); constants below must match ANT there.
#include "evoxmi_common.h"

namespace {

constexpr float DT = 0.01f, GEAR = 150.f, ARM = 30.f, JD = 1.f, LIMK = 500.f;
constexpr float HIP_LO = -0.5236f, HIP_HI = 0.5236f, ANK_LO = 0.5236f, ANK_HI = 1.2217f;
constexpr float L1 = 0.2828f, L2 = 0.5657f, HIPR = 0.2828f, ADAMP = 0.5f, LDAMP = 0.05f;
constexpr float M1 = 0.8f, M2 = 1.2f;                     // thigh, shin
constexpr float I1 = M1 * L1 * L1 / 12.f, I2 = M2 * L2 * L2 / 12.f;
constexpr float MTOT = 10.f + 4.f * (M1 + M2);
constexpr float IC = 4.474515846961317f;                  // ant_derived()["i_c"] in envs.py
constexpr float RAD = 0.08f, KC = 2000.f, CC = 60.f, MU = 1.f, EPSV = 0.05f, GRAV = 9.81f;
constexpr float RK = HIPR + L1, R1 = HIPR + 0.5f * L1;
constexpr int SUB = 5;
__constant__ float LEG_ANG[4] = {0.7854f, 2.3562f, 3.9270f, 5.4978f};
__constant__ float ANK_SGN[4] = {1.f, -1.f, -1.f, 1.f};

struct AntBody {
  float p[3], q[4], v[3], w[3];
};

__device__ __forceinline__ void cross(const float* a, const float* b, float* o) {
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}

__device__ __forceinline__ void qrot(const float* q, const float* v, float* o) {
  float t[3], u[3];
  const float xyz[3] = {q[1], q[2], q[3]};
  cross(xyz, v, t);
  t[0] *= 2.f; t[1] *= 2.f; t[2] *= 2.f;
  cross(xyz, t, u);
  for (int k = 0; k < 3; ++k) o[k] = v[k] + q[0] * t[k] + u[k];
}

// Lane-split sub-step for the register kernel: the four legs are evaluated in
// parallel by lane groups (leg = lane & 3) instead of redundantly by every lane,
// and the per-leg force/torque are summed across each quad with two DPP
// quad-permutes.  Joint and body integration stay lane-uniform.
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

__device__ __forceinline__ void qrot_inv(const float* q, const float* v, float* o) {
  const float qc[4] = {q[0], -q[1], -q[2], -q[3]};
  qrot(qc, v, o);
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

// leg's linear / angular momentum relative to the torso frame (angular about the torso
// origin); mirrors Ant._rel_momentum in envs.py
__device__ __forceinline__ void leg_momentum(float cphi, float sphi, float ca, float sa, float phid, float ad, float* p, float* L) {
  const float er[3] = {cphi, sphi, 0.f}, ep[3] = {-sphi, cphi, 0.f};
  const float r2 = RK + 0.5f * L2 * ca;
  const float c1[3] = {R1 * cphi, R1 * sphi, 0.f};
  const float c2[3] = {r2 * cphi, r2 * sphi, -0.5f * L2 * sa};
  float v1[3], v2[3], t1[3], t2[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    v1[k] = R1 * phid * ep[k];
    v2[k] = r2 * phid * ep[k] - 0.5f * L2 * sa * ad * er[k];
  }
  v2[2] -= 0.5f * L2 * ca * ad;
  cross(c1, v1, t1);
  cross(c2, v2, t2);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    p[k] = M1 * v1[k] + M2 * v2[k];
    L[k] = M1 * t1[k] + M2 * t2[k] + I2 * ad * ep[k];
  }
  L[2] += (I1 + I2 * ca * ca) * phid;
}

// penalty contact of a capsule end-cap sphere at torso-frame point x (joint-driven velocity
// xd): world force f, its torque about the torso origin, and the torso-frame force
__device__ __forceinline__ void cap_contact(const AntBody& s, const float* R, const float* x, const float* xd, float* F, float* T,
                                            float* ft) {
  float r[3], dr[3], wr[3];
  mrot(R, x, r);
  mrot(R, xd, dr);
  cross(s.w, r, wr);
  const float pz = s.p[2] + r[2];
  const float pv[3] = {s.v[0] + wr[0] + dr[0], s.v[1] + wr[1] + dr[1], s.v[2] + wr[2] + dr[2]};
  const float pen = fmaxf(RAD - pz, 0.f);
  const float fn = fmaxf(KC * pen - CC * pv[2] * (pen > 0.f ? 1.f : 0.f), 0.f);
  const float ivn = rsqrtf(pv[0] * pv[0] + pv[1] * pv[1] + EPSV * EPSV);
  const float f[3] = {-MU * fn * pv[0] * ivn, -MU * fn * pv[1] * ivn, fn};
  float tq[3];
  cross(r, f, tq);
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    F[k] += f[k];
    T[k] += tq[k];
  }
  mrot_t(R, f, ft);
}

// One sub-step of the articulated Ant for this lane's leg (hip yaw q_h, ankle q_a with
// sign sg, base yaw angle base); pm / Lm: the leg's relative momentum after the previous
// sub-step (a function of the joint state, carried to avoid recomputing it).  Mirrors
// Ant._substep in envs.py.
__device__ __forceinline__ void art_substep(AntBody& s, float& hq, float& aq, float& hqd, float& aqd, float th, float ta,
                                            float base, float sg, float* pm, float* Lm, float* tc) {
  const float phid = hqd, ad = aqd * sg;
  const float cphi = tc[0], sphi = tc[1], ca = tc[2], sa = tc[3];  // of the current joint state
  float R[9];
  quat_mat(s.q, R);
  const float er[3] = {cphi, sphi, 0.f}, ep[3] = {-sphi, cphi, 0.f};
  const float rf = RK + L2 * ca;
  float F[3] = {0.f, 0.f, 0.f}, T[3] = {0.f, 0.f, 0.f}, fk[3], ff[3];
  {
    const float xk[3] = {RK * cphi, RK * sphi, 0.f};
    const float vk[3] = {RK * phid * ep[0], RK * phid * ep[1], 0.f};
    cap_contact(s, R, xk, vk, F, T, fk);
    const float xf[3] = {rf * cphi, rf * sphi, -L2 * sa};
    const float vf[3] = {rf * phid * ep[0] - L2 * sa * ad * er[0], rf * phid * ep[1] - L2 * sa * ad * er[1], -L2 * ca * ad};
    cap_contact(s, R, xf, vf, F, T, ff);
  }
  const float gt[3] = {-GRAV * R[6], -GRAV * R[7], -GRAV * R[8]};  // Rᵀ (0, 0, −g)
  const float r2 = RK + 0.5f * L2 * ca;
  const float gp = gt[0] * ep[0] + gt[1] * ep[1], gr = gt[0] * er[0] + gt[1] * er[1];
  const float Qphi = (M1 * R1 + M2 * r2) * gp + RK * (fk[0] * ep[0] + fk[1] * ep[1]) + rf * (ff[0] * ep[0] + ff[1] * ep[1]);
  const float Qa = M2 * (-0.5f * L2) * (sa * gr + ca * gt[2]) + L2 * (-sa * (ff[0] * er[0] + ff[1] * er[1]) - ca * ff[2]);
  const float mag = aq * sg;
  const float vh = fmaxf(HIP_LO - hq, 0.f) - fmaxf(hq - HIP_HI, 0.f);
  const float va = fmaxf(ANK_LO - mag, 0.f) - fmaxf(mag - ANK_HI, 0.f);
  const float Qh = th - JD * hqd + LIMK * vh + Qphi;
  const float Qq = ta - JD * aqd + LIMK * va * sg + sg * Qa;
  const float H11 = ARM + M1 * R1 * R1 + I1 + M2 * r2 * r2 + I2 * ca * ca;
  const float H22 = ARM + M2 * (0.25f * L2 * L2) + I2;
  const float dH = -M2 * L2 * r2 * sa - 2.f * I2 * ca * sa;
  const float hdd = (Qh - dH * hqd * ad) * __builtin_amdgcn_rcpf(H11);
  const float add = (Qq + sg * 0.5f * dH * hqd * hqd) * __builtin_amdgcn_rcpf(H22);
  hqd += DT * hdd;
  aqd += DT * add;
  hq += DT * hqd;
  aq += DT * aqd;
  float p1[3], L1m[3];
  {
    const float phi1 = base + hq, a1 = aq * sg;
    tc[0] = __cosf(phi1);
    tc[1] = __sinf(phi1);
    tc[2] = __cosf(a1);
    tc[3] = __sinf(a1);
    leg_momentum(tc[0], tc[1], tc[2], tc[3], hqd, aqd * sg, p1, L1m);
  }
  // per leg, torso frame: momentum change, first moment of the link masses
  // this leg's wrench on the torso (world frame): contact forces / torques, minus the rate
  // of the leg's relative momentum, plus the gravity torque of its links — rotated per lane
  // so that only 6 values need the quad sum
  float dpl[3], dLl[3], cgl[3];
  {
    float t0[3], t1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      t0[k] = p1[k] - pm[k];
      t1[k] = L1m[k] - Lm[k];
      pm[k] = p1[k];
      Lm[k] = L1m[k];
    }
    const float cg[3] = {(M1 * R1 + M2 * r2) * cphi, (M1 * R1 + M2 * r2) * sphi, -M2 * 0.5f * L2 * sa};
    mrot(R, t0, dpl);
    mrot(R, t1, dLl);
    mrot(R, cg, cgl);
  }
  float X[6];
  // cross(R·cg, (0, 0, −g)) = (−g·cg_y, g·cg_x, 0)
  X[0] = F[0] - dpl[0] * (1.f / DT);
  X[1] = F[1] - dpl[1] * (1.f / DT);
  X[2] = F[2] - dpl[2] * (1.f / DT);
  X[3] = T[0] - dLl[0] * (1.f / DT) - GRAV * cgl[1];
  X[4] = T[1] - dLl[1] * (1.f / DT) + GRAV * cgl[0];
  X[5] = T[2] - dLl[2] * (1.f / DT);
#pragma unroll
  for (int k = 0; k < 6; ++k) X[k] = quad_sum(X[k]);
  const float gw[3] = {0.f, 0.f, -GRAV};
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float force = X[k] + MTOT * gw[k] - LDAMP * s.v[k];
    const float torque = X[3 + k] - ADAMP * s.w[k];
    s.v[k] += DT * force * (1.f / MTOT);
    s.w[k] += DT * torque * (1.f / IC);
    s.p[k] += DT * s.v[k];
  }
  const float w = s.q[0], x = s.q[1], y = s.q[2], z = s.q[3];
  const float ox = s.w[0], oy = s.w[1], oz = s.w[2];
  float nq[4] = {w + DT * 0.5f * (-ox * x - oy * y - oz * z), x + DT * 0.5f * (ox * w + oy * z - oz * y),
                 y + DT * 0.5f * (oy * w + oz * x - ox * z), z + DT * 0.5f * (oz * w + ox * y - oy * x)};
  const float in = rsqrtf(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
#pragma unroll
  for (int c = 0; c < 4; ++c) s.q[c] = nq[c] * in;
}

__device__ __forceinline__ void init_leg_momentum(float hq, float aq, float hqd, float aqd, float base, float sg, float* pm, float* Lm,
                                                  float* tc) {
  const float phi = base + hq, a = aq * sg;
  tc[0] = __cosf(phi);
  tc[1] = __sinf(phi);
  tc[2] = __cosf(a);
  tc[3] = __sinf(a);
  leg_momentum(tc[0], tc[1], tc[2], tc[3], hqd, aqd * sg, pm, Lm);
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
  for (int i = 0; i < 3; ++i) s.p[i] = init[i];
  for (int i = 0; i < 4; ++i) s.q[i] = init[3 + i];
  for (int i = 0; i < 3; ++i) s.v[i] = init[7 + i];
  for (int i = 0; i < 3; ++i) s.w[i] = init[10 + i];
  const int leg = lane & 3;
  float hq = init[13 + 2 * leg], aq = init[14 + 2 * leg], hqd = init[21 + 2 * leg], aqd = init[22 + 2 * leg];
  float pm[3], Lm[3], tc[4];
  init_leg_momentum(hq, aq, hqd, aqd, LEG_ANG[leg], ANK_SGN[leg], pm, Lm, tc);
  float total = 0.f;
  int t = 0;
  for (; t < cap; ++t) {
    // observation → LDS (the joints come from the leg-owning lanes 0-3)
    float jq[8], jqd[8];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      jq[2 * l] = rl(hq, l);
      jq[2 * l + 1] = rl(aq, l);
      jqd[2 * l] = rl(hqd, l);
      jqd[2 * l + 1] = rl(aqd, l);
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
    for (int k = 0; k < SUB; ++k) art_substep(s, hq, aq, hqd, aqd, th, ta, LEG_ANG[leg], ANK_SGN[leg], pm, Lm, tc);
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

__global__ void __launch_bounds__(64, 2) ant_rollout_reg_kernel(const float* __restrict__ W, int64_t P, int N, int h1, int h2,
                                                              const float* __restrict__ init, int cap, float* __restrict__ ret,
                                                              int* __restrict__ steps_out) {
  __shared__ float a1s[64];
  const int lane = threadIdx.x & 63;
  // one wave per workgroup: a finished episode frees its slot immediately, which
  // matters because episode lengths differ by orders of magnitude
  const int ind = blockIdx.x;
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
  AntBody s;
  for (int i = 0; i < 3; ++i) s.p[i] = init[i];
  for (int i = 0; i < 4; ++i) s.q[i] = init[3 + i];
  for (int i = 0; i < 3; ++i) s.v[i] = init[7 + i];
  for (int i = 0; i < 3; ++i) s.w[i] = init[10 + i];
  const int lg = lane & 3;
  float hq = init[13 + 2 * lg], aq = init[14 + 2 * lg], hqd = init[21 + 2 * lg], aqd = init[22 + 2 * lg];
  const bool hb5 = lane & 32, hb4 = lane & 16, hb3 = lane & 8;
  const int leg = lane & 3;
  const float lbase = LEG_ANG[leg], lsg = ANK_SGN[leg];
  float pm[3], Lm[3], tc[4];
  init_leg_momentum(hq, aq, hqd, aqd, lbase, lsg, pm, Lm, tc);
  float total = 0.f;
  int t = 0;
  for (; t < cap; ++t) {
    float o[27];
    o[0] = s.p[2];
#pragma unroll
    for (int i = 0; i < 4; ++i) o[1 + i] = s.q[i];
#pragma unroll
    for (int l = 0; l < 4; ++l) {
      o[5 + 2 * l] = rl(hq, l);
      o[6 + 2 * l] = rl(aq, l);
      o[19 + 2 * l] = rl(hqd, l);
      o[20 + 2 * l] = rl(aqd, l);
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
    float c4[4] = {b2, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const float4 a = reinterpret_cast<const float4*>(a1s)[i];
      c4[0] = fmaf(a.x, w2[4 * i], c4[0]);
      c4[1] = fmaf(a.y, w2[4 * i + 1], c4[1]);
      c4[2] = fmaf(a.z, w2[4 * i + 2], c4[2]);
      c4[3] = fmaf(a.w, w2[4 * i + 3], c4[3]);
    }
    const float a2 = fast_tanh((c4[0] + c4[1]) + (c4[2] + c4[3]));
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
    for (int k = 0; k < SUB; ++k) art_substep(s, hq, aq, hqd, aqd, th, ta, lbase, lsg, pm, Lm, tc);
    const bool healthy = (s.p[2] >= 0.2f) && (s.p[2] <= 1.0f);
    if (!healthy) break;
    total += (s.p[0] - x0) * (1.f / (DT * SUB)) + 1.f - 0.5f * csum;
  }
  if (lane == 0) {
    ret[ind] = total;
    if (steps_out) steps_out[ind] = t;
  }
}

}  // namespace

int64_t evx_ant_lds_bytes(int64_t P, int h1, int h2, int waves) { return (P + 32 + h1 + h2 + 8) * 4 * waves; }

void evx_ant_rollout(const float* W, int64_t P, int N, int h1, int h2, const float* init, int cap, float* ret, int* steps, hipStream_t s) {
  if (h1 <= 64 && h2 <= 64) {
    ant_rollout_reg_kernel<<<N, 64, 0, s>>>(W, P, N, h1, h2, init, cap, ret, steps);
    return;
  }
  const int64_t per = (P + 32 + h1 + h2 + 8) * 4;
  int waves = 4;
  while (waves > 1 && per * waves > 160 * 1024) --waves;
  const int blocks = (N + waves - 1) / waves;
  (void)hipFuncSetAttribute((const void*)ant_rollout_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(per * waves));
  ant_rollout_kernel<<<blocks, 64 * waves, per * waves, s>>>(W, P, N, h1, h2, init, cap, ret, steps, waves);
}
