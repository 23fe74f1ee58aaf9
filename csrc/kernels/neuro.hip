// Persistent neuroevolution rollout (K15): Brax-style Ant + per-individual MLP policy.
//
// One wave64 owns one individual for the whole episode: its MLP weights are copied
// into LDS once and reused for every control step (no per-step weight traffic from
// HBM), the forward pass is lane-parallel over hidden units (lane j computes units
// j, j+64, ...; weights are stored (in, out) row-major so a row read is contiguous
// across lanes → bank-conflict free), and the physics (5 semi-implicit 10 ms
// sub-steps, feet by forward kinematics, penalty contacts with smooth friction) is
// evaluated redundantly by every lane from register state, so the only
// synchronisation inside the episode is the wave's own LDS exchange of the
// activations.  Waves leave the loop independently when their episode ends
// (sticky done), so there are no block barriers after the weight load.
//
// Semantics mirror evoxmi/problems/neuroevolution/reinforcement_learning/envs.py:Ant
// (the CPU reference); constants below must match ANT there.
#include "evoxmi_common.h"

namespace {

constexpr float DT = 0.01f, GEAR = 150.f, JI = 30.f, JD = 1.f, LIMK = 500.f;
constexpr float HIP_LO = -0.5236f, HIP_HI = 0.5236f, ANK_LO = 0.5236f, ANK_HI = 1.2217f;
constexpr float L1 = 0.2828f, L2 = 0.5657f, HIPR = 0.2828f, MASS = 10.f, INERTIA = 1.f, ADAMP = 0.5f, LDAMP = 0.05f;
constexpr float KC = 2000.f, CC = 60.f, MU = 1.f, EPSV = 0.05f, GRAV = 9.81f;
constexpr int SUB = 5;
__constant__ float LEG_ANG[4] = {0.7854f, 2.3562f, 3.9270f, 5.4978f};
__constant__ float ANK_SGN[4] = {1.f, -1.f, -1.f, 1.f};

struct AntState {
  float p[3], q[4], v[3], w[3], jq[8], jqd[8];
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

__device__ void substep(AntState& s, const float* tau) {
  // joints
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int leg = j >> 1;
    const bool ankle = j & 1;
    const float sg = ankle ? ANK_SGN[leg] : 1.f;
    const float lo = ankle ? ANK_LO : HIP_LO, hi = ankle ? ANK_HI : HIP_HI;
    const float mag = s.jq[j] * sg;
    const float viol = fmaxf(lo - mag, 0.f) - fmaxf(mag - hi, 0.f);
    const float acc = (tau[j] - JD * s.jqd[j] + LIMK * viol * sg) / JI;
    s.jqd[j] += DT * acc;
    s.jq[j] += DT * s.jqd[j];
  }
  float F[3] = {0.f, 0.f, -MASS * GRAV}, T[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float sg = ANK_SGN[k];
    const float hip = s.jq[2 * k], ank = s.jq[2 * k + 1], hipd = s.jqd[2 * k], ankd = s.jqd[2 * k + 1];
    const float phi = LEG_ANG[k] + hip, a = ank * sg;
    const float ca = cosf(a), sa = sinf(a), cphi = cosf(phi), sphi = sinf(phi);
    const float reach = HIPR + L1 + L2 * ca;
    const float loc[3] = {reach * cphi, reach * sphi, -L2 * sa};
    const float dreach = -L2 * sa * ankd * sg;
    const float dloc[3] = {dreach * cphi - reach * sphi * hipd, dreach * sphi + reach * cphi * hipd, -L2 * ca * ankd * sg};
    float r[3], dr[3], wr[3];
    qrot(s.q, loc, r);
    qrot(s.q, dloc, dr);
    cross(s.w, r, wr);
    const float fz = s.p[2] + r[2];
    const float fv[3] = {s.v[0] + wr[0] + dr[0], s.v[1] + wr[1] + dr[1], s.v[2] + wr[2] + dr[2]};
    const float pen = fmaxf(-fz, 0.f);
    const float fn = fmaxf(KC * pen - CC * fv[2] * (pen > 0.f ? 1.f : 0.f), 0.f);
    const float vn = sqrtf(fv[0] * fv[0] + fv[1] * fv[1] + EPSV * EPSV);
    const float f[3] = {-MU * fn * fv[0] / vn, -MU * fn * fv[1] / vn, fn};
    float t[3];
    cross(r, f, t);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      F[c] += f[c];
      T[c] += t[c];
    }
  }
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    F[c] -= LDAMP * s.v[c];
    T[c] -= ADAMP * s.w[c];
    s.v[c] += DT * F[c] / MASS;
    s.w[c] += DT * T[c] / INERTIA;
    s.p[c] += DT * s.v[c];
  }
  const float w = s.q[0], x = s.q[1], y = s.q[2], z = s.q[3];
  const float ox = s.w[0], oy = s.w[1], oz = s.w[2];
  float nq[4] = {w + DT * 0.5f * (-ox * x - oy * y - oz * z), x + DT * 0.5f * (ox * w + oy * z - oz * y),
                 y + DT * 0.5f * (oy * w + oz * x - ox * z), z + DT * 0.5f * (oz * w + ox * y - oy * x)};
  const float n = sqrtf(nq[0] * nq[0] + nq[1] * nq[1] + nq[2] * nq[2] + nq[3] * nq[3]);
#pragma unroll
  for (int c = 0; c < 4; ++c) s.q[c] = nq[c] / n;
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
  AntState s;
  for (int i = 0; i < 3; ++i) s.p[i] = init[i];
  for (int i = 0; i < 4; ++i) s.q[i] = init[3 + i];
  for (int i = 0; i < 3; ++i) s.v[i] = init[7 + i];
  for (int i = 0; i < 3; ++i) s.w[i] = init[10 + i];
  for (int i = 0; i < 8; ++i) s.jq[i] = init[13 + i];
  for (int i = 0; i < 8; ++i) s.jqd[i] = init[21 + i];
  float total = 0.f;
  int t = 0;
  for (; t < cap; ++t) {
    // observation → LDS (static register indices: one lane writes all 27 values)
    if (lane == 0) {
      a0[0] = s.p[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a0[1 + i] = s.q[i];
#pragma unroll
      for (int i = 0; i < 8; ++i) a0[5 + i] = s.jq[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) a0[13 + i] = s.v[i];
#pragma unroll
      for (int i = 0; i < 3; ++i) a0[16 + i] = s.w[i];
#pragma unroll
      for (int i = 0; i < 8; ++i) a0[19 + i] = s.jqd[i];
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
    for (int k = 0; k < SUB; ++k) substep(s, tau);
    const bool healthy = (s.p[2] >= 0.2f) && (s.p[2] <= 1.0f);
    if (!healthy) break;  // sticky done: the terminating step earns nothing
    total += (s.p[0] - x0) / (DT * SUB) + 1.f - 0.5f * csum;
  }
  if (lane == 0) {
    ret[ind] = total;
    if (steps_out) steps_out[ind] = t;
  }
}

}  // namespace

int64_t evx_ant_lds_bytes(int64_t P, int h1, int h2, int waves) { return (P + 32 + h1 + h2 + 8) * 4 * waves; }

void evx_ant_rollout(const float* W, int64_t P, int N, int h1, int h2, const float* init, int cap, float* ret, int* steps, hipStream_t s) {
  const int64_t per = (P + 32 + h1 + h2 + 8) * 4;
  int waves = 4;
  while (waves > 1 && per * waves > 160 * 1024) --waves;
  const int blocks = (N + waves - 1) / waves;
  hipFuncSetAttribute((const void*)ant_rollout_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)(per * waves));
  ant_rollout_kernel<<<blocks, 64 * waves, per * waves, s>>>(W, P, N, h1, h2, init, cap, ret, steps, waves);
}
