// Device helpers shared by the sorted-block-refinement kernels (eigh_sbr16.hip, eigh_sbr_dev.hip).
#pragma once
#include "evoxmi_common.h"

// α = min(1, τ / sqrt(max_c ‖V3_c‖ / ‖V2_c‖)) of the power-step vectors, reduced by one
// 256-thread workgroup (every workgroup that calls it computes the same bits)
__device__ __forceinline__ float evx_sbr_damping_alpha(const float* __restrict__ V2, const float* __restrict__ V3, int n, float tau) {
  __shared__ float red[2][8][4];
  __shared__ float out;
  float s2[8] = {}, s3[8] = {};
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float a = V2[(int64_t)j * 8 + c], b = V3[(int64_t)j * 8 + c];
      s2[c] = fmaf(a, a, s2[c]);
      s3[c] = fmaf(b, b, s3[c]);
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    s2[c] = evx::wave_sum(s2[c]);
    s3[c] = evx::wave_sum(s3[c]);
    if (lane == 0) {
      red[0][c][w] = s2[c];
      red[1][c][w] = s3[c];
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float lam = 0.f;
    for (int c = 0; c < 8; ++c) {
      const float a = red[0][c][0] + red[0][c][1] + red[0][c][2] + red[0][c][3];
      const float b = red[1][c][0] + red[1][c][1] + red[1][c][2] + red[1][c][3];
      lam = fmaxf(lam, sqrtf(b) / fmaxf(sqrtf(a), 1e-30f));
    }
    out = fminf(1.f, tau / sqrtf(fmaxf(lam, 1e-30f)));
  }
  __syncthreads();
  return out;
}


// Bounds of ‖X‖₂² for the skew generator X from the stats partials of its X² = −X·Xᵀ GEMM
// (gemm_ks MODE 1: per workgroup [Σ offdiag², Σ diag², min diag, max diag]): the diagonal of X²
// is −‖row_i‖², so max_i ‖row_i‖² = −min diag ≤ ‖X‖₂² ≤ ‖X‖_F² = −Σ diag ≤ sqrt(n · Σ diag²).
// Free — the GEMM's epilogue computed them — and every workgroup that calls it gets the same bits.
__device__ __forceinline__ float2 evx_sbr_xbounds(const double* __restrict__ part, int nparts, int n) {
  __shared__ double red[2][4];
  __shared__ float2 out;
  double s = 0.0, mn = 0.0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) {
    s += part[4 * i + 1];
    mn = fmin(mn, part[4 * i + 2]);
  }
  s = evx::wave_sum_d(s);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mn = fmin(mn, __shfl_xor(mn, o));
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = mn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0, m = 0.0;
    for (int w = 0; w < (int)(blockDim.x + 63) / 64; ++w) {
      t += red[0][w];
      m = fmin(m, red[1][w]);
    }
    out = make_float2((float)(-m), (float)sqrt((double)n * t));  // (lower, upper) bound of ‖X‖₂²
  }
  __syncthreads();
  return out;
}

// Whether the damping's power iteration runs for a far step (control word c2 of the device
// schedule: 0 the κ rule asked for it, 2 the bounds decide, else skipped): never when the
// upper bound proves ‖X‖₂ ≤ τ (α = 1 exact); with c2 = 2 only when some row of X is longer
// than τ/2 (the lower bound), where an undamped step is at risk
__device__ __forceinline__ bool evx_sbr_damp_runs(int c2, float2 b, float tau2) {
  if (c2 == 0) return !(b.y <= tau2);
  if (c2 == 2) return b.x > 0.25f * tau2 && !(b.y <= tau2);
  return false;
}
