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

