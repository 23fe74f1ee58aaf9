// Fused DTLZ1–4 evaluation: one wave64 per population row.
//
// The distance function g is a row reduction over x[m-1:] (lanes stride the tail,
// reduced with xor-shuffles); then lanes 0..m-1 each build one objective
//   f_j = s·(1+g) · prod_{i < m-1-j} h(x_i) · (j > 0 ? t(x_{m-1-j}) : 1)
// directly (m ≤ 16, so the m-1 term product per lane is cheap) and write it, so the
// (n, m) output is produced in one pass over X with no intermediate tensors.
// Reference semantics: problems/numerical/dtlz.py:8-200.
#include "evoxmi_common.h"

namespace {
using namespace evx;

constexpr float PI_F = 3.14159265358979323846f;

template <int V>
__global__ void __launch_bounds__(256) dtlz_kernel(const float* __restrict__ X, float* __restrict__ F, int N, int D, int M) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= N) return;
  const float* x = X + (int64_t)row * D;
  float s = 0.f;
  for (int j = M - 1 + lane; j < D; j += 64) {
    const float y = x[j] - 0.5f;
    if (V == 1 || V == 3)
      s += y * y - cosf(20.f * PI_F * y);
    else
      s += y * y;
  }
  s = wave_sum(s);
  const float g = (V == 1 || V == 3) ? 100.f * ((float)(D - M + 1) + s) : s;
  if (lane < M) {
    const int j = lane;
    float f = (V == 1 ? 0.5f : 1.f) * (1.f + g);
    const int np = M - 1 - j;
    for (int i = 0; i < np; ++i) {
      float xi = x[i];
      if (V == 4) xi = powf(xi, 100.f);
      f *= (V == 1) ? xi : fmaxf(cosf(xi * PI_F * 0.5f), 0.f);
    }
    if (j > 0) {
      float xi = x[np];
      if (V == 4) xi = powf(xi, 100.f);
      f *= (V == 1) ? (1.f - xi) : sinf(xi * PI_F * 0.5f);
    }
    F[(int64_t)row * M + j] = f;
  }
}

}  // namespace

void evx_dtlz(const float* X, float* F, int N, int D, int M, int variant, hipStream_t s) {
  const dim3 block(256), grid((N + 3) / 4);
  switch (variant) {
    case 1: dtlz_kernel<1><<<grid, block, 0, s>>>(X, F, N, D, M); break;
    case 2: dtlz_kernel<2><<<grid, block, 0, s>>>(X, F, N, D, M); break;
    case 3: dtlz_kernel<3><<<grid, block, 0, s>>>(X, F, N, D, M); break;
    default: dtlz_kernel<4><<<grid, block, 0, s>>>(X, F, N, D, M); break;
  }
}
