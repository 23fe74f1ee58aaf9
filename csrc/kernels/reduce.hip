// Row reductions of populations (K3 support).
//   weighted_rowsum: partial[c][j] = Σ_{k in chunk c} w[k] · (X[idx[k]][j] − sub[j])
// Grid = (column blocks of 256) × chunks; lanes read consecutive columns of the same
// gathered row (coalesced 1 KiB per wave-instruction), no atomics (deterministic).
#include "evoxmi_common.h"

namespace {
__global__ void __launch_bounds__(256) weighted_rowsum_kernel(const float* __restrict__ X, int64_t ldx,
                                                              const int32_t* __restrict__ idx, const float* __restrict__ w,
                                                              const float* __restrict__ sub, int K, int D,
                                                              float* __restrict__ partial, int chunks) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int c = blockIdx.y;
  const int per = (K + chunks - 1) / chunks;
  const int k0 = c * per, k1 = min(K, k0 + per);
  if (j >= D) return;
  const float m = sub ? sub[j] : 0.f;
  // 4 rows in flight per iteration (independent gathers), fixed summation order
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  int k = k0;
  for (; k + 3 < k1; k += 4) {
    int64_t r0 = k, r1 = k + 1, r2 = k + 2, r3 = k + 3;
    if (idx) {
      r0 = idx[k];
      r1 = idx[k + 1];
      r2 = idx[k + 2];
      r3 = idx[k + 3];
    }
    const float x0 = X[r0 * ldx + j], x1 = X[r1 * ldx + j], x2 = X[r2 * ldx + j], x3 = X[r3 * ldx + j];
    a0 = fmaf(w[k], x0 - m, a0);
    a1 = fmaf(w[k + 1], x1 - m, a1);
    a2 = fmaf(w[k + 2], x2 - m, a2);
    a3 = fmaf(w[k + 3], x3 - m, a3);
  }
  for (; k < k1; ++k) {
    const int64_t r = idx ? (int64_t)idx[k] : (int64_t)k;
    a0 = fmaf(w[k], X[r * ldx + j] - m, a0);
  }
  partial[(int64_t)c * D + j] = (a0 + a1) + (a2 + a3);
}
// out[j] = Σ_c partial[c][j] in a fixed order (deterministic): 64 columns per workgroup, its
// 4 waves sum the chunks c ≡ wave (mod 4) with 4 loads in flight, then wave 0 adds the 4
// partials in wave order
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ partial, int chunks, int D, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + lane;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (j < D) {
    int c = w;
    for (; c + 12 < chunks; c += 16) {
      a0 += partial[(int64_t)c * D + j];
      a1 += partial[(int64_t)(c + 4) * D + j];
      a2 += partial[(int64_t)(c + 8) * D + j];
      a3 += partial[(int64_t)(c + 12) * D + j];
    }
    for (; c < chunks; c += 4) a0 += partial[(int64_t)c * D + j];
  }
  red[w][lane] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (w == 0 && j < D) out[j] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}
}  // namespace

void evx_colsum(const float* partial, int chunks, int D, float* out, hipStream_t s) {
  colsum_kernel<<<(D + 63) / 64, 256, 0, s>>>(partial, chunks, D, out);
}

void evx_weighted_rowsum(const float* X, int64_t ldx, const int32_t* idx, const float* w, const float* sub, int K, int D,
                         float* partial, int chunks, hipStream_t s) {
  dim3 grid((D + 255) / 256, chunks);
  weighted_rowsum_kernel<<<grid, 256, 0, s>>>(X, ldx, idx, w, sub, K, D, partial, chunks);
}
