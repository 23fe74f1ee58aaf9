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
// out[j] = Σ_c partial[c][j] in chunk order (deterministic); one thread per column,
// consecutive threads read consecutive columns of each chunk row
__global__ void __launch_bounds__(256) colsum_kernel(const float* __restrict__ partial, int chunks, int D, float* __restrict__ out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= D) return;
  float a0 = 0.f, a1 = 0.f;
  int c = 0;
  for (; c + 1 < chunks; c += 2) {
    a0 += partial[(int64_t)c * D + j];
    a1 += partial[(int64_t)(c + 1) * D + j];
  }
  if (c < chunks) a0 += partial[(int64_t)c * D + j];
  out[j] = a0 + a1;
}
}  // namespace

void evx_colsum(const float* partial, int chunks, int D, float* out, hipStream_t s) {
  colsum_kernel<<<(D + 255) / 256, 256, 0, s>>>(partial, chunks, D, out);
}

void evx_weighted_rowsum(const float* X, int64_t ldx, const int32_t* idx, const float* w, const float* sub, int K, int D,
                         float* partial, int chunks, hipStream_t s) {
  dim3 grid((D + 255) / 256, chunks);
  weighted_rowsum_kernel<<<grid, 256, 0, s>>>(X, ldx, idx, w, sub, K, D, partial, chunks);
}
