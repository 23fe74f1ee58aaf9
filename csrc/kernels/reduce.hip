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
  float acc = 0.f;
  for (int k = k0; k < k1; ++k) {
    const int64_t r = idx ? (int64_t)idx[k] : (int64_t)k;
    acc = fmaf(w[k], X[r * ldx + j] - m, acc);
  }
  partial[(int64_t)c * D + j] = acc;
}
}  // namespace

void evx_weighted_rowsum(const float* X, int64_t ldx, const int32_t* idx, const float* w, const float* sub, int K, int D,
                         float* partial, int chunks, hipStream_t s) {
  dim3 grid((D + 255) / 256, chunks);
  weighted_rowsum_kernel<<<grid, 256, 0, s>>>(X, ldx, idx, w, sub, K, D, partial, chunks);
}
