// Sequential MOEA/D-style neighbourhood replacement scan (K14) as ONE wave64.
//
// MOEA/D-DRA (reference moeaddra.py:137-203) and EAG-MOEA/D (eagmoead.py:131-160)
// let offspring i = 0..R-1 replace, in order, the neighbours p = P[i, :] whose
// aggregated value does not get worse (g_old >= g_new), at most `nr` of them
// (first in P order), optionally after updating the ideal point z with offspring i.
// Every step depends on the previous one (z and the occupants change), so instead of
// R dependent launches this runs the whole scan in a single wave: lane t handles
// neighbour t (T <= 64), the "first nr" rule is a ballot + popcount prefix, and the
// occupants' objective rows are updated in place in global memory (L2-resident).
// Output: owner[s] = index of the offspring that finally occupies slot s (or -1), the
// updated objective matrix and z.  Decision vectors are gathered afterwards in one
// pass (population[s] = offspring[owner[s]]), so d never enters the sequential part.
#include "evoxmi_common.h"

namespace {

constexpr int MAXM = 16;

__device__ __forceinline__ float agg(int func, const float* f, const float* w, const float* z, int M) {
  if (func == 2) {  // weighted sum
    float s = 0.f;
    for (int k = 0; k < M; ++k) s += f[k] * w[k];
    return s;
  }
  if (func == 1) {  // PBI, theta = 5
    float nw = 0.f, d1 = 0.f;
    for (int k = 0; k < M; ++k) {
      nw += w[k] * w[k];
      d1 += (f[k] - z[k]) * w[k];
    }
    nw = sqrtf(nw);
    d1 /= nw;
    float d2 = 0.f;
    for (int k = 0; k < M; ++k) {
      const float r = f[k] - z[k] - d1 * w[k] / nw;
      d2 += r * r;
    }
    return d1 + 5.f * sqrtf(d2);
  }
  float g = -INFINITY;
  for (int k = 0; k < M; ++k) {
    const float a = fabsf(f[k] - z[k]);
    g = fmaxf(g, func == 3 ? a / w[k] : a * w[k]);  // 3: modified Tchebycheff, 0: Tchebycheff
  }
  return g;
}

__global__ void __launch_bounds__(64) moead_scan_kernel(float* __restrict__ objs, const float* __restrict__ off_objs,
                                                        const int32_t* __restrict__ P, const float* __restrict__ W,
                                                        float* __restrict__ z_io, int32_t* __restrict__ owner, int N, int R,
                                                        int T, int M, int func, int nr, int update_z) {
  const int lane = threadIdx.x;
  float z[MAXM];
  for (int k = 0; k < M; ++k) z[k] = z_io[k];
  for (int s = lane; s < N; s += 64) owner[s] = -1;
  __syncthreads();
  for (int i = 0; i < R; ++i) {
    float fo[MAXM];
    for (int k = 0; k < M; ++k) fo[k] = off_objs[(int64_t)i * M + k];
    if (update_z)
      for (int k = 0; k < M; ++k) z[k] = fminf(z[k], fo[k]);
    bool pred = false;
    int slot = 0;
    if (lane < T) {
      slot = P[(int64_t)i * T + lane];
      float fs[MAXM], w[MAXM];
      for (int k = 0; k < M; ++k) {
        fs[k] = objs[(int64_t)slot * M + k];
        w[k] = W[(int64_t)slot * M + k];
      }
      pred = agg(func, fs, w, z, M) >= agg(func, fo, w, z, M);
    }
    const unsigned long long mask = __ballot(pred);
    const int rank = __popcll(mask & ((1ull << lane) - 1ull));
    if (pred && rank < nr) {
      for (int k = 0; k < M; ++k) objs[(int64_t)slot * M + k] = fo[k];
      owner[slot] = i;
    }
    __threadfence_block();
    __syncthreads();
  }
  if (lane == 0)
    for (int k = 0; k < M; ++k) z_io[k] = z[k];
}

}  // namespace

void evx_moead_scan(float* objs, const float* off_objs, const int32_t* P, const float* W, float* z, int32_t* owner, int N, int R,
                    int T, int M, int func, int nr, int update_z, hipStream_t s) {
  moead_scan_kernel<<<1, 64, 0, s>>>(objs, off_objs, P, W, z, owner, N, R, T, M, func, nr, update_z);
}
