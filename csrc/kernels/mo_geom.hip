// Geometry kernels of the multi-objective zoo.
//
// knn_kernel (K17): the T nearest rows of Y for every row of X (euclidean), sorted by
//   (distance, index) — MOEA/D weight neighbourhoods (reference moead.py:65-67 argsorts a
//   full N×N distance matrix), IGD/GD nearest distances (metrics/igd.py:7-21, T = 1),
//   SPEA2 / KnEA k-th neighbour distances.  One thread per query row keeps its top-T in
//   registers (branch-free insertion, T ≤ 32); the candidates stream through LDS in tiles
//   shared by the 256 rows of a workgroup.  No N×M matrix is ever materialised: MOEA/D
//   at N = 16384 needs 16384 × T floats instead of 1 GiB.
//
// hv_count_kernel / hv_contrib_kernel (K18): Monte-Carlo hypervolume.  count[s] = number
//   of points that dominate sample s (strict "sample < point" for the HV metric on
//   |objs − ref|, reference metrics/hypervolume.py:7-59; "point ≤ sample" for HypE,
//   hype.py:21-53).  HypE's contribution f[i] = Σ_s [point i dominates s] · α[count[s] − 1]
//   is a second pass with one workgroup per point and a fixed-order reduction
//   (deterministic, no float atomics).
#include "evoxmi_common.h"
#include <float.h>

namespace {

constexpr int kKnnThreads = 256;

// Σ (x − y)² unfused, in index order (no FMA contraction despite -ffp-contract=fast):
// bit-identical to the CPU oracle ((x − y)²).sum(-1), so exactly tied distances (lattice
// weight vectors) order identically on both
__device__ __forceinline__ float sqdist(const float (&x)[64], const float* y, int m) {
#pragma clang fp contract(off)
  float d2 = 0.f;
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    if (k < m) {
      const float df = x[k] - y[k];
      d2 = d2 + df * df;
    }
  }
  return d2;
}
constexpr int kKnnTile = 4096;  // floats of Y per LDS tile (16 KiB)

template <int T>
__global__ void __launch_bounds__(kKnnThreads) knn_kernel(const float* __restrict__ X, const float* __restrict__ Y, int N, int M,
                                                         int m, int t_out, float* __restrict__ out_d, int32_t* __restrict__ out_i) {
  __shared__ float ys[kKnnTile];
  const int row = blockIdx.x * kKnnThreads + threadIdx.x;
  float x[64];
  const bool live = row < N;
#pragma unroll
  for (int k = 0; k < 64; ++k) x[k] = (live && k < m) ? X[(int64_t)row * m + k] : 0.f;
  float bd[T];
  int bi[T];
#pragma unroll
  for (int t = 0; t < T; ++t) {  // empty slots: (+inf, INT_MAX) — any candidate beats them
    bd[t] = INFINITY;
    bi[t] = 0x7fffffff;
  }
  const int rows_per_tile = kKnnTile / m;
  for (int j0 = 0; j0 < M; j0 += rows_per_tile) {
    const int nr = min(rows_per_tile, M - j0);
    __syncthreads();
    for (int e = threadIdx.x; e < nr * m; e += kKnnThreads) ys[e] = Y[(int64_t)j0 * m + e];
    __syncthreads();
    if (!live) continue;
    for (int jj = 0; jj < nr; ++jj) {
      const float* y = ys + jj * m;  // same address in every lane: LDS broadcast
      // a NaN distance ranks first (key −inf, reported as NaN: torch.cdist(..).min() and the
      // reference propagate it); (key, index) order, so an inf distance still fills an
      // empty slot and an equal key never displaces an earlier index
      float d2 = sqdist(x, y, m);
      d2 = (d2 != d2) ? -INFINITY : d2;
      const int j = j0 + jj;
      if (d2 < bd[T - 1] || (d2 == bd[T - 1] && j < bi[T - 1])) {
#pragma unroll
        for (int t = T - 1; t > 0; --t) {
          const bool shift = d2 < bd[t - 1] || (d2 == bd[t - 1] && j < bi[t - 1]);
          const bool here = !shift && (d2 < bd[t] || (d2 == bd[t] && j < bi[t]));
          bd[t] = shift ? bd[t - 1] : (here ? d2 : bd[t]);
          bi[t] = shift ? bi[t - 1] : (here ? j : bi[t]);
        }
        if (d2 < bd[0] || (d2 == bd[0] && j < bi[0])) {
          bd[0] = d2;
          bi[0] = j;
        }
      }
    }
  }
  if (!live) return;
#pragma unroll
  for (int t = 0; t < T; ++t) {
    if (t < t_out) {
      out_d[(int64_t)row * t_out + t] = bd[t] == -INFINITY ? NAN : sqrtf(bd[t]);
      out_i[(int64_t)row * t_out + t] = bi[t];
    }
  }
}

// count[s] = #{i : dom(point_i, sample_s)}; strict: sample < point in every objective,
// else point ≤ sample in every objective.  Points staged through LDS.
__global__ void __launch_bounds__(256) hv_count_kernel(const float* __restrict__ S, const float* __restrict__ P, int ns, int np, int m,
                                                       int strict, int32_t* __restrict__ count) {
  __shared__ float ps[4096];
  const int s = blockIdx.x * 256 + threadIdx.x;
  float x[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) x[k] = (s < ns && k < m) ? S[(int64_t)s * m + k] : 0.f;
  int c = 0;
  const int per = 4096 / m;
  for (int i0 = 0; i0 < np; i0 += per) {
    const int nr = min(per, np - i0);
    __syncthreads();
    for (int e = threadIdx.x; e < nr * m; e += 256) ps[e] = P[(int64_t)i0 * m + e];
    __syncthreads();
    for (int i = 0; i < nr; ++i) {
      const float* p = ps + i * m;
      bool dom = true;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k < m) dom = dom && (strict ? (x[k] < p[k]) : (p[k] <= x[k]));
      c += dom ? 1 : 0;
    }
  }
  if (s < ns) count[s] = c;
}

// f[i] = Σ_s [point i ≤ sample s] · alpha[count[s] − 1]: one workgroup per point, strided
// samples, fixed-order tree reduction
__global__ void __launch_bounds__(256) hv_contrib_kernel(const float* __restrict__ S, const float* __restrict__ P,
                                                         const int32_t* __restrict__ count, const float* __restrict__ alpha, int ns,
                                                         int np, int m, float* __restrict__ f) {
  __shared__ float red[256];
  const int i = blockIdx.x;
  float p[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) p[k] = k < m ? P[(int64_t)i * m + k] : 0.f;
  float acc = 0.f;
  for (int s = threadIdx.x; s < ns; s += 256) {
    bool dom = true;
#pragma unroll
    for (int k = 0; k < 16; ++k)
      if (k < m) dom = dom && (p[k] <= S[(int64_t)s * m + k]);
    const int c = count[s];
    acc += (dom && c > 0) ? alpha[c - 1] : 0.f;
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) f[i] = red[0];
}

}  // namespace

int evx_knn_max_t() { return 32; }
int evx_knn_max_m() { return 64; }

void evx_knn(const float* X, const float* Y, int N, int M, int m, int T, float* out_d, int32_t* out_i, hipStream_t s) {
  const dim3 g((N + kKnnThreads - 1) / kKnnThreads), b(kKnnThreads);
  if (T <= 1) knn_kernel<1><<<g, b, 0, s>>>(X, Y, N, M, m, T, out_d, out_i);
  else if (T <= 4) knn_kernel<4><<<g, b, 0, s>>>(X, Y, N, M, m, T, out_d, out_i);
  else if (T <= 8) knn_kernel<8><<<g, b, 0, s>>>(X, Y, N, M, m, T, out_d, out_i);
  else if (T <= 16) knn_kernel<16><<<g, b, 0, s>>>(X, Y, N, M, m, T, out_d, out_i);
  else knn_kernel<32><<<g, b, 0, s>>>(X, Y, N, M, m, T, out_d, out_i);
}

int evx_hv_max_m() { return 16; }

void evx_hv_count(const float* S, const float* P, int ns, int np, int m, int strict, int32_t* count, hipStream_t s) {
  hv_count_kernel<<<(ns + 255) / 256, 256, 0, s>>>(S, P, ns, np, m, strict, count);
}

void evx_hv_contrib(const float* S, const float* P, const int32_t* count, const float* alpha, int ns, int np, int m, float* f,
                    hipStream_t s) {
  hv_contrib_kernel<<<np, 256, 0, s>>>(S, P, count, alpha, ns, np, m, f);
}
