// Non-dominated sorting on the GPU (K9).
//
// 1. dominance kernel: DT[j][w] bit b set ⇔ individual i = 32w + b dominates j
//    (minimisation: ≤ in every objective, < in at least one).  Each thread builds one
//    32-bit word from 32 compares of m objectives; objectives of the 32 candidates are
//    staged in LDS.  cnt[j] = popcount over the row = number of dominators of j.
// 2. peel kernel: ONE workgroup (1024 threads) peels the fronts without returning to
//    the host: the current front is kept as a bitmask F (n/32 words in LDS) plus the
//    list of its non-zero words; each unranked j subtracts Σ popcount(DT[j][w] & F[w])
//    over that list.  The loop runs until every row is ranked.
#include "evoxmi_common.h"

namespace {

template <int M>
__global__ void __launch_bounds__(256) dominance_kernel(const float* __restrict__ f, int n, int m, int nw,
                                                        uint32_t* __restrict__ DT) {
  // grid.x over words w (blockDim.y = 1), each thread a row j
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int w = blockIdx.y;
  __shared__ float cand[32 * 8];
  const int mm = M > 0 ? M : m;
  for (int e = threadIdx.x; e < 32 * mm; e += blockDim.x) {
    const int b = e / mm, k = e - b * mm;
    const int i = 32 * w + b;
    cand[b * mm + k] = i < n ? f[(int64_t)i * m + k] : INFINITY;
  }
  __syncthreads();
  if (j >= n) return;
  float fj[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) fj[k] = k < mm ? f[(int64_t)j * m + k] : 0.f;
  uint32_t word = 0;
  for (int b = 0; b < 32; ++b) {
    if (32 * w + b >= n) break;
    bool le = true, lt = false;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < mm) {
        const float a = cand[b * mm + k];
        le = le && (a <= fj[k]);
        lt = lt || (a < fj[k]);
      }
    }
    if (le && lt) word |= (1u << b);
  }
  DT[(int64_t)j * nw + w] = word;
}

__global__ void __launch_bounds__(1024) peel_kernel(const uint32_t* __restrict__ DT, int n, int nw, int32_t* __restrict__ rank,
                                                    int32_t* __restrict__ cnt_g) {
  extern __shared__ uint32_t smem[];
  uint32_t* F = smem;                         // nw words: current front bitmask
  uint32_t* nzw = smem + nw;                  // list of non-zero word ids
  __shared__ int nnz, front_size;
  // dominator counts
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    int c = 0;
    for (int w = 0; w < nw; ++w) c += __popc(DT[(int64_t)j * nw + w]);
    cnt_g[j] = c;
    rank[j] = -1;
  }
  __syncthreads();
  for (int r = 0;; ++r) {
    for (int w = threadIdx.x; w < nw; w += blockDim.x) F[w] = 0;
    if (threadIdx.x == 0) { nnz = 0; front_size = 0; }
    __syncthreads();
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
      if (rank[j] < 0 && cnt_g[j] == 0) {
        rank[j] = r;
        atomicOr(&F[j >> 5], 1u << (j & 31));
        atomicAdd(&front_size, 1);
      }
    }
    __syncthreads();
    if (front_size == 0) break;
    for (int w = threadIdx.x; w < nw; w += blockDim.x)
      if (F[w]) nzw[atomicAdd(&nnz, 1)] = w;
    __syncthreads();
    const int nz = nnz;
    for (int j = threadIdx.x; j < n; j += blockDim.x) {
      if (rank[j] >= 0) continue;
      int dec = 0;
      const uint32_t* row = DT + (int64_t)j * nw;
      for (int q = 0; q < nz; ++q) {
        const int w = nzw[q];
        dec += __popc(row[w] & F[w]);
      }
      cnt_g[j] -= dec;
    }
    __syncthreads();
  }
}

}  // namespace

void evx_nds(const float* f, int n, int m, uint32_t* DT, int32_t* rank, int32_t* cnt, hipStream_t s) {
  const int nw = (n + 31) / 32;
  dim3 grid((n + 255) / 256, nw);
  if (m == 2) dominance_kernel<2><<<grid, 256, 0, s>>>(f, n, m, nw, DT);
  else if (m == 3) dominance_kernel<3><<<grid, 256, 0, s>>>(f, n, m, nw, DT);
  else dominance_kernel<0><<<grid, 256, 0, s>>>(f, n, m, nw, DT);
  const size_t shm = 2 * (size_t)nw * sizeof(uint32_t);
  peel_kernel<<<1, 1024, shm, s>>>(DT, n, nw, rank, cnt);
}
