// Non-dominated sorting on the GPU (K9 of SURVEY §2.10; reference
// operators/selection/non_dominate.py:30-113).
//
// 1. dominance kernel: word-major bit matrix DW[w][j], bit b set ⇔ individual
//    i = 32w + b dominates j (minimisation: ≤ in every objective, < in at least one).
//    Word-major so a wave's 64 lanes (64 consecutive j) read 256 contiguous bytes.
//    The 32 candidates of word w are staged in LDS.
// 2. peel kernel: a chip-wide persistent grid (≤ 256 workgroups of 64 rows × 4 word
//    quarters, all co-resident on the 256 CUs) computes one front per iteration.  j joins front k iff every
//    dominator of j is already ranked:  DW[w][j] & ~R[w] == 0 for all w, where R is
//    the ranked bitset (early exit at the first word with an unranked dominator; the
//    next front's test of the same row resumes at that word).  R is double-buffered and only ever OR-ed
//    (R_next |= R_cur | new-front bits), so one grid barrier per front suffices; the
//    loop ends when the per-iteration "still unranked" counter is zero or at least
//    `limit` rows are ranked (NSGA-II only needs fronts until N survivors are
//    covered: the rest get rank = n).  The barrier spins with a bound: on timeout
//    the kernel sets an error flag and every wave exits (no hang is possible).
#include "evoxmi_common.h"
#include <stdlib.h>

namespace {

template <int M>
__global__ void __launch_bounds__(256) dominance_kernel(const float* __restrict__ f, int n, int m, int nw,
                                                        uint32_t* __restrict__ DW) {
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
  const int nb = min(32, n - 32 * w);
  for (int b = 0; b < nb; ++b) {
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
  DW[(int64_t)w * n + j] = word;
}

// workspace layout (uint32): [0] barrier count, [1] barrier generation, [2] error flag,
// [3] ranked total, [4 .. 4+nw) R0, [4+nw .. 4+2nw) R1, [4+2nw .. 4+2nw+n+1) left[k],
// then 4n words: per-(row, word-quarter) resume word (words before it hold only ranked
// dominators, and R only grows, so each scan continues where the previous front's stopped)
constexpr int kSpinLimit = 1 << 24;

__device__ __forceinline__ bool grid_barrier(uint32_t* ws, uint32_t nblocks, uint32_t& gen) {
  __syncthreads();
  __shared__ int ok;
  if (threadIdx.x == 0) {
    ok = 1;
    __threadfence();
    const uint32_t arrived = __hip_atomic_fetch_add(&ws[0], 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) + 1;
    if (arrived == nblocks) {
      __hip_atomic_store(&ws[0], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&ws[1], gen + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    } else {
      int spins = 0;
      while (__hip_atomic_load(&ws[1], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == gen) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > kSpinLimit) {
          __hip_atomic_store(&ws[2], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = 0;
          break;
        }
      }
    }
    __threadfence();
  }
  __syncthreads();
  gen += 1;
  return ok && __hip_atomic_load(&ws[2], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
}

// Peel layout: a workgroup owns 64 rows j (one per lane) and its four waves split each
// row's dominance words into quarters, so the sequential early-exit scan of a row is a
// quarter as long; words are loaded CHUNK at a time (independent loads in flight), the
// ranked bitset of the front is copied to LDS once per front, and every (row, quarter)
// keeps a resume pointer (words before it hold only ranked dominators; R only grows).
constexpr int PEEL_CHUNK = 16;
constexpr int PEEL_PARTS = 8;  // waves per workgroup = word parts per row
constexpr int PEEL_MAXW = 2048;  // n <= 65536

__global__ void __launch_bounds__(64 * PEEL_PARTS) peel_kernel(const uint32_t* __restrict__ DW, int n, int nw, int limit,
                                                   int32_t* __restrict__ rank, uint32_t* __restrict__ ws, int32_t* __restrict__ err,
                                                   int barrier_extra) {
  uint32_t* R[2] = {ws + 4, ws + 4 + nw};
  uint32_t* left = ws + 4 + 2 * nw;
  uint32_t* wptr = left + n + 1;  // 4 per row
  const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
  const int qlen = (nw + PEEL_PARTS - 1) / PEEL_PARTS, w0q = q * qlen, w1q = min(nw, w0q + qlen);
  __shared__ uint32_t Rs[PEEL_MAXW];
  __shared__ uint8_t fail_q[PEEL_PARTS][64];
  __shared__ uint8_t done_s[4][64];  // ranked flags of this workgroup's rows (≤ 4 passes: n ≤ 65536)
  __shared__ uint32_t wg_left;
  uint32_t gen = 0;
  const int rows_per_pass = gridDim.x * 64;
  for (int j = blockIdx.x * 64 + lane; j < n; j += rows_per_pass)
    if (q == 0) rank[j] = -1;
  if (q < 4) done_s[q][lane] = 0;
  for (int j = blockIdx.x * 64 + lane; j < n; j += rows_per_pass) wptr[PEEL_PARTS * (int64_t)j + q] = (uint32_t)w0q;
  for (int k = 0;; ++k) {
    const uint32_t* Rc = R[k & 1];
    uint32_t* Rn = R[(k + 1) & 1];
    if (threadIdx.x == 0) wg_left = 0;
    for (int w = threadIdx.x; w < nw; w += blockDim.x) Rs[w] = __hip_atomic_load(&Rc[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // carry the ranked set into the next buffer (it holds R_{k-1} ⊆ R_k)
    for (int w = blockIdx.x * blockDim.x + threadIdx.x; w < nw; w += gridDim.x * blockDim.x) {
      const uint32_t v = __hip_atomic_load(&Rc[w], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (v) __hip_atomic_fetch_or(&Rn[w], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    uint32_t my_left = 0, my_ranked = 0;  // my_ranked: lane-uniform in wave 0
    for (int jb = blockIdx.x * 64, pass = 0; jb < n; jb += rows_per_pass, ++pass) {
      const int j = jb + lane;
      const bool active = j < n && !done_s[pass][lane];
      bool fail = false;
      if (active) {
        int w = (int)wptr[PEEL_PARTS * (int64_t)j + q];
        while (w < w1q && !fail) {
          uint32_t d[PEEL_CHUNK];
#pragma unroll
          for (int u = 0; u < PEEL_CHUNK; ++u) d[u] = (w + u < w1q) ? DW[(int64_t)(w + u) * n + j] : 0u;
          int f = PEEL_CHUNK;
#pragma unroll
          for (int u = PEEL_CHUNK - 1; u >= 0; --u)
            if (w + u < w1q && (d[u] & ~Rs[w + u])) f = u;
          if (f < PEEL_CHUNK) { w += f; fail = true; }
          else w += PEEL_CHUNK;
        }
        wptr[PEEL_PARTS * (int64_t)j + q] = (uint32_t)min(w, w1q);
      }
      fail_q[q][lane] = fail;
      __syncthreads();
      if (q == 0) {
        // wave 0 owns the 64 rows: ballot the new front members, one atomic OR per 32-row
        // word (jb is a multiple of 64) and one ranked-count add per workgroup per front
        bool any_fail = false;
#pragma unroll
        for (int p2 = 0; p2 < PEEL_PARTS; ++p2) any_fail |= fail_q[p2][lane];
        const bool free_ = active && !any_fail;
        const uint64_t m = __ballot(free_);
        if (free_) {
          rank[j] = k;
          done_s[pass][lane] = 1;
        } else if (active) {
          ++my_left;
        }
        if (lane == 0 && (uint32_t)m) __hip_atomic_fetch_or(&Rn[jb >> 5], (uint32_t)m, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (lane == 32 && (uint32_t)(m >> 32)) __hip_atomic_fetch_or(&Rn[(jb >> 5) + 1], (uint32_t)(m >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        my_ranked += __popcll(m);
      }
      __syncthreads();
    }
    if (my_left) atomicAdd(&wg_left, my_left);
    __syncthreads();
    if (threadIdx.x == 0 && wg_left)
      __hip_atomic_fetch_add(&left[k], wg_left, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (threadIdx.x == 0 && my_ranked)
      __hip_atomic_fetch_add(&ws[3], my_ranked, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (!grid_barrier(ws, gridDim.x + barrier_extra, gen)) {
      // a workgroup never arrived (not co-resident): rows not ranked yet go last (rank n,
      // never the best front) and the sticky device error word tells the host
      for (int jb = blockIdx.x * 64, pass = 0; jb < n; jb += rows_per_pass, ++pass)
        if (q == 0 && jb + lane < n && !done_s[pass][lane]) rank[jb + lane] = n;
      if (threadIdx.x == 0 && err) __hip_atomic_fetch_or(err, 4, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return;
    }
    const uint32_t still = __hip_atomic_load(&left[k], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t done = __hip_atomic_load(&ws[3], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (still == 0) return;
    if ((int)done >= limit || k + 1 >= n) {
      for (int jb = blockIdx.x * 64, pass = 0; jb < n; jb += rows_per_pass, ++pass)
        if (q == 0 && jb + lane < n && !done_s[pass][lane]) rank[jb + lane] = n;
      return;
    }
  }
}

__global__ void __launch_bounds__(256) zero_kernel(uint32_t* __restrict__ p, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) p[i] = 0u;
}

}  // namespace

size_t evx_nds_workspace_words(int n) { return 4 + 2 * (size_t)((n + 31) / 32) + (PEEL_PARTS + 1) * (size_t)n + 1; }

// Workgroups the persistent peel may use: every one must be co-resident for the grid
// barrier, so the grid is capped by the device's CU count × the kernel's occupancy
// (hipOccupancy… on this kernel), not by a hard-coded 256.  Returns 0 if the peel cannot
// run co-resident at this n (the caller falls back to the host-orchestrated peel).
int evx_nds_peel_blocks(int n) {
  static int capacity = -1;
  if (capacity < 0) {
    int dev = 0, cus = 0, per_cu = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, peel_kernel, 64 * PEEL_PARTS, 0) != hipSuccess) per_cu = 0;
    capacity = cus * per_cu;
  }
  static const int cap = [] { const char* e = getenv("EVOXMI_NDS_BLOCKS"); const int v = e ? atoi(e) : (1 << 30); return v < 1 ? 1 : v; }();
  int blocks = min(min((n + 63) / 64, cap), capacity);
  const int need = (n + 255) / 256;  // the kernel keeps ≤ 4 row passes per workgroup in LDS
  if (blocks < need) return 0;
  return blocks;
}

void evx_nds(const float* f, int n, int m, int limit, uint32_t* DW, int32_t* rank, uint32_t* ws, int32_t* err, int blocks,
             hipStream_t s) {
  const int nw = (n + 31) / 32;
  dim3 grid((n + 255) / 256, nw);
  if (m == 2) dominance_kernel<2><<<grid, 256, 0, s>>>(f, n, m, nw, DW);
  else if (m == 3) dominance_kernel<3><<<grid, 256, 0, s>>>(f, n, m, nw, DW);
  else dominance_kernel<0><<<grid, 256, 0, s>>>(f, n, m, nw, DW);
  // a kernel, not hipMemsetAsync: the workspace must be zeroed inside captured hipGraphs too
  const int64_t nws = (int64_t)evx_nds_workspace_words(n);
  const int zb = (int)((nws + 255) / 256 < 64 ? (nws + 255) / 256 : 64);
  zero_kernel<<<zb, 256, 0, s>>>(ws, nws);
  // fault-injection hook for the error-path test: the barrier then waits for a workgroup
  // that is never launched, times out, and the sticky error word must report it
  static const int extra = getenv("EVOXMI_NDS_FAULT_TEST") ? 1 : 0;
  peel_kernel<<<blocks, 64 * PEEL_PARTS, 0, s>>>(DW, n, nw, limit, rank, ws, err, extra);
}
