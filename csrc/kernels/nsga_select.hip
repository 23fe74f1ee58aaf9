// NSGA-II environmental selection after the non-dominated sort (K10 of SURVEY §2.10;
// reference algorithms/mo/nsga2.py:86-100 and operators/selection/non_dominate.py:116-204).
//
// Semantics reproduced exactly: worst = sorted(rank)[mask_pos]; crowding distance on the
// front `rank == worst` (per objective: stable sort by cost, extremes +inf, interior
// (c[p+1] − c[p−1]) / (c[last] − c[0]), summed over objectives; rows outside the front
// get −inf); survivors = lexsort((−cd, rank))[:N] (stable: ties by row index).
//
// One workgroup of 1024 threads × 8 items does it all on chip (n ≤ 8192).  Every sort is
// rocPRIM's stable LDS block radix sort with the items held in registers (blocked
// arrangement), so a sort is a handful of 4-bit digit passes instead of the 91
// compare-exchange rounds of a bitonic network:
//   1. (rank, row) over only the bits the ranks use → the survivors of ranks < worst in
//      output order, and the worst front [lo, hi) in row order;
//   2. per objective, (cost, slot) over the front → crowding distance, neighbours
//      exchanged through DPP shuffles + one LDS word per wave;
//   3. (−cd, slot) → the remaining survivors.
// Steps 2–3 sort 1024·IT keys with IT ∈ {1, 2, 4, 8} picked from the front size.
// Float keys are canonicalised first (NaN → +qNaN, −0 → +0) so the bit-order radix sort
// agrees with torch.sort (NaN last, ±0 equal, stable ties).
// It replaces ~60 small library launches (sorts, gathers, scatters, lexsort) per
// generation with one.
#include <rocprim/block/block_radix_sort.hpp>

#include "evoxmi_common.h"

namespace {

constexpr int SEL_THREADS = 1024;
constexpr int SEL_ITEMS = 8;
constexpr int SEL_MAXN = SEL_THREADS * SEL_ITEMS;  // 8192
constexpr int SEL_WAVES = SEL_THREADS / 64;

using rank_sort_t = rocprim::block_radix_sort<uint32_t, SEL_THREADS, SEL_ITEMS, uint32_t>;
template <int IT>
using key_sort_t = rocprim::block_radix_sort<float, SEL_THREADS, IT, uint32_t>;

union SortStorage {
  typename rank_sort_t::storage_type r;
  typename key_sort_t<1>::storage_type k1;
  typename key_sort_t<2>::storage_type k2;
  typename key_sort_t<4>::storage_type k4;
  typename key_sort_t<8>::storage_type k8;
};

template <int IT>
__device__ __forceinline__ typename key_sort_t<IT>::storage_type& key_storage(SortStorage& st) {
  if constexpr (IT == 1) return st.k1;
  else if constexpr (IT == 2) return st.k2;
  else if constexpr (IT == 4) return st.k4;
  else return st.k8;
}

__device__ __forceinline__ float canon(float x) {
  if (x != x) return __int_as_float(0x7fc00000);
  return x == 0.f ? 0.f : x;
}

struct SelShared {
  SortStorage sort;
  uint32_t srow[SEL_MAXN];  // rows in (rank, row) order
  uint32_t srank[SEL_MAXN];
  float cd[SEL_MAXN];       // crowding distance per front slot
  float wave_first[SEL_WAVES], wave_last[SEL_WAVES];
  float key0, keyl;
  int lo, hi, maxr;
};

// Crowding distance on the front slots [0, F) (rows srow[lo + slot]) and the `need`
// best slots by (−cd, slot); IT items per thread cover F <= 1024·IT, so a small worst
// front sorts IT·1024 keys instead of 8192.
template <int IT>
__device__ void crowd_select(SelShared& sh, const float* __restrict__ f, int m, int lo, int F, int need, int64_t* __restrict__ keep) {
  const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
  const int base = t * IT;
  using sort_t = key_sort_t<IT>;
#pragma unroll
  for (int i = 0; i < IT; ++i) sh.cd[base + i] = 0.f;
  for (int obj = 0; obj < m; ++obj) {
    float k[IT];
    uint32_t v[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int s = base + i;
      // +qNaN padding ties with real NaNs but sits after them (stable: larger slots)
      k[i] = s < F ? canon(f[(int64_t)sh.srow[lo + s] * m + obj]) : __int_as_float(0x7fc00000);
      v[i] = (uint32_t)s;
    }
    __syncthreads();  // sort storage reuse and the cd writes of the previous objective
    sort_t().sort(k, v, key_storage<IT>(sh.sort));
    // neighbour keys across the thread boundary: shuffles within the wave, LDS across waves
    float prev = __shfl_up(k[IT - 1], 1);
    float next = __shfl_down(k[0], 1);
    if (lane == 0) sh.wave_first[wave] = k[0];
    if (lane == 63) sh.wave_last[wave] = k[IT - 1];
    if (t == 0) sh.key0 = k[0];
#pragma unroll
    for (int i = 0; i < IT; ++i)
      if (base + i == F - 1) sh.keyl = k[i];
    __syncthreads();
    if (lane == 0 && wave > 0) prev = sh.wave_last[wave - 1];
    if (lane == 63 && wave < SEL_WAVES - 1) next = sh.wave_first[wave + 1];
    const float rng = sh.keyl - sh.key0;
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int p = base + i;
      if (p < F) {
        const float kp = i > 0 ? k[i - 1] : prev;
        const float kn = i < IT - 1 ? k[i + 1] : next;
        const float d = (p == 0 || p == F - 1) ? INFINITY : (kn - kp) / rng;
        sh.cd[v[i]] += d;  // v is a permutation of the slots: no two threads share a slot
      }
    }
  }
  __syncthreads();
  // remaining survivors: the worst front by (−cd, slot)
  float k[IT];
  uint32_t v[IT];
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int s = base + i;
    k[i] = s < F ? canon(-sh.cd[s]) : __int_as_float(0x7fc00000);
    v[i] = (uint32_t)s;
  }
  sort_t().sort(k, v, key_storage<IT>(sh.sort));
#pragma unroll
  for (int i = 0; i < IT; ++i) {
    const int p = base + i;
    if (p < need) keep[lo + p] = (int64_t)sh.srow[lo + v[i]];
  }
}

__global__ void __launch_bounds__(SEL_THREADS) nsga_select_kernel(const int32_t* __restrict__ rank, const float* __restrict__ f, int n, int m,
                                                                   int N, int mask_pos, int64_t* __restrict__ keep) {
  __shared__ SelShared sh;
  const int t = threadIdx.x;
  const int base = t * SEL_ITEMS;

  // 1. stable sort of rows by rank.  Unranked rows (rank n, past the early stop) map to
  // max ranked + 1, so the radix sort only walks the bits the ranks actually use.
  uint32_t k[SEL_ITEMS], v[SEL_ITEMS];
  int mr = -1;
#pragma unroll
  for (int i = 0; i < SEL_ITEMS; ++i) {
    const int r = base + i;
    k[i] = r < n ? (uint32_t)min(max(rank[r], 0), n) : (uint32_t)n;
    if ((int)k[i] < n) mr = max(mr, (int)k[i]);
    v[i] = (uint32_t)r;
  }
  if (t == 0) { sh.lo = n; sh.hi = n; sh.maxr = -1; }
  __syncthreads();
  mr = (int)evx::wave_max((float)mr);  // exact: ranks ≤ 8192
  if ((t & 63) == 0) atomicMax(&sh.maxr, mr);
  __syncthreads();
  const uint32_t cap = (uint32_t)(sh.maxr + 1);  // ≤ n ≤ 8192
  int bits = 1;
  while ((1u << bits) <= cap) ++bits;
#pragma unroll
  for (int i = 0; i < SEL_ITEMS; ++i) k[i] = k[i] > cap ? cap : k[i];
  rank_sort_t().sort(k, v, sh.sort.r, 0, bits);
#pragma unroll
  for (int i = 0; i < SEL_ITEMS; ++i) { sh.srank[base + i] = k[i]; sh.srow[base + i] = v[i]; }
  __syncthreads();
  const uint32_t worst = sh.srank[mask_pos];
#pragma unroll
  for (int i = 0; i < SEL_ITEMS; ++i) {
    const int p = base + i;
    if (p < n) {
      const uint32_t r = sh.srank[p];
      const uint32_t rp = p > 0 ? sh.srank[p - 1] : 0xFFFFFFFFu;
      if (r == worst && (p == 0 || rp != worst)) sh.lo = p;  // first slot of the worst front
      if (r > worst && (p == 0 || rp <= worst)) sh.hi = p;   // first slot after it
    }
  }
  __syncthreads();
  const int lo = sh.lo, hi = sh.hi, F = hi - lo;
  // survivors of ranks < worst, already in (rank, row) order
  for (int i = t; i < lo && i < N; i += SEL_THREADS) keep[i] = (int64_t)sh.srow[i];
  const int need = N - lo;
  if (need <= 0) return;  // uniform: every thread leaves together
  if (F <= SEL_THREADS) crowd_select<1>(sh, f, m, lo, F, need, keep);
  else if (F <= 2 * SEL_THREADS) crowd_select<2>(sh, f, m, lo, F, need, keep);
  else if (F <= 4 * SEL_THREADS) crowd_select<4>(sh, f, m, lo, F, need, keep);
  else crowd_select<8>(sh, f, m, lo, F, need, keep);
}

}  // namespace

void evx_nsga_select(const int32_t* rank, const float* f, int n, int m, int N, int mask_pos, int64_t* keep, hipStream_t s) {
  nsga_select_kernel<<<1, SEL_THREADS, 0, s>>>(rank, f, n, m, N, mask_pos, keep);
}
