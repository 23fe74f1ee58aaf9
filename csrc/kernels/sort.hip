// Single-workgroup argsort (K19) for populations up to 16384 — register + LDS bitonic.
//
// Keys are f32 fitness values mapped to order-preserving u32 and packed with the
// 32-bit index into one u64, so a single 64-bit compare orders by (key, index):
// deterministic and identical to a stable sort (torch semantics: NaN is the largest
// value).  1024 threads each hold E = NP/1024 consecutive elements in registers:
//   * compare-exchange stages with stride j < E run entirely in registers (the stage
//     structure is unrolled at compile time so no register is indexed dynamically);
//   * stages with j ≥ E exchange whole per-thread runs with partner thread t ^ (j/E)
//     through LDS: one vectorised write (ds_write_b128), barrier, one vectorised read
//     of the partner's run, barrier.  Runs are padded to 144 B so the ds_read_b128 lane
//     groups hit distinct banks.
// At NP = 16384: 55 LDS stages instead of the 105 of an all-LDS bitonic network.
#include "evoxmi_common.h"
#include <float.h>
#include <rocprim/block/block_radix_sort.hpp>

namespace {

__device__ __forceinline__ uint32_t f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}

template <int E>
struct Run {
  unsigned long long v[E];
};

// in-register compare-exchange for all strides j < E of phase k (e0 = global index of v[0])
template <int E>
__device__ __forceinline__ void reg_stages(Run<E>& R, int k, int e0) {
#pragma unroll
  for (int j = E / 2; j > 0; j >>= 1) {
#pragma unroll
    for (int r = 0; r < E; ++r) {
      if ((r & j) == 0) {
        const int e = e0 + r;
        const bool up = (e & k) == 0;
        unsigned long long a = R.v[r], b = R.v[r + j];
        const bool sw = (a > b) == up;
        R.v[r] = sw ? b : a;
        R.v[r + j] = sw ? a : b;
      }
    }
  }
}

template <int LOGN>
__global__ void __launch_bounds__(1024) bitonic_argsort_kernel(const float* __restrict__ keys, int n, int descending,
                                                               float* __restrict__ out_keys, int32_t* __restrict__ out_idx) {
  // one workgroup per row (batched runs sort their rows in one launch)
  keys += (int64_t)blockIdx.x * n;
  out_idx += (int64_t)blockIdx.x * n;
  if (out_keys) out_keys += (int64_t)blockIdx.x * n;
  constexpr int NP = 1 << LOGN;
  constexpr int T = 1024;
  constexpr int E = NP / T;  // 1..16
  constexpr int RUN_U64 = E < 2 ? E : E + 2;  // pad runs (144 B for E = 16) to spread banks
  __shared__ unsigned long long s[T * RUN_U64];
  const int t = threadIdx.x;
  const int e0 = t * E;
  Run<E> R;
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const int i = e0 + r;
    unsigned long long v = 0xFFFFFFFFFFFFFFFFull;
    if (i < n) {
      const float k = keys[i];
      uint32_t o = (k != k) ? (descending ? 0u : 0xFFFFFFFFu) : f2ord(descending ? -k : k);
      v = ((unsigned long long)o << 32) | (uint32_t)i;
    }
    R.v[r] = v;
  }
  // phases k ≤ E: entirely in registers
#pragma unroll
  for (int k = 2; k <= E; k <<= 1) {
#pragma unroll
    for (int j = k / 2; j > 0; j >>= 1) {
#pragma unroll
      for (int r = 0; r < E; ++r) {
        if ((r & j) == 0) {
          const bool up = ((e0 + r) & k) == 0;
          unsigned long long a = R.v[r], b = R.v[r + j];
          const bool sw = (a > b) == up;
          R.v[r] = sw ? b : a;
          R.v[r + j] = sw ? a : b;
        }
      }
    }
  }
  for (int k = 2 * E; k <= NP; k <<= 1) {
    for (int j = k >> 1; j >= E; j >>= 1) {
      const int pt = t ^ (j / E);
      unsigned long long* mine = s + t * RUN_U64;
      const unsigned long long* theirs = s + pt * RUN_U64;
#pragma unroll
      for (int r = 0; r < E; ++r) mine[r] = R.v[r];
      __syncthreads();
      const bool lower = (t & (j / E)) == 0;
#pragma unroll
      for (int r = 0; r < E; ++r) {
        const int e = e0 + r;
        const bool up = (e & k) == 0;
        unsigned long long a = R.v[r], b = theirs[r];
        // lower element keeps min when ascending, upper keeps max
        const bool take_min = (lower == up);
        R.v[r] = take_min ? (a < b ? a : b) : (a > b ? a : b);
      }
      __syncthreads();
    }
    reg_stages<E>(R, k, e0);
  }
#pragma unroll
  for (int r = 0; r < E; ++r) {
    const int i = e0 + r;
    if (i < n) {
      const int32_t src = (int32_t)(R.v[r] & 0xFFFFFFFFu);
      if (out_keys) out_keys[i] = keys[src];
      out_idx[i] = src;
    }
  }
}

// Single-workgroup LDS radix argsort (rocPRIM block radix sort, 1024 threads × IT keys
// held in registers, 8-bit digits): 4 scatter passes through LDS instead of the bitonic
// network's 55 LDS stages.  Stable: keys are loaded in blocked order with index payloads,
// padding (the extreme NaN bit pattern, index ≥ n) sorts behind every real key, so ties
// break by index as in torch.sort(stable=True).
template <int IT>
__global__ void __launch_bounds__(1024) radix_argsort_kernel(const float* __restrict__ keys, int n, int descending,
                                                             float* __restrict__ out_keys, int32_t* __restrict__ out_idx) {
  using sort_t = rocprim::block_radix_sort<float, 1024, IT, int32_t>;
  __shared__ typename sort_t::storage_type storage;
  const float* kb = keys + (int64_t)blockIdx.x * n;
  float k[IT];
  int32_t v[IT];
  // padding sorts behind every real key, NaNs included (largest / smallest NaN bit patterns)
  const float pad = __uint_as_float(descending ? 0xffffffffu : 0x7fffffffu);
  // every NaN (either sign bit) becomes the largest key 0x7fffffff, so NaNs sort last when
  // ascending (tied with the padding, which follows by index) and first when descending, as
  // torch.sort does; -0.0 becomes +0.0 (torch treats them as equal keys: index order)
  const float qnan = __uint_as_float(0x7fffffffu);
#pragma unroll
  for (int r = 0; r < IT; ++r) {
    const int i = threadIdx.x * IT + r;
    float x = i < n ? kb[i] : pad;
    if (i < n) x = (x != x) ? qnan : (x == 0.f ? 0.f : x);
    k[r] = x;
    v[r] = i;
  }
  if (descending)
    sort_t().sort_desc(k, v, storage);
  else
    sort_t().sort(k, v, storage);
  float* ok = out_keys ? out_keys + (int64_t)blockIdx.x * n : nullptr;
  int32_t* oi = out_idx + (int64_t)blockIdx.x * n;
#pragma unroll
  for (int r = 0; r < IT; ++r) {
    const int i = threadIdx.x * IT + r;
    if (i < n) {
      if (ok) ok[i] = kb[v[r]];  // the original bits (NaN payloads, signed zeros)
      oi[i] = v[r];
    }
  }
}

// Rank-by-counting argsort (K19 at 10⁴-class n): rank(i) = #{j : k_j < k_i or (k_j = k_i and j < i)}
// on order-preserving u32 keys, so the result is a stable sort.  All n keys sit in LDS; a
// workgroup ranks 64 consecutive elements (one per lane), its WAVES waves splitting the key
// range and reading four keys per LDS broadcast into four independent counters.  The tie
// test is needed only for j inside the workgroup's own 64 elements: below them every j < i
// (count k_j ≤ k_i), above them none (count k_j < k_i) — one compare + one add per key.
// 16 waves per workgroup (4 per SIMD) hide the LDS latency of the broadcast chain; the
// single-wave-per-SIMD first cut ran 53.6 µs at n = 16384 (profiles/r3_sort_microbench.log).
__device__ __forceinline__ uint32_t ord_key(float x, bool desc) {
  x = (x != x) ? __uint_as_float(0x7fffffffu) : (x == 0.f ? 0.f : x);  // NaN largest, -0 == +0
  const uint32_t o = f2ord(x);
  return desc ? ~o : o;
}

//
// Chunked mode (m > 0, the first pass of the merge sort below): blockIdx.y = row * C + chunk, the
// workgroup ranks inside its m-key chunk only and writes the chunk-sorted ORDERED keys to ws_keys and
// the row-global indices to out_idx, both at row * N + chunk * m + rank.
template <int WAVES>
__global__ void __launch_bounds__(64 * WAVES) rank_argsort_kernel(const float* __restrict__ keys, int N, int desc,
                                                                  float* __restrict__ out_keys, int32_t* __restrict__ out_idx,
                                                                  int m = 0, uint32_t* __restrict__ ws_keys = nullptr) {
  extern __shared__ uint4 sk4[];  // 16-byte aligned: the compare loops read four keys per ds_read_b128
  __shared__ int part[WAVES][64];
  uint32_t* sk = reinterpret_cast<uint32_t*>(sk4);
  const int C = m > 0 ? (N + m - 1) / m : 1;
  const int row = blockIdx.y / C, cb = m > 0 ? (int)(blockIdx.y % C) * m : 0;
  const int n = m > 0 ? min(m, N - cb) : N;  // keys in this workgroup's chunk
  const float* kb = keys + (int64_t)row * N + cb;
  const int np = (n + 3) & ~3;
  const bool d = desc != 0;
  if (((n | N | cb) & 3) == 0) {  // 16-byte aligned: float4 loads, all in flight before the first use
    const float4* kb4 = reinterpret_cast<const float4*>(kb);
#pragma unroll 4
    for (int v = threadIdx.x; v < (n >> 2); v += 64 * WAVES) {
      const float4 x = kb4[v];
      sk4[v] = make_uint4(ord_key(x.x, d), ord_key(x.y, d), ord_key(x.z, d), ord_key(x.w, d));
    }
  } else {
#pragma unroll 4
    for (int i = threadIdx.x; i < np; i += 64 * WAVES) sk[i] = i < n ? ord_key(kb[min(i, n - 1)], d) : 0xffffffffu;  // pads: never counted
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int b = blockIdx.x * 64, i = b + lane;
  const uint32_t ki = i < n ? sk[i] : 0u;
  const int q = ((np >> 2) + WAVES - 1) / WAVES * 4;
  const int lo = min(np, w * q), hi = min(np, lo + q);
  int c0 = 0, c1 = 0, c2 = 0, c3 = 0;
  const int e0 = min(hi, b), s1 = max(lo, b), e1 = min(hi, b + 64), s2 = max(lo, b + 64);
  // [lo, b): every j < i
  for (int j = lo; j < e0; j += 4) {
    const uint4 k4 = sk4[j >> 2];
    c0 += k4.x <= ki;
    c1 += k4.y <= ki;
    c2 += k4.z <= ki;
    c3 += k4.w <= ki;
  }
  // the workgroup's own elements: explicit index tie-break
  for (int j = s1; j < e1; j += 4) {
    const uint4 k4 = sk4[j >> 2];
    c0 += (k4.x < ki) | ((k4.x == ki) & (j < i));
    c1 += (k4.y < ki) | ((k4.y == ki) & (j + 1 < i));
    c2 += (k4.z < ki) | ((k4.z == ki) & (j + 2 < i));
    c3 += (k4.w < ki) | ((k4.w == ki) & (j + 3 < i));
  }
  // [b + 64, hi): every j > i
  for (int j = s2; j < hi; j += 4) {
    const uint4 k4 = sk4[j >> 2];
    c0 += k4.x < ki;
    c1 += k4.y < ki;
    c2 += k4.z < ki;
    c3 += k4.w < ki;
  }
  part[w][lane] = (c0 + c1) + (c2 + c3);
  __syncthreads();
  if (w == 0 && i < n) {
    int r = 0;
#pragma unroll
    for (int v = 0; v < WAVES; ++v) r += part[v][lane];
    const int64_t o = (int64_t)row * N + cb + r;
    out_idx[o] = cb + i;
    if (ws_keys) ws_keys[o] = ki;
    else if (out_keys) out_keys[o] = kb[i];
  }
}

// Second pass of the merge sort for n beyond one LDS-resident row: element p of chunk c (sorted by the
// chunked rank pass) lands at  p - c·m + Σ_{c' ≠ c} #{keys of chunk c' before it}, counting equal keys of
// earlier chunks (smaller indices) and not those of later ones — the stable-sort position.  The CMAX
// binary searches run in lockstep, branch-free over the fixed log2(m) + 1 levels, so each level issues up to
// CMAX - 1 independent L2 loads per lane instead of one dependent chain per chunk.
template <int CMAX, int LOGM>
__global__ void __launch_bounds__(256) corank_merge_kernel(const float* __restrict__ keys, const uint32_t* __restrict__ wk,
                                                           const int32_t* __restrict__ wi, int N, float* __restrict__ out_keys,
                                                           int32_t* __restrict__ out_idx) {
  constexpr int M = 1 << LOGM;
  const int row = blockIdx.y, p = blockIdx.x * 256 + threadIdx.x;
  if (p >= N) return;
  const int C = (N + M - 1) >> LOGM;
  const uint32_t* rk = wk + (int64_t)row * N;
  const uint32_t k = rk[p];
  const int c = p >> LOGM;
  int base[CMAX];
#pragma unroll
  for (int c2 = 0; c2 < CMAX; ++c2) base[c2] = 0;  // #keys of chunk c2 that go before k
#pragma unroll
  for (int half = M; half >= 1; half >>= 1) {  // halves sum to 2M - 1: a whole chunk of M keys can be before k
#pragma unroll
    for (int c2 = 0; c2 < CMAX; ++c2) {
      if (c2 >= C || c2 == c) continue;
      const int len = min(M, N - (c2 << LOGM));
      const int probe = base[c2] + half;  // is the key at position probe - 1 before k?
      if (probe <= len) {
        const uint32_t v = rk[(c2 << LOGM) + probe - 1];
        if (c2 < c ? v <= k : v < k) base[c2] = probe;
      }
    }
  }
  int pos = p - (c << LOGM);
#pragma unroll
  for (int c2 = 0; c2 < CMAX; ++c2) pos += base[c2];
  const int gi = wi[(int64_t)row * N + p];
  out_idx[(int64_t)row * N + pos] = gi;
  if (out_keys) out_keys[(int64_t)row * N + pos] = keys[(int64_t)row * N + gi];
}


// The same merge with the row's chunk-sorted keys staged in LDS (n ≤ 32768: 128 KiB), so the
// log2(m) + 1 search levels are LDS round trips instead of L2 ones.
template <int CMAX, int LOGM>
__global__ void __launch_bounds__(1024) corank_merge_lds_kernel(const float* __restrict__ keys, const uint32_t* __restrict__ wk,
                                                                const int32_t* __restrict__ wi, int N, float* __restrict__ out_keys,
                                                                int32_t* __restrict__ out_idx) {
  extern __shared__ uint32_t srk[];
  constexpr int M = 1 << LOGM;
  const int row = blockIdx.y, p = blockIdx.x * 1024 + threadIdx.x;
  const uint32_t* rk = wk + (int64_t)row * N;
#pragma unroll 4
  for (int j = threadIdx.x; j < N; j += 1024) srk[j] = rk[j];
  __syncthreads();
  if (p >= N) return;
  const int C = (N + M - 1) >> LOGM;
  const uint32_t k = srk[p];
  const int c = p >> LOGM;
  int base[CMAX];
#pragma unroll
  for (int c2 = 0; c2 < CMAX; ++c2) base[c2] = 0;
#pragma unroll
  for (int half = M; half >= 1; half >>= 1) {
#pragma unroll
    for (int c2 = 0; c2 < CMAX; ++c2) {
      if (c2 >= C || c2 == c) continue;
      const int len = min(M, N - (c2 << LOGM));
      const int probe = base[c2] + half;
      if (probe <= len) {
        const uint32_t v = srk[(c2 << LOGM) + probe - 1];
        if (c2 < c ? v <= k : v < k) base[c2] = probe;
      }
    }
  }
  int pos = p - (c << LOGM);
#pragma unroll
  for (int c2 = 0; c2 < CMAX; ++c2) pos += base[c2];
  const int gi = wi[(int64_t)row * N + p];
  out_idx[(int64_t)row * N + pos] = gi;
  if (out_keys) out_keys[(int64_t)row * N + pos] = keys[(int64_t)row * N + gi];
}

}  // namespace

void evx_radix_argsort(const float* keys, int n, int descending, float* out_keys, int32_t* out_idx, hipStream_t s, int batch) {
  if (n <= 2048) radix_argsort_kernel<2><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx);
  else if (n <= 4096) radix_argsort_kernel<4><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx);
  else if (n <= 8192) radix_argsort_kernel<8><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx);
  else if (n <= 10240) radix_argsort_kernel<10><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx);
  else if (n <= 12288) radix_argsort_kernel<12><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx);
  else radix_argsort_kernel<16><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx);
}

int evx_argsort_max_n() { return 16384; }

void evx_argsort(const float* keys, int n, int descending, float* out_keys, int32_t* out_idx, hipStream_t s, int batch) {
  int logn = 10;
  while ((1 << logn) < n) ++logn;
  switch (logn) {
    case 10: bitonic_argsort_kernel<10><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
    case 11: bitonic_argsort_kernel<11><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
    case 12: bitonic_argsort_kernel<12><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
    case 13: bitonic_argsort_kernel<13><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
    default: bitonic_argsort_kernel<14><<<batch, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
  }
}

int evx_rank_argsort_max_n() { return 16384; }

void evx_rank_argsort(const float* keys, int n, int descending, float* out_keys, int32_t* out_idx, hipStream_t s, int batch) {
  const int np = (n + 3) & ~3;
  const size_t lds = (size_t)np * 4;
  const dim3 grid((n + 63) / 64, batch);
  if (n < 256) {
    rank_argsort_kernel<4><<<grid, 256, lds, s>>>(keys, n, descending, out_keys, out_idx);
  } else {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)rank_argsort_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    rank_argsort_kernel<16><<<grid, 1024, lds, s>>>(keys, n, descending, out_keys, out_idx);
  }
}

int evx_merge_argsort_max_n() { return 16 * 4096; }

void evx_merge_argsort(const float* keys, int n, int descending, float* out_keys, int32_t* out_idx, uint32_t* ws_keys,
                       int32_t* ws_idx, hipStream_t s, int batch) {
  constexpr int LOGM = 12, M = 1 << LOGM;
  const int C = (n + M - 1) / M;
  rank_argsort_kernel<16><<<dim3(M / 64, batch * C), 1024, M * 4, s>>>(keys, n, descending, nullptr, ws_idx, M, ws_keys);
  if ((size_t)n * 4 <= 128 * 1024) {  // the whole chunk-sorted row fits in LDS: search there
    const dim3 g((n + 1023) / 1024, batch);
    const size_t lds = (size_t)n * 4;
    if (lds > 64 * 1024) {
      (void)hipFuncSetAttribute((const void*)corank_merge_lds_kernel<4, LOGM>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      (void)hipFuncSetAttribute((const void*)corank_merge_lds_kernel<8, LOGM>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    }
    if (C <= 4)
      corank_merge_lds_kernel<4, LOGM><<<g, 1024, lds, s>>>(keys, ws_keys, ws_idx, n, out_keys, out_idx);
    else
      corank_merge_lds_kernel<8, LOGM><<<g, 1024, lds, s>>>(keys, ws_keys, ws_idx, n, out_keys, out_idx);
    return;
  }
  const dim3 grid((n + 255) / 256, batch);
  if (C <= 4)
    corank_merge_kernel<4, LOGM><<<grid, 256, 0, s>>>(keys, ws_keys, ws_idx, n, out_keys, out_idx);
  else if (C <= 8)
    corank_merge_kernel<8, LOGM><<<grid, 256, 0, s>>>(keys, ws_keys, ws_idx, n, out_keys, out_idx);
  else
    corank_merge_kernel<16, LOGM><<<grid, 256, 0, s>>>(keys, ws_keys, ws_idx, n, out_keys, out_idx);
}
