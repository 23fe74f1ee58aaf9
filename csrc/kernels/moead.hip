// MOEA/D generation kernels (K11/K12 of SURVEY §2.10; reference
// algorithms/mo/moead.py:87-134, operators/crossover/sbx.py, operators/mutation/pm_mutation.py).
//
// At the north-star shape (N = 16 290 subproblems, T = 1 629 neighbours, d = 10 000)
// a generation is four passes:
//   1. parents: per subproblem, the first two entries of a uniform random permutation
//      of its neighbour list = the two smallest (u, j) of uniform(key, (N, T)) row i
//      (stable-argsort tie order).  One wave per row, (u24, j) packed into a u64 key.
//   2. variation: offspring i = clip(PM(SBX_type2(pop[p0_i], pop[p1_i]))) in ONE pass:
//      gathers the two parent rows, regenerates the SBX word (μ, sign, skip) and the PM
//      site uniform from Philox counters in-register — four consecutive genes share
//      one Philox block, so 2 blocks per 4 genes; PM's μ is drawn only at the rare
//      mutation sites — and writes the child once.  Same counters as the unfused
//      operators (operators/crossover/sbx.py, mutation), so results agree with them.
//   3. replace: the reference's sequential scan leaves slot s holding the FIRST
//      minimiser of agg(·, w_s) over [occupant, offspring i ∈ revN(s) ascending] with
//      strict improvement; one wave per slot walks its reverse-neighbour CSR row and
//      reduces (value, i) with lowest-index tie-break.  Only objective vectors move.
//   4. select rows: pop'[s] = win_s ≥ 0 ? off[win_s] : pop[s] (float4 copy).
#include "evoxmi_common.h"

namespace {
using namespace evx;

constexpr int MAXM = 16;

__device__ __forceinline__ uint32_t word_at(uint64_t i, uint32_t k0, uint32_t k1) {
  u4 w = philox_block(i >> 2, k0, k1);
  const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
  return ws[i & 3];
}

// 0 tchebycheff, 1 pbi (theta 5), 2 weighted sum, 3 modified tchebycheff, 4 normalised tchebycheff
__device__ __forceinline__ float agg(int func, const float* f, const float* w, const float* z, const float* zmax, int M) {
  if (func == 2) {
    float s = 0.f;
    for (int k = 0; k < M; ++k) s += f[k] * w[k];
    return s;
  }
  if (func == 1) {
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
    float v;
    if (func == 3) v = a / w[k];
    else if (func == 4) v = a / (zmax[k] - z[k]) * w[k];
    else v = a * w[k];
    g = fmaxf(g, v);
  }
  return g;
}

__device__ __forceinline__ void min2_merge(uint64_t& a1, uint64_t& a2, uint64_t b1, uint64_t b2) {
  const uint64_t lo = a1 < b1 ? a1 : b1, hi = a1 < b1 ? b1 : a1;
  const uint64_t s = a2 < b2 ? a2 : b2;
  a1 = lo;
  a2 = hi < s ? hi : s;
}

// rows [row0, row0 + N) of the (global) neighbour table; counters use the global row, so a
// rank drawing only its own slots' parents gets the full launch's values
__global__ void __launch_bounds__(256) parents_kernel(const int64_t* __restrict__ nb, int N, int T, const int64_t* __restrict__ key,
                                                      int32_t* __restrict__ p0, int32_t* __restrict__ p1, int row0) {
  const int lane = threadIdx.x & 63;
  const int row = row0 + blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= row0 + N) return;
  uint32_t k0, k1;
  load_key(key, k0, k1);
  uint64_t m1 = ~0ull, m2 = ~0ull;
  const uint64_t base = (uint64_t)row * T;
  for (int j = lane; j < T; j += 64) {
    const uint64_t kv = ((uint64_t)(word_at(base + j, k0, k1) >> 8) << 32) | (uint32_t)j;
    if (kv < m1) { m2 = m1; m1 = kv; }
    else if (kv < m2) m2 = kv;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t b1 = __shfl_xor(m1, o, 64), b2 = __shfl_xor(m2, o, 64);
    min2_merge(m1, m2, b1, b2);
  }
  if (lane == 0) {
    const int j1 = (int)(uint32_t)m1, j2 = (int)(uint32_t)(T > 1 ? m2 : m1);
    p0[row] = (int32_t)nb[(int64_t)row * T + j1];
    p1[row] = (int32_t)nb[(int64_t)row * T + j2];
  }
}

struct VarKeys {
  uint32_t g0, g1, pr0, pr1;  // SBX: split(key_x, 2) → per-gene word, per-pair rate
  uint32_t st0, st1, pm0, pm1;  // PM:  split(key_m, 2) → site, mu
};

// keys live on the device (graph-capturable): uniform scalar loads at kernel start
__device__ __forceinline__ VarKeys load_keys(const int64_t* __restrict__ kx, const int64_t* __restrict__ km) {
  return VarKeys{(uint32_t)kx[0], (uint32_t)kx[1], (uint32_t)kx[2], (uint32_t)kx[3],
                 (uint32_t)km[0], (uint32_t)km[1], (uint32_t)km[2], (uint32_t)km[3]};
}

// SBX child from the per-gene word: μ = top 24 bits, bit 0 = sign of β, bit 1 = skip gene
__device__ __forceinline__ float sbx_child(float a, float b, uint32_t w, bool no_x, float e) {
  float beta = 1.f;
  if (!no_x && !(w & 2u)) {
    const float mu = u24(w);
    beta = mu <= 0.5f ? exp2f(e * __log2f(2.f * mu)) : exp2f(-e * __log2f(2.f - 2.f * mu));
    if (w & 1u) beta = -beta;
  }
  return 0.5f * (a + b) + beta * (0.5f * (a - b));
}

// PM at one gene; μ is drawn (one more Philox block) only at the rare mutation sites
__device__ __forceinline__ float pm_gene(float v, float lo, float hi, uint32_t wst, uint64_t t, const VarKeys& K, float pr, float e1,
                                         float inv) {
  v = fmaxf(fminf(v, hi), lo);
  if (u24(wst) < pr) {
    const float span = hi - lo;
    const float mu = u24(word_at(t, K.pm0, K.pm1));
    if (mu <= 0.5f) {
      const float nrm = (v - lo) / span;
      v = v + span * (powf(2.f * mu + (1.f - 2.f * mu) * powf(1.f - nrm, e1), inv) - 1.f);
    } else {
      const float nrm = (hi - v) / span;
      v = v + span * (1.f - powf(2.f * (1.f - mu) + 2.f * (mu - 0.5f) * powf(1.f - nrm, e1), inv));
    }
  }
  return v;
}

// one thread = 4 consecutive genes (d % 4 == 0 ⇒ they share one Philox block per stream):
// 2 Philox blocks per 4 genes (SBX word + PM site) plus one per row for the pair rate
// Output row r holds offspring i = row0 + r, or (SELECT) i = win[r] with a copy of pop[r]
// where win[r] < 0: the population-sharded MOEA/D regenerates the winning offspring rows
// from the replicated population instead of shipping them between GPUs.  Counters use
// the global offspring index i, so every row is bit-identical to the full launch.
template <bool SELECT>
__global__ void __launch_bounds__(256) variation4_kernel(const float* __restrict__ pop, const int32_t* __restrict__ p0,
                                                         const int32_t* __restrict__ p1, float* __restrict__ out, int N, int d,
                                                         const int64_t* __restrict__ kx, const int64_t* __restrict__ km,
                                                         const float* __restrict__ lb, const float* __restrict__ ub,
                                                         float pro_c, float dis_c, float pro_m, float dis_m, int nm, int row0,
                                                         const int32_t* __restrict__ win) {
  const VarKeys K = load_keys(kx, km);
  const int q = d >> 2;
  const int64_t total = (int64_t)N * q;
  const float e = 1.f / (dis_c + 1.f), e1 = dis_m + 1.f, inv = 1.f / (dis_m + 1.f), pr = pro_m / d;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(t / q), c = (int)(t - (int64_t)r * q);
    const int j = c << 2;
    int i = row0 + r;
    if (SELECT) {
      i = win[r];
      if (i < 0) {
        *reinterpret_cast<float4*>(out + (int64_t)r * d + j) = *reinterpret_cast<const float4*>(pop + (int64_t)r * d + j);
        continue;
      }
    }
    const uint64_t g0 = (uint64_t)i * d + j;
    const float4 a = *reinterpret_cast<const float4*>(pop + (int64_t)p0[i] * d + j);
    const float4 b = *reinterpret_cast<const float4*>(pop + (int64_t)p1[i] * d + j);
    const float4 lo = *reinterpret_cast<const float4*>(lb + j);
    const float4 hi = *reinterpret_cast<const float4*>(ub + j);
    const u4 w = philox_block(g0 >> 2, K.g0, K.g1);
    const bool no_x = u24(word_at((uint64_t)i, K.pr0, K.pr1)) > pro_c;
    float4 y;
    y.x = sbx_child(a.x, b.x, w.x, no_x, e);
    y.y = sbx_child(a.y, b.y, w.y, no_x, e);
    y.z = sbx_child(a.z, b.z, w.z, no_x, e);
    y.w = sbx_child(a.w, b.w, w.w, no_x, e);
    if (i < nm) {
      const u4 ws = philox_block(g0 >> 2, K.st0, K.st1);
      y.x = pm_gene(y.x, lo.x, hi.x, ws.x, g0, K, pr, e1, inv);
      y.y = pm_gene(y.y, lo.y, hi.y, ws.y, g0 + 1, K, pr, e1, inv);
      y.z = pm_gene(y.z, lo.z, hi.z, ws.z, g0 + 2, K, pr, e1, inv);
      y.w = pm_gene(y.w, lo.w, hi.w, ws.w, g0 + 3, K, pr, e1, inv);
    }
    y.x = fmaxf(fminf(y.x, hi.x), lo.x);
    y.y = fmaxf(fminf(y.y, hi.y), lo.y);
    y.z = fmaxf(fminf(y.z, hi.z), lo.z);
    y.w = fmaxf(fminf(y.w, hi.w), lo.w);
    *reinterpret_cast<float4*>(out + (int64_t)r * d + j) = y;
  }
}

// generic d: one thread per gene
template <bool SELECT>
__global__ void __launch_bounds__(256) variation1_kernel(const float* __restrict__ pop, const int32_t* __restrict__ p0,
                                                         const int32_t* __restrict__ p1, float* __restrict__ out, int N, int d,
                                                         const int64_t* __restrict__ kx, const int64_t* __restrict__ km,
                                                         const float* __restrict__ lb, const float* __restrict__ ub,
                                                         float pro_c, float dis_c, float pro_m, float dis_m, int nm, int row0,
                                                         const int32_t* __restrict__ win) {
  const VarKeys K = load_keys(kx, km);
  const int64_t total = (int64_t)N * d;
  const float e = 1.f / (dis_c + 1.f), e1 = dis_m + 1.f, inv = 1.f / (dis_m + 1.f), pr = pro_m / d;
  for (int64_t tt = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; tt < total; tt += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(tt / d), j = (int)(tt - (int64_t)r * d);
    int i = row0 + r;
    if (SELECT) {
      i = win[r];
      if (i < 0) {
        out[tt] = pop[tt];
        continue;
      }
    }
    const int64_t t = (int64_t)i * d + j;  // global gene counter
    const float a = pop[(int64_t)p0[i] * d + j], b = pop[(int64_t)p1[i] * d + j];
    const bool no_x = u24(word_at((uint64_t)i, K.pr0, K.pr1)) > pro_c;
    float y = sbx_child(a, b, word_at(t, K.g0, K.g1), no_x, e);
    const float lo = lb[j], hi = ub[j];
    if (i < nm) y = pm_gene(y, lo, hi, word_at(t, K.st0, K.st1), (uint64_t)t, K, pr, e1, inv);
    out[tt] = fmaxf(fminf(y, hi), lo);
  }
}

// best candidate (lexicographic (value, offspring index)) of slot s over its CSR range, one wave:
// each slot has ~T candidates (T = ⌈N/10⌉, the reference's neighbourhood: 1629 at the
// north-star shape), so the scan is the work — every lane keeps U independent candidate chains
// (owner index → objective row → aggregation) in flight instead of one dependent chain per
// candidate (92.8 → 40.6 µs for the owner-mode halo at world 8)
template <int MA, int U>
__device__ __forceinline__ void scan_candidates(const float* __restrict__ off_obj, const int32_t* __restrict__ owner, int b, int e,
                                                const float* w, const float* z, const float* zm, int M, int func, float& best,
                                                int& bi) {
  const int lane = threadIdx.x & 63;
  best = INFINITY;
  bi = 0x7fffffff;
  for (int q0 = b + lane; q0 < e; q0 += U * 64) {
    int ii[U];
#pragma unroll
    for (int u = 0; u < U; ++u) ii[u] = q0 + 64 * u < e ? owner[q0 + 64 * u] : -1;
    float fv[U][MA];
#pragma unroll
    for (int u = 0; u < U; ++u)
      for (int k = 0; k < M; ++k) fv[u][k] = ii[u] >= 0 ? off_obj[(int64_t)ii[u] * M + k] : 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ii[u] < 0) continue;
      const float v = agg(func, fv[u], w, z, zm, M);
      if (v < best || (v == best && ii[u] < bi)) { best = v; bi = ii[u]; }
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float ob = __shfl_xor(best, o, 64);
    const int oi = __shfl_xor(bi, o, 64);
    if (ob < best || (ob == best && oi < bi)) { best = ob; bi = oi; }
  }
}

template <int MT>
__global__ void __launch_bounds__(256) replace_kernel(const float* __restrict__ pop_obj, const float* __restrict__ off_obj,
                                                      const float* __restrict__ W, const float* __restrict__ zp,
                                                      const float* __restrict__ zmaxp, const int32_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ owner, int N, int Mrt, int func,
                                                      int32_t* __restrict__ win, float* __restrict__ new_obj) {
  constexpr int MA = MT > 0 ? MT : MAXM;
  const int M = MT > 0 ? MT : Mrt;
  const int lane = threadIdx.x & 63;
  const int s = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (s >= N) return;
  float w[MA], z[MA], zm[MA], f[MA];
  for (int k = 0; k < M; ++k) {
    w[k] = W[(int64_t)s * M + k];
    z[k] = zp[k];
    zm[k] = zmaxp[k];
  }
  float best;
  int bi;
  scan_candidates<MA, (MT > 0 ? 8 : 4)>(off_obj, owner, rowptr[s], rowptr[s + 1], w, z, zm, M, func, best, bi);
  for (int k = 0; k < M; ++k) f[k] = pop_obj[(int64_t)s * M + k];
  const float old = agg(func, f, w, z, zm, M);
  const bool take = bi != 0x7fffffff && best < old;
  if (lane == 0) win[s] = take ? bi : -1;
  if (lane < M) new_obj[(int64_t)s * M + lane] = take ? off_obj[(int64_t)bi * M + lane] : pop_obj[(int64_t)s * M + lane];
}

__global__ void __launch_bounds__(256) select_rows_kernel(const float* __restrict__ pop, const float* __restrict__ off,
                                                          const int32_t* __restrict__ win, float* __restrict__ out, int N, int d) {
  const int row = blockIdx.y;
  const int w = win[row];
  const float* src = w >= 0 ? off + (int64_t)w * d : pop + (int64_t)row * d;
  float* dst = out + (int64_t)row * d;
  if ((d & 3) == 0) {
    const int q = d >> 2;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < q; c += gridDim.x * blockDim.x)
      reinterpret_cast<float4*>(dst)[c] = reinterpret_cast<const float4*>(src)[c];
  } else {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < d; c += gridDim.x * blockDim.x) dst[c] = src[c];
  }
}

// in-place variant: only the winning slots' rows are written (pop[s] = off[win[s]]); the
// hipGraph path updates the captured population buffer directly instead of building a new
// population that the graph's state write-back then copies back (2 × 651 MB per generation at
// the north-star shape)
__global__ void __launch_bounds__(256) select_rows_inplace_kernel(float* __restrict__ pop, const float* __restrict__ off,
                                                                  const int32_t* __restrict__ win, int N, int d) {
  const int row = blockIdx.y;
  const int w = win[row];
  if (w < 0) return;
  const float* src = off + (int64_t)w * d;
  float* dst = pop + (int64_t)row * d;
  if ((d & 3) == 0) {
    const int q = d >> 2;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < q; c += gridDim.x * blockDim.x)
      reinterpret_cast<float4*>(dst)[c] = reinterpret_cast<const float4*>(src)[c];
  } else {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < d; c += gridDim.x * blockDim.x) dst[c] = src[c];
  }
}

// Owner-computes MOEA/D (population-sharded): the replacement of only the slots a rank
// must keep current (its halo: every neighbour of its own slots), in place on the
// objective matrix (a slot reads and writes only its own row).
// owner mode: the same scan for the halo slots only, in place on the objective matrix
template <int MT>
__global__ void __launch_bounds__(256) halo_replace_kernel(float* __restrict__ obj, const float* __restrict__ off_obj,
                                                           const float* __restrict__ W, const float* __restrict__ zp,
                                                           const float* __restrict__ zmaxp, const int32_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ owner, const int32_t* __restrict__ slots,
                                                           int H, int Mrt, int func, int32_t* __restrict__ win_h) {
  constexpr int MA = MT > 0 ? MT : MAXM;
  const int M = MT > 0 ? MT : Mrt;
  const int lane = threadIdx.x & 63;
  const int h = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (h >= H) return;
  const int s = slots[h];
  float w[MA], z[MA], zm[MA], f[MA];
  for (int k = 0; k < M; ++k) {
    w[k] = W[(int64_t)s * M + k];
    z[k] = zp[k];
    zm[k] = zmaxp[k];
  }
  float best;
  int bi;
  scan_candidates<MA, (MT > 0 ? 8 : 4)>(off_obj, owner, rowptr[s], rowptr[s + 1], w, z, zm, M, func, best, bi);
  for (int k = 0; k < M; ++k) f[k] = obj[(int64_t)s * M + k];
  const float old = agg(func, f, w, z, zm, M);
  const bool take = bi != 0x7fffffff && best < old;
  if (lane == 0) win_h[h] = take ? bi : -1;
  if (take && lane < M) obj[(int64_t)s * M + lane] = off_obj[(int64_t)bi * M + lane];
}

// halo row update: slot slots[h] takes offspring win_h[h], read straight from the memory of
// the rank that generated it (peer[q] = that rank's offspring buffer, IPC-mapped over xGMI:
// a direct mesh read, no collective), rows of rank q start at starts[q]
// first[w] = INT_MAX for every offspring, then the lowest halo index that takes offspring w
__global__ void __launch_bounds__(256) halo_first_fill_kernel(int32_t* __restrict__ first, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < N) first[i] = INT_MAX;
}

__global__ void __launch_bounds__(256) halo_first_kernel(const int32_t* __restrict__ win_h, int H, int32_t* __restrict__ first, int N) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < H) {
    const int w = win_h[i];
    if (w >= 0 && w < N) atomicMin(first + w, i);
  }
}

// pop[slots[h]] ← offspring win_h[h] from the generating rank's buffer.  With `first`
// (deduplicated form) only the first halo slot taking an offspring reads it — an offspring that
// wins several of this rank's halo slots crosses xGMI once — and dup_copy_kernel then fills the
// other slots from that local row.
typedef float f32x4v __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) halo_gather_kernel(float* __restrict__ pop, const int32_t* __restrict__ slots,
                                                          const int32_t* __restrict__ win_h, const int64_t* __restrict__ peer,
                                                          const int32_t* __restrict__ starts, int world, int d,
                                                          const int32_t* __restrict__ first) {
  const int h = blockIdx.y;
  const int w = win_h[h];
  if (w < 0) return;
  if (first && first[w] != h) return;
  int q = 0;
  while (q + 1 < world && starts[q + 1] <= w) ++q;
  const float* src = reinterpret_cast<const float*>(peer[q]) + (int64_t)(w - starts[q]) * d;
  float* dst = pop + (int64_t)slots[h] * d;
  // (peer-buffer contract, parallel/peer.py: the peer_acquire launch before this kernel has
  // invalidated every XCD's caches at system scope; one fence per reading wave here measured
  // 0.678 vs 0.464 ms per MOEA/D generation at rank 0 of 8)
  if ((d & 3) == 0) {
    const int n4 = d >> 2;
    // peer rows are read once: non-temporal, so they do not displace this rank's own data in L2
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n4; c += gridDim.x * blockDim.x)
      reinterpret_cast<f32x4v*>(dst)[c] = __builtin_nontemporal_load(reinterpret_cast<const f32x4v*>(src) + c);
  } else {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < d; c += gridDim.x * blockDim.x) dst[c] = __builtin_nontemporal_load(src + c);
  }
}

__global__ void __launch_bounds__(256) halo_dup_copy_kernel(float* __restrict__ pop, const int32_t* __restrict__ slots,
                                                            const int32_t* __restrict__ win_h, const int32_t* __restrict__ first, int d) {
  const int h = blockIdx.y;
  const int w = win_h[h];
  if (w < 0) return;
  const int f = first[w];
  if (f == h) return;
  const float* src = pop + (int64_t)slots[f] * d;
  float* dst = pop + (int64_t)slots[h] * d;
  if ((d & 3) == 0) {
    const int n4 = d >> 2;
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < n4; c += gridDim.x * blockDim.x)
      reinterpret_cast<float4*>(dst)[c] = reinterpret_cast<const float4*>(src)[c];
  } else {
    for (int c = blockIdx.x * blockDim.x + threadIdx.x; c < d; c += gridDim.x * blockDim.x) dst[c] = src[c];
  }
}

int grid1(int64_t work) {
  int64_t g = (work + 255) / 256;
  return (int)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

}  // namespace

void evx_moead_parents(const int64_t* nb, int N, int T, const int64_t* key, int32_t* p0, int32_t* p1, hipStream_t s, int row0) {
  parents_kernel<<<(N + 3) / 4, 256, 0, s>>>(nb, N, T, key, p0, p1, row0);
}

void evx_moead_variation(const float* pop, const int32_t* p0, const int32_t* p1, float* out, int N, int d, const int64_t* kx,
                         const int64_t* km, const float* lb, const float* ub, float pro_c, float dis_c, float pro_m, float dis_m,
                         int nm, hipStream_t s, int row0, const int32_t* win) {
  if ((d & 3) == 0) {
    const int g = grid1((int64_t)N * (d >> 2));
    if (win) variation4_kernel<true><<<g, 256, 0, s>>>(pop, p0, p1, out, N, d, kx, km, lb, ub, pro_c, dis_c, pro_m, dis_m, nm, row0, win);
    else variation4_kernel<false><<<g, 256, 0, s>>>(pop, p0, p1, out, N, d, kx, km, lb, ub, pro_c, dis_c, pro_m, dis_m, nm, row0, win);
  } else {
    const int g = grid1((int64_t)N * d);
    if (win) variation1_kernel<true><<<g, 256, 0, s>>>(pop, p0, p1, out, N, d, kx, km, lb, ub, pro_c, dis_c, pro_m, dis_m, nm, row0, win);
    else variation1_kernel<false><<<g, 256, 0, s>>>(pop, p0, p1, out, N, d, kx, km, lb, ub, pro_c, dis_c, pro_m, dis_m, nm, row0, win);
  }
}

void evx_moead_replace(const float* pop_obj, const float* off_obj, const float* W, const float* z, const float* zmax,
                       const int32_t* rowptr, const int32_t* owner, int N, int M, int func, int32_t* win, float* new_obj,
                       hipStream_t s) {
  const int g = (N + 3) / 4;
  if (M == 3) replace_kernel<3><<<g, 256, 0, s>>>(pop_obj, off_obj, W, z, zmax, rowptr, owner, N, M, func, win, new_obj);
  else if (M == 2) replace_kernel<2><<<g, 256, 0, s>>>(pop_obj, off_obj, W, z, zmax, rowptr, owner, N, M, func, win, new_obj);
  else replace_kernel<0><<<g, 256, 0, s>>>(pop_obj, off_obj, W, z, zmax, rowptr, owner, N, M, func, win, new_obj);
}

void evx_moead_select_rows(const float* pop, const float* off, const int32_t* win, float* out, int N, int d, hipStream_t s) {
  const int q = (d & 3) == 0 ? d >> 2 : d;
  dim3 grid((q + 255) / 256 < 16 ? (q + 255) / 256 : 16, N);
  select_rows_kernel<<<grid, 256, 0, s>>>(pop, off, win, out, N, d);
}

void evx_moead_select_rows_inplace(float* pop, const float* off, const int32_t* win, int N, int d, hipStream_t s) {
  const int q = (d & 3) == 0 ? d >> 2 : d;
  dim3 grid((q + 255) / 256 < 16 ? (q + 255) / 256 : 16, N);
  select_rows_inplace_kernel<<<grid, 256, 0, s>>>(pop, off, win, N, d);
}

void evx_moead_halo_replace(float* obj, const float* off_obj, const float* W, const float* z, const float* zmax, const int32_t* rowptr,
                            const int32_t* owner, const int32_t* slots, int H, int M, int func, int32_t* win_h, hipStream_t s) {
  if (H <= 0) return;
  const int g = (H + 3) / 4;
  if (M == 3) halo_replace_kernel<3><<<g, 256, 0, s>>>(obj, off_obj, W, z, zmax, rowptr, owner, slots, H, M, func, win_h);
  else if (M == 2) halo_replace_kernel<2><<<g, 256, 0, s>>>(obj, off_obj, W, z, zmax, rowptr, owner, slots, H, M, func, win_h);
  else halo_replace_kernel<0><<<g, 256, 0, s>>>(obj, off_obj, W, z, zmax, rowptr, owner, slots, H, M, func, win_h);
}

// Peer-buffer contract (parallel/peer.py).  Writer side: a system-scope RELEASE after the kernels
// that wrote this rank's peer-visible buffer, stream-ordered before the collective that publishes
// it — dirty lines of EVERY XCD's L2 are written back to HBM, where peers' xGMI reads land (per-XCD
// L2s are not coherent with each other or with other GPUs, MI355X_MICROARCH.md).  Reader side: a
// system-scope ACQUIRE before the gather, so no XCD serves a peer row from a line cached by the
// previous generation's reads.  A fence acts on the issuing CU's L1 and its XCD's L2, so each runs
// in one lane of kPeerFenceBlocks workgroups: blocks are dealt round-robin over the 8 XCDs, and 8
// per XCD cover every XCD whatever the start.
constexpr int kPeerFenceBlocks = 64;

__global__ void peer_release_kernel() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

__global__ void peer_acquire_kernel() {
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
}

void evx_peer_release(hipStream_t s) { peer_release_kernel<<<kPeerFenceBlocks, 64, 0, s>>>(); }
void evx_peer_acquire(hipStream_t s) { peer_acquire_kernel<<<kPeerFenceBlocks, 64, 0, s>>>(); }

void evx_moead_halo_gather(float* pop, const int32_t* slots, const int32_t* win_h, int H, const int64_t* peer, const int32_t* starts,
                           int world, int d, hipStream_t s, int32_t* first, int N) {
  if (H <= 0) return;
  const int q = (d & 3) == 0 ? d >> 2 : d;
  dim3 grid((q + 255) / 256 < 16 ? (q + 255) / 256 : 16, H);
  if (first) {
    halo_first_fill_kernel<<<(N + 255) / 256, 256, 0, s>>>(first, N);
    halo_first_kernel<<<(H + 255) / 256, 256, 0, s>>>(win_h, H, first, N);
  }
  evx_peer_acquire(s);
  halo_gather_kernel<<<grid, 256, 0, s>>>(pop, slots, win_h, peer, starts, world, d, first);
  if (first) halo_dup_copy_kernel<<<grid, 256, 0, s>>>(pop, slots, win_h, first, d);
}
