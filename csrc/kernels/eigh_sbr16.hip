// Sorted-block refinement with 16-wide blocks in a cyclically shifted sorted order (K4, v3).
//
// The block step of SBR (eigh_sbr.hip) diagonalises the near (clustered) pairs of the
// sorted diagonal exactly.  With 64-wide blocks that is 126 dependent Jacobi rounds per
// iteration in 16 workgroups (≈134 µs, a third of the converged solve): the chip idles
// on a latency chain.  Measured on CMA-ES matrices at d = 1000 (CPU reference, five
// generation depths), 16-wide blocks with a far-pair threshold of thr_fac = 0.5 converge in
// the same number of refinement iterations once past the first generations (4 at gens 25 /
// 40; 26 vs 24 iterations summed over gens 4-40), because the far step's atan generator
// already handles every pair whose gap exceeds 8·thr_fac·spread/n.  A 16×16 block is 30
// rounds of one wave, ~60 workgroups instead of 16.
//
// Layout: position j of the shifted sorted order is index perm[j] = argsort(diag)[(j + shift)
// mod n]; blocks are always [16k, 16k + 16) of that order (shift = 0 / 8 on alternate
// iterations so that rank-adjacent pairs share a block in one of two iterations).  Because
// the blocks are aligned, the generator / Bq kernels work on 64×64 tiles that contain
// exactly four blocks and contract only over 16-wide block-diagonal factors (4× fewer
// FMAs than a dense 64-wide product).
//
//   sbr16_rank_kernel   perm by rank counting (strict total order on (diag, index))
//   sbr16_block_kernel  one wave per 16-block: 2 cyclic Jacobi sweeps in LDS → Q, dq
//   sbr16_far_kernel    X = ½·atan(2·A1/(d_e − d_c)) on far cross-block pairs,
//                       A1 = blockdiag(Q)ᵀ A[perm, perm] blockdiag(Q)
//   sbr16_bq_kernel     Bq = B[:, perm] · blockdiag(Q)
// evoxmi/ops/sbr.py holds the torch reference of each step and the host driver.
#include "evoxmi_common.h"
#include "evoxmi_sbr.h"
#include <float.h>
#include <math.h>
#include <cstdlib>

namespace {

// block size SB ∈ {16, 32} is a template parameter; LDS pitch SB + 1 (odd: conflict-free columns)
constexpr int TL = 64;            // tile of the generator / Bq kernels (four blocks)
// LDS pitches of the 64-wide tiles, chosen for the f32 MFMA fragment reads (ds_read_b32 banks =
// word address mod 32 per 32-lane half; lanes (m = lane & 15, kq = lane >> 4)):
//  * TP (≡ 16 mod 32): tiles read along rows, lane m ↔ column, kq ↔ row (Q tiles, the
//    generator's gathered block as the B operand) — kq = 0 / 1 land on banks 0-15 / 16-31;
//  * TC (≡ 2 mod 32): tiles read along columns, lane m ↔ row (T and the Bq rows as the A
//    operand) — rows 2 banks apart, kq = 0 / 1 on the even / odd banks.
constexpr int TP = 80;
constexpr int TC = 66;
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int BQR = 32;  // rows of a Bq tile: twice the workgroups of 64-row tiles, better latency hiding
constexpr int kRankMax = 8192;    // largest n of the rank kernel (32 KB of keys in LDS)

__device__ __forceinline__ float sort_key(float v) { return isnan(v) ? INFINITY : v; }

// ------------------------------------------------------------------ 1. ranks → shifted perm
// 64 indices per workgroup; its 16 waves each count over a sixteenth of the keys (16 waves:
// the counting loop is 4× shorter than with 4, and the launch stays at ⌈n/64⌉ workgroups)
constexpr int kRankWaves = 16;
__global__ void __launch_bounds__(64 * kRankWaves) sbr16_rank_kernel(const float* __restrict__ A, int n, int64_t lda, int shift,
                                                                     int* __restrict__ perm, const int* __restrict__ skip) {
  if (skip && *skip) return;
  __shared__ __attribute__((aligned(16))) float key[kRankMax + 16];
  __shared__ int part[kRankWaves][64];
  const int np = (n + 15) & ~15;  // padded with +inf: never below a real key (NaN keys are +inf too, ties by index)
  for (int i = threadIdx.x; i < np; i += blockDim.x) key[i] = i < n ? sort_key(A[(int64_t)i * lda + i]) : INFINITY;
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane;
  const float ki = i < n ? key[i] : 0.f;
  // each wave counts over a sixteenth of the keys, 4 keys per LDS broadcast read (ds_read_b128)
  const int q = ((np / kRankWaves) + 3) & ~3, j0 = min(np, w * q), j1 = min(np, j0 + q);
  int cnt = 0;
#pragma unroll 4
  for (int j = j0; j < j1; j += 4) {
    const float4 k4 = *(const float4*)(key + j);  // same address across the wave: broadcast
    cnt += (k4.x < ki) | ((k4.x == ki) & (j < i));
    cnt += (k4.y < ki) | ((k4.y == ki) & (j + 1 < i));
    cnt += (k4.z < ki) | ((k4.z == ki) & (j + 2 < i));
    cnt += (k4.w < ki) | ((k4.w == ki) & (j + 3 < i));
  }
  part[w][lane] = cnt;
  __syncthreads();
  if (w == 0 && i < n) {
    int r = 0;
#pragma unroll
    for (int v = 0; v < kRankWaves; ++v) r += part[v][lane];
    int pos = r - shift;
    if (pos < 0) pos += n;
    perm[pos] = i;
  }
}

// circle-method round robin on SB slots: round r pairs (SB−1, r) and ((r+i) mod (SB−1), (r−i) mod (SB−1))
template <int SB>
__device__ __forceinline__ int2 rr16(int r, int i) {
  int a = SB - 1, b = r;
  if (i) {
    a = r + i;
    if (a >= SB - 1) a -= SB - 1;
    b = r - i;
    if (b < 0) b += SB - 1;
  }
  return make_int2(min(a, b), max(a, b));
}

// (c, s, t) of the Jacobi rotation annihilating [[app, apq], [apq, aqq]]; only on a
// normal-range coupling (a denormal apq would overflow the reciprocal)
__device__ __forceinline__ float3 rot16(float app, float aqq, float apq) {
  const bool on = fabsf(apq) >= FLT_MIN;
  const float theta = (aqq - app) * (0.5f * __builtin_amdgcn_rcpf(on ? apq : 1.f));
  float t = copysignf(__builtin_amdgcn_rcpf(fabsf(theta) + __builtin_amdgcn_sqrtf(fmaf(theta, theta, 1.f))), theta);
  t = on ? t : 0.f;
  const float c = __builtin_amdgcn_rsqf(fmaf(t, t, 1.f));
  return make_float3(c, t * c, t);
}

// ------------------------------------------------------------------ 2. block solve
// One wave per block.  Per round: lanes 0-7 compute the 8 rotations (→ LDS), then lane
// {u ≤ v} (36 items) forms the 2×2 blocks (u, v) and (v, u) of S' = Jᵀ S J (written as exact
// transposes: S stays symmetric; pair u's own block set exactly), and every lane rotates a
// 2×2 block of Q' = Q J (rows 2(L/8)+{0,1}, column pair L mod 8).  All updates are in place:
// the 2×2 blocks of one round partition S and Q.
// (A fused-rank variant — every workgroup ranking the keys itself, one launch per slot fewer —
// measured slower: 1.867 vs 1.689 ms per flagship generation in round 5, 42 vs 27 + 8 µs per
// executed solve in round 4; removed in round 6, profiles/NOTES.md.)

// Threads: 2·SB²/4 — the first SB²/4 (waves 0-3 for SB = 32) rotate Q, the others (the
// SB/2·(SB/2+1)/2 items {u ≤ v}) update S, so the two updates of a round run side by side on
// different SIMDs instead of one after the other in every lane; the round-robin pairs come from
// a table built once in LDS (the index arithmetic was a third of the round's instructions).
template <int SB>
__global__ void __launch_bounds__(SB * SB / 2) sbr16_block_kernel(const float* __restrict__ A, int n, int64_t lda,
                                                                 int* __restrict__ perm, int sweeps, float* __restrict__ Q_out,
                                                                 float* __restrict__ dq_out, const int* __restrict__ skip, int shift,
                                                                 float skip_tol) {
  if (skip && *skip) return;
  constexpr int SP = SB + 1, NT = SB * SB / 4, NH = SB / 2;
  __shared__ float S[SB * SP];
  __shared__ float Qm[SB * SP];
  __shared__ float4 rot[NH];
  __shared__ int members[SB];
  __shared__ int2 ptab[(SB - 1) * NH];
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int s0 = blockIdx.x * SB, m = min(SB, n - s0);
  for (int e = tid; e < (SB - 1) * NH; e += nthr) ptab[e] = rr16<SB>(e / NH, e % NH);
  if (tid < SB) members[tid] = tid < m ? perm[s0 + tid] : -1;
  __syncthreads();
  for (int e = tid; e < SB * SB; e += nthr) {
    const int a = e / SB, c = e % SB;
    const int ra = members[a], rc = members[c];
    S[a * SP + c] = (ra >= 0 && rc >= 0) ? A[(int64_t)ra * lda + rc] : 0.f;
    Qm[a * SP + c] = a == c ? 1.f : 0.f;
  }
  __syncthreads();
  const bool qlane = tid < NT;
  // Q lanes: row qrow, column pairs qv0 and qv0 + SB/4 — the 32 lanes of a half-wave share one
  // pair and cover 32 rows, so their Q reads and writes hit 32 distinct banks (row pitch ≡ 1 mod
  // 32); the round-4 map (two rows × 16 pairs per half-wave) conflicted whenever two pairs' columns
  // differed by the row offset (SQ_LDS_BANK_CONFLICT 48 %, profiles/r5_pmc_flagship.txt)
  const int qrow = tid % SB, qv0 = tid / SB;
  // S lanes: item {u ≤ v}
  int u = 0, rem = tid - NT;
  while (u < NH - 1 && rem >= NH - u) {
    rem -= NH - u;
    ++u;
  }
  const int v = u + rem;
  const bool item = !qlane && rem >= 0 && (tid - NT) < NH * (NH + 1) / 2;
  const bool dg = u == v;
  const int G = (SB - 1) * sweeps;
  __shared__ float s_off[SB * SB / 128], s_dg[SB * SB / 128];
  __shared__ int s_done;
  for (int g = 0; g < G; ++g) {
    const int r = g % (SB - 1);
    if (r == 0 && skip_tol > 0.f) {
      // before every sweep: a block already diagonal to skip_tol (relative off-diagonal norm)
      // skips its remaining sweeps — after one sweep of the quadratically converging cyclic
      // Jacobi the second one is usually below rounding in the later refinement iterations
      float off = 0.f, dg = 0.f;
      for (int e = tid; e < SB * SB; e += nthr) {
        const int a = e / SB, c = e % SB;
        const float v = S[a * SP + c];
        if (a == c) dg = fmaf(v, v, dg);
        else off = fmaf(v, v, off);
      }
      off = evx::wave_sum(off);
      dg = evx::wave_sum(dg);
      if ((tid & 63) == 0) {
        s_off[tid >> 6] = off;
        s_dg[tid >> 6] = dg;
      }
      __syncthreads();
      if (tid == 0) {
        float o = 0.f, d = 0.f;
        for (int w = 0; w < nthr / 64; ++w) {
          o += s_off[w];
          d += s_dg[w];
        }
        s_done = o <= skip_tol * skip_tol * d ? 1 : 0;
      }
      __syncthreads();
      if (s_done) break;
    }
    const int2* pr = ptab + r * NH;
    if (tid < NH) {
      const int2 p = pr[tid];
      const float3 cs = rot16(S[p.x * SP + p.x], S[p.y * SP + p.y], S[p.x * SP + p.y]);
      rot[tid] = make_float4(cs.x, cs.y, cs.z, 0.f);
    }
    __syncthreads();
    if (qlane) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int qv = qv0 + h * (SB / 4);
        const int2 pq = pr[qv];
        const float4 rq = rot[qv];
        const float x0 = Qm[qrow * SP + pq.x], y0 = Qm[qrow * SP + pq.y];
        Qm[qrow * SP + pq.x] = rq.x * x0 - rq.y * y0;
        Qm[qrow * SP + pq.y] = rq.y * x0 + rq.x * y0;
      }
    } else if (item) {
      const int2 pu = pr[u], pv = pr[v];
      const float4 ru = rot[u], rv = rot[v];
      const int ux = pu.x * SP, uy = pu.y * SP, vx = pv.x * SP, vy = pv.y * SP;
      const float a = S[ux + pv.x], b = S[ux + pv.y], c = S[uy + pv.x], d = S[uy + pv.y];
      // O = J_uᵀ S[u rows, v cols] J_v: columns first (p' = c·p − s·q, q' = s·p + c·q), then rows
      const float a1 = rv.x * a - rv.y * b, b1 = rv.y * a + rv.x * b;
      const float c1 = rv.x * c - rv.y * d, d1 = rv.y * c + rv.x * d;
      float o00 = ru.x * a1 - ru.y * c1, o01 = ru.x * b1 - ru.y * d1;
      float o10 = ru.y * a1 + ru.x * c1, o11 = ru.y * b1 + ru.x * d1;
      o00 = dg ? a - ru.z * b : o00;
      o11 = dg ? d + ru.z * b : o11;
      o01 = dg ? 0.f : o01;
      o10 = dg ? 0.f : o10;
      S[ux + pv.x] = o00;
      S[ux + pv.y] = o01;
      S[uy + pv.x] = o10;
      S[uy + pv.y] = o11;
      if (!dg) {
        S[vx + pu.x] = o00;
        S[vy + pu.x] = o01;
        S[vx + pu.y] = o10;
        S[vy + pu.y] = o11;
      }
    }
    __syncthreads();
  }
  float* Qo = Q_out + (int64_t)blockIdx.x * SB * SB;
  for (int e = tid; e < SB * SB; e += nthr) Qo[e] = Qm[(e / SB) * SP + (e % SB)];
  if (tid < m) dq_out[s0 + tid] = S[tid * SP + tid];
}

// ------------------------------------------------------------------ block-diagonal tile helpers
// Qt[a][c] (64×64 in LDS, pitch TP) = blockdiag of the four 16×16 Q blocks of tile t (0 elsewhere
// is never read: the contractions below stay inside a block)
template <int SB>
__device__ __forceinline__ void load_qtile(const float* __restrict__ Q, int nb, int t, float* Qt) {
  for (int e = threadIdx.x; e < TL * SB; e += blockDim.x) {
    const int blk = e / (SB * SB), a = (e / SB) % SB, c = e % SB;
    const int gb = (TL / SB) * t + blk;
    Qt[(blk * SB + a) * TP + blk * SB + c] = gb < nb ? Q[(int64_t)gb * SB * SB + a * SB + c] : (a == c ? 1.f : 0.f);
  }
}

// ------------------------------------------------------------------ 3. far-pair generator
struct FarSmem {
  float G[TL * TP];  // the gathered block (pitch TP), then T (pitch TC ≤ TP)
  float Qk[TL * TP];
  float Ql[TL * TP];
  int pk[TL], pl[TL];
  float dk[TL], dl[TL], tk[TL], tl[TL];
};

template <int SB>
__device__ __forceinline__ void far_tile(const float* __restrict__ A, int n, int64_t lda, const int* __restrict__ perm,
                                         const float* __restrict__ Q, const float* __restrict__ dq, const double* __restrict__ stats,
                                         float thr_fac, float theta, float* __restrict__ X, int64_t ldx, int K, int L, FarSmem& sm,
                                         bool mirror = false, bool pre = false) {
  float* G = sm.G;
  float* Qk = sm.Qk;
  float* Ql = sm.Ql;
  int* pk = sm.pk;
  int* pl = sm.pl;
  float* dk = sm.dk;
  float* dl = sm.dl;
  float* tk = sm.tk;
  float* tl = sm.tl;
  const int nb = (n + SB - 1) / SB;
  const int sk = K * TL, sl = L * TL;
  const int mk = min(TL, n - sk), ml = min(TL, n - sl);
  const float gthr = thr_fac * (0.5f * SB) * (float)(stats[3] - stats[2]) / (float)n;
  if (threadIdx.x < 2 * TL) {
    // per position: global threshold capped by the local one (local_threshold in sbr.py)
    const int t = threadIdx.x & (TL - 1), side = threadIdx.x >> 6;
    const int s0 = side ? sl : sk, mm = side ? ml : mk, j = s0 + t;
    float d = 0.f, th = gthr;
    if (t < mm) {
      d = dq[j];
      if (theta > 0.f) {
        const float up = j + SB / 2 < n ? fabsf(dq[j + SB / 2] - d) : INFINITY;
        const float dn = j >= SB / 2 ? fabsf(d - dq[j - SB / 2]) : INFINITY;
        th = fminf(th, theta * fminf(up, dn));
      }
    }
    if (side) {
      pl[t] = t < mm ? perm[j] : -1;
      dl[t] = d;
      tl[t] = th;
    } else {
      pk[t] = t < mm ? perm[j] : -1;
      dk[t] = d;
      tk[t] = th;
    }
  }
  load_qtile<SB>(Q, nb, K, Qk);
  load_qtile<SB>(Q, nb, L, Ql);
  __syncthreads();
  for (int e = threadIdx.x; e < TL * TL; e += blockDim.x) {
    const int a = e >> 6, f = e & 63;
    if (pre) {  // A already in the shifted sorted order (sbr16_permute_kernel): a contiguous tile
      G[a * TP + f] = (a < mk && f < ml) ? A[(int64_t)(sk + a) * lda + sl + f] : 0.f;
    } else {
      const int ra = pk[a], rf = pl[f];
      G[a * TP + f] = (ra >= 0 && rf >= 0) ? A[(int64_t)ra * lda + rf] : 0.f;
    }
  }
  __syncthreads();
  // both contractions on the f32 matrix cores (v_mfma_f32_16x16x4f32: the exact f32 product of
  // an fmaf chain): wave w owns rows [16w, 16w + 16) of T and A1, four 16×16 column tiles each.
  // Lane (m, kq): A operand A[m][kq], B operand B[kq][m], accumulator rows 4kq + i, column m.
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4;
  // T[c][f] = Σ_{a in block(c)} Qk[a][c] G[a][f]
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
  {
    const int ab = (16 * w) & ~(SB - 1);
#pragma unroll
    for (int s4 = 0; s4 < SB / 4; ++s4) {
      const int a = ab + 4 * s4 + kq;
      const float av = Qk[a * TP + 16 * w + m];
#pragma unroll
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, G[a * TP + 16 * t + m], acc[t], 0, 0, 0);
    }
  }
  __syncthreads();  // all reads of G done: T overwrites it (pitch TC: read by columns below)
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) G[(16 * w + 4 * kq + i) * TC + 16 * t + m] = acc[t][i];
  __syncthreads();
  // A1[c][e] = Σ_{f in block(e)} T[c][f] Ql[f][e]
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int fb = (16 * t) & ~(SB - 1);
#pragma unroll
    for (int s4 = 0; s4 < SB / 4; ++s4) {
      const int f = fb + 4 * s4 + kq;
      acc[t] = __builtin_amdgcn_mfma_f32_16x16x4f32(G[(16 * w + m) * TC + f], Ql[f * TP + 16 * t + m], acc[t], 0, 0, 0);
    }
  }
  // element (c, e) = (16w + 4kq + i, 16t + m) of the generator tile
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int e = 16 * t + m;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = 16 * w + 4 * kq + i;
      float x = 0.f;
      if (c < mk && e < ml) {
        const float den = dl[e] - dk[c];
        // the 2×2 Jacobi angle ½·atan(2a/den): a/den to first order for well-separated pairs,
        // saturating at π/4 for strongly coupled ones
        const bool far = ((sl + e) / SB) != ((sk + c) / SB) && fabsf(den) > fminf(tk[c], tl[e]);
        x = far ? 0.5f * atanf(2.f * acc[t][i] / den) : 0.f;
        X[(int64_t)(sk + c) * ldx + sl + e] = x;
      }
      acc[t][i] = x;
    }
  }
  if (mirror && K != L) {
    // X is skew: tile (L, K) = −(tile (K, L))ᵀ, written from here through LDS (coalesced rows)
    __syncthreads();  // every read of G (T) is done
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int i = 0; i < 4; ++i) G[(16 * t + m) * TP + 16 * w + 4 * kq + i] = acc[t][i];
    __syncthreads();
    for (int e = threadIdx.x; e < TL * TL; e += blockDim.x) {
      const int er = e >> 6, cc = e & 63;
      if (er < ml && cc < mk) X[(int64_t)(sl + er) * ldx + sk + cc] = -G[er * TP + cc];
    }
  }
}

template <int SB>
__global__ void __launch_bounds__(256) sbr16_far_kernel(const float* __restrict__ A, int n, int64_t lda,
                                                        const int* __restrict__ perm, const float* __restrict__ Q,
                                                        const float* __restrict__ dq, const double* __restrict__ stats,
                                                        float thr_fac, float theta, float* __restrict__ X, int64_t ldx,
                                                        const float* __restrict__ theta_ptr, const int* __restrict__ skip) {
  if (skip && *skip) return;
  if (theta_ptr) theta = *theta_ptr;  // device-side local-threshold switch (ops/sbr_device.py)
  __shared__ __attribute__((aligned(16))) FarSmem sm;
  far_tile<SB>(A, n, lda, perm, Q, dq, stats, thr_fac, theta, X, ldx, blockIdx.y, blockIdx.x, sm);
}

// ------------------------------------------------------------------ 4. Bq = B[:, perm]·blockdiag(Q)
template <int SB>
__device__ __forceinline__ void bq_tile(const float* __restrict__ B, int rows, int n, int64_t ldb, const int* __restrict__ perm,
                                        const float* __restrict__ Q, float* __restrict__ Bq, int64_t ldq, int rt, int L, float* G,
                                        float* Ql, int* pl, bool pre = false) {
  const int nb = (n + SB - 1) / SB;
  const int sl = L * TL, ml = min(TL, n - sl);
  if (threadIdx.x < TL) pl[threadIdx.x] = threadIdx.x < ml ? perm[sl + threadIdx.x] : -1;
  load_qtile<SB>(Q, nb, L, Ql);
  __syncthreads();
  for (int e = threadIdx.x; e < BQR * TL; e += blockDim.x) {
    const int r = e >> 6, f = e & 63;
    const int row = rt * BQR + r;
    if (pre) {  // B's columns already permuted: a contiguous tile
      G[r * TC + f] = (row < rows && f < ml) ? B[(int64_t)row * ldb + sl + f] : 0.f;
    } else {
      const int col = pl[f];
      G[r * TC + f] = (row < rows && col >= 0) ? B[(int64_t)row * ldb + col] : 0.f;
    }
  }
  __syncthreads();
  // a BQR (32)-row tile on the f32 matrix cores: wave w takes 16-row tile w & 1 and the column
  // tiles 2(w >> 1), 2(w >> 1) + 1 (see far_tile for the lane map)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, m = lane & 15, kq = lane >> 4;
  const int rl = 16 * (w & 1);
  const int row0 = rt * BQR + rl + 4 * kq;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int t = 2 * (w >> 1) + tt;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int fb = (16 * t) & ~(SB - 1);
#pragma unroll
    for (int s4 = 0; s4 < SB / 4; ++s4) {
      const int f = fb + 4 * s4 + kq;
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(G[(rl + m) * TC + f], Ql[f * TP + 16 * t + m], acc, 0, 0, 0);
    }
    const int e = 16 * t + m;
    if (e < ml) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (row0 + i < rows) Bq[(int64_t)(row0 + i) * ldq + sl + e] = acc[i];
    }
  }
}


template <int SB>
__global__ void __launch_bounds__(256) sbr16_bq_kernel(const float* __restrict__ B, int rows, int n, int64_t ldb,
                                                       const int* __restrict__ perm, const float* __restrict__ Q,
                                                       float* __restrict__ Bq, int64_t ldq, const int* __restrict__ skip) {
  if (skip && *skip) return;
  __shared__ __attribute__((aligned(16))) float G[TL * TP];
  __shared__ __attribute__((aligned(16))) float Ql[TL * TP];
  __shared__ int pl[TL];
  bq_tile<SB>(B, rows, n, ldb, perm, Q, Bq, ldq, blockIdx.y, blockIdx.x, G, Ql, pl);
}

// far generator and Bq in ONE launch (device schedule): both read only the block solve's
// perm / Q, so the (nt × nt) far tiles and the (row tiles × nt) Bq tiles run side by side —
// one launch boundary fewer per refinement iteration, and the Bq tiles fill the CUs the far
// tiles leave idle.  skip_far / skip_bq: the two parts' own control words.  (A row-wise
// pre-permutation of A and B before the tiles measured no faster — far+Bq 30.0 vs 28 µs plus 6 µs
// for the gather — and was removed in round 6; the `pre` path reads already-permuted operands.)
template <int SB>
__global__ void __launch_bounds__(256) sbr16_far_bq_kernel(const float* __restrict__ A, int n, int64_t lda, const int* __restrict__ perm,
                                                           const float* __restrict__ Q, const float* __restrict__ dq,
                                                           const double* __restrict__ stats, float thr_fac,
                                                           const float* __restrict__ theta_ptr, float* __restrict__ X, int64_t ldx,
                                                           const float* __restrict__ B, int rows, int64_t ldb, float* __restrict__ Bq,
                                                           int64_t ldq, const int* __restrict__ skip_far, const int* __restrict__ skip_bq,
                                                           bool pre) {
  __shared__ __attribute__((aligned(16))) FarSmem sm;
  const int nt = gridDim.x;
  if ((int)blockIdx.y < nt) {
    // upper tiles only (K ≤ L): each writes its mirror tile −Xᵀ as well
    if (*skip_far || blockIdx.y > blockIdx.x) return;
    far_tile<SB>(A, n, lda, perm, Q, dq, stats, thr_fac, *theta_ptr, X, ldx, blockIdx.y, blockIdx.x, sm, true, pre);
  } else {
    if (*skip_bq) return;
    bq_tile<SB>(B, rows, n, ldb, perm, Q, Bq, ldq, blockIdx.y - nt, blockIdx.x, sm.G, sm.Ql, sm.pl, pre);
  }
}

// ------------------------------------------------------------------ 5. step-size cap (damping)
// ‖X‖₂ of the skew generator from three power steps on −X² (8 probe vectors): one wave per
// row of Vout = −X²·Vin (n×8, row-major), then one workgroup forms
// α = min(1, τ / sqrt(max_j ‖V3_j‖ / ‖V2_j‖)).  Replaces ~15 small library launches.
__global__ void __launch_bounds__(256) sbr_power_step_kernel(const float* __restrict__ X2, int n, int64_t ldx,
                                                             const float* __restrict__ Vin, float* __restrict__ Vout,
                                                             const int* __restrict__ skip, const double* __restrict__ xpart = nullptr,
                                                             int nparts = 0, float tau2 = 0.f) {
  if (xpart) {  // the free ‖X‖ bounds decide (evx_sbr_damp_runs; the prep kernel applies the same test)
    if (!evx_sbr_damp_runs(skip ? *skip : 0, evx_sbr_xbounds(xpart, nparts, n), tau2)) return;
  } else if (skip && *skip) {
    return;
  }
  const int lane = threadIdx.x & 63;
  // rows stride over the grid (n > 1024)
  for (int row = blockIdx.x * 4 + (threadIdx.x >> 6); row < n; row += gridDim.x * 4) {
  const float* x = X2 + (int64_t)row * ldx;
  float acc[8] = {};
#pragma unroll 4
  for (int j = lane; j < n; j += 64) {
    const float a = x[j];
    const float4 v0 = *(const float4*)(Vin + (int64_t)j * 8), v1 = *(const float4*)(Vin + (int64_t)j * 8 + 4);
    acc[0] = fmaf(a, v0.x, acc[0]);
    acc[1] = fmaf(a, v0.y, acc[1]);
    acc[2] = fmaf(a, v0.z, acc[2]);
    acc[3] = fmaf(a, v0.w, acc[3]);
    acc[4] = fmaf(a, v1.x, acc[4]);
    acc[5] = fmaf(a, v1.y, acc[5]);
    acc[6] = fmaf(a, v1.z, acc[6]);
    acc[7] = fmaf(a, v1.w, acc[7]);
  }
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = evx::wave_sum(acc[c]);
  if (lane == 0) {
    *(float4*)(Vout + (int64_t)row * 8) = make_float4(-acc[0], -acc[1], -acc[2], -acc[3]);
    *(float4*)(Vout + (int64_t)row * 8 + 4) = make_float4(-acc[4], -acc[5], -acc[6], -acc[7]);
  }
  }
}

__global__ void __launch_bounds__(256) sbr_damping_final_kernel(const float* __restrict__ V2, const float* __restrict__ V3, int n,
                                                                float tau, float* __restrict__ alpha, const int* __restrict__ skip) {
  if (skip && *skip) return;
  const float a = evx_sbr_damping_alpha(V2, V3, n, tau);
  if (threadIdx.x == 0) alpha[0] = a;
}



// Taylor-4 operands: exp(αX) ≈ M + X²·P with M = I + αX + α²X²/2, P = α²(αX/6 + α²X²/24)
__global__ void __launch_bounds__(256) sbr_taylor4_prep_kernel(const float* __restrict__ X, const float* __restrict__ X2, int n,
                                                               const float* __restrict__ alpha, float* __restrict__ P,
                                                               float* __restrict__ M, int mt) {
  // mt = 1: M of exp(−αX) (odd term negated): Vᵀ = M(−α) + X²·Pᵀ (ops/sbr.py)
  const float a = alpha ? alpha[0] : 1.f, a2 = a * a;
  const float so = mt ? -1.f : 1.f;
  const int64_t total = (int64_t)n * n;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const float x = a * X[e], x2 = a2 * X2[e];
    P[e] = a2 * (x * (1.f / 6.f) + x2 * (1.f / 24.f));
    const int64_t i = e / n, j = e - i * n;
    M[e] = (i == j ? 1.f : 0.f) + so * x + 0.5f * x2;
  }
}

}  // namespace

int evx_sbr16_nblocks(int n, int sb) { return (n + sb - 1) / sb; }
int evx_sbr16_max_n() { return kRankMax; }

void evx_sbr16_block(const float* A, int n, int64_t lda, int shift, int sweeps, int* perm, float* Q, float* dq, int sb, hipStream_t s,
                     const int* skip, float skip_tol) {
  sbr16_rank_kernel<<<(n + 63) / 64, 64 * kRankWaves, 0, s>>>(A, n, lda, shift, perm, skip);
  if (sb == 32)
    sbr16_block_kernel<32><<<(n + 31) / 32, 512, 0, s>>>(A, n, lda, perm, sweeps, Q, dq, skip, shift, skip_tol);
  else
    sbr16_block_kernel<16><<<(n + 15) / 16, 128, 0, s>>>(A, n, lda, perm, sweeps, Q, dq, skip, shift, skip_tol);
}

void evx_sbr16_far(const float* A, int n, int64_t lda, const int* perm, const float* Q, const float* dq, const double* stats,
                   float thr_fac, float theta, float* X, int64_t ldx, int sb, hipStream_t s, const float* theta_ptr,
                   const int* skip) {
  const int nt = (n + TL - 1) / TL;
  if (sb == 32)
    sbr16_far_kernel<32><<<dim3(nt, nt), 256, 0, s>>>(A, n, lda, perm, Q, dq, stats, thr_fac, theta, X, ldx, theta_ptr, skip);
  else
    sbr16_far_kernel<16><<<dim3(nt, nt), 256, 0, s>>>(A, n, lda, perm, Q, dq, stats, thr_fac, theta, X, ldx, theta_ptr, skip);
}

void evx_sbr16_bq(const float* B, int rows, int n, int64_t ldb, const int* perm, const float* Q, float* Bq, int64_t ldq, int sb,
                  hipStream_t s, const int* skip) {
  const int nt = (n + TL - 1) / TL;
  if (sb == 32)
    sbr16_bq_kernel<32><<<dim3(nt, (rows + BQR - 1) / BQR), 256, 0, s>>>(B, rows, n, ldb, perm, Q, Bq, ldq, skip);
  else
    sbr16_bq_kernel<16><<<dim3(nt, (rows + BQR - 1) / BQR), 256, 0, s>>>(B, rows, n, ldb, perm, Q, Bq, ldq, skip);
}


void evx_sbr16_far_bq(const float* A, int n, int64_t lda, const int* perm, const float* Q, const float* dq, const double* stats,
                      float thr_fac, const float* theta_ptr, float* X, int64_t ldx, const float* B, int rows, int64_t ldb, float* Bq,
                      int64_t ldq, int sb, hipStream_t s, const int* skip_far, const int* skip_bq, bool pre) {
  const int nt = (n + TL - 1) / TL, rt = (rows + BQR - 1) / BQR;
  const dim3 grid(nt, nt + rt);
  if (sb == 32)
    sbr16_far_bq_kernel<32><<<grid, 256, 0, s>>>(A, n, lda, perm, Q, dq, stats, thr_fac, theta_ptr, X, ldx, B, rows, ldb, Bq, ldq, skip_far,
                                                 skip_bq, pre);
  else
    sbr16_far_bq_kernel<16><<<grid, 256, 0, s>>>(A, n, lda, perm, Q, dq, stats, thr_fac, theta_ptr, X, ldx, B, rows, ldb, Bq, ldq, skip_far,
                                                 skip_bq, pre);
}


void evx_sbr_damping(const float* X2, int n, int64_t ldx, const float* V, float* work, float tau, float* alpha, hipStream_t s,
                     const int* skip, int no_final, const double* xpart, int nparts) {
  float* V1 = work;
  float* V2 = work + (int64_t)n * 8;
  float* V3 = work + (int64_t)n * 16;
  // one row per wave up to n = 1024 (a 64-workgroup grid made an executed step 12 vs 5.5 µs —
  // profiles/r5_pmc_flagship.txt — for ≈1 µs less per empty launch)
  const int g = (n + 3) / 4 < 256 ? (n + 3) / 4 : 256;
  const float t2 = tau * tau;
  sbr_power_step_kernel<<<g, 256, 0, s>>>(X2, n, ldx, V, V1, skip, xpart, nparts, t2);
  sbr_power_step_kernel<<<g, 256, 0, s>>>(X2, n, ldx, V1, V2, skip, xpart, nparts, t2);
  sbr_power_step_kernel<<<g, 256, 0, s>>>(X2, n, ldx, V2, V3, skip, xpart, nparts, t2);
  // no_final: the consumer (the device schedule's Taylor prep) forms α from V2 / V3 itself
  if (!no_final) sbr_damping_final_kernel<<<1, 256, 0, s>>>(V2, V3, n, tau, alpha, skip);
}

void evx_sbr_taylor4_prep(const float* X, const float* X2, int n, const float* alpha, float* P, float* M, hipStream_t s, int mt) {
  const int64_t total = (int64_t)n * n;
  int g = (int)((total + 255) / 256);
  if (g > 2048) g = 2048;
  sbr_taylor4_prep_kernel<<<g, 256, 0, s>>>(X, X2, n, alpha, P, M, mt);
}
