// Sorted-block refinement (SBR) of a warm-started symmetric eigendecomposition (K4).
//
// CMA-ES decomposes C every generation; B (previous eigenbasis) makes A = Bᵀ C B
// nearly diagonal, but the spectrum is tightly clustered relative to the rank-μ
// perturbation (eigenvalue gaps ≈1e-4 vs off-diagonal entries ≈1e-4), so plain
// Jacobi converges only linearly (profiles/r1_jacobi_convergence_probe.log).  One SBR
// iteration instead
//
//   1. sorts diag(A) and cuts the sorted order into blocks of 64 (offset 0 or 32 on
//      alternate iterations, so every pair of rank distance < 32 shares a block in one
//      of two consecutive iterations) and diagonalises each 64×64 block with two
//      cyclic Jacobi sweeps in LDS                                 (sbr_block_kernel)
//   2. forms A1 = Qᵀ A[perm,perm] Q tile by tile and the first-order (Newton) rotation
//      generator X_ij = A1_ij / (d_j − d_i) for pairs in different blocks whose gap
//      exceeds a threshold (0 otherwise)                            (sbr_far_kernel)
//   3. Bq = B[:, perm] · blockdiag(Q)                                (sbr_bq_kernel)
// after which the host finishes with plain GEMMs: V = Taylor(exp X), B ← Bq·V, one
// Newton–Schulz re-orthonormalisation and A ← Bᵀ C B.  Far pairs converge
// quadratically through X, near (clustered) pairs through the exact block solves.
// sbr_stats_kernel reports ‖offdiag A‖², ‖diag A‖², min/max diag for the host's
// convergence / hand-off decisions (evoxmi/ops/sbr.py).
#include "evoxmi_common.h"
#include <float.h>

namespace {

constexpr int BK = 64;        // block size
constexpr int LP = 65;        // LDS pitch of the Jacobi block (odd ⇒ column walks conflict-free)
constexpr int TP = 68;        // LDS pitch of the tile kernels (float4 aligned)
constexpr int kStatParts = 128;
constexpr int kMaxN = 2048;   // largest n handled by the block kernel (LDS sort of diag(A))
constexpr int kWaves = 16;    // waves per block-solve workgroup (b32 LDS reads need ~4 waves per SIMD for full rate)

// ------------------------------------------------------------------ stats
__global__ void __launch_bounds__(256) sbr_stats_kernel(const float* __restrict__ A, int n, int64_t lda, double* __restrict__ part) {
  __shared__ double s_off[256], s_dg[256];
  __shared__ float s_mn[256], s_mx[256];
  double off = 0.0, dg = 0.0;
  float mn = FLT_MAX, mx = -FLT_MAX;
  for (int r = blockIdx.x; r < n; r += gridDim.x) {
    const float* row = A + (int64_t)r * lda;
    float acc = 0.f;
    for (int c = threadIdx.x; c < n; c += blockDim.x) {
      float v = row[c];
      if (c == r) {
        dg += (double)v * v;
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
      } else {
        acc = fmaf(v, v, acc);
      }
    }
    off += acc;
  }
  s_off[threadIdx.x] = off;
  s_dg[threadIdx.x] = dg;
  s_mn[threadIdx.x] = mn;
  s_mx[threadIdx.x] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      s_off[threadIdx.x] += s_off[threadIdx.x + o];
      s_dg[threadIdx.x] += s_dg[threadIdx.x + o];
      s_mn[threadIdx.x] = fminf(s_mn[threadIdx.x], s_mn[threadIdx.x + o]);
      s_mx[threadIdx.x] = fmaxf(s_mx[threadIdx.x], s_mx[threadIdx.x + o]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[4 * blockIdx.x + 0] = s_off[0];
    part[4 * blockIdx.x + 1] = s_dg[0];
    part[4 * blockIdx.x + 2] = s_mn[0];
    part[4 * blockIdx.x + 3] = s_mx[0];
  }
}

// fixed-order tree reduction of `nparts` partials (deterministic); out = [off², diag², dmin, dmax]
__global__ void __launch_bounds__(256) sbr_stats_final_kernel(const double* __restrict__ part, int nparts, double* __restrict__ out) {
  __shared__ double s[4][256];
  const int t = threadIdx.x;
  double off = 0.0, dg = 0.0, mn = DBL_MAX, mx = -DBL_MAX;
  for (int i = t; i < nparts; i += 256) {
    off += part[4 * i];
    dg += part[4 * i + 1];
    mn = fmin(mn, part[4 * i + 2]);
    mx = fmax(mx, part[4 * i + 3]);
  }
  s[0][t] = off;
  s[1][t] = dg;
  s[2][t] = mn;
  s[3][t] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      s[0][t] += s[0][t + o];
      s[1][t] += s[1][t + o];
      s[2][t] = fmin(s[2][t], s[2][t + o]);
      s[3][t] = fmax(s[3][t], s[3][t + o]);
    }
    __syncthreads();
  }
  if (t < 4) out[t] = s[t][0];
}

// A = (T + Tᵀ)/2 and its stats partials, one 64×64 tile per workgroup (the mirrored tile is
// read through LDS so both global reads are row-contiguous)
__global__ void __launch_bounds__(256) sbr_symstats_kernel(const float* __restrict__ T, int n, int64_t ldt, float* __restrict__ A,
                                                           int64_t lda, double* __restrict__ part) {
  __shared__ float M[64][65];
  __shared__ double r_off[256], r_dg[256];
  __shared__ float r_mn[256], r_mx[256];
  const int bi = blockIdx.y, bj = blockIdx.x;
  // mirrored tile T[bj-block rows][bi-block cols] → M (row-contiguous loads)
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e >> 6, c = e & 63;
    const int gr = bj * 64 + r, gc = bi * 64 + c;
    M[r][c] = (gr < n && gc < n) ? T[(int64_t)gr * ldt + gc] : 0.f;
  }
  __syncthreads();
  double off = 0.0, dg = 0.0;
  float mn = FLT_MAX, mx = -FLT_MAX;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int r = e >> 6, c = e & 63;
    const int gr = bi * 64 + r, gc = bj * 64 + c;
    if (gr < n && gc < n) {
      const float v = 0.5f * (T[(int64_t)gr * ldt + gc] + M[c][r]);
      A[(int64_t)gr * lda + gc] = v;
      if (gr == gc) {
        dg += (double)v * v;
        mn = fminf(mn, v);
        mx = fmaxf(mx, v);
      } else {
        off += (double)v * v;
      }
    }
  }
  const int t = threadIdx.x;
  r_off[t] = off;
  r_dg[t] = dg;
  r_mn[t] = mn;
  r_mx[t] = mx;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) {
      r_off[t] += r_off[t + o];
      r_dg[t] += r_dg[t + o];
      r_mn[t] = fminf(r_mn[t], r_mn[t + o]);
      r_mx[t] = fmaxf(r_mx[t], r_mx[t + o]);
    }
    __syncthreads();
  }
  if (t == 0) {
    const int64_t b = (int64_t)bi * gridDim.x + bj;
    part[4 * b + 0] = r_off[0];
    part[4 * b + 1] = r_dg[0];
    part[4 * b + 2] = r_mn[0];
    part[4 * b + 3] = r_mx[0];
  }
}

// Taylor terms of exp(αX) (α: damping factor on the device, 1 if null):
// P = α³(Y/24 + Y²/120 + Y³/720), M = I + Y + Y²/2 + Y³/6 with Y = αX, so that
// exp(αX) ≈ M + X³·P (one pass; X³·P carries the α³ of Y³)
// mt = 1: M of exp(−αX) = exp(αX)ᵀ (odd terms negated) — with P unchanged the transposed
// product Vᵀ = M(−α) − X³·Pᵀ is an A·Bᵀ GEMM on P's rows (ops/sbr.py)
__global__ void __launch_bounds__(256) sbr_taylor_prep_kernel(const float* __restrict__ X, const float* __restrict__ X2,
                                                              const float* __restrict__ X3, int n, const float* __restrict__ alpha,
                                                              float* __restrict__ P, float* __restrict__ M, int mt) {
  const float a = alpha ? alpha[0] : 1.f, a2 = a * a, a3 = a2 * a;
  const float so = mt ? -1.f : 1.f;
  const int64_t total = (int64_t)n * n;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const float x = a * X[e], x2 = a2 * X2[e], x3 = a3 * X3[e];
    P[e] = a3 * (x * (1.f / 24.f) + x2 * (1.f / 120.f) + x3 * (1.f / 720.f));
    const int64_t i = e / n, j = e - i * n;
    M[e] = (i == j ? 1.f : 0.f) + so * x + 0.5f * x2 + so * x3 * (1.f / 6.f);
  }
}

// ------------------------------------------------------------------ block layout
// blocks of BK in sorted order; with off = BK/2 the first block is [0, off)
__device__ __forceinline__ void block_range(int blk, int off, int n, int& s, int& e) {
  if (off == 0) {
    s = blk * BK;
    e = s + BK;
  } else {
    s = blk == 0 ? 0 : off + (blk - 1) * BK;
    e = blk == 0 ? off : s + BK;
  }
  if (e > n) e = n;
}

// bitonic sort of (key, idx) pairs in LDS, ascending by (key, idx); P is a power of 2
__device__ void lds_bitonic(float* key, int* idx, int P) {
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int ixj = i ^ j;
        if (ixj > i) {
          const float a = key[i], b = key[ixj];
          const int ia = idx[i], ib = idx[ixj];
          const bool gt = (a > b) || (a == b && ia > ib);
          const bool up = (i & k) == 0;
          if (gt == up) {
            key[i] = b;
            key[ixj] = a;
            idx[i] = ib;
            idx[ixj] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
}

// pair i of round r of the circle-method round robin on 64 slots: (63, r) for i = 0, else
// ((r + i) mod 63, (r − i) mod 63); returned as (p, q) with p < q
__device__ __forceinline__ int2 rr_pair(int r, int i) {
  int a = BK - 1, b = r;
  if (i) {
    a = r + i;
    if (a >= BK - 1) a -= BK - 1;
    b = r - i;
    if (b < 0) b += BK - 1;
  }
  return make_int2(min(a, b), max(a, b));
}

// ------------------------------------------------------------------ 1. block solves
// One workgroup (512 threads) per block.  Every workgroup sorts the full diagonal (≤ 2048
// entries, a few µs in LDS) so no separate sort launch / global permutation buffer is
// needed before the gathers.  Round-robin (circle method) parallel Jacobi on 64 slots
// (slots ≥ m are zero padding: their couplings are exact zeros, so they never rotate).
// Per round: 32 threads compute the 32 rotations; barrier; every thread updates two 2×2
// blocks of S' = Jᵀ S J and four row-pairs of Q' = Q J in place; barrier.
template <int PROBE>
__global__ void __launch_bounds__(1024) sbr_block_kernel(const float* __restrict__ A, int n, int64_t lda, int off, int sweeps,
                                                        int* __restrict__ perm_out, float* __restrict__ Q_out,
                                                        float* __restrict__ dq_out, long long* __restrict__ dbg) {
  // S and Q are updated in place: the 2×2 groups {p_u, q_u}×{p_v, q_v} of a round partition
  // S, and the (row, pair) items partition Q, so no thread reads what another one writes
  // within a round (the rotations are read after a barrier, before any update).
  __shared__ float Sc[BK * LP];
  __shared__ float Qc[BK * LP];
  __shared__ float4 rcs[32];  // (c, s, t, ·) of the round's 32 rotations
  __shared__ float key[kMaxN];
  __shared__ int idx[kMaxN];
  __shared__ int members[BK];
  int P = 1;
  while (P < n) P <<= 1;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  for (int i = tid; i < P; i += blockDim.x) {
    key[i] = i < n ? A[(int64_t)i * lda + i] : FLT_MAX;
    idx[i] = i;
  }
  __syncthreads();
  lds_bitonic(key, idx, P);
  int s, e;
  block_range(blockIdx.x, off, n, s, e);
  const int m = e - s;
  if (tid < BK) {
    members[tid] = tid < m ? idx[s + tid] : -1;
    if (tid < m) perm_out[s + tid] = idx[s + tid];
  }
  __syncthreads();
  // gather S = A[members, members] (zero padding), Q = I
  for (int i = tid; i < BK * BK; i += blockDim.x) {
    const int a = i >> 6, c = i & 63;
    const int ra = members[a], rc = members[c];
    Sc[a * LP + c] = (ra >= 0 && rc >= 0) ? A[(int64_t)ra * lda + rc] : 0.f;
    Qc[a * LP + c] = a == c ? 1.f : 0.f;
  }
  __syncthreads();
  long long tA = 0, tB = 0, tS = dbg ? clock64() : 0;  // dbg: per-phase cycle counts (probe tool)
  for (int sw = 0; sw < sweeps; ++sw) {
    for (int r = 0; r < BK - 1; ++r) {
      const long long c0 = dbg ? clock64() : 0;
      if (tid < 32) {
        const int2 pq = rr_pair(r, tid);
        const int p = pq.x, q = pq.y;
        // all three loads issued before any branch (one LDS round trip)
        const float app = Sc[p * LP + p], aqq = Sc[q * LP + q], apq = Sc[p * LP + q];
        // rotate only on a normal-range coupling: a denormal apq would make the
        // reciprocal overflow (advisor note on the round-1 rotation)
        const bool rot_on = fabsf(apq) >= FLT_MIN;
        const float theta = (aqq - app) * (0.5f * __builtin_amdgcn_rcpf(rot_on ? apq : 1.f));
        const float at = fabsf(theta);
        float t = at > 1e15f ? 0.5f * __builtin_amdgcn_rcpf(theta)
                             : copysignf(__builtin_amdgcn_rcpf(at + __builtin_amdgcn_sqrtf(fmaf(theta, theta, 1.f))), theta);
        t = rot_on ? t : 0.f;
        const float c = __builtin_amdgcn_rsqf(fmaf(t, t, 1.f));
        rcs[tid] = make_float4(c, t * c, t, 0.f);
      }
      __syncthreads();
      const long long c1 = dbg ? clock64() : 0;
      tA += c1 - c0;
      // Phase B, conflict-free LDS: lane c of a wave owns column c.  Its column's pair,
      // partner c̄ and role come from the round in registers; the rotation of that pair
      // (c_c, s_c) is one b128 read reused for every row the wave updates.
      {
        const int c = lane;
        int d = c - r;
        if (d < 0) d += BK - 1;
        int cp, cb;  // pair index of column c, partner column
        if (c == BK - 1) {
          cp = 0;
          cb = r;
        } else if (d == 0) {
          cp = 0;
          cb = BK - 1;
        } else if (d < BK / 2) {
          cp = d;
          cb = r - d;
          if (cb < 0) cb += BK - 1;
        } else {
          cp = BK - 1 - d;
          cb = r + cp;
          if (cb >= BK - 1) cb -= BK - 1;
        }
        const float4 rc = rcs[cp];
        const float cc = rc.x, sc = c < cb ? -rc.y : rc.y;  // new col c = c_c·col c + σ_c·s_c·col c̄
        // S' = Jᵀ S J for the wave's row pairs u = wave + 8j (rows p_u, q_u at column c) and
        // Q' = Q J for its rows k = wave + 8j.  Every load is issued before any store (the
        // in-place update is race-free: rows are owned by one wave, loads precede stores).
        constexpr int NU = BK / 2 / kWaves, NQ = BK / kWaves;
        int2 pu[NU];
        float4 ru[NU];
        float x0[NU], x1[NU], y0[NU], y1[NU], q0[NQ], q1[NQ];
#pragma unroll
        for (int j = 0; j < NU && !(PROBE & 1); ++j) {
          pu[j] = rr_pair(r, wave + j * kWaves);
          ru[j] = rcs[wave + j * kWaves];
          x0[j] = Sc[pu[j].x * LP + c];
          x1[j] = Sc[pu[j].x * LP + cb];
          y0[j] = Sc[pu[j].y * LP + c];
          y1[j] = Sc[pu[j].y * LP + cb];
        }
#pragma unroll
        for (int j = 0; j < NQ && !(PROBE & 2); ++j) {
          const int k = wave + j * kWaves;
          q0[j] = Qc[k * LP + c];
          q1[j] = Qc[k * LP + cb];
        }
#pragma unroll
        for (int j = 0; j < NU && !(PROBE & 1); ++j) {
          const float np_ = cc * x0[j] + sc * x1[j], nq = cc * y0[j] + sc * y1[j];
          float op = ru[j].x * np_ - ru[j].y * nq, oq = ru[j].y * np_ + ru[j].x * nq;
          if (c == pu[j].x) {  // the annihilated 2×2 block, set exactly
            op = x0[j] - ru[j].z * x1[j];
            oq = 0.f;
          } else if (c == pu[j].y) {
            op = 0.f;
            oq = y0[j] + ru[j].z * y1[j];
          }
          Sc[pu[j].x * LP + c] = op;
          Sc[pu[j].y * LP + c] = oq;
        }
#pragma unroll
        for (int j = 0; j < NQ && !(PROBE & 2); ++j) Qc[(wave + j * kWaves) * LP + c] = cc * q0[j] + sc * q1[j];
      }
      __syncthreads();
      if (dbg) tB += clock64() - c1;
    }
  }
  if (dbg && tid == 0) {
    dbg[3 * blockIdx.x] = tA;
    dbg[3 * blockIdx.x + 1] = tB;
    dbg[3 * blockIdx.x + 2] = clock64() - tS;
  }
  float* Qo = Q_out + (int64_t)blockIdx.x * BK * BK;
  for (int i = tid; i < BK * BK; i += blockDim.x) {
    const int a = i >> 6, c = i & 63;
    Qo[i] = Qc[a * LP + c];
  }
  if (tid < m) dq_out[s + tid] = Sc[tid * LP + tid];
}

// Jacobi rotation (c, s, t) annihilating the (p, q) entry of [[app, apq], [apq, aqq]]
__device__ __forceinline__ float3 jacobi_rot(float app, float aqq, float apq) {
  // rotate only on a normal-range coupling: a denormal apq would make the reciprocal overflow.
  // Branch-free: for |θ| ≳ 1e19, θ² = inf gives t = 0 (the exact t ≈ 1/(2θ) < 1e-19).
  const bool rot_on = fabsf(apq) >= FLT_MIN;
  const float theta = (aqq - app) * (0.5f * __builtin_amdgcn_rcpf(rot_on ? apq : 1.f));
  const float at = fabsf(theta);
  float t = copysignf(__builtin_amdgcn_rcpf(at + __builtin_amdgcn_sqrtf(fmaf(theta, theta, 1.f))), theta);
  t = rot_on ? t : 0.f;
  const float c = __builtin_amdgcn_rsqf(fmaf(t, t, 1.f));
  return make_float3(c, t * c, t);
}

// Version 2 of the block solve: double-buffered S, one barrier per round, Q in registers.
//
// 528 "S threads" (9 waves): thread {u ≤ v} owns the 2×2 blocks {p_u, q_u}×{p_v, q_v} of
// S' = Jᵀ S J and their transposes (written as the exact transpose: S stays symmetric).  It
// recomputes the rotations of pairs u and v itself from the round's input buffer (pure
// functions of S: every thread gets bit-identical values) — no separate parameter phase,
// no second barrier.  The pair-u diagonal block is set exactly.
//
// One "Q wave" accumulates Q' = Q J with lane k = row k of Q in 64 registers: column
// pairs of a circle-method round sit at fixed register slots when the 63 rotating slots
// shift by one per round (slot s holds column (s + r) mod 63, slot 63 column 63), so
// every index is static.  The S threads publish (c, σ·s) per pair (σ: orientation of the
// pair in slot order) and the Q wave applies round g after the barrier that ends it,
// concurrently with the S threads' round g + 1.  63·sweeps rounds return the slots to
// the identity mapping; the wave shifts its register file once per 7 rounds (static
// indices in between).
constexpr int kPairItems = (BK / 2) * (BK / 2 + 1) / 2;  // 528 unordered pairs {u ≤ v}
constexpr int kSThreads = 576;                             // 9 waves
// PROBE (tools/probe_sbr_block.py): bit 1 skips the Q work, bit 2 the S block updates, bit 4
// reuses pair u's rotation for pair v (cost of the per-thread rotation recomputation)
template <int PROBE>
__global__ void __launch_bounds__(kSThreads + 64) sbr_block2_kernel(const float* __restrict__ A, int n, int64_t lda, int off,
                                                                   int sweeps, int* __restrict__ perm_out, float* __restrict__ Q_out,
                                                                   float* __restrict__ dq_out) {
  __shared__ float Sb[2][BK * LP];
  __shared__ __attribute__((aligned(16))) float2 rq[2][BK / 2];
  __shared__ float key[kMaxN];
  __shared__ int idx[kMaxN];
  __shared__ int members[BK];
  int P = 1;
  while (P < n) P <<= 1;
  const int tid = threadIdx.x;
  for (int i = tid; i < P; i += blockDim.x) {
    key[i] = i < n ? A[(int64_t)i * lda + i] : FLT_MAX;
    idx[i] = i;
  }
  __syncthreads();
  lds_bitonic(key, idx, P);
  int s0, e0;
  block_range(blockIdx.x, off, n, s0, e0);
  const int m = e0 - s0;
  if (tid < BK) {
    members[tid] = tid < m ? idx[s0 + tid] : -1;
    if (tid < m) perm_out[s0 + tid] = idx[s0 + tid];
  }
  __syncthreads();
  for (int i = tid; i < BK * BK; i += blockDim.x) {
    const int a = i >> 6, c = i & 63;
    const int ra = members[a], rc = members[c];
    Sb[0][a * LP + c] = (ra >= 0 && rc >= 0) ? A[(int64_t)ra * lda + rc] : 0.f;
  }
  __syncthreads();
  const int G = (BK - 1) * sweeps;
  if (tid < kSThreads) {
    // thread ↔ unordered pair-of-pairs {u ≤ v} (528 of them): it owns the 2×2 blocks
    // (u, v) and (v, u) = (u, v)ᵀ, so it needs only the two rotations u and v
    const bool active = tid < kPairItems;
    int u = 0, rem = active ? tid : 0;  // inactive threads (528…575) map to item 0, never store
    while (u < BK / 2 - 1 && rem >= BK / 2 - u) {
      rem -= BK / 2 - u;
      ++u;
    }
    const int v = u + rem;
    const bool dg = u == v;
    for (int g = 0; g < G; ++g) {
      const int r = g % (BK - 1);
      const float* Si = Sb[g & 1];
      float* So = Sb[(g + 1) & 1];
      if (active) {
        const int2 pu = rr_pair(r, u), pv = rr_pair(r, v);
        const int ux = pu.x * LP, uy = pu.y * LP, vx = pv.x * LP, vy = pv.y * LP;
        const float u_pp = Si[ux + pu.x], u_qq = Si[uy + pu.y], u_pq = Si[ux + pu.y];
        const float v_pp = Si[vx + pv.x], v_qq = Si[vy + pv.y], v_pq = Si[vx + pv.y];
        const float a = Si[ux + pv.x], b = Si[ux + pv.y], c = Si[uy + pv.x], d = Si[uy + pv.y];
        const float3 ru = (PROBE & 4) ? make_float3(1.f, 0.f, 0.f) : jacobi_rot(u_pp, u_qq, u_pq);
        const float3 rv = jacobi_rot(v_pp, v_qq, v_pq);
        if (dg) {
          // publish in slot orientation for the Q wave: the first slot of pair 0 is slot 63
          // (column 63 = q), of pair v ≥ 1 slot v (column (r + v) mod 63)
          const int f = v == 0 ? BK - 1 : (r + v) % (BK - 1);
          rq[g & 1][v] = make_float2(rv.x, f == pv.x ? rv.y : -rv.y);
        }
        if (!(PROBE & 2)) {
          // O = J_uᵀ S[u rows, v cols] J_v: right (col p' = c·p − s·q, col q' = s·p + c·q), then left
          const float a1 = rv.x * a - rv.y * b, b1 = rv.y * a + rv.x * b;
          const float c1 = rv.x * c - rv.y * d, d1 = rv.y * c + rv.x * d;
          float o00 = ru.x * a1 - ru.y * c1, o01 = ru.x * b1 - ru.y * d1;
          float o10 = ru.y * a1 + ru.x * c1, o11 = ru.y * b1 + ru.x * d1;
          o00 = dg ? a - ru.z * b : o00;  // pair u's own block: set exactly
          o11 = dg ? d + ru.z * b : o11;
          o01 = dg ? 0.f : o01;
          o10 = dg ? 0.f : o10;
          So[ux + pv.x] = o00;
          So[ux + pv.y] = o01;
          So[uy + pv.x] = o10;
          So[uy + pv.y] = o11;
          So[vx + pu.x] = o00;
          So[vy + pu.x] = o01;
          So[vx + pu.y] = o10;
          So[vy + pu.y] = o11;
        } else if (dg) {
          So[ux + pu.x] = ru.x;
        }
      }
      __syncthreads();
    }
  } else {
    const int k = tid - kSThreads;  // row of Q
    float q[BK];
#pragma unroll
    for (int j = 0; j < BK; ++j) q[j] = j == k ? 1.f : 0.f;
    // 7 rounds with statically shifted slot indices, then one 7-slot shift of the register
    // file (63 = 9·7, so the shift never straddles a sweep)
    for (int g0 = 0; g0 < G; g0 += 7) {
#pragma unroll
      for (int t = 0; t < 7; ++t) {
        __syncthreads();
        if (PROBE & 1) continue;
        const float2* R = rq[(g0 + t) & 1];
        // rotations in 4 groups of 8 (one LDS wait per group; keeps the VGPR budget of
        // 3 waves per SIMD without spilling the 64-entry row)
#pragma unroll
        for (int i0 = 0; i0 < BK / 2; i0 += 8) {
          float2 cs[8];
#pragma unroll
          for (int i = 0; i < 8; ++i) cs[i] = R[i0 + i];
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const int pi = i0 + i;
            // pair 0: (slot 63, slot t); pair i ≥ 1: (slot i, slot 63 − i), shifted by t
            const int si = pi == 0 ? BK - 1 : (pi + t) % (BK - 1);
            const int sj = pi == 0 ? t : (BK - 1 - pi + t) % (BK - 1);
            const float x = q[si], y = q[sj];
            q[si] = cs[i].x * x - cs[i].y * y;
            q[sj] = cs[i].y * x + cs[i].x * y;
          }
        }
      }
      float tmp[7];
#pragma unroll
      for (int j = 0; j < 7; ++j) tmp[j] = q[j];
#pragma unroll
      for (int j = 0; j < BK - 1 - 7; ++j) q[j] = q[j + 7];
#pragma unroll
      for (int j = 0; j < 7; ++j) q[BK - 1 - 7 + j] = tmp[j];
    }
    float* Qo = Q_out + (int64_t)blockIdx.x * BK * BK + (int64_t)k * BK;
#pragma unroll
    for (int j = 0; j < BK; j += 4) *reinterpret_cast<float4*>(Qo + j) = make_float4(q[j], q[j + 1], q[j + 2], q[j + 3]);
  }
  __syncthreads();
  if (tid < m) dq_out[s0 + tid] = Sb[G & 1][tid * LP + tid];
}

// 64×64×64 product in LDS: Out[c][e] (+)= Σ_a L[a][c]·R[a][e] (TA: L read transposed) or
// Σ_a L[c][a]·R[a][e]; every thread owns a 4×4 micro-tile.
template <bool TA>
__device__ __forceinline__ void tile_mm(const float* L, const float* R, float acc[4][4]) {
  const int r0 = (threadIdx.x >> 4) << 2, c0 = (threadIdx.x & 15) << 2;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = 0.f;
#pragma unroll 4
  for (int a = 0; a < BK; ++a) {
    float l[4];
    if (TA) {
      const float4 lv = *(const float4*)(L + a * TP + r0);
      l[0] = lv.x; l[1] = lv.y; l[2] = lv.z; l[3] = lv.w;
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) l[i] = L[(r0 + i) * TP + a];
    }
    const float4 rv = *(const float4*)(R + a * TP + c0);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i][0] = fmaf(l[i], rv.x, acc[i][0]);
      acc[i][1] = fmaf(l[i], rv.y, acc[i][1]);
      acc[i][2] = fmaf(l[i], rv.z, acc[i][2]);
      acc[i][3] = fmaf(l[i], rv.w, acc[i][3]);
    }
  }
}

__device__ __forceinline__ void load_q(const float* __restrict__ Qg, float* Ql) {
  for (int i = threadIdx.x; i < BK * BK / 4; i += blockDim.x) {
    const int a = i >> 4, c = (i & 15) << 2;
    *(float4*)(Ql + a * TP + c) = *(const float4*)(Qg + a * BK + c);
  }
}

// ------------------------------------------------------------------ 2. far-pair generator
// tile (k, l) of the sorted coordinates: A1 = Q_kᵀ A[perm_k, perm_l] Q_l, X = A1 / (d_l − d_k)
// on cross-block pairs with |d_l − d_k| > thr, 0 elsewhere.  thr = thr_fac·(BK/2)·spread/n with
// the spread of diag(A) read from the stats buffer (no host round trip).
__global__ void __launch_bounds__(256) sbr_far_kernel(const float* __restrict__ A, int n, int64_t lda, int off,
                                                      const int* __restrict__ perm, const float* __restrict__ Q,
                                                      const float* __restrict__ dq, const double* __restrict__ stats,
                                                      float thr_fac, float* __restrict__ X, int64_t ldx) {
  __shared__ __attribute__((aligned(16))) float G[BK * TP];
  __shared__ __attribute__((aligned(16))) float Qk[BK * TP];
  __shared__ __attribute__((aligned(16))) float Qlv[BK * TP];
  __shared__ int pk[BK], pl[BK];
  __shared__ float dk[BK], dl[BK];
  const int k = blockIdx.y, l = blockIdx.x;
  int sk, ek, sl, el;
  block_range(k, off, n, sk, ek);
  block_range(l, off, n, sl, el);
  const int mk = ek - sk, ml = el - sl;
  const int r0 = (threadIdx.x >> 4) << 2, c0 = (threadIdx.x & 15) << 2;
  if (k == l) {
    for (int i = threadIdx.x; i < BK * BK; i += blockDim.x) {
      const int c = i >> 6, e = i & 63;
      if (c < mk && e < ml) X[(int64_t)(sk + c) * ldx + sl + e] = 0.f;
    }
    return;
  }
  if (threadIdx.x < BK) {
    const int t = threadIdx.x;
    pk[t] = t < mk ? perm[sk + t] : -1;
    pl[t] = t < ml ? perm[sl + t] : -1;
    dk[t] = t < mk ? dq[sk + t] : 0.f;
    dl[t] = t < ml ? dq[sl + t] : 0.f;
  }
  load_q(Q + (int64_t)k * BK * BK, Qk);
  load_q(Q + (int64_t)l * BK * BK, Qlv);
  __syncthreads();
  for (int i = threadIdx.x; i < BK * BK; i += blockDim.x) {
    const int a = i >> 6, f = i & 63;
    const int ra = pk[a], rf = pl[f];
    G[a * TP + f] = (ra >= 0 && rf >= 0) ? A[(int64_t)ra * lda + rf] : 0.f;
  }
  __syncthreads();
  float acc[4][4];
  tile_mm<true>(Qk, G, acc);  // T = Q_kᵀ G
  __syncthreads();             // every thread is done reading G: T overwrites it (LDS < 64 KB)
#pragma unroll
  for (int i = 0; i < 4; ++i) *(float4*)(G + (r0 + i) * TP + c0) = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
  __syncthreads();
  tile_mm<false>(G, Qlv, acc);  // A1 = T Q_l
  const float spread = (float)(stats[3] - stats[2]);
  const float thr = thr_fac * (0.5f * BK) * spread / (float)n;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = r0 + i;
    if (c >= mk) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int e = c0 + j;
      if (e >= ml) continue;
      const float den = dl[e] - dk[c];
      // the 2×2 Jacobi angle ½·atan(2a/den): a/den to first order for well-separated
      // pairs, saturating at π/4 for strongly coupled ones (no blow-up near the threshold)
      X[(int64_t)(sk + c) * ldx + sl + e] = fabsf(den) > thr ? 0.5f * atanf(2.f * acc[i][j] / den) : 0.f;
    }
  }
}

// ------------------------------------------------------------------ 3. Bq = B[:, perm]·blockdiag(Q)
__global__ void __launch_bounds__(256) sbr_bq_kernel(const float* __restrict__ B, int rows, int n, int64_t ldb, int off,
                                                     const int* __restrict__ perm, const float* __restrict__ Q,
                                                     float* __restrict__ Bq, int64_t ldq) {
  __shared__ __attribute__((aligned(16))) float G[BK * TP];
  __shared__ __attribute__((aligned(16))) float Qlv[BK * TP];
  __shared__ int pl[BK];
  const int rt = blockIdx.y, l = blockIdx.x;
  int sl, el;
  block_range(l, off, n, sl, el);
  const int ml = el - sl;
  if (threadIdx.x < BK) pl[threadIdx.x] = threadIdx.x < ml ? perm[sl + threadIdx.x] : -1;
  load_q(Q + (int64_t)l * BK * BK, Qlv);
  __syncthreads();
  // G[r][f] stored transposed-as-needed: Out[r][e] = Σ_f B[row r][perm f] Q[f][e]; tile_mm<false>
  // reads L[(r)*TP + f]
  for (int i = threadIdx.x; i < BK * BK; i += blockDim.x) {
    const int r = i >> 6, f = i & 63;
    const int row = rt * BK + r, col = pl[f];
    G[r * TP + f] = (row < rows && col >= 0) ? B[(int64_t)row * ldb + col] : 0.f;
  }
  __syncthreads();
  float acc[4][4];
  tile_mm<false>(G, Qlv, acc);
  const int r0 = (threadIdx.x >> 4) << 2, c0 = (threadIdx.x & 15) << 2;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int row = rt * BK + r0 + i;
    if (row >= rows) continue;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (c0 + j < ml) Bq[(int64_t)row * ldq + sl + c0 + j] = acc[i][j];
  }
}

}  // namespace

int evx_sbr_nblocks(int n, int off) { return off == 0 ? (n + BK - 1) / BK : 1 + (n - off + BK - 1) / BK; }

void evx_sbr_stats(const float* A, int n, int64_t lda, double* part, double* out, hipStream_t s) {
  sbr_stats_kernel<<<kStatParts, 256, 0, s>>>(A, n, lda, part);
  sbr_stats_final_kernel<<<1, 256, 0, s>>>(part, kStatParts, out);
}

int evx_sbr_stat_parts() { return kStatParts; }

int evx_sbr_symstats_parts(int n) {
  const int nt = (n + 63) / 64;
  return nt * nt;
}

void evx_sbr_symstats(const float* T, int n, int64_t ldt, float* A, int64_t lda, double* part, double* out, hipStream_t s) {
  const int nt = (n + 63) / 64;
  sbr_symstats_kernel<<<dim3(nt, nt), 256, 0, s>>>(T, n, ldt, A, lda, part);
  sbr_stats_final_kernel<<<1, 256, 0, s>>>(part, nt * nt, out);
}

void evx_sbr_taylor_prep(const float* X, const float* X2, const float* X3, int n, const float* alpha, float* P, float* M,
                         hipStream_t s, int mt) {
  const int64_t total = (int64_t)n * n;
  int g = (int)((total + 255) / 256);
  if (g > 2048) g = 2048;
  sbr_taylor_prep_kernel<<<g, 256, 0, s>>>(X, X2, X3, n, alpha, P, M, mt);
}

void evx_sbr_block(const float* A, int n, int64_t lda, int off, int sweeps, int* perm, float* Q, float* dq, hipStream_t s,
                   long long* dbg) {
  int probe = sweeps >> 8;  // diagnostic variants (tools/probe_sbr_block.py): 1 no S update, 2 no Q update
  sweeps &= 255;
  const dim3 g(evx_sbr_nblocks(n, off)), b(64 * kWaves);
  if (probe == 0 && !dbg) {
    sbr_block2_kernel<0><<<g, kSThreads + 64, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq);
    return;
  }
  if (probe >= 8) {  // version-2 probes
    switch (probe - 8) {
      case 1: sbr_block2_kernel<1><<<g, kSThreads + 64, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq); break;
      case 2: sbr_block2_kernel<2><<<g, kSThreads + 64, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq); break;
      case 3: sbr_block2_kernel<3><<<g, kSThreads + 64, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq); break;
      case 4: sbr_block2_kernel<4><<<g, kSThreads + 64, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq); break;
      case 5: sbr_block2_kernel<5><<<g, kSThreads + 64, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq); break;
      case 7: sbr_block2_kernel<7><<<g, kSThreads + 64, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq); break;
      default: sbr_block2_kernel<0><<<g, kSThreads + 64, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq); break;
    }
    return;
  }
  if (probe == 4) probe = 0;  // version 1 (probe tool: sweeps | 4 << 8)
  if (probe == 1) sbr_block_kernel<1><<<g, b, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq, dbg);
  else if (probe == 2) sbr_block_kernel<2><<<g, b, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq, dbg);
  else if (probe == 3) sbr_block_kernel<3><<<g, b, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq, dbg);
  else sbr_block_kernel<0><<<g, b, 0, s>>>(A, n, lda, off, sweeps, perm, Q, dq, dbg);
}

void evx_sbr_far(const float* A, int n, int64_t lda, int off, const int* perm, const float* Q, const float* dq,
                 const double* stats, float thr_fac, float* X, int64_t ldx, hipStream_t s) {
  const int nb = evx_sbr_nblocks(n, off);
  sbr_far_kernel<<<dim3(nb, nb), 256, 0, s>>>(A, n, lda, off, perm, Q, dq, stats, thr_fac, X, ldx);
}

void evx_sbr_bq(const float* B, int rows, int n, int64_t ldb, int off, const int* perm, const float* Q, float* Bq, int64_t ldq,
                hipStream_t s) {
  const int nb = evx_sbr_nblocks(n, off);
  sbr_bq_kernel<<<dim3(nb, (rows + BK - 1) / BK), 256, 0, s>>>(B, rows, n, ldb, off, perm, Q, Bq, ldq);
}
