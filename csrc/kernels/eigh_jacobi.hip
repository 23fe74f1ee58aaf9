// Warm-started two-sided block Jacobi for the symmetric eigenproblem (K4).
//
// A (np × np, np = nb·16, nb even) is nearly diagonal (A = Bᵀ C B with the previous
// generation's eigenbasis B).  One sweep = nb−1 tournament rounds; in round t the nb
// blocks of 16 indices are paired into nb/2 "pairs" P = (I, J) of 32 indices.
//
//  * jacobi_solve : one wave64 per pair.  The 32×32 subproblem S = A[P,P] is loaded
//    into LDS, symmetrised, and diagonalised with cyclic parallel Jacobi (31 rounds
//    of 16 rotations per inner sweep, convergence checked per sweep); the accumulated
//    orthogonal V_P (32×32) goes to global memory.
//  * jacobi_apply : A ← Jᵀ A J and B ← B J with J = ⊕_P V_P.  Output tile (P,Q) of A
//    depends only on A[P,Q], V_P and V_Q, so every tile is independent and updated in
//    place: one wave per 32×32 tile, T = A[P,Q]·V_Q with v_mfma_f32_32x32x2_f32 (16
//    MFMAs), then V_Pᵀ·T with T taken straight from the accumulator registers as the
//    B operand (no LDS round trip; the k order is permuted to the accumulator's row
//    map).  B tiles (32 rows × pair Q) need only the first product.
//  * jacobi_offnorm / jacobi_flag : Σ off-diagonal² vs tol²·Σ diagonal² → device flag.
//    Every kernel returns immediately once the flag says "converged", so a fixed
//    number of sweeps can be captured in a hipGraph without host round trips.
#include "evoxmi_common.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

constexpr int BS = 16;   // block size
constexpr int PS = 32;   // pair size
constexpr int LDP = 33;  // padded LDS row (apply kernel tiles)
// solve kernel pitches: S rows at 49 floats (odd ⇒ transposed reads conflict-free; the
// 2×2-block reads of lanes (k, l), (k+1, l) land 17 banks apart), V rows at 40 floats
// (rows 2k and 2k+2 land 16 banks apart)
constexpr int LDS_S = 49;
constexpr int LDS_V = 40;

// Block pairing of one outer round.  tab != nullptr: a row of the host schedule table
// (jacobi.py:_schedule_cpu).  Otherwise the same pairing computed in registers — round 0
// pairs (2P, 2P+1), round t ≥ 1 is circle-method rotation r = t−1 with block 0 fixed —
// so the subproblem / tile gathers do not wait behind a dependent schedule load.
struct RoundMap {
  const int* tab;
  int t, nb;
};
template <bool TAB>
__device__ __forceinline__ int round_blk(const RoundMap m, int P, int side) {
  if (TAB) return m.tab[2 * P + side];
  if (m.t == 0) return 2 * P + side;
  const int i = side ? m.nb - 1 - P : P;
  int x = i + m.t - 2;  // < 2(nb−1) for i, t in [1, nb)
  if (x >= m.nb - 1) x -= m.nb - 1;
  return i == 0 ? 0 : x + 1;
}

// inner circle-method schedule on 32 items: position i in round r
__device__ __forceinline__ int rr_item(int i, int r) { return i == 0 ? 0 : ((i - 1 + r) % 31) + 1; }

__device__ __forceinline__ void rot_params(float app, float aqq, float apq, float& c, float& s) {
  c = 1.f;
  s = 0.f;
  if (apq != 0.f) {
    float tau = (aqq - app) / (2.f * apq);
    float t = copysignf(1.f, tau) / (fabsf(tau) + sqrtf(fmaf(tau, tau, 1.f)));
    c = rsqrtf(fmaf(t, t, 1.f));
    s = t * c;
  }
}

// DPP row_newbcast:0 — lane 0 of each 16-lane row to the whole row (one VALU op)
__device__ __forceinline__ float row_bcast0(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x150, 0xf, 0xf, false));
}

// 256 threads per 32×32 subproblem: thread t owns the 2×2 block (row pair k = t>>4,
// col pair l = (t + k) & 15) of S and the V items (rows 2k, 2k+1 × col pair l).  Each thread
// computes ONE rotation (its column pair l) from S; the row-pair rotation k is computed by
// lane 0 of the thread's 16-lane row (l = k there) and broadcast with DPP.  Per inner round: one
// LDS read phase, barrier, one LDS write phase, barrier.
// MODE 0 ("cross"): 16 inner rounds pairing I[x] with J[(x + r) mod 16] — only the
//   coupling block A_IJ is annihilated; within-block pairs are handled by MODE 1.
// MODE 1 ("within"): 15 circle-method rounds inside I and inside J simultaneously.
// S is double-buffered: a round reads Sc and writes every element of Sn (the 2×2 blocks
// of the 256 threads tile the 32×32 matrix), so the read and write phases need no
// barrier in between; V has one owner per element within a round (single buffer).
struct SolveSmem {
  float Sbuf[2][PS * LDS_S];
  float V[PS * LDS_V];
  float red[8];
};

template <int MODE>
__device__ __forceinline__ void solve_pair(const float* __restrict__ A, int np, int blkI, int blkJ, int P, float* __restrict__ Vout,
                           float tol, int max_inner, SolveSmem& sm, int stop) {
  float (*Sbuf)[PS * LDS_S] = sm.Sbuf;
  float* V = sm.V;
  float* red = sm.red;
  float* S = Sbuf[0];
  const int t = threadIdx.x;
  // fixed trip count (blockDim = 256): the eight gathers (S[i][j] and its mirror, symmetrised
  // in registers — a + b is commutative, so both halves get the same value) are issued back
  // to back and share one memory latency; no separate LDS symmetrisation pass
  float g[4], gt[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = t + 256 * u, i = e >> 5, j = e & 31;
    const int gi = (i < 16 ? blkI : blkJ) * BS + (i & 15);
    const int gj = (j < 16 ? blkI : blkJ) * BS + (j & 15);
    g[u] = A[(int64_t)gi * np + gj];
    gt[u] = A[(int64_t)gj * np + gi];
  }
#pragma unroll
  for (int u = 0; u < 4; ++u) g[u] = 0.5f * (g[u] + gt[u]);
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = t + 256 * u, i = e >> 5, j = e & 31;
    S[i * LDS_S + j] = g[u];
    V[i * LDS_V + j] = (i == j) ? 1.f : 0.f;
  }
  __syncthreads();
  if (stop) return;  // uniform
  // column pairs are skewed by the row pair, l = (lane-in-row + k) mod 16, so lane 0 of
  // every 16-lane row owns l = k: the row-pair rotation it computes is broadcast to its
  // row with one DPP op (was: 4 v_readlane + select per value)
  const int k = t >> 4, l = (t + k) & 15;
  const int vr0 = 2 * k, vr1 = 2 * k + 1;
  for (int sweep = 0; sweep < max_inner; ++sweep) {
    // the first inner sweep always runs (on a converged subproblem its rotations are
    // ≈ identity); the convergence test (a block reduction + two barriers) only gates
    // the further sweeps
    if (sweep > 0) {
      float off = 0.f, dia = 0.f;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int e = t + 256 * u, i = e >> 5, j = e & 31;
        float v = S[i * LDS_S + j];
        if (i == j) dia += v * v; else off += v * v;
      }
      off = evx::wave_sum(off);
      dia = evx::wave_sum(dia);
      if ((t & 63) == 0) { red[t >> 6] = off; red[4 + (t >> 6)] = dia; }
      __syncthreads();
      off = red[0] + red[1] + red[2] + red[3];
      dia = red[4] + red[5] + red[6] + red[7];
      __syncthreads();
      if (off <= tol * tol * dia || off == 0.f) break;
    }
    constexpr int ROUNDS = MODE == 0 ? 16 : 15;
#pragma unroll
    for (int r = 0; r < ROUNDS; ++r) {
      int pk, qk, pl, ql;
      if (MODE == 0) {
        pk = k; qk = 16 + ((k + r) & 15);
        pl = l; ql = 16 + ((l + r) & 15);
      } else {
        const int kb = (k & 8) << 1, kk = k & 7, lb = (l & 8) << 1, ll = l & 7;
        pk = kb + (kk == 0 ? 0 : ((kk - 1 + r) % 15) + 1);
        qk = kb + ((14 - kk + r) % 15) + 1;
        pl = lb + (ll == 0 ? 0 : ((ll - 1 + r) % 15) + 1);
        ql = lb + ((14 - ll + r) % 15) + 1;
      }
      // ---- read phase (current buffer)
      float* Sn = (S == Sbuf[0]) ? Sbuf[1] : Sbuf[0];
      float alp = S[pl * LDS_S + pl], alq = S[ql * LDS_S + ql], alo = S[pl * LDS_S + ql];
      float x00 = S[pk * LDS_S + pl], x01 = S[pk * LDS_S + ql], x10 = S[qk * LDS_S + pl], x11 = S[qk * LDS_S + ql];
      float v0a = V[vr0 * LDS_V + pl], v0b = V[vr0 * LDS_V + ql];
      float v1a = V[vr1 * LDS_V + pl], v1b = V[vr1 * LDS_V + ql];
      // branch-free (a divergent `if (alo != 0)` let the compiler sink the alp/alq reads
      // into the branch: a second LDS round trip on every inner round's critical path) and
      // with the hardware v_sqrt_f32 (1 ulp; the IEEE sqrtf expands to ≈20 dependent
      // instructions).  alo = 0 gives inf/NaN in tau, replaced by the identity below.
      const float tau = (alq - alp) * __builtin_amdgcn_rcpf(2.f * alo);
      const float tt = copysignf(1.f, tau) * __builtin_amdgcn_rcpf(fabsf(tau) + __builtin_amdgcn_sqrtf(fmaf(tau, tau, 1.f)));
      const float cr = __builtin_amdgcn_rsqf(fmaf(tt, tt, 1.f));
      // normal-range couplings only: a denormal alo makes rcp(2·alo) overflow to inf and, with
      // alq == alp, tau = 0·inf = NaN (IEEE denormals under -O3)
      const bool rot = fabsf(alo) >= 1.17549435e-38f;
      const float cl = rot ? cr : 1.f, sl = rot ? tt * cr : 0.f;
      // row-pair rotation from lane (k, l = k) = lane 0 of this 16-lane row
      const float ck = row_bcast0(cl);
      const float sk = row_bcast0(sl);
      float y00 = ck * x00 - sk * x10, y01 = ck * x01 - sk * x11;
      float y10 = sk * x00 + ck * x10, y11 = sk * x01 + ck * x11;
      float o00 = y00 * cl - y01 * sl, o01 = y00 * sl + y01 * cl;
      float o10 = y10 * cl - y11 * sl, o11 = y10 * sl + y11 * cl;
      if (k == l) { o01 = 0.f; o10 = 0.f; }
      // ---- write phase (next buffer)
      Sn[pk * LDS_S + pl] = o00;
      Sn[pk * LDS_S + ql] = o01;
      Sn[qk * LDS_S + pl] = o10;
      Sn[qk * LDS_S + ql] = o11;
      V[vr0 * LDS_V + pl] = v0a * cl - v0b * sl;
      V[vr0 * LDS_V + ql] = v0a * sl + v0b * cl;
      V[vr1 * LDS_V + pl] = v1a * cl - v1b * sl;
      V[vr1 * LDS_V + ql] = v1a * sl + v1b * cl;
      S = Sn;
      __syncthreads();
    }
  }
  float* Vo = Vout + (int64_t)P * PS * PS;
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int e = t + 256 * u;
    Vo[e] = V[(e >> 5) * LDS_V + (e & 31)];
  }
  __syncthreads();  // LDS reuse by the caller
}

// flag must be non-null; its load overlaps the subproblem gather and the exit is taken after it
template <int MODE, bool TAB>
__global__ void __launch_bounds__(256) jacobi_solve_kernel(const float* __restrict__ A, int np, const RoundMap rm,
                                                           float* __restrict__ Vout, const int* __restrict__ flag,
                                                           float tol, int max_inner) {
  const int stop = *flag;
  __shared__ SolveSmem sm;
  const int P = blockIdx.x;
  solve_pair<MODE>(A, np, round_blk<TAB>(rm, P, 0), round_blk<TAB>(rm, P, 1), P, Vout, tol, max_inner, sm, stop);
}

// ---------------------------------------------------------------------------------- apply
// One wave per 32×32 tile; all global loads of the tile and of V_Q / V_P are issued up
// front (independent registers) so one memory latency covers the whole tile.
typedef __attribute__((address_space(1))) float gf32;

// PUBLISH: the A tile is stored write-through (sc1, agent-scope relaxed atomic stores) so
// a workgroup on another XCD can read it in the same launch after an acquire
template <bool PUBLISH, bool TAB>
__device__ __forceinline__ void apply_tile(float* __restrict__ A, float* __restrict__ B, int np, const RoundMap rm,
                                           const float* __restrict__ Vp, int tile, float* T0, int stop = 0) {
  const int lane = threadIdx.x & 63;
  const int npairs = np / PS;
  const int nA = npairs * npairs;
  const bool isA = tile < nA;
  int P = 0, Q, row0 = 0;
  if (isA) { P = tile / npairs; Q = tile % npairs; }
  else { int tt = tile - nA; row0 = (tt / npairs) * PS; Q = tt % npairs; }
  float* M = isA ? A : B;
  const int h = lane >> 5, c = lane & 31;
  const int qI = round_blk<TAB>(rm, Q, 0), qJ = round_blk<TAB>(rm, Q, 1);
  const int gj = (c < 16 ? qI : qJ) * BS + (c & 15);
  int pI = 0, pJ = 0;
  if (isA) { pI = round_blk<TAB>(rm, P, 0); pJ = round_blk<TAB>(rm, P, 1); }
  // tile gather: iteration it covers rows 2it, 2it+1 (one per half-wave), 32 columns
  float tv[16];
#pragma unroll
  for (int it = 0; it < 16; ++it) {
    const int i = 2 * it + h;
    const int gi = isA ? ((i < 16 ? pI : pJ) * BS + (i & 15)) : row0 + i;
    tv[it] = M[(int64_t)gi * np + gj];
  }
  const float* VQ = Vp + (int64_t)Q * PS * PS;
  const float* VP = Vp + (int64_t)P * PS * PS;
  float bq[16], ap[16];
#pragma unroll
  for (int s = 0; s < 16; ++s) bq[s] = VQ[(2 * s + h) * PS + c];
  if (isA) {
#pragma unroll
    for (int r = 0; r < 16; ++r) ap[r] = VP[((r & 3) + 8 * (r >> 2) + 4 * h) * PS + c];
  }
  if (stop) return;  // converged: the flag load overlapped the gathers above
#pragma unroll
  for (int it = 0; it < 16; ++it) T0[(2 * it + h) * LDP + c] = tv[it];
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_wave_barrier();
  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;
#pragma unroll
  for (int s = 0; s < 16; ++s) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(T0[c * LDP + 2 * s + h], bq[s], acc, 0, 0, 0);
  f32x16 out = acc;
  if (isA) {
#pragma unroll
    for (int r = 0; r < 16; ++r) out[r] = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) out = __builtin_amdgcn_mfma_f32_32x32x2f32(ap[r], acc[r], out, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = (r & 3) + 8 * (r >> 2) + 4 * h;
    const int gi = isA ? ((i < 16 ? pI : pJ) * BS + (i & 15)) : row0 + i;
    if (PUBLISH && isA) __hip_atomic_store((gf32*)(M + (int64_t)gi * np + gj), out[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else M[(int64_t)gi * np + gj] = out[r];
  }
}

template <bool TAB>
__global__ void __launch_bounds__(256) jacobi_apply_kernel(float* __restrict__ A, float* __restrict__ B, int np,
                                                           const RoundMap rm, const float* __restrict__ Vp,
                                                           const int* __restrict__ flag, int tile0, int tile_end) {
  const int stop = *flag;  // non-null; waited on only after the tile gathers are issued
  __shared__ float T0s[4][PS * LDP];
  const int wv = threadIdx.x >> 6;
  const int tile = __builtin_amdgcn_readfirstlane(tile0 + blockIdx.x * 4 + wv);  // wave-uniform: scalar index math
  if (tile >= tile_end) return;
  apply_tile<false, TAB>(A, B, np, rm, Vp, tile, T0s[wv], stop);
}

// ------------------------------------------------------------------------- solve ‖ B update
// Round t's subproblem solves on workgroups [0, npairs) and, in the same launch, the
// eigenbasis update B ← B·J_{t−1} of the previous round on the workgroups behind them.
// The solve occupies only npairs CUs and is the critical path (latency-bound); B is
// read by nothing but these updates, so its 32-row tiles fill the otherwise idle CUs
// and leave the separate apply launch with the A tiles only.  V is double-buffered
// by round parity.  Workgroups dispatch in blockIdx order, so the solves start first.
union SolveApplySmem {
  SolveSmem s;
  float T0s[4][PS * LDP];
};

template <int MODE>
__global__ void __launch_bounds__(256) jacobi_solve_applyB_kernel(float* __restrict__ A, float* __restrict__ B, int np,
                                                                  const RoundMap rm, float* __restrict__ Vout,
                                                                  const RoundMap rm_prev, const float* __restrict__ Vprev,
                                                                  const int* __restrict__ flag, float tol, int max_inner) {
  const int stop = *flag;
  __shared__ SolveApplySmem sm;
  const int npairs = np / PS;
  if ((int)blockIdx.x < npairs) {
    const int P = blockIdx.x;
    solve_pair<MODE>(A, np, round_blk<false>(rm, P, 0), round_blk<false>(rm, P, 1), P, Vout, tol, max_inner, sm.s, stop);
    return;
  }
  const int wv = threadIdx.x >> 6;
  const int nA = npairs * npairs;
  const int tile = __builtin_amdgcn_readfirstlane(nA + ((int)blockIdx.x - npairs) * 4 + wv);
  if (tile >= 2 * nA) return;
  apply_tile<false, false>(A, B, np, rm_prev, Vprev, tile, sm.T0s[wv], stop);
}

// ------------------------------------------------------------------------- fused apply + next solve
// Round t's apply, and the subproblem solves of round t+1 in the same launch: the next
// pair P' = (X, Y) reads the blocks (X,X), (X,Y), (Y,X), (Y,Y) of the updated A, which
// live in 1 (X, Y from one current pair) or 4 current tiles.  A tiles are stored
// write-through (sc1: the XCDs' L2s are not coherent with each other, and a per-workgroup
// buffer_wbl2 release made the first version 5x slower), each wave drains its stores,
// and after the workgroup barrier one lane per tile counts the tile's contributions on a
// per-(round, pair) counter (relaxed agent-scope atomic); the workgroup that completes a
// pair's count acquires (L1 invalidate) and solves it while other tiles are still being
// applied.  This removes the separate solve launch and overlaps the
// latency-bound 32×32 solves with the tail of the apply.
constexpr int MAXNB = 256;  // np ≤ 4096

__global__ void __launch_bounds__(256) jacobi_apply_solve_kernel(float* __restrict__ A, float* __restrict__ B, int np,
                                                                 const int* __restrict__ sched, const float* __restrict__ Vp,
                                                                 const int* __restrict__ flag, const int* __restrict__ sched_next,
                                                                 int mode_next, float* __restrict__ Vnext, int* __restrict__ counters,
                                                                 float tol, int max_inner) {
  if (flag && *flag) return;
  __shared__ float T0s[4][PS * LDP];
  __shared__ SolveSmem sm;
  __shared__ int pair_cur[MAXNB], pair_next[MAXNB];
  __shared__ int todo[8], ntodo;
  const int wv = threadIdx.x >> 6;
  const int npairs = np / PS, nb = np / BS;
  const int nA = npairs * npairs;
  const int tile = blockIdx.x * 4 + wv;
  if (tile < 2 * nA) apply_tile<true, true>(A, B, np, RoundMap{sched, 0, nb}, Vp, tile, T0s[wv]);
  // block → pair maps of this round and the next
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    pair_cur[sched[i]] = i >> 1;
    pair_next[sched_next[i]] = i >> 1;
  }
  if (threadIdx.x == 0) ntodo = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  if (threadIdx.x < 4) {
    const int tl = blockIdx.x * 4 + threadIdx.x;
    if (tl < nA) {
      const int P = tl / npairs, Q = tl % npairs;
      const int rb[2] = {sched[2 * P], sched[2 * P + 1]}, cb[2] = {sched[2 * Q], sched[2 * Q + 1]};
      int seen[4], ns = 0;
      for (int x = 0; x < 2; ++x)
        for (int y = 0; y < 2; ++y) {
          const int pn = pair_next[rb[x]];
          if (pn != pair_next[cb[y]]) continue;
          bool dup = false;
          for (int u = 0; u < ns; ++u) dup |= seen[u] == pn;
          if (dup) continue;
          seen[ns++] = pn;
          const int X = sched_next[2 * pn], Y = sched_next[2 * pn + 1];
          const int target = pair_cur[X] == pair_cur[Y] ? 1 : 4;
          if (atomicAdd(&counters[pn], 1) + 1 == target) todo[atomicAdd(&ntodo, 1)] = pn;
        }
    }
  }
  __syncthreads();
  const int nt = ntodo;
  if (nt == 0) return;  // uniform
  // acquire: one lane invalidates this CU's L1, waits for it, and the barrier releases
  // the other waves' loads behind it
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  for (int i = 0; i < nt; ++i) {
    const int pn = todo[i];
    if (mode_next) solve_pair<1>(A, np, sched_next[2 * pn], sched_next[2 * pn + 1], pn, Vnext, tol, max_inner, sm, 0);
    else solve_pair<0>(A, np, sched_next[2 * pn], sched_next[2 * pn + 1], pn, Vnext, tol, max_inner, sm, 0);
  }
}

// ---------------------------------------------------------------------------------- convergence
__global__ void __launch_bounds__(256) jacobi_offnorm_kernel(const float* __restrict__ A, int np, double* __restrict__ part,
                                                             const int* __restrict__ flag) {
  if (flag && *flag) return;
  __shared__ float scratch[8];
  double off = 0.0, dia = 0.0;
  // row-strided (no 64-bit division per element); np % 4 == 0, rows are float4-aligned
  for (int i = blockIdx.x; i < np; i += gridDim.x) {
    const float4* row = reinterpret_cast<const float4*>(A + (int64_t)i * np);
    for (int j4 = threadIdx.x; j4 < (np >> 2); j4 += blockDim.x) {
      const float4 v = row[j4];
      const float e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const double d = (double)e[q] * e[q];
        if (4 * j4 + q == i) dia += d; else off += d;
      }
    }
  }
  off = evx::wave_sum_d(off);
  dia = evx::wave_sum_d(dia);
  __shared__ double so[4], sd[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) { so[w] = off; sd[w] = dia; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double a = 0, b = 0;
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) { a += so[i]; b += sd[i]; }
    part[2 * blockIdx.x] = a;
    part[2 * blockIdx.x + 1] = b;
  }
  (void)scratch;
}

__global__ void jacobi_flag_kernel(const double* __restrict__ part, int nparts, int* __restrict__ flag, double tol2,
                                   double* __restrict__ last_off) {
  if (*flag) return;
  double off = 0, dia = 0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) { off += part[2 * i]; dia += part[2 * i + 1]; }
  off = evx::wave_sum_d(off);
  dia = evx::wave_sum_d(dia);
  if (threadIdx.x == 0) {
    if (last_off) { last_off[0] = off; last_off[1] = dia; }
    if (off <= tol2 * dia) *flag = 1;
  }
}

}  // namespace

constexpr int kOffParts = 128;

void evx_jacobi_round(float* A, float* B, int np, int round, float* Vbuf, const int* flag, float inner_tol, int max_inner,
                      hipStream_t s) {
  const int npairs = np / PS;
  const RoundMap rm{nullptr, round, np / BS};
  if (round != 0)
    jacobi_solve_kernel<0, false><<<npairs, 256, 0, s>>>(A, np, rm, Vbuf, flag, inner_tol, max_inner);
  else
    jacobi_solve_kernel<1, false><<<npairs, 256, 0, s>>>(A, np, rm, Vbuf, flag, inner_tol, max_inner);
  const int tiles = 2 * npairs * npairs;
  jacobi_apply_kernel<false><<<(tiles + 3) / 4, 256, 0, s>>>(A, B, np, rm, Vbuf, flag, 0, tiles);
}

void evx_jacobi_sweep_overlapB(float* A, float* B, int np, float* V0, float* V1, const int* flag, float inner_tol,
                               int max_inner, hipStream_t s) {
  const int npairs = np / PS, nb = np / BS, nA = npairs * npairs;
  float* V[2] = {V0, V1};
  const int gridB = (nA + 3) / 4;
  for (int t = 0; t < nb; ++t) {
    const RoundMap rm{nullptr, t, nb};
    if (t == 0) {
      jacobi_solve_kernel<1, false><<<npairs, 256, 0, s>>>(A, np, rm, V[0], flag, inner_tol, max_inner);
    } else {
      const RoundMap rp{nullptr, t - 1, nb};
      jacobi_solve_applyB_kernel<0><<<npairs + gridB, 256, 0, s>>>(A, B, np, rm, V[t & 1], rp, V[(t - 1) & 1], flag,
                                                                   inner_tol, max_inner);
    }
    jacobi_apply_kernel<false><<<gridB, 256, 0, s>>>(A, B, np, rm, V[t & 1], flag, 0, nA);
  }
  // the last round's B update, before the convergence check can set the flag
  jacobi_apply_kernel<false><<<gridB, 256, 0, s>>>(A, B, np, RoundMap{nullptr, nb - 1, nb}, V[(nb - 1) & 1], flag, nA, 2 * nA);
}

void evx_jacobi_solve(const float* A, int np, const int* sched_t, float* Vbuf, const int* flag, float inner_tol, int max_inner,
                      int mode, hipStream_t s) {
  const int npairs = np / PS;
  const RoundMap rm{sched_t, 0, np / BS};
  if (mode == 0)
    jacobi_solve_kernel<0, true><<<npairs, 256, 0, s>>>(A, np, rm, Vbuf, flag, inner_tol, max_inner);
  else
    jacobi_solve_kernel<1, true><<<npairs, 256, 0, s>>>(A, np, rm, Vbuf, flag, inner_tol, max_inner);
}

void evx_jacobi_apply_solve(float* A, float* B, int np, const int* sched_t, const float* Vcur, const int* flag,
                            const int* sched_next, int mode_next, float* Vnext, int* counters, float inner_tol, int max_inner,
                            hipStream_t s) {
  const int npairs = np / PS;
  const int tiles = 2 * npairs * npairs;
  if (sched_next == nullptr) {
    jacobi_apply_kernel<true><<<(tiles + 3) / 4, 256, 0, s>>>(A, B, np, RoundMap{sched_t, 0, np / BS}, Vcur, flag, 0, tiles);
    return;
  }
  jacobi_apply_solve_kernel<<<(tiles + 3) / 4, 256, 0, s>>>(A, B, np, sched_t, Vcur, flag, sched_next, mode_next, Vnext, counters,
                                                            inner_tol, max_inner);
}

void evx_jacobi_check(const float* A, int np, double* part, int* flag, double tol2, double* last_off, hipStream_t s) {
  jacobi_offnorm_kernel<<<kOffParts, 256, 0, s>>>(A, np, part, flag);
  jacobi_flag_kernel<<<1, 64, 0, s>>>(part, kOffParts, flag, tol2, last_off);
}

int evx_jacobi_parts() { return kOffParts; }
