// f32 GEMM family for the CMA-ES / SBR hot path on CDNA4 matrix cores
// (v_mfma_f32_16x16x4_f32: exact f32 fmaf chains, 32-cycle issue, 40-cycle latency).
//
//   C[m, n] = s · Σ_k A[m, k] · B[k, n]  (+ bias_n[n])  (+ beta · Cin[m, n]),  s = alpha · (*alpha_ptr)
//
// Why a second GEMM next to gemm_f32.hip.  The flagship's products are 1000 × 1000 × 1000
// (eigensolver, invsqrtC), 1000 × 1000 × 5000 (rank-μ) and 10 000 × 1000 × 1000 (sampling,
// CEC rotation), all f32.  At 1000² a chip of 256 CUs holds exactly one 64 × 64 output tile
// per CU, so the classic LDS-shared 2 × 2-wave tile spends its time in per-K-tile barriers
// and pipeline refills instead of MFMAs (hipBLASLt: 22–23 µs per 1000³ product = 56 % of
// the f32 matrix peak).  Here the four waves of a workgroup split K instead of the tile:
//
//   * every wave accumulates the WHOLE BM × BN tile (TM × TN 16 × 16 accumulators) over a
//     quarter of K, loading its operand fragments straight from global memory into
//     registers (float4 along k for K-contiguous operands) three 16-k groups ahead — no LDS
//     and no barrier in the main loop, so each SIMD's matrix pipe sees back-to-back MFMAs;
//   * the four partial tiles are summed once through LDS in the epilogue;
//   * operand bytes per CU are the same as with a shared tile (each wave reads a disjoint
//     K range of the same row panels), and an XCD-aware grouped tile order keeps the row
//     panels a group of workgroups shares inside that XCD's 4 MB L2.
//
// Symmetric / skew-symmetric outputs (MODE 1 / 2: Bᵀ C B, X², BᵀB, the rank-μ product,
// (B/D)Bᵀ / X²·X) compute only the tiles with tm ≤ tn and write the mirrored tile
// transposed (negated for skew): 231 instead of 441 48 × 48 tiles at n = 1000, i.e. one
// tile per CU, ≈0.56× the time of the full product.
//
// Operand layouts (template): KC = element (row, k) at p[row·ld + k] (k contiguous),
// RC = element (row, k) at p[k·ld + row] (rows contiguous: four dword loads per group).
// A skew-symmetric or symmetric operand can always be read KC (Xᵀ = −X, Cᵀ = C).
//
// ``skip``: a device word; when non-null and non-zero every workgroup returns at once
// (device-side control of the eigensolver's fixed iteration schedule, ops/sbr_device.py).
#include "evoxmi_common.h"
#include "evoxmi_launchers.h"
#include <float.h>
#include <type_traits>

#include "../host/gemm_tiles.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

namespace {

// ---- bf16x6: f32-accurate products on the bf16 matrix pipe (PREC = 1) ----
// An f32 value splits EXACTLY into three bf16 (8-bit significand) parts a = h + m + l
// (round-to-nearest-even at each step: |m| ≤ 2⁻⁹|a|, |l| ≤ 2⁻¹⁸|a|; exact because the
// f32 significand has 24 bits).  a·b is then the sum of nine bf16 × bf16 products, each
// exact in the f32 accumulator; the six kept (hh, hm, mh, hl, lh, mm) leave out terms of
// at most 2⁻²⁶|a·b|, below the f32 rounding of the accumulation itself.  The bf16 MFMA
// (v_mfma_f32_16x16x32_bf16, ≈16 cycles for 8192 MACs) runs 16× the f32 MFMA rate
// (v_mfma_f32_16x16x4_f32, 32 cycles for 1024 MACs), so six of them cost 3/8 of the f32
// product; the split is ≈4.5 VALU instructions per operand element, co-issued with the
// MFMAs of the previous block.
#ifndef EVX_X6_SPLIT
// 0: round-to-nearest parts (v_cvt_pk_bf16_f32, unbiased); 1: truncated parts (and / sub / perm):
// 15 % fewer loop cycles but its dropped terms share the sign of a·b, so a same-sign sum (a
// Gram diagonal over K = 5000) drifts past the f32 bound — measured, not used
#define EVX_X6_SPLIT 0
#endif
__device__ __forceinline__ void split3(const float4& v0, const float4& v1, bf16x8& h, bf16x8& m, bf16x8& l) {
  u32x4 H, M, L;
#if EVX_X6_SPLIT == 0
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float4& q = p < 2 ? v0 : v1;
    // scalar residuals (gemm_ks.hip is built without SLP vectorisation: a packed
    // v_pk_add_f32 beside MFMAs costs ≈3× two scalar subtractions, MI355X_MICROARCH.md)
    const float a0 = (p & 1) ? q.z : q.x, a1 = (p & 1) ? q.w : q.y;
    const bf16x2 hb = __builtin_convertvector(f32x2{a0, a1}, bf16x2);
    const f32x2 hf = __builtin_convertvector(hb, f32x2);
    const float r10 = a0 - hf.x, r11 = a1 - hf.y;
    const bf16x2 mb = __builtin_convertvector(f32x2{r10, r11}, bf16x2);
    const f32x2 mf = __builtin_convertvector(mb, f32x2);
    const bf16x2 lb = __builtin_convertvector(f32x2{r10 - mf.x, r11 - mf.y}, bf16x2);
    H[p] = __builtin_bit_cast(unsigned, hb);
    M[p] = __builtin_bit_cast(unsigned, mb);
    L[p] = __builtin_bit_cast(unsigned, lb);
  }
#else
  // truncated parts: h = the top 8 significand bits of a (mask), m = the top 8 of the exact
  // remainder, l = what is left — at most 8 significant bits, so l is a bf16 exactly; every
  // part is an f32 with a zero low half, packed pairwise with one byte permute
  const float a[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
  unsigned hu[8], mu[8], lu[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    const unsigned ab = __float_as_uint(a[c]);
    hu[c] = ab & 0xFFFF0000u;
    const float r1 = a[c] - __uint_as_float(hu[c]);
    mu[c] = __float_as_uint(r1) & 0xFFFF0000u;
    lu[c] = __float_as_uint(r1 - __uint_as_float(mu[c]));
  }
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    // high halves of (x0, x1) → one dword (x1 in the high half)
    H[p] = __builtin_amdgcn_perm(hu[2 * p + 1], hu[2 * p], 0x07060302u);
    M[p] = __builtin_amdgcn_perm(mu[2 * p + 1], mu[2 * p], 0x07060302u);
    L[p] = __builtin_amdgcn_perm(lu[2 * p + 1], lu[2 * p], 0x07060302u);
  }
#endif
  h = __builtin_bit_cast(bf16x8, H);
  m = __builtin_bit_cast(bf16x8, M);
  l = __builtin_bit_cast(bf16x8, L);
}

// ---- bf16x3: correction products (PREC = 3) ----
// a = h + m + ε with two RNE bf16 parts (|ε| ≤ 2⁻¹⁸|a|); a·b ≈ hh + hm + mh drops m·m and the
// split remainders: ≤ ≈3·2⁻¹⁸ ≈ 1.1e-5 |a·b| per product.  Used for the eigensolver products
// that form a SMALL correction (exp(αX) − I, its Taylor terms, Newton–Schulz T·(BᵀB − I)): the
// result carries ≈16 good bits relative to the correction's own size (‖X‖ ≈ 1e-3 in settled
// solves ⇒ ≈1e-8 of the basis), while the residual products (Bᵀ C B, BᵀB) stay bf16x6.  Half
// the MFMAs of bf16x6 and two instead of three conversions per operand element.
__device__ __forceinline__ void split2(const float4& v0, const float4& v1, bf16x8& h, bf16x8& m) {
  u32x4 H, M;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const float4& q = p < 2 ? v0 : v1;
    const float a0 = (p & 1) ? q.z : q.x, a1 = (p & 1) ? q.w : q.y;
    const bf16x2 hb = __builtin_convertvector(f32x2{a0, a1}, bf16x2);
    const f32x2 hf = __builtin_convertvector(hb, f32x2);
    const bf16x2 mb = __builtin_convertvector(f32x2{a0 - hf.x, a1 - hf.y}, bf16x2);
    H[p] = __builtin_bit_cast(unsigned, hb);
    M[p] = __builtin_bit_cast(unsigned, mb);
  }
  h = __builtin_bit_cast(bf16x8, H);
  m = __builtin_bit_cast(bf16x8, M);
}

__device__ __forceinline__ f32x4 mfma_x3(const bf16x8& ah, const bf16x8& am, const bf16x8& bh, const bf16x8& bm, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 mfma_x6w(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                           const bf16x8& bm, const bf16x8& bl, f32x16 c) {
  // v_mfma_f32_32x32x16_bf16: 32 cycles, holds vector issue for 8 of them (24 free cycles per
  // MFMA for the split VALU work, against 8 of 16 for the 16x16x32 form)
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, c, 0, 0, 0);
}

__device__ __forceinline__ f32x4 mfma_x6(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                         const bf16x8& bm, const bf16x8& bl, f32x4 c) {
  // smallest terms first
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, c, 0, 0, 0);
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, c, 0, 0, 0);
}


// DPP row_ror:m (rotation by m lanes inside each 16-lane row)
__device__ __forceinline__ float row_ror(float v, int m) {
  switch (m) {
    case 8: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));
    case 4: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));
    case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xF, 0xF, false));
    default: return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xF, 0xF, false));
  }
}

// One lane's four k values k .. k + 3 of one operand row.  Full 16-k groups load without
// masks; only the tail group (K % 16 != 0, handled once after the main loop) masks, with
// a clamped (valid) address and a select (KC operands need K % 4 == 0: a float4 is either
// wholly inside K or wholly outside; the launcher checks).
template <bool KC>
__device__ __forceinline__ float4 load_full(const float* __restrict__ p, int64_t ld, int k) {
  if (KC) return *reinterpret_cast<const float4*>(p + k);
  const float* q = p + (int64_t)k * ld;
  return make_float4(q[0], q[ld], q[2 * ld], q[3 * ld]);
}

template <bool KC>
__device__ __forceinline__ float4 load_tail(const float* __restrict__ p, int64_t ld, int k, int K) {
  if (KC) {
    const bool in = k < K;
    const float4 t = *reinterpret_cast<const float4*>(p + (in ? k : 0));
    return in ? t : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  float v[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const bool in = k + c < K;
    const float t = p[(int64_t)(in ? k + c : 0) * ld];
    v[c] = in ? t : 0.f;
  }
  return make_float4(v[0], v[1], v[2], v[3]);
}

// (tm, tn) of workgroup `bid` (already XCD-remapped: consecutive ids share an XCD).
// Full grid: groups of 4 tile rows, column-major inside a group.  Triangle (tm ≤ tn):
// 4 × 4 super-tiles enumerated row-major over the upper triangle, tiles row-major inside.
template <int MODE>
__device__ __forceinline__ void decode_tile(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
  if (MODE == 0) {
    constexpr int GM = 4;
    const int width = GM * tiles_n;
    const int grp = bid / width, fm = grp * GM;
    const int gm = min(GM, tiles_m - fm), rem = bid - grp * width;
    tm = fm + rem % gm;
    tn = rem / gm;
    return;
  }
  constexpr int G = 4;
  const int T = tiles_m;
  const int S = (T + G - 1) / G;
  int acc = 0;
  for (int I = 0; I < S; ++I) {
    const int rI = min(G, T - I * G);
    for (int J = I; J < S; ++J) {
      const int cJ = min(G, T - J * G);
      const int cnt = (I == J) ? rI * (rI + 1) / 2 : rI * cJ;
      if (bid < acc + cnt) {
        int t = bid - acc;
        if (I < J) {
          tm = I * G + t / cJ;
          tn = J * G + t % cJ;
        } else {
          int row = 0;
          while (t >= rI - row) {
            t -= rI - row;
            ++row;
          }
          tm = I * G + row;
          tn = I * G + row + t;
        }
        return;
      }
      acc += cnt;
    }
  }
  tm = tn = 0;
}

// PREC 0: f32 MFMA (16x16x4, KH float4 per lane and 16-row block per k-group); PREC 3: bf16x3
// (the PREC 1 fragment map with two bf16 parts and three products);
// PREC 1: bf16x6 (KH = 2: a 32-k group is one 16x16x32 bf16 step — lane (r, q) holds
// fragment element j ↔ k = 32·group + 16·(j >> 2) + 4q + (j & 3), the same k map for A and B,
// so the f32 path's loads are reused unchanged).
// NW: waves per workgroup, each owning 1/NW of K.  8 for grids that cannot fill the chip twice
// (the 1000³ eigensolver products: 256 tiles for 256 CUs): two waves per SIMD, so one wave's loads
// are in flight while the other computes; the first 4 waves then run the 4-wave epilogue.
// PL (operands as pre-split bf16x6 fragment planes) is no longer launched: the round-4 opt-in
// measured no gain inside the generation (profiles/NOTES.md); the template keeps PL = 0.
template <int TM, int TN, int KH, bool AKC, bool BKC, int MODE, int PREC, int PL = 0, int NW = 4>
__global__ void __launch_bounds__(64 * NW) gemm_ks_kernel(EvxGemmKs p) {
  static_assert(NW == 4 || NW == 8, "4 or 8 waves");
  static_assert(PREC == 0 || KH == 2, "bf16x6 groups hold two float4 per lane and block");
  static_assert(PL == 0 || (PREC == 1 && AKC && BKC), "fragment planes: bf16x6 on 16x16x32, K-contiguous operands");
  static_assert(PREC != 3 || PL == 0, "bf16x3 splits in registers");
  constexpr bool APL = PL & 1, BPL = PL & 2;
  static_assert(PREC != 2 || (TM % 2 == 0 && TN % 2 == 0), "32x32 MFMA tiles need even 16-blocks");
  if (p.skip && *p.skip) return;
  if (p.sel && *p.sel) {
    if (p.A2) p.A = p.A2;
    p.alpha = p.alpha2;
    if (p.C2) p.C = p.C2;
  }
  constexpr int BM = 16 * TM, BN = 16 * TN;
  // PREC 2 works on 32-row operand blocks (v_mfma_f32_32x32x16_bf16), the others on 16-row ones
  constexpr int RB = PREC == 2 ? 32 : 16;
  constexpr int NA = BM / RB, NB = BN / RB;
  constexpr int NE = PREC == 2 ? 16 : 4;  // accumulator registers per block pair
  // k per group: PREC 0: KH float4 per lane (16-row blocks, 4 lanes along k); PREC 1: 32
  // (16x16x32 step); PREC 2: 16 (32x32x16 step, two lane halves along k)
  constexpr int KG = PREC == 2 ? 16 : 16 * KH;
  // LDS row pitch ≡ 16 (mod 32) floats: the partial-tile writes (16 columns × 4 rows per
  // wave instruction) hit 32 distinct banks per half-wave
  constexpr int P = (BN % 32 == 16) ? BN : BN + 16;
  // two partial-tile buffers (the four K-partials are summed pairwise): 40 KB for a 64 × 64
  // tile, so LDS never limits residency below what the registers allow
  __shared__ __attribute__((aligned(16))) float red[(NW == 8 ? 4 : 2) * BM * P];

  int tm, tn;
  decode_tile<MODE>(evx::xcd_remap(blockIdx.x, gridDim.x), p.tiles_m, p.tiles_n, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  // wave index as a scalar: the K range, loop bounds and slot branches below are then
  // wave-uniform (scalar branches, and the waitcnt pass can count loads across them)
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 15, q = lane >> 4;
  const int rw = lane & 31, hw = lane >> 5;  // PREC 2 lane map: operand row, k half
  const int rl = PREC == 2 ? rw : r;

  // this wave's K range in full KG-groups (wave 0 has the fewest and also takes the tail)
  const int K = p.K;
  const int ngf = K / KG;
  const int g0 = (w * ngf) / NW, g1 = ((w + 1) * ngf) / NW;

  const float* ap[NA];
  const float* bp[NB];
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const int row = min(m0 + RB * i + rl, p.M - 1);
    ap[i] = AKC ? p.A + (int64_t)row * p.lda : p.A + row;
  }
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int col = min(n0 + RB * j + rl, p.N - 1);
    bp[j] = BKC ? p.B + (int64_t)col * p.ldb : p.B + col;
  }

  // fragment-plane operands: lane (r, q) reads the 16 bytes of its 8 k values of a 32-k group at
  // plane[row][32·group + 8q] (h, m and l planes 3 × 16 B apart by a plane stride)
  const uint16_t* apl[APL ? NA : 1];
  const uint16_t* bpl[BPL ? NB : 1];
  const int64_t pl_kp = p.pl_kp;
  if constexpr (APL) {
#pragma unroll
    for (int i = 0; i < NA; ++i) apl[i] = p.a_pl + (int64_t)min(m0 + RB * i + rl, p.M - 1) * pl_kp + 8 * q;
  }
  if constexpr (BPL) {
#pragma unroll
    for (int j = 0; j < NB; ++j) bpl[j] = p.b_pl + (int64_t)min(n0 + RB * j + rl, p.N - 1) * pl_kp + 8 * q;
  }
  const int64_t a_plane = (int64_t)p.a_pl_rows * pl_kp, b_plane = (int64_t)p.b_pl_rows * pl_kp;

  using AccT = typename std::conditional<PREC == 2, f32x16, f32x4>::type;
  AccT acc[NA][NB];
#pragma unroll
  for (int i = 0; i < NA; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j)
#pragma unroll
      for (int e = 0; e < NE; ++e) acc[i][j][e] = 0.f;

  // loads per slot: one float4 (KC) or four dwords (RC) per block and float4 slot; at most
  // 63 vector loads can be counted in flight (vmcnt)
  constexpr int LPS = KH * (NA * (AKC ? 1 : 4) + NB * (BKC ? 1 : 4)) + (APL ? NA : 0) + (BPL ? NB : 0);
#ifdef EVX_KS_DEPTH  // tools/gemm_ks_probe.cpp experiments
  constexpr int D = EVX_KS_DEPTH;
#else
  constexpr int D = (3 * LPS <= 63) ? 3 : 2;
#endif
  float4 fa[D][KH][APL ? 1 : NA], fb[D][KH][BPL ? 1 : NB];
  uint4 pa[D][3][APL ? NA : 1], pb[D][3][BPL ? NB : 1];
  const int64_t lda = p.lda, ldb = p.ldb;
  // k of float4 h of a lane: PREC 0/1: KG·group + 16h + 4q + c (lane (r, q));
  // PREC 2: KG·group + 8·hw + 4h + c (lane (rw, hw)) — the same map for A and B, so the
  // MFMA k order inside a group is a consistent permutation
  auto kof = [&](int grp, int h) { return PREC == 2 ? KG * grp + 8 * hw + 4 * h : KG * grp + 16 * h + 4 * q; };
  // fused A prologue A(m, k) − sub[k] (the CEC shift x − o): the shift float4 of a lane's k
  // values rides along with the operand loads, the subtraction runs just before the MFMAs
  const float* __restrict__ asub = (p.a_sub_k && p.sub_cols > 0) ? p.a_sub_k + (int64_t)(n0 / p.sub_cols) * p.sub_ld : p.a_sub_k;
  float4 fs[D][KH];
  constexpr int NAF = APL ? 1 : NA, NBF = BPL ? 1 : NB;
  auto load_slot = [&](float4 (&xa)[KH][NAF], float4 (&xb)[KH][NBF], float4 (&xs)[KH], uint4 (&ya)[3][APL ? NA : 1],
                       uint4 (&yb)[3][BPL ? NB : 1], int grp) {
#pragma unroll
    for (int h = 0; h < KH; ++h) {
      const int k = kof(grp, h);
      if (AKC && asub && !APL) xs[h] = *reinterpret_cast<const float4*>(asub + k);
      if constexpr (!APL) {
#pragma unroll
        for (int i = 0; i < NA; ++i) xa[h][i] = load_full<AKC>(ap[i], lda, k);
      }
      if constexpr (!BPL) {
#pragma unroll
        for (int j = 0; j < NB; ++j) xb[h][j] = load_full<BKC>(bp[j], ldb, k);
      }
    }
    if constexpr (APL) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int i = 0; i < NA; ++i) ya[c][i] = *reinterpret_cast<const uint4*>(apl[i] + c * a_plane + 32 * grp);
    }
    if constexpr (BPL) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int j = 0; j < NB; ++j) yb[c][j] = *reinterpret_cast<const uint4*>(bpl[j] + c * b_plane + 32 * grp);
    }
  };
  auto compute_slot = [&](float4 (&xa)[KH][NAF], const float4 (&xb)[KH][NBF], const float4 (&xs)[KH], const uint4 (&ya)[3][APL ? NA : 1],
                          const uint4 (&yb)[3][BPL ? NB : 1]) {
    if (AKC && asub && !APL) {
#pragma unroll
      for (int h = 0; h < KH; ++h)
#pragma unroll
        for (int i = 0; i < NA; ++i) {
          xa[h][i].x -= xs[h].x;
          xa[h][i].y -= xs[h].y;
          xa[h][i].z -= xs[h].z;
          xa[h][i].w -= xs[h].w;
        }
    }
    if constexpr (PREC == 3) {
      bf16x8 bh[NB], bm[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) split2(xb[0][j], xb[1][j], bh[j], bm[j]);
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        bf16x8 ah, am;
        split2(xa[0][i], xa[1][i], ah, am);
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = mfma_x3(ah, am, bh[j], bm[j], acc[i][j]);
      }
    } else if constexpr (PREC >= 1) {
      bf16x8 bh[NB], bm[NB], bl[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        if constexpr (BPL) {
          bh[j] = __builtin_bit_cast(bf16x8, yb[0][j]);
          bm[j] = __builtin_bit_cast(bf16x8, yb[1][j]);
          bl[j] = __builtin_bit_cast(bf16x8, yb[2][j]);
        } else {
          split3(xb[0][BPL ? 0 : j], xb[1][BPL ? 0 : j], bh[j], bm[j], bl[j]);
        }
      }
#pragma unroll
      for (int i = 0; i < NA; ++i) {
        bf16x8 ah, am, al;
        if constexpr (APL) {
          ah = __builtin_bit_cast(bf16x8, ya[0][i]);
          am = __builtin_bit_cast(bf16x8, ya[1][i]);
          al = __builtin_bit_cast(bf16x8, ya[2][i]);
        } else {
          split3(xa[0][APL ? 0 : i], xa[1][APL ? 0 : i], ah, am, al);
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          if constexpr (PREC == 2) acc[i][j] = mfma_x6w(ah, am, al, bh[j], bm[j], bl[j], acc[i][j]);
          else acc[i][j] = mfma_x6(ah, am, al, bh[j], bm[j], bl[j], acc[i][j]);
        }
      }
    } else {
#pragma unroll
      for (int h = 0; h < KH; ++h)
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < NA; ++i)
#pragma unroll
            for (int j = 0; j < NB; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32((&xa[h][APL ? 0 : i].x)[e], (&xb[h][BPL ? 0 : j].x)[e], acc[i][j], 0, 0, 0);
    }
  };
  // Loads are issued unconditionally (group index clamped to the wave's last group, so the
  // addresses stay valid and the surplus loads are never consumed): the loop body is then
  // straight-line between scalar branches and the waitcnt pass keeps D − 1 groups in flight
  // (a conditional issue makes it wait for everything at the join).
  // (g0 ≤ ngf − 1 whenever ngf ≥ 1; with K < KG there is no full group at all and group 0
  // would read past the last row's K floats: nothing is loaded, the tail below does it all)
  const int glast = max(g1 - 1, g0);
  if (ngf > 0) {
#pragma unroll
    for (int s = 0; s < D - 1; ++s) load_slot(fa[s], fb[s], fs[s], pa[s], pb[s], min(g0 + s, glast));
  }
  // chunks of D groups with no branch inside (load group g + s + D − 1, compute group g + s),
  // then the < D remaining groups, whose data the last chunk (or the prologue) loaded
  int g = g0;
  for (; g + D <= g1; g += D) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
#ifndef EVX_KS_NO_LOADS  // probe: MFMA loop alone (operands of the prologue reused)
#ifdef EVX_KS_FAKE_LOADS  // probe: every group re-reads group g0 (L1-resident operands)
      load_slot(fa[(s + D - 1) % D], fb[(s + D - 1) % D], fs[(s + D - 1) % D], pa[(s + D - 1) % D], pb[(s + D - 1) % D], g0);
#else
      load_slot(fa[(s + D - 1) % D], fb[(s + D - 1) % D], fs[(s + D - 1) % D], pa[(s + D - 1) % D], pb[(s + D - 1) % D],
                min(g + s + D - 1, glast));
#endif
#endif
      // keep the issue order (loads of group g + s + D − 1 before the MFMAs of group g + s):
      // left alone, the scheduler sinks the loads behind the MFMAs and the prefetch distance
      // collapses to one group
      __builtin_amdgcn_sched_barrier(0);
      compute_slot(fa[s], fb[s], fs[s], pa[s], pb[s]);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int s = 0; s < D - 1; ++s)
    if (g + s < g1) compute_slot(fa[s], fb[s], fs[s], pa[s], pb[s]);
  if (w == 0 && K % KG) {  // tail (masked loads; fragment planes are zero-padded to kp)
#pragma unroll
    for (int h = 0; h < KH; ++h) {
      const int k = kof(ngf, h);
      if (AKC && asub && !APL) fs[0][h] = load_tail<true>(asub, 0, k, K);
      if constexpr (!APL) {
#pragma unroll
        for (int i = 0; i < NA; ++i) fa[0][h][i] = load_tail<AKC>(ap[i], lda, k, K);
      }
      if constexpr (!BPL) {
#pragma unroll
        for (int j = 0; j < NB; ++j) fb[0][h][j] = load_tail<BKC>(bp[j], ldb, k, K);
      }
    }
    if constexpr (APL) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int i = 0; i < NA; ++i) pa[0][c][i] = *reinterpret_cast<const uint4*>(apl[i] + c * a_plane + 32 * ngf);
    }
    if constexpr (BPL) {
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int j = 0; j < NB; ++j) pb[0][c][j] = *reinterpret_cast<const uint4*>(bpl[j] + c * b_plane + 32 * ngf);
    }
    compute_slot(fa[0], fb[0], fs[0], pa[0], pb[0]);
  }

  // ---- epilogue: sum the four K-partials through LDS, pairwise: waves 2, 3 park theirs,
  // waves 0, 1 add them (fixed order: deterministic), park the sums; all threads add the two
  // accumulator maps: 16x16: col = lane & 15, row = 4·(lane >> 4) + reg;
  // 32x32: col = lane & 31, row = (reg & 3) + 8·(reg >> 2) + 4·(lane >> 5)
  auto elem = [&](int i, int j, int e) {
    return PREC == 2 ? (32 * i + (e & 3) + 8 * (e >> 2) + 4 * hw) * P + 32 * j + rw : (16 * i + 4 * q + e) * P + 16 * j + r;
  };
  auto park = [&](int buf) {
    float* my = red + buf * BM * P;
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int e = 0; e < NE; ++e) my[elem(i, j, e)] = acc[i][j][e];
  };
  if constexpr (NW == 8) {  // 8 → 4: waves 4-7 park, waves 0-3 add (fixed order)
    if (w >= 4) park(w - 4);
    __syncthreads();
    if (w < 4) {
      const float* his = red + w * BM * P;
#pragma unroll
      for (int i = 0; i < NA; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
          for (int e = 0; e < NE; ++e) acc[i][j][e] += his[elem(i, j, e)];
    }
    __syncthreads();
  }
  // the epilogue below runs on the first 256 threads (waves 4-7 only meet its barriers)
  const bool epi = threadIdx.x < 256;
  if (w >= 2 && w < 4) park(w - 2);
  __syncthreads();
  if (w < 2) {
    const float* his = red + w * BM * P;
#pragma unroll
    for (int i = 0; i < NA; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int e = 0; e < NE; ++e) acc[i][j][e] += his[elem(i, j, e)];
  }
  __syncthreads();
  if (w < 2) park(w);
  __syncthreads();
  const float sc = p.alpha * (p.alpha_ptr ? p.alpha_ptr[0] : 1.f);
  // stats partials (symmetric mode): mirrored tiles count twice, diagonal tiles their upper
  // triangle twice and the diagonal once
  double st_off = 0.0, st_dg = 0.0;
  float st_mn = FLT_MAX, st_mx = -FLT_MAX;
  constexpr int NV4 = BM * BN / 4;
  constexpr int PER = (NV4 + 255) / 256;
  float4 out[PER];
  float rt1[PER], rt2[PER];  // row-terms partials (MODE 0 with row_terms)
  const bool zak = p.row_fid == 0;
#pragma unroll
  for (int v = 0; v < PER; ++v) {
    const int e = threadIdx.x + 256 * v;
    if (epi && e < NV4) {
      const int row = e / (BN / 4), c = (e % (BN / 4)) * 4;
      float4 t = *reinterpret_cast<const float4*>(&red[row * P + c]);
      {
        const float4 u = *reinterpret_cast<const float4*>(&red[BM * P + row * P + c]);
        t.x += u.x;
        t.y += u.y;
        t.z += u.z;
        t.w += u.w;
      }
      t.x *= sc;
      t.y *= sc;
      t.z *= sc;
      t.w *= sc;
      const int gr = m0 + row, gc = n0 + c;
      if (MODE == 0 && BN == 64 && p.row_terms) {
        // fused CEC'22 basic-function row reduction: this float4's two additive terms
        // (branch-free; columns past N contribute 0), reduced across the row after the loop
        const float vv[4] = {t.x, t.y, t.z, t.w};
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          const float z = gc + e2 < p.N ? vv[e2] : 0.f;
          if (zak) {
            s1 = fmaf(z, z, s1);
            s2 = fmaf(0.5f * (float)(gc + e2 + 1), z, s2);
          } else {  // Rastrigin (z · 0.0512 as in the CEC'22 basic function); v_cos takes revolutions
            const float y = 0.0512f * z;
            s1 += y * y - 10.f * __builtin_amdgcn_cosf(y) + 10.f;
          }
        }
        rt1[v] = s1;
        rt2[v] = s2;
        continue;
      }
      if (p.bias_n) {
        if (gc < p.N) t.x += p.bias_n[gc];
        if (gc + 1 < p.N) t.y += p.bias_n[gc + 1];
        if (gc + 2 < p.N) t.z += p.bias_n[gc + 2];
        if (gc + 3 < p.N) t.w += p.bias_n[gc + 3];
      }
      if (gr < p.M) {
        float* crow = p.C + (int64_t)gr * p.ldc;
        if (p.Cin) {
          const float* cin = p.Cin + (int64_t)gr * p.ldcin;
          if (gc < p.N) t.x += p.beta * cin[gc];
          if (gc + 1 < p.N) t.y += p.beta * cin[gc + 1];
          if (gc + 2 < p.N) t.z += p.beta * cin[gc + 2];
          if (gc + 3 < p.N) t.w += p.beta * cin[gc + 3];
        }
        if (p.diag_add != 0.f) {
          // the diagonal element of this float4, if any (explicit selects: HIP's float4 members
          // are accessor objects, not an indexable array)
          const int dd = gr - gc;
          if (dd == 0) t.x += p.diag_add;
          else if (dd == 1) t.y += p.diag_add;
          else if (dd == 2) t.z += p.diag_add;
          else if (dd == 3) t.w += p.diag_add;
        }
        if (MODE != 0 && tm == tn) {
          // diagonal tile: only its upper triangle is stored here (the mirror pass writes the
          // lower one from it), so the output is exactly (skew-)symmetric; skew diagonal = 0
          const float vv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
          for (int e2 = 0; e2 < 4; ++e2) {
            const int cc = c + e2;
            if (gc + e2 < p.N && row <= cc) crow[gc + e2] = (MODE == 2 && row == cc) ? 0.f : vv[e2];
          }
        } else if (gc + 3 < p.N && p.c_vec4) {
          *reinterpret_cast<float4*>(crow + gc) = t;
        } else {
          if (gc < p.N) crow[gc] = t.x;
          if (gc + 1 < p.N) crow[gc + 1] = t.y;
          if (gc + 2 < p.N) crow[gc + 2] = t.z;
          if (gc + 3 < p.N) crow[gc + 3] = t.w;
        }
      }
      out[v] = t;
      if (MODE == 1 && p.stat_part && gr < p.M && (!p.stat_diag_only || tm == tn)) {
        const float vv[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          const int cc = c + e2;
          if (gc + e2 >= p.N) continue;
          if (p.stat_diag_only && row != cc) continue;
          const double d2 = (double)vv[e2] * vv[e2];
          if (tm != tn || row < cc) st_off += 2.0 * d2;
          else if (row == cc) {
            st_dg += d2;
            st_mn = fminf(st_mn, vv[e2]);
            st_mx = fmaxf(st_mx, vv[e2]);
          }
        }
      }
    }
  }
  if (MODE == 0 && BN == 64 && p.row_terms) {
    // DPP row rotations by 8, 4, 2, 1 inside the 16-lane row that holds one tile row, all
    // PER rows of this thread interleaved (independent chains); every lane ends with the sum
#pragma unroll
    for (int m = 8; m >= 1; m >>= 1) {
#pragma unroll
      for (int v = 0; v < PER; ++v) {
        rt1[v] += row_ror(rt1[v], m);
        rt2[v] += row_ror(rt2[v], m);
      }
    }
    if (epi && (threadIdx.x & 15) == 0) {
#pragma unroll
      for (int v = 0; v < PER; ++v) {
        const int gr = m0 + (threadIdx.x + 256 * v) / (BN / 4);
        if (gr < p.M) *reinterpret_cast<float2*>(p.row_terms + ((int64_t)tn * p.M + gr) * 2) = make_float2(rt1[v], rt2[v]);
      }
    }
    return;
  }
  if (MODE == 1 && p.stat_part) {
    st_off = evx::wave_sum_d(st_off);
    st_dg = evx::wave_sum_d(st_dg);
    st_mn = evx::wave_min(st_mn);
    st_mx = evx::wave_max(st_mx);
    __shared__ double s_st[4][4];
    if (lane == 0 && w < 4) {
      s_st[w][0] = st_off;
      s_st[w][1] = st_dg;
      s_st[w][2] = st_mn;
      s_st[w][3] = st_mx;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      double* o = p.stat_part + 4 * (int64_t)blockIdx.x;
      o[0] = (s_st[0][0] + s_st[1][0]) + (s_st[2][0] + s_st[3][0]);
      o[1] = (s_st[0][1] + s_st[1][1]) + (s_st[2][1] + s_st[3][1]);
      o[2] = fmin(fmin(s_st[0][2], s_st[1][2]), fmin(s_st[2][2], s_st[3][2]));
      o[3] = fmax(fmax(s_st[0][3], s_st[1][3]), fmax(s_st[2][3], s_st[3][3]));
    }
  }
  if (MODE == 0) return;
  // mirrored tile C[n0 + c][m0 + r] = ±v(r, c), stored with consecutive threads on
  // consecutive r (coalesced rows of the mirrored tile)
  __syncthreads();
#pragma unroll
  for (int v = 0; v < PER; ++v) {
    const int e = threadIdx.x + 256 * v;
    if (epi && e < NV4) {
      const int row = e / (BN / 4), c = (e % (BN / 4)) * 4;
      *reinterpret_cast<float4*>(&red[row * P + c]) = out[v];
    }
  }
  __syncthreads();
  const float sgn = MODE == 2 ? -1.f : 1.f;
  const bool diag = tm == tn;
  for (int e = threadIdx.x; e < BM * BN; e += 64 * NW) {
    const int rr = e % BM, cc = e / BM;
    const int gr = n0 + cc, gc = m0 + rr;
    if (gr < p.N && gc < p.M && (!diag || rr < cc)) p.C[(int64_t)gr * p.ldc + gc] = sgn * red[rr * P + cc];
  }
}

#ifndef EVX_KS_KH
#define EVX_KS_KH 1
#endif

int g_ks_prec = 1;  // 1: bf16x6 on 16x16x32 (default), 2: bf16x6 on 32x32x16 where the tile allows, 0: f32 MFMA

template <int TM, int TN, int MODE, int PREC, int NW>
void launch_prec_nw(const EvxGemmKs& a, int tiles, hipStream_t s) {
  constexpr int KH = PREC >= 1 ? 2 : EVX_KS_KH;
  const dim3 grid(tiles), block(64 * NW);
  if (a.a_kc && a.b_kc) gemm_ks_kernel<TM, TN, KH, true, true, MODE, PREC, 0, NW><<<grid, block, 0, s>>>(a);
  else if (a.a_kc && !a.b_kc) gemm_ks_kernel<TM, TN, KH, true, false, MODE, PREC, 0, NW><<<grid, block, 0, s>>>(a);
  else if (!a.a_kc && a.b_kc) gemm_ks_kernel<TM, TN, KH, false, true, MODE, PREC, 0, NW><<<grid, block, 0, s>>>(a);
  else gemm_ks_kernel<TM, TN, KH, false, false, MODE, PREC, 0, NW><<<grid, block, 0, s>>>(a);
}

// 8-wave workgroups for grids of at most this many tiles whose K gives every wave ≥ 12 k-groups
// (0: never).  Measured (tools/bench_gemm.py, profiles/r4_gemm_nw8.log): the 1000×1000×5000
// rank-μ product 55.8 → 47.8 µs and the 1000³ symmetric TN 17.9 → 16.8, but the short-K 1000³
// full products slower (NT 24.4 → 51.7: 4 k-groups per wave leave the prefetch pipeline empty)
int g_ks_nw8_tiles = 384;
constexpr int kNw8MinK = 3072;

template <int TM, int TN, int MODE, int PREC>
void launch_prec(const EvxGemmKs& a, int tiles, hipStream_t s) {
  if constexpr (TM <= 4 && TN <= 4) {
    if (tiles <= g_ks_nw8_tiles && a.K >= kNw8MinK) return launch_prec_nw<TM, TN, MODE, PREC, 8>(a, tiles, s);
  }
  launch_prec_nw<TM, TN, MODE, PREC, 4>(a, tiles, s);
}

template <int TM, int TN, int MODE>
void launch_layout(const EvxGemmKs& a, int tiles, hipStream_t s) {
  {
    if (a.prec == 3) return launch_prec<TM, TN, MODE, 3>(a, tiles, s);
    if constexpr (TM % 2 == 0 && TN % 2 == 0) {
      if (g_ks_prec == 2) return launch_prec<TM, TN, MODE, 2>(a, tiles, s);
    }
    if (g_ks_prec >= 1) launch_prec<TM, TN, MODE, 1>(a, tiles, s);
    else launch_prec<TM, TN, MODE, 0>(a, tiles, s);
  }
}

template <int TM, int TN>
void launch_tile(EvxGemmKs a, hipStream_t s) {
  a.tiles_m = (a.M + 16 * TM - 1) / (16 * TM);
  a.tiles_n = (a.N + 16 * TN - 1) / (16 * TN);
  if (a.mode == 0) launch_layout<TM, TN, 0>(a, a.tiles_m * a.tiles_n, s);
  else if (a.mode == 1) launch_layout<TM, TN, 1>(a, a.tiles_m * (a.tiles_m + 1) / 2, s);
  else launch_layout<TM, TN, 2>(a, a.tiles_m * (a.tiles_m + 1) / 2, s);
}

int g_ks_tile_override = 0;

}  // namespace

void evx_gemm_ks_set_tile(int t) { g_ks_tile_override = t; }

void evx_gemm_ks_set_prec(int prec) { g_ks_prec = prec; }

void evx_gemm_ks_set_nw8(int tiles) { g_ks_nw8_tiles = tiles; }

int evx_gemm_ks_prec() { return g_ks_prec; }

int evx_gemm_ks_tile(int M, int N, int mode) { return evx_host::gemm_ks_tile(M, N, mode, g_ks_tile_override); }

int evx_gemm_ks_grid(int M, int N, int mode) { return (int)evx_host::gemm_ks_grid(M, N, mode, g_ks_tile_override); }

int evx_gemm_ks_tiles_n(int M, int N, int mode) { return (int)evx_host::gemm_ks_tiles_n(M, N, mode, g_ks_tile_override); }

void evx_gemm_ks(const EvxGemmKs& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return;
  switch (a.force_tile ? a.force_tile : evx_gemm_ks_tile(a.M, a.N, a.mode)) {
    case 2: launch_tile<2, 2>(a, s); break;
    case 3: launch_tile<3, 3>(a, s); break;
    case 8: launch_tile<8, 4>(a, s); break;  // tall products (M ≫ N), full mode only
    default: launch_tile<4, 4>(a, s); break;
  }
}
