// LDS-staged bf16x6 GEMM for the tall f32 products of the flagship (CDNA4 matrix cores).
//
//   C[m, n] = s · Σ_k A[m, k] · B[n, k]  (+ bias_n[n]),   s = alpha · (*alpha_ptr)
//
// The CMA-ES sampling product X = mean + σ·Z·(B∘D)ᵀ and the CEC'22 rotation (X − o)·Mᵀ are
// 10 000 × 1000 × 1000 NT products that the reference evaluates every generation
// (/root/reference/src/evox/algorithms/so/es_variants/cma_es.py:130-137,
//  /root/reference/src/evox/problems/numerical/cec2022_so.py:109-119).  gemm_ks.hip runs them
// register-direct: every A element is split into its three bf16 parts once per 64-column
// tile (16 times per product), which made that kernel VALU- and issue-bound at one wave per
// SIMD (27 % of the bf16x6 ceiling).  Here the operands arrive ALREADY split:
//
//   * "blocked planes": an f32 matrix (rows × K) is stored as bf16 [K/16][Rp][3][16] — for
//     every 16-k block and row the high, middle and low bf16 parts of its 16 values, 96
//     contiguous bytes (split_blk_kernel / philox_blk_kernel write them; a producer that
//     already streams the operand writes its planes instead of f32).  The 16-k block of BM
//     consecutive rows is ONE contiguous run of BM·96 bytes, so a stage is a plain memcpy;
//   * a stage (one 16-k block of the 320-row A panel and the 128-row B panel, 42 KiB) goes
//     global → LDS by LDS-DMA (global_load_lds_dwordx4, 1 KiB per wave instruction), three
//     stages in flight, one barrier per stage, a counted vmcnt that leaves the next stage's
//     copies outstanding across it;
//   * the six kept products per k (hh, hm, mh, hl, mm, lh: each dropped term ≤ 2⁻²⁶|ab|, see
//     gemm_ks.hip split3) are three v_mfma_f32_16x16x32_bf16 per 16-row × 16-column block and
//     16-k block: a 32-deep k' step pairs two 16-k plane slices per lane quarter (lane q
//     reads A plane PA[c][q>>1] and B plane PB[c][q>>1] at k = 8(q&1) … +7):
//       c = 0: A (h, h) · B (h, m)   c = 1: A (m, h) · B (h, l)   c = 2: A (m, l) · B (m, h);
//     the 96-byte row pitch puts the 16 lanes of every ds_read_b128 lane group on 16 distinct
//     16-byte bank slots (6r + 2p + (q & 1) mod 16 is a bijection over a group's lanes);
//   * 320 × 128 output tiles, 8 waves as 4 (M) × 2 (N) of 80 × 64, two waves per SIMD: at
//     10 000 × 1000 that is 32 × 8 = 256 tiles, one per CU, with an XCD-aware order (each XCD
//     owns 4 row panels × all 8 column tiles, so an A panel is fetched into one L2 once).
#include "evoxmi_common.h"
#include "evoxmi_launchers.h"
#include <cstdlib>
#include <stdexcept>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

namespace {

constexpr int kRowB = 96;  // bytes per (row, 16-k block): 3 planes × 16 bf16

// exact RNE split of 16 f32 into their h / m / l bf16 parts, stored as the 96-byte row record
__device__ __forceinline__ void split16_store(const float (&v)[16], uint4* __restrict__ dst) {
  unsigned H[8], M[8], L[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const float a0 = v[2 * p], a1 = v[2 * p + 1];
    const bf16x2 hb = __builtin_convertvector(f32x2{a0, a1}, bf16x2);
    const f32x2 hf = __builtin_convertvector(hb, f32x2);
    const float r0 = a0 - hf.x, r1 = a1 - hf.y;
    const bf16x2 mb = __builtin_convertvector(f32x2{r0, r1}, bf16x2);
    const f32x2 mf = __builtin_convertvector(mb, f32x2);
    const bf16x2 lb = __builtin_convertvector(f32x2{r0 - mf.x, r1 - mf.y}, bf16x2);
    H[p] = __builtin_bit_cast(unsigned, hb);
    M[p] = __builtin_bit_cast(unsigned, mb);
    L[p] = __builtin_bit_cast(unsigned, lb);
  }
  dst[0] = make_uint4(H[0], H[1], H[2], H[3]);
  dst[1] = make_uint4(H[4], H[5], H[6], H[7]);
  dst[2] = make_uint4(M[0], M[1], M[2], M[3]);
  dst[3] = make_uint4(M[4], M[5], M[6], M[7]);
  dst[4] = make_uint4(L[0], L[1], L[2], L[3]);
  dst[5] = make_uint4(L[4], L[5], L[6], L[7]);
}

// thread per (16-k block, row), rows fastest (the 96-byte records of consecutive threads are
// contiguous); rows ≥ `rows` and k ≥ K are written as zeros
__global__ void __launch_bounds__(256) split_blk_kernel(const float* __restrict__ X, int64_t ld, int64_t rows, int K,
                                                        const float* __restrict__ sub_k, const float* __restrict__ colscale,
                                                        uint16_t* __restrict__ out, int64_t Rp, int KB, int vec) {
  const int64_t total = (int64_t)KB * Rp;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = t % Rp;
    const int kb = (int)(t / Rp), k0 = 16 * kb;
    float v[16];
    if (row < rows) {
      const float* x = X + row * ld + k0;
      if (vec && k0 + 16 <= K) {
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const float4 f = reinterpret_cast<const float4*>(x)[c];
          v[4 * c] = f.x;
          v[4 * c + 1] = f.y;
          v[4 * c + 2] = f.z;
          v[4 * c + 3] = f.w;
        }
      } else {
#pragma unroll
        for (int c = 0; c < 16; ++c) v[c] = k0 + c < K ? x[c] : 0.f;
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        const bool in = k0 + c < K;
        if (sub_k && in) v[c] -= sub_k[k0 + c];
        if (colscale && in) v[c] *= colscale[k0 + c];
      }
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) v[c] = 0.f;
    }
    split16_store(v, reinterpret_cast<uint4*>(out + t * 48));
  }
}

// the blocked planes of rows [row0, row0 + rows) of the virtual matrix normal(key, (·, d))
// (rng.hip's philox_fill arithmetic: element e is word e mod 4 of Philox block e / 4, Box–Muller
// on word pairs) — the f32 noise is never written
__global__ void __launch_bounds__(256) philox_blk_kernel(const int64_t* __restrict__ key, int64_t rows, int d, int64_t row0,
                                                         uint16_t* __restrict__ out, int64_t Rp, int KB) {
  uint32_t k0, k1;
  evx::load_key(key, k0, k1);
  const int64_t total = (int64_t)KB * Rp;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t row = t % Rp;
    const int kb = (int)(t / Rp);
    float v[16];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = 16 * kb + 4 * c;
      float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < rows && k < d) {  // d % 4 == 0: the four values are one Philox block
        const int64_t e = (row0 + row) * (int64_t)d + k;
        f = evx::normal4(evx::philox_block((uint64_t)(e >> 2), k0, k1));
      }
      v[4 * c] = f.x;
      v[4 * c + 1] = f.y;
      v[4 * c + 2] = f.z;
      v[4 * c + 3] = f.w;
    }
    split16_store(v, reinterpret_cast<uint4*>(out + t * 48));
  }
}

__device__ __forceinline__ void glds16(const void* src, void* dst) {
  typedef const __attribute__((address_space(1))) void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
}

// VAR (probes, tools/bench_gemm_blk.py --variant): 0 the kernel; 1 no main-loop copies (the
// prologue's stages are re-read: the MFMA / LDS-read ceiling); 2 no MFMAs (copies, barriers
// and fragment reads only); 3 s_setprio(1) around each stage's MFMAs
template <int WM, int WN, int TMW, int TNW, int NS, int VAR = 0>
__global__ void __launch_bounds__(64 * WM * WN) gemm_blk_kernel(EvxGemmBlk p) {
  constexpr int NW = WM * WN;
  constexpr int BM = 16 * TMW * WM, BN = 16 * TNW * WN;
  constexpr int AB = BM * kRowB, BB = BN * kRowB, SB = AB + BB;
  static_assert(AB % 1024 == 0 && BB % 1024 == 0, "a stage is whole 1 KiB wave copies");
  constexpr int APC = AB / 1024, PC = SB / 1024;
  constexpr int PMAX = (PC + NW - 1) / NW, PMIN = PC / NW;  // copies per wave and stage
  static_assert(PMIN >= 1 && PMIN <= 15, "vmcnt range");
  // ALL of the kernel's LDS in this one array (a second __shared__ object makes hipcc wait for
  // every LDS-DMA before the first ds_read of a stage)
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NS * SB];
  if (p.skip && *p.skip) return;

  int tm, tn;
  {  // XCD-aware order: groups of 4 row panels, column-major inside a group
    const int bid = evx::xcd_remap(blockIdx.x, gridDim.x);
    constexpr int GM = 4;
    const int width = GM * p.tiles_n;
    const int grp = bid / width, fm = grp * GM;
    const int gm = min(GM, p.tiles_m - fm), rem = bid - grp * width;
    tm = fm + rem % gm;
    tn = rem / gm;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w / WN, wn = w % WN;
  const int r = lane & 15, q = lane >> 4;

  const unsigned char* a_base = reinterpret_cast<const unsigned char*>(p.A) + (int64_t)m0 * kRowB + lane * 16;
  const unsigned char* b_base = reinterpret_cast<const unsigned char*>(p.B) + (int64_t)n0 * kRowB + lane * 16;
  const int64_t a_ks = p.a_rows * kRowB, b_ks = p.b_rows * kRowB;

  auto issue = [&](int kb, int buf) {
    unsigned char* dst = lds + buf * SB;
    const unsigned char* as = a_base + kb * a_ks;
    const unsigned char* bs = b_base + kb * b_ks;
#pragma unroll
    for (int i = 0; i < PMAX; ++i) {
      const int pc = w + NW * i;  // wave-uniform
      if (pc < PC) glds16(pc < APC ? as + pc * 1024 : bs + (pc - APC) * 1024, dst + pc * 1024);
    }
  };

  // lane (r, q) reads k = 8(q & 1) … +7 of plane PA / PB[c][q >> 1] (0 h, 1 m, 2 l)
  const int hq = q >> 1, e16 = 16 * (q & 1);
  const int oa0 = e16, oa1 = e16 + 32 * (hq ? 0 : 1), oa2 = e16 + 32 * (hq ? 2 : 1);
  const int ob0 = e16 + 32 * (hq ? 1 : 0), ob1 = e16 + 32 * (hq ? 2 : 0), ob2 = e16 + 32 * (hq ? 0 : 1);
  const int arow = (wm * TMW * 16 + r) * kRowB, brow = AB + (wn * TNW * 16 + r) * kRowB;

  f32x4 acc[TMW][TNW];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TNW; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const unsigned char* sa = lds + buf * SB + arow;
    const unsigned char* sb = lds + buf * SB + brow;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int oa = c == 0 ? oa0 : (c == 1 ? oa1 : oa2);
      const int ob = c == 0 ? ob0 : (c == 1 ? ob1 : ob2);
      bf16x8 af[TMW], bfr[TNW];
#pragma unroll
      for (int i = 0; i < TMW; ++i) af[i] = *reinterpret_cast<const bf16x8*>(sa + i * 16 * kRowB + oa);
#pragma unroll
      for (int j = 0; j < TNW; ++j) bfr[j] = *reinterpret_cast<const bf16x8*>(sb + j * 16 * kRowB + ob);
      if constexpr (VAR == 2) {
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
          for (int j = 0; j < TNW; ++j) acc[i][j][0] += (float)af[i][0] * (float)bfr[j][0];
      } else {
        if constexpr (VAR == 3) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < TMW; ++i)
#pragma unroll
          for (int j = 0; j < TNW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if constexpr (VAR == 3) __builtin_amdgcn_s_setprio(0);
      }
    }
  };

  const int KB = p.KB;
  issue(0, 0);
  if (KB > 1) issue(1, 1);
  int cur = 0, nxt = 2 % NS;
  for (int t = 0; t < KB; ++t) {
    // stage t landed in this wave's copies (the next stage's may stay in flight), this wave's
    // reads of the buffer about to be refilled are done; then every wave's
    if (t + 1 < KB) asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(PMIN) : "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    if (VAR != 1 && t + 2 < KB) issue(t + 2, nxt);
    compute(cur);
    cur = cur + 1 == NS ? 0 : cur + 1;
    nxt = nxt + 1 == NS ? 0 : nxt + 1;
  }

  // epilogue: 16x16 accumulator map col = lane & 15, row = 4·(lane >> 4) + e
  const float s = p.alpha * (p.alpha_ptr ? p.alpha_ptr[0] : 1.f);
#pragma unroll
  for (int j = 0; j < TNW; ++j) {
    const int col = n0 + (wn * TNW + j) * 16 + r;
    const bool cin = col < p.N;
    const float bias = (p.bias_n && cin) ? p.bias_n[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      const int rowb = m0 + (wm * TMW + i) * 16 + 4 * q;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = rowb + e;
        if (cin && row < p.M) p.C[(int64_t)row * p.ldc + col] = fmaf(s, acc[i][j][e], bias);
      }
    }
  }
}

// ============================================================================ f16x3 planes
// An f32 value split into two f16 (11-bit significand) parts with round-to-nearest-even,
// after a per-row power-of-two scale that puts the row's largest |x| at ≤ 2¹⁵:
//   x·2^e = h + m + ε,  |m| ≤ 2⁻¹¹|x·2^e|,  |ε| ≤ max(2⁻²²|x·2^e|, 2⁻²⁴ · 2⁻¹⁴)
// (the 13 low bits of the remainder x − h are exact in f32 and m keeps 11 of them, as long as
// m is a normal f16: for elements more than ≈2¹⁸ below the row max, m falls into the f16
// subnormals and the error is bounded absolutely instead, |ε| ≤ 2⁻⁴⁰·rowmax·2^e after the
// scale).  The scale exponent is clamped (e ≤ 125) so a row of tiny magnitude never scales
// to inf; the Σ|ab| bound below holds either way (tests/test_gemm_blk.py, tiny and
// wide-range rows).  A
// product a·b is kept as h_a h_b + h_a m_b + m_a h_b — three v_mfma_f32_32x32x16_f16, each
// product of two f16 exact in the f32 accumulator — with the dropped m_a m_b ≤ 2⁻²²|ab|: at
// most ≈3·2⁻²² ≈ 7e-7 |a·b| per product in the worst case, unbiased (RNE), inside the
// 2e-6·Σ|a·b| bound every framework GEMM is tested to (tests/test_gemm_blk.py).  Against the
// bf16x6 split this halves the MFMAs (3 instead of 6 per k) and the operand bytes go from 6 to
// 4 per element, which is what bounds a 256-tile launch's global → LDS stream.
//
// Record layout: f16 [K/16][Rp][2][16] — per 16-k block and row 64 bytes = four 16-byte slots
// (h k0-7, h k8-15, m k0-7, m k8-15), slot s stored at position s ^ ((row >> 2) & 3) so the 16
// lanes of a ds_read_b128 lane group (32x32x16 operand map: lane l reads row l & 31, k half
// l >> 5) land on 16 distinct bank slots.  Row scales 2^-e are a separate f32 vector.
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kRowH = 64;

// s_waitcnt immediate (gfx9 encoding): vmcnt(n) [3:0] + [15:14], expcnt(7) [6:4] = no wait, lgkmcnt(0) [11:8]
constexpr int waitcnt_vm_lgkm0(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4); }  // bytes per (row, 16-k block): 2 planes × 16 f16

__device__ __forceinline__ void split16h_store(const float (&v)[16], float sc, int64_t row, uint4* __restrict__ dst) {
  unsigned H[8], M[8];
#pragma unroll
  for (int p = 0; p < 8; ++p) {
    const float a0 = v[2 * p] * sc, a1 = v[2 * p + 1] * sc;
    const f16x2 hb = __builtin_convertvector(f32x2{a0, a1}, f16x2);
    const f32x2 hf = __builtin_convertvector(hb, f32x2);
    const f16x2 mb = __builtin_convertvector(f32x2{a0 - hf.x, a1 - hf.y}, f16x2);
    H[p] = __builtin_bit_cast(unsigned, hb);
    M[p] = __builtin_bit_cast(unsigned, mb);
  }
  const int sw = (int)((row >> 2) & 3);
  dst[0 ^ sw] = make_uint4(H[0], H[1], H[2], H[3]);
  dst[1 ^ sw] = make_uint4(H[4], H[5], H[6], H[7]);
  dst[2 ^ sw] = make_uint4(M[0], M[1], M[2], M[3]);
  dst[3 ^ sw] = make_uint4(M[4], M[5], M[6], M[7]);
}

// 2^e with e = 15 − ⌈log₂ max⌉ (max > 0, finite), else 1; e ≤ 125 (a row whose max is below
// ≈2⁻¹¹⁰ would otherwise get a scale past 2¹²⁸ = inf and NaN planes)
__device__ __forceinline__ float row_scale(float mx) {
  if (!(mx > 0.f) || !(mx < 3.0e38f)) return 1.f;
  int ex;
  frexpf(mx, &ex);  // mx = f·2^ex, f ∈ [0.5, 1): mx < 2^ex
  return ldexpf(1.f, 15 - max(ex, -110));
}

// one wave per row: lane j owns the 16-k blocks j, j + 64, …; row max → scale → split
__global__ void __launch_bounds__(256) split_h_kernel(const float* __restrict__ X, int64_t ld, int64_t rows, int K,
                                                      const float* __restrict__ sub_k, const float* __restrict__ colscale,
                                                      uint16_t* __restrict__ out, float* __restrict__ rinv, int64_t Rp, int KB, int vec) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= Rp) return;
  // the first 16-k block of each lane stays in registers (K ≤ 1024: the whole row); blocks past
  // it are re-read for the split (L2-resident: the row was just read for its max)
  float v0[16];
  float mx = 0.f;
  auto load_blk = [&](int kb, float (&o)[16]) {
    const int k0 = 16 * kb;
    const float* x = X + row * ld + k0;
    if (vec && k0 + 16 <= K) {
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 f = reinterpret_cast<const float4*>(x)[c];
        o[4 * c] = f.x;
        o[4 * c + 1] = f.y;
        o[4 * c + 2] = f.z;
        o[4 * c + 3] = f.w;
      }
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) o[c] = k0 + c < K ? x[c] : 0.f;
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      const bool in = k0 + c < K;
      if (sub_k && in) o[c] -= sub_k[k0 + c];
      if (colscale && in) o[c] *= colscale[k0 + c];
    }
  };
  const bool live = row < rows;
#pragma unroll
  for (int c = 0; c < 16; ++c) v0[c] = 0.f;
  if (live) {
    if (lane < KB) load_blk(lane, v0);
#pragma unroll
    for (int c = 0; c < 16; ++c) mx = fmaxf(mx, fabsf(v0[c]));
    for (int kb = lane + 64; kb < KB; kb += 64) {
      float t[16];
      load_blk(kb, t);
#pragma unroll
      for (int c = 0; c < 16; ++c) mx = fmaxf(mx, fabsf(t[c]));
    }
  }
  mx = evx::wave_max(mx);
  const float sc = live ? row_scale(mx) : 1.f;
  if (lane == 0) rinv[row] = live ? 1.f / sc : 0.f;
  for (int kb = lane; kb < KB; kb += 64) {
    float t[16];
    if (kb == lane) {
#pragma unroll
      for (int c = 0; c < 16; ++c) t[c] = v0[c];
    } else if (live) {
      load_blk(kb, t);
    } else {
#pragma unroll
      for (int c = 0; c < 16; ++c) t[c] = 0.f;
    }
    split16h_store(t, sc, row, reinterpret_cast<uint4*>(out + ((int64_t)kb * Rp + row) * 32));
  }
}

// 16 rows per 256-thread workgroup.  Phase 1: each wave reads 4 whole rows (coalesced, lane j
// takes the 16-k block j, j + 64, …) and reduces the row's max |x| to its scale (LDS).  Phase
// 2: thread (record, slot) computes one 16-byte slot (8 values of the h or m plane) of a
// record, so each store instruction writes 1 KiB contiguous (16 rows of one 16-k block); its
// 32-byte operand read hits L2 (the workgroup's 64 KiB of rows were just read).
__global__ void __launch_bounds__(256) split_h2_kernel(const float* __restrict__ X, int64_t ld, int64_t rows, int K,
                                                       const float* __restrict__ sub_k, const float* __restrict__ colscale,
                                                       uint16_t* __restrict__ out, float* __restrict__ rinv, int64_t Rp, int KB) {
  __shared__ float s_sc[16];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 16;
  auto val = [&](int64_t row, int k) {
    float x = X[row * ld + k];
    if (sub_k) x -= sub_k[k];
    if (colscale) x *= colscale[k];
    return x;
  };
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int64_t row = r0 + 4 * w + i;
    float mx = 0.f;
    if (row < rows) {
      for (int k = 4 * lane; k < K; k += 256) {
        if (k + 3 < K && ((ld | (int64_t)k) & 3) == 0 && !sub_k && !colscale) {
          const float4 f = *reinterpret_cast<const float4*>(X + row * ld + k);
          mx = fmaxf(mx, fmaxf(fmaxf(fabsf(f.x), fabsf(f.y)), fmaxf(fabsf(f.z), fabsf(f.w))));
        } else {
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (k + c < K) mx = fmaxf(mx, fabsf(val(row, k + c)));
        }
      }
    }
    mx = evx::wave_max(mx);
    if (lane == 0) {
      const float sc = row < rows ? row_scale(mx) : 1.f;
      s_sc[4 * w + i] = sc;
      if (row < Rp) rinv[row] = row < rows ? 1.f / sc : 0.f;
    }
  }
  __syncthreads();
  // phase 2: 16 rows × 4 slots = 64 threads per 16-k block, 4 blocks per pass
  const int rl = (threadIdx.x >> 2) & 15, pos = threadIdx.x & 3;
  const int64_t row = r0 + rl;
  const float sc = s_sc[rl];
  const int sw = (int)((row >> 2) & 3), slot = pos ^ sw, plane = slot >> 1, kh = slot & 1;
  for (int kb = threadIdx.x >> 6; kb < KB; kb += 4) {
    const int k0 = 16 * kb + 8 * kh;
    float v[8];
    if (row < rows) {
      if (k0 + 8 <= K && ((ld | (int64_t)k0) & 3) == 0) {
        const float4 f0 = *reinterpret_cast<const float4*>(X + row * ld + k0);
        const float4 f1 = *reinterpret_cast<const float4*>(X + row * ld + k0 + 4);
        v[0] = f0.x; v[1] = f0.y; v[2] = f0.z; v[3] = f0.w;
        v[4] = f1.x; v[5] = f1.y; v[6] = f1.z; v[7] = f1.w;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          if (sub_k) v[c] -= sub_k[k0 + c];
          if (colscale) v[c] *= colscale[k0 + c];
        }
      } else {
#pragma unroll
        for (int c = 0; c < 8; ++c) v[c] = k0 + c < K ? val(row, k0 + c) : 0.f;
      }
    } else {
#pragma unroll
      for (int c = 0; c < 8; ++c) v[c] = 0.f;
    }
    unsigned o[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float a0 = v[2 * p] * sc, a1 = v[2 * p + 1] * sc;
      const f16x2 hb = __builtin_convertvector(f32x2{a0, a1}, f16x2);
      if (plane == 0) {
        o[p] = __builtin_bit_cast(unsigned, hb);
      } else {
        const f32x2 hf = __builtin_convertvector(hb, f32x2);
        o[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a0 - hf.x, a1 - hf.y}, f16x2));
      }
    }
    *reinterpret_cast<uint4*>(out + (((int64_t)kb * Rp + row) * 4 + pos) * 8) = make_uint4(o[0], o[1], o[2], o[3]);
  }
}

// 4 rows per 256-thread workgroup (one per wave; K ≤ 1024).  Phase 1: the wave issues all its
// row's loads at once (4 float4 per lane), stages the shifted / scaled row in LDS and reduces
// its max |x| to the row scale.  Phase 2: thread (record, slot) computes one 16-byte slot (8
// values of the h or m plane) from LDS — 16 consecutive threads write the 4 rows' records of
// one 16-k block, 256 contiguous bytes.  ncomp > 1: one plane set per shift row of sub_k
// (sub_ld apart; sets pstride elements and Rp row scales apart) from ONE read of X — the
// stacked composition GEMM's per-component operands (x − o_c).
__global__ void __launch_bounds__(256) split_h4_kernel(const float* __restrict__ X, int64_t ld, int64_t rows, int K,
                                                       const float* __restrict__ sub_k, const float* __restrict__ colscale,
                                                       uint16_t* __restrict__ out, float* __restrict__ rinv, int64_t Rp, int KB, int vec,
                                                       int64_t sub_ld, int ncomp, int64_t pstride) {
  __shared__ __attribute__((aligned(16))) float s_row[4][1024 + 16];
  __shared__ float s_sc[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t r0 = (int64_t)blockIdx.x * 4;
  float4 f[4];
  {
    const int64_t row = r0 + w;
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int k = 4 * lane + 256 * c;
      f[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < rows) {
        if (vec && k + 3 < K) {
          f[c] = *reinterpret_cast<const float4*>(X + row * ld + k);
        } else {
          float t[4];
#pragma unroll
          for (int e = 0; e < 4; ++e) t[e] = k + e < K ? X[row * ld + k + e] : 0.f;
          f[c] = make_float4(t[0], t[1], t[2], t[3]);
        }
      }
    }
  }
  for (int comp = 0; comp < ncomp; ++comp) {
    const float* sub = sub_k ? sub_k + comp * sub_ld : nullptr;
    if (comp) __syncthreads();  // the previous component's phase 2 is done with s_row / s_sc
    {
      const int64_t row = r0 + w;
      float mx = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int k = 4 * lane + 256 * c;
        float t[4] = {f[c].x, f[c].y, f[c].z, f[c].w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bool in = k + e < K && row < rows;
          if (sub && in) t[e] -= sub[k + e];
          if (colscale && in) t[e] *= colscale[k + e];
          if (!in) t[e] = 0.f;
          mx = fmaxf(mx, fabsf(t[e]));
        }
        *reinterpret_cast<float4*>(&s_row[w][k]) = make_float4(t[0], t[1], t[2], t[3]);
      }
      mx = evx::wave_max(mx);
      if (lane == 0) {
        const float sc = row < rows ? row_scale(mx) : 1.f;
        s_sc[w] = sc;
        if (row < Rp) rinv[comp * Rp + row] = row < rows ? 1.f / sc : 0.f;
      }
    }
    __syncthreads();
    const int rl = (threadIdx.x >> 2) & 3, pos = threadIdx.x & 3;
    const int64_t row = r0 + rl;
    const float sc = s_sc[rl];
    const int sw = (int)((row >> 2) & 3), slot = pos ^ sw, plane = slot >> 1, kh = slot & 1;
    uint16_t* o_c = out + comp * pstride;
    for (int kb = threadIdx.x >> 4; kb < KB; kb += 16) {
      const float* src = &s_row[rl][16 * kb + 8 * kh];
      const float4 f0 = *reinterpret_cast<const float4*>(src);
      const float4 f1 = *reinterpret_cast<const float4*>(src + 4);
      const float v[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
      unsigned o[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float a0 = v[2 * p] * sc, a1 = v[2 * p + 1] * sc;
        const f16x2 hb = __builtin_convertvector(f32x2{a0, a1}, f16x2);
        if (plane == 0) {
          o[p] = __builtin_bit_cast(unsigned, hb);
        } else {
          const f32x2 hf = __builtin_convertvector(hb, f32x2);
          o[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a0 - hf.x, a1 - hf.y}, f16x2));
        }
      }
      *reinterpret_cast<uint4*>(o_c + (((int64_t)kb * Rp + row) * 4 + pos) * 8) = make_uint4(o[0], o[1], o[2], o[3]);
    }
  }
}

// Philox normals straight into f16x3 records at the fixed scale 2¹³ (|z| < 6.7 for 32-bit
// uniforms: ≤ 5.5e4 < 65504).  Thread (record, half): 8 normals (two Philox blocks), their h
// and m slots; consecutive threads fill consecutive records.
__global__ void __launch_bounds__(256) philox_h_kernel(const int64_t* __restrict__ key, int64_t rows, int d, int64_t row0,
                                                       uint16_t* __restrict__ out, float* __restrict__ rinv, int64_t Rp, int KB) {
  uint32_t k0, k1;
  evx::load_key(key, k0, k1);
  // 32-bit record index (the launcher checks KB·Rp < 2³¹): a 64-bit division here was ≈ 10 %
  // of this VALU-bound kernel's issue
  const uint32_t total = (uint32_t)KB * (uint32_t)Rp * 2u, rp = (uint32_t)Rp;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < total; t += gridDim.x * blockDim.x) {
    const int half = (int)(t & 1);
    const uint32_t rec = t >> 1, kb32 = rec / rp;
    const int64_t row = rec - kb32 * rp;
    const int kb = (int)kb32;
    float v[8];
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int k = 16 * kb + 8 * half + 4 * c;
      float4 f = make_float4(0.f, 0.f, 0.f, 0.f);
      if (row < rows && k < d) {
        const int64_t e = (row0 + row) * (int64_t)d + k;
        f = evx::normal4(evx::philox_block((uint64_t)(e >> 2), k0, k1));
      }
      v[4 * c] = f.x;
      v[4 * c + 1] = f.y;
      v[4 * c + 2] = f.z;
      v[4 * c + 3] = f.w;
    }
    unsigned H[4], M[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const float a0 = v[2 * p] * 8192.f, a1 = v[2 * p + 1] * 8192.f;
      const f16x2 hb = __builtin_convertvector(f32x2{a0, a1}, f16x2);
      const f32x2 hf = __builtin_convertvector(hb, f32x2);
      H[p] = __builtin_bit_cast(unsigned, hb);
      M[p] = __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{a0 - hf.x, a1 - hf.y}, f16x2));
    }
    const int sw = (int)((row >> 2) & 3);
    uint4* dst = reinterpret_cast<uint4*>(out + (int64_t)rec * 32);
    dst[half ^ sw] = make_uint4(H[0], H[1], H[2], H[3]);
    dst[(2 + half) ^ sw] = make_uint4(M[0], M[1], M[2], M[3]);
    if (kb == 0 && half == 0) rinv[row] = row < rows ? 1.f / 8192.f : 0.f;
  }
}

// WM × WN waves, each TMW 32-row blocks × TNW 32-column blocks; NS stages of one 16-k block
template <int WM, int WN, int TMW, int TNW, int NS, int VAR = 0>
__global__ void __launch_bounds__(64 * WM * WN) gemm_h3_kernel(EvxGemmBlk p) {
  constexpr int NW = WM * WN;
  constexpr int BM = 32 * TMW * WM, BN = 32 * TNW * WN;
  constexpr int AB = BM * kRowH, BB = BN * kRowH, SB = AB + BB;
  static_assert(AB % 1024 == 0 && BB % 1024 == 0, "a stage is whole 1 KiB wave copies");
  constexpr int APC = AB / 1024, PC = SB / 1024;
  constexpr int PMAX = (PC + NW - 1) / NW, PMIN = PC / NW;
  static_assert(PMIN >= 1 && PMIN * (NS - 2) <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NS * SB];
  if (p.skip && *p.skip) return;

  int tm, tn;
  {
    const int bid = evx::xcd_remap(blockIdx.x, gridDim.x);
    constexpr int GM = 4;
    const int width = GM * p.tiles_n;
    const int grp = bid / width, fm = grp * GM;
    const int gm = min(GM, p.tiles_m - fm), rem = bid - grp * width;
    tm = fm + rem % gm;
    tn = rem / gm;
  }
  const int m0 = tm * BM, n0 = tn * BN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w / WN, wn = w % WN;
  const int r = lane & 31, h2 = lane >> 5;

  // stacked operands (sub_cols > 0): column block n0 / sub_cols reads A's plane set of that
  // component (a tile never straddles two blocks: sub_cols is a multiple of BN)
  const int comp = p.sub_cols > 0 ? n0 / p.sub_cols : 0;
  const unsigned char* a_base =
      reinterpret_cast<const unsigned char*>(p.A + comp * p.a_comp_stride) + (int64_t)m0 * kRowH + lane * 16;
  const float* a_rinv = p.a_rinv + (int64_t)comp * p.a_rows;
  const unsigned char* b_base = reinterpret_cast<const unsigned char*>(p.B) + (int64_t)n0 * kRowH + lane * 16;
  const int64_t a_ks = p.a_rows * kRowH, b_ks = p.b_rows * kRowH;
  auto issue = [&](int kb, int buf) {
    unsigned char* dst = lds + buf * SB;
    const unsigned char* as = a_base + kb * a_ks;
    const unsigned char* bs = b_base + kb * b_ks;
#pragma unroll
    for (int i = 0; i < PMAX; ++i) {
      const int pc = w + NW * i;
      if (pc < PC) glds16(pc < APC ? as + pc * 1024 : bs + (pc - APC) * 1024, dst + pc * 1024);
    }
  };

  // lane (r, h2): 8 values k = 8·h2 … of the h / m plane of its row, slot-swizzled by row
  const int sw = (r >> 2) & 3;
  const int oh = ((0 + h2) ^ sw) * 16, om = ((2 + h2) ^ sw) * 16;
  const int arow = (wm * TMW * 32 + r) * kRowH, brow = AB + (wn * TNW * 32 + r) * kRowH;

  f32x16 acc[TMW][TNW];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int j = 0; j < TNW; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  // fragments of one stage: h and m planes of the wave's TMW A blocks and TNW B blocks
  struct Frag {
    f16x8 ah[TMW], am[TMW], bh[TNW], bm[TNW];
  };
  auto read_frag = [&](Frag& f, int buf) {
    const unsigned char* sa = lds + buf * SB + arow;
    const unsigned char* sb = lds + buf * SB + brow;
#pragma unroll
    for (int j = 0; j < TNW; ++j) {
      f.bh[j] = *reinterpret_cast<const f16x8*>(sb + j * 32 * kRowH + oh);
      f.bm[j] = *reinterpret_cast<const f16x8*>(sb + j * 32 * kRowH + om);
    }
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      f.ah[i] = *reinterpret_cast<const f16x8*>(sa + i * 32 * kRowH + oh);
      f.am[i] = *reinterpret_cast<const f16x8*>(sa + i * 32 * kRowH + om);
    }
  };
  auto mfma_frag = [&](const Frag& f) {
    if constexpr (VAR == 2) {
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j][0] += (float)f.ah[i][0] * (float)f.bm[j][0] + (float)f.am[i][0] * (float)f.bh[j][0];
    } else {
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.ah[i], f.bh[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.ah[i], f.bm[j], acc[i][j], 0, 0, 0);
#pragma unroll
      for (int i = 0; i < TMW; ++i)
#pragma unroll
        for (int j = 0; j < TNW; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.am[i], f.bh[j], acc[i][j], 0, 0, 0);
    }
  };

  // software pipeline: the fragment reads of stage t are issued right after the barrier that
  // publishes it and run under the MFMAs of stage t − 1 (two fragment sets in registers); the
  // reads are complete (lgkmcnt(0)) before the next barrier, which also guards the buffer refill
  const int KB = p.KB;
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < KB) issue(s, s);
  Frag fr[2];
  int cur = 0, nxt = NS - 1;
  auto sync_stage = [&](int t) {
    // stage t landed (this wave's copies; later stages' stay in flight), this wave's reads of
    // the buffer refilled next are done — then every wave's, at the barrier.  The wait is the
    // builtin (the waitcnt pass then knows every fragment read is complete and inserts no
    // lgkmcnt(0) in front of the next MFMAs); the barrier is asm with a memory clobber so no
    // LDS read moves above it
    const int after = min(NS - 2, KB - 1 - t);
    if (after >= 6 && NS >= 8) __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(6 * PMIN));
    else if (after == 5 && NS >= 7) __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(5 * PMIN));
    else if (after == 4 && NS >= 6) __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(4 * PMIN));
    else if (after >= 3 && NS >= 5) __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(3 * PMIN));
    else if (after == 2 && NS >= 4) __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(2 * PMIN));
    else if (after == 1) __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(PMIN));
    else __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(0));
    if (VAR != 4) asm volatile("s_barrier" ::: "memory");
  };
  sync_stage(0);
  if (VAR != 1 && VAR != 4 && NS - 1 < KB) issue(NS - 1, nxt);
  read_frag(fr[0], cur);
  cur = cur + 1 == NS ? 0 : cur + 1;
  nxt = nxt + 1 == NS ? 0 : nxt + 1;
  int t = 1;
  for (; t + 1 < KB; t += 2) {  // two stages per trip: the fragment sets swap roles statically
    sync_stage(t);
    if (VAR != 1 && VAR != 4 && t + NS - 1 < KB) issue(t + NS - 1, nxt);
    read_frag(fr[1], cur);
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(fr[0]);
    __builtin_amdgcn_sched_barrier(0);
    cur = cur + 1 == NS ? 0 : cur + 1;
    nxt = nxt + 1 == NS ? 0 : nxt + 1;
    sync_stage(t + 1);
    if (VAR != 1 && VAR != 4 && t + NS < KB) issue(t + NS, nxt);
    read_frag(fr[0], cur);
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(fr[1]);
    __builtin_amdgcn_sched_barrier(0);
    cur = cur + 1 == NS ? 0 : cur + 1;
    nxt = nxt + 1 == NS ? 0 : nxt + 1;
  }
  if (t < KB) {  // one stage left: its reads under the MFMAs of the stage before
    sync_stage(t);
    read_frag(fr[1], cur);
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(fr[0]);
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(fr[1]);
  } else {
    mfma_frag(fr[0]);
  }

  // epilogue: 32x32 accumulator map col = lane & 31, row = (e & 3) + 8·(e >> 2) + 4·(lane >> 5)
  if constexpr (VAR == 5) {  // probe: no output stores (one value per lane keeps the MFMAs live)
    float z = 0.f;
#pragma unroll
    for (int i = 0; i < TMW; ++i)
#pragma unroll
      for (int j = 0; j < TNW; ++j)
#pragma unroll
        for (int e = 0; e < 16; ++e) z += acc[i][j][e];
    if (z == 1.2345f) p.C[threadIdx.x] = z;
    return;
  }
  const float s = p.alpha * (p.alpha_ptr ? p.alpha_ptr[0] : 1.f);
  if (p.row_terms) {
    // CEC'22 basic-function row terms of z = this tile's columns (Zakharov: Σ z², Σ ½(j+1) z;
    // Rastrigin: Σ y² − 10 cos 2πy + 10 with y = 0.0512 z, 0): per 32-column block a
    // transposing butterfly over the 32 lanes of each half (16 values → one sum per lane pair,
    // 16 shuffles instead of 80), then the WN column blocks through LDS, one write per row
    static_assert(TNW == 1, "row terms: one 32-column block per wave");
    float* part = reinterpret_cast<float*>(lds);  // [WN][BM][2], the stages are free now
    __syncthreads();
    const int col = n0 + wn * 32 + r;
    const bool cin = col < p.N;
    const float cs = cin ? s * p.b_rinv[col] : 0.f;
    const float cj = 0.5f * (float)(col + 1);
    const bool zak = p.row_fid == 0;
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      const int rowb = m0 + (wm * TMW + i) * 32 + 4 * h2;
      float t1[16], t2[16];
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = rowb + (e & 3) + 8 * (e >> 2);
        const float rv = row < p.M ? p.a_rinv[row] : 0.f;
        const float z = cs * rv * acc[i][0][e];
        if (zak) {
          t1[e] = z * z;
          t2[e] = cj * z;
        } else {  // v_cos takes revolutions: cos(2πy)
          const float y = 0.0512f * z;
          t1[e] = cin ? y * y - 10.f * __builtin_amdgcn_cosf(y) + 10.f : 0.f;
          t2[e] = 0.f;
        }
      }
#pragma unroll
      for (int w2 = 16; w2 >= 1; w2 >>= 1) {  // 16 → 8 → 4 → 2 → 1 values per lane
        const bool hi = (r & w2) != 0;
        const int nv = w2 == 1 ? 1 : w2 / 2;  // values kept after this step (xor 1: the final sum)
        if (w2 == 1) {
          t1[0] += __shfl_xor(t1[0], 1);
          t2[0] += __shfl_xor(t2[0], 1);
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            if (k < nv) {
              const float s1 = hi ? t1[k] : t1[k + nv], s2 = hi ? t2[k] : t2[k + nv];
              const float k1 = hi ? t1[k + nv] : t1[k], k2 = hi ? t2[k + nv] : t2[k];
              t1[k] = k1 + __shfl_xor(s1, w2);
              t2[k] = k2 + __shfl_xor(s2, w2);
            }
          }
        }
      }
      // lane (r even, h2) holds the 32-column sums of value e = (r >> 1) & 15
      if ((r & 1) == 0) {
        const int e = (r >> 1) & 15;
        const int lr = (wm * TMW + i) * 32 + 4 * h2 + (e & 3) + 8 * (e >> 2);
        part[(wn * BM + lr) * 2] = t1[0];
        part[(wn * BM + lr) * 2 + 1] = t2[0];
      }
    }
    __syncthreads();
    for (int lr = threadIdx.x; lr < BM; lr += 64 * NW) {
      const int row = m0 + lr;
      if (row >= p.M) continue;
      float a = 0.f, b = 0.f;
#pragma unroll
      for (int q = 0; q < WN; ++q) {  // fixed order: deterministic
        a += part[(q * BM + lr) * 2];
        b += part[(q * BM + lr) * 2 + 1];
      }
      *reinterpret_cast<float2*>(p.row_terms + ((int64_t)tn * p.M + row) * 2) = make_float2(a, b);
    }
    return;
  }
  // the lane's 16 rows of a 32-row block are 4 runs of 4 (rows 8q + 4·h2 … +3): their row
  // scales arrive as 4 float4 loads per block, all issued before the first store
  // (rinv has Rp ≥ the tile's rows rounded to 64 entries; rows past M read zeros / slack)
  float4 ra[TMW][4];
#pragma unroll
  for (int i = 0; i < TMW; ++i)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int row = m0 + (wm * TMW + i) * 32 + 8 * q + 4 * h2;
      ra[i][q] = row < p.M ? *reinterpret_cast<const float4*>(a_rinv + row) : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
  for (int j = 0; j < TNW; ++j) {
    const int col = n0 + (wn * TNW + j) * 32 + r;
    const bool cin = col < p.N;
    const float bias = (p.bias_n && cin) ? p.bias_n[col] : 0.f;
    const float cs = cin ? s * p.b_rinv[col] : 0.f;
#pragma unroll
    for (int i = 0; i < TMW; ++i) {
      const int rowb = m0 + (wm * TMW + i) * 32 + 4 * h2;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int row = rowb + (e & 3) + 8 * (e >> 2);
        const float4 q4 = ra[i][e >> 2];
        const float rv = (e & 3) == 0 ? q4.x : (e & 3) == 1 ? q4.y : (e & 3) == 2 ? q4.z : q4.w;
        if (cin && row < p.M) __builtin_nontemporal_store(fmaf(cs * rv, acc[i][j][e], bias), p.C + (int64_t)row * p.ldc + col);
      }
    }
  }
}

template <int WM, int WN, int TMW, int TNW, int NS>
void launch_h3(EvxGemmBlk a, hipStream_t s, int var) {
  constexpr int BM = 32 * TMW * WM, BN = 32 * TNW * WN;
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  const dim3 grid(a.tiles_m * a.tiles_n), block(64 * WM * WN);
  switch (var) {
    case 1: gemm_h3_kernel<WM, WN, TMW, TNW, NS, 1><<<grid, block, 0, s>>>(a); break;
    case 2: gemm_h3_kernel<WM, WN, TMW, TNW, NS, 2><<<grid, block, 0, s>>>(a); break;
    case 4: gemm_h3_kernel<WM, WN, TMW, TNW, NS, 4><<<grid, block, 0, s>>>(a); break;
    case 5: gemm_h3_kernel<WM, WN, TMW, TNW, NS, 5><<<grid, block, 0, s>>>(a); break;
    default: gemm_h3_kernel<WM, WN, TMW, TNW, NS, 0><<<grid, block, 0, s>>>(a); break;
  }
}

int g_h3_ns = -1;
int g_h3_cfg = -1;

int g_blk_variant = -1;

template <int WM, int WN, int TMW, int TNW, int NS>
void launch_cfg(EvxGemmBlk a, hipStream_t s) {
  constexpr int BM = 16 * TMW * WM, BN = 16 * TNW * WN;
  a.tiles_m = (a.M + BM - 1) / BM;
  a.tiles_n = (a.N + BN - 1) / BN;
  if (g_blk_variant < 0) {
    const char* e = getenv("EVOXMI_BLK_VARIANT");
    g_blk_variant = e ? atoi(e) : 0;
  }
  const dim3 grid(a.tiles_m * a.tiles_n), block(64 * WM * WN);
  switch (g_blk_variant) {
    case 1: gemm_blk_kernel<WM, WN, TMW, TNW, NS, 1><<<grid, block, 0, s>>>(a); break;
    case 2: gemm_blk_kernel<WM, WN, TMW, TNW, NS, 2><<<grid, block, 0, s>>>(a); break;
    case 3: gemm_blk_kernel<WM, WN, TMW, TNW, NS, 3><<<grid, block, 0, s>>>(a); break;
    default: gemm_blk_kernel<WM, WN, TMW, TNW, NS, 0><<<grid, block, 0, s>>>(a); break;
  }
}

}  // namespace

int64_t evx_blk_rows(int64_t rows) { return (rows + 63) / 64 * 64; }

int64_t evx_blk_elems(int64_t rows, int K) { return ((int64_t)((K + 15) / 16) * evx_blk_rows(rows) + kEvxBlkSlackRows) * 48; }

void evx_split_blk(const float* X, int64_t ld, int64_t rows, int K, const float* sub_k, const float* colscale, uint16_t* out,
                   hipStream_t s) {
  const int KB = (K + 15) / 16;
  const int64_t Rp = evx_blk_rows(rows), total = (int64_t)KB * Rp;
  const int vec = (reinterpret_cast<uintptr_t>(X) % 16 == 0) && (ld % 4 == 0);
  int g = (int)((total + 255) / 256);
  if (g > 8192) g = 8192;
  if (g > 0) split_blk_kernel<<<g, 256, 0, s>>>(X, ld, rows, K, sub_k, colscale, out, Rp, KB, vec);
}

void evx_philox_blk(const int64_t* key, int64_t rows, int d, int64_t row0, uint16_t* out, hipStream_t s) {
  const int KB = (d + 15) / 16;
  const int64_t Rp = evx_blk_rows(rows), total = (int64_t)KB * Rp;
  int g = (int)((total + 255) / 256);
  if (g > 8192) g = 8192;
  if (g > 0) philox_blk_kernel<<<g, 256, 0, s>>>(key, rows, d, row0, out, Rp, KB);
}

int64_t evx_h3_elems(int64_t rows, int K) { return ((int64_t)((K + 15) / 16) * evx_blk_rows(rows) + kEvxBlkSlackRows) * 32; }

void evx_split_h3(const float* X, int64_t ld, int64_t rows, int K, const float* sub_k, const float* colscale, uint16_t* out,
                  float* rinv, hipStream_t s, int ncomp, int64_t sub_ld) {
  const int KB = (K + 15) / 16;
  const int64_t Rp = evx_blk_rows(rows), pstride = evx_h3_elems(rows, K);
  const int vec = (reinterpret_cast<uintptr_t>(X) % 16 == 0) && (ld % 4 == 0);
  if (ncomp < 1) ncomp = 1;
  if (K <= 1024) {
    split_h4_kernel<<<(unsigned)(Rp / 4), 256, 0, s>>>(X, ld, rows, K, sub_k, colscale, out, rinv, Rp, KB, vec, sub_ld, ncomp,
                                                        pstride);
    return;
  }
  for (int c = 0; c < ncomp; ++c) {  // long rows: one pass per component
    const float* sub = sub_k ? sub_k + c * sub_ld : nullptr;
    if (reinterpret_cast<uintptr_t>(X) % 16 == 0)
      split_h2_kernel<<<(unsigned)(Rp / 16), 256, 0, s>>>(X, ld, rows, K, sub, colscale, out + c * pstride, rinv + c * Rp, Rp, KB);
    else
      split_h_kernel<<<(unsigned)((Rp + 3) / 4), 256, 0, s>>>(X, ld, rows, K, sub, colscale, out + c * pstride, rinv + c * Rp, Rp, KB, 0);
  }
}

void evx_philox_h3(const int64_t* key, int64_t rows, int d, int64_t row0, uint16_t* out, float* rinv, hipStream_t s) {
  const int KB = (d + 15) / 16;
  const int64_t Rp = evx_blk_rows(rows), total = (int64_t)KB * Rp * 2;
  if (total >= (int64_t)1 << 31) throw std::runtime_error("evx_philox_h3: rows · d too large for the 32-bit record index");
  int g = (int)((total + 255) / 256);
  if (g > 8192) g = 8192;
  if (g > 0) philox_h_kernel<<<g, 256, 0, s>>>(key, rows, d, row0, out, rinv, Rp, KB);
}

void evx_gemm_h3(const EvxGemmBlk& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return;
  if (g_blk_variant < 0) {
    const char* e = getenv("EVOXMI_BLK_VARIANT");
    g_blk_variant = e ? atoi(e) : 0;
  }
  if (g_h3_ns < 0) {
    const char* e = getenv("EVOXMI_H3_NS");
    g_h3_ns = e ? atoi(e) : 5;
  }
  // Tile height by how the product fills 256 CUs: the shortest of 64 / 128 / 192 / 320 rows
  // (× 128 columns, 8 waves) whose tiles fit in one wave of tiles — a population shard has
  // fewer rows than the flagship's 10 000 (5000 at 2 ranks, 1250 at 8), and 320-row tiles
  // would leave half / seven eighths of the chip idle.  Measured (eager, µs; tools/
  // bench_gemm_blk.py --only-h3, profiles/r6_h3_tile_heights.jsonl) at × 1000 × 1000:
  //   rows    320    192    128(NS6)  64     160×128 on 4 waves
  //   10000   82.2   97.1   102.6     99.8   108.6
  //    5000   72.0   52.8    67.8     60.4    58.1
  //    2500   65.7   46.3    36.4     39.9    53.0
  //    1250   66.8   44.0    33.7     29.7    51.2
  // (64 rows with 8 stages, 128 with 4, 32 × 128 on 4 waves: no better — removed).
  if (g_h3_cfg < 0) {
    const char* e = getenv("EVOXMI_H3_CFG");  // probe override: 1 = 320, 2 = 192, 3 = 128, 4 = 64 rows
    g_h3_cfg = e ? atoi(e) : 0;
  }
  int cfg = g_h3_cfg;
  if (cfg < 1 || cfg > 4) {
    const int64_t tn = (a.N + 127) / 128;
    auto fits = [&](int bm) { return (int64_t)((a.M + bm - 1) / bm) * tn <= 256; };
    cfg = fits(64) ? 4 : fits(128) ? 3 : fits(192) ? 2 : 1;
  }
  if (cfg == 2) {
    launch_h3<2, 4, 3, 1, 5>(a, s, g_blk_variant);
    return;
  }
  if (cfg == 3) {
    launch_h3<2, 4, 2, 1, 6>(a, s, g_blk_variant);
    return;
  }
  if (cfg == 4) {
    launch_h3<2, 4, 1, 1, 5>(a, s, g_blk_variant);
    return;
  }
  switch (g_h3_ns) {
    case 3: launch_h3<2, 4, 5, 1, 3>(a, s, g_blk_variant); break;
    case 4: launch_h3<2, 4, 5, 1, 4>(a, s, g_blk_variant); break;
    default: launch_h3<2, 4, 5, 1, 5>(a, s, g_blk_variant); break;
  }
}

int evx_gemm_blk_tile_m() { return 320; }
int evx_gemm_h3_tiles_n(int N) { return (N + 127) / 128; }
int evx_gemm_blk_tile_n() { return 128; }

void evx_gemm_blk(const EvxGemmBlk& a, hipStream_t s) {
  if (a.M <= 0 || a.N <= 0) return;
  launch_cfg<4, 2, 5, 4, 3>(a, s);
}
