// LDS-staged bf16x6 GEMM for the eigensolver's square products (1000 × 1000 × 1000:
// Bᵀ C, W B, X Xᵀ, X² Xᵀ, X² Pᵀ, Bq Vᵀ, Tᵀ T, T G) — the same interface and epilogue as
// gemm_ks (EvxGemmKs: α / *α, bias, β·Cin, device-selected A2 / α2 / C2, skip word,
// symmetric / skew-symmetric upper-tile mode with the mirrored write and the stats partials).
//
// STATUS: opt-in experiment, off by default (measurements below, at evx_gemm_sq_shape).
//
// Why a second kernel for these shapes.  gemm_ks loads every operand fragment straight into
// registers three 16-k groups ahead and splits it there; at 1000³ its 256 workgroups hold one
// wave per SIMD with ≈200 VGPRs, and the MFMA pipe idles behind the loads (≈24 µs per product
// in the flagship's kernel trace against ≈5 µs of bf16x6 MFMA work per CU).  Here:
//
//   * 64 × 64 output tile per workgroup, four waves, each one 32 × 32 v_mfma_f32_32x32x16_bf16
//     block; the six bf16x6 products of a 16-k stage go to two accumulators (the three
//     small-term products and the three large ones: two independent MFMA chains);
//   * operands move global → LDS by LDS-DMA (global_load_lds, 16 B per lane) NS stages ahead —
//     no VGPRs held by in-flight loads, so the prefetch depth is set by LDS (8 KB per stage),
//     not by the register file;
//   * each wave reads its fragments from LDS (ds_read_b128 for k-contiguous operands, on a
//     row-swizzled image that is conflict-free for the MFMA lane map; ds_read_b32 columns for
//     row-contiguous ones) and splits them into bf16 h / m / l in registers (exact, as gemm_ks);
//   * the epilogue is gemm_ks's: the tile goes through LDS once, then bias / β·Cin / the
//     (skew-)symmetric diagonal tile and mirror / stats partials.
//
// Requirements (checked by evx_gemm_sq_ok): M, N, K, the leading dimensions and the element
// offsets of every operand multiples of 4 floats, 16-byte aligned pointers, no fused shift /
// row terms / pre-split planes.  The launcher in gemm_ks.hip routes qualifying products here.
#include "evoxmi_common.h"
#include "evoxmi_launchers.h"
#include <float.h>

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int kBM = 64, kBN = 64;  // output tile
constexpr int kStageK = 16;
constexpr int kOpBytes = 64 * kStageK * 4;        // one operand's stage image: 4 KB
constexpr int kStageBytes = 2 * kOpBytes;         // A and B: 8 KB = 8 one-KiB wave copies
constexpr int kNW = 4;                            // waves
constexpr int kPiecesPerWave = kStageBytes / 1024 / kNW;  // 2
constexpr int kP = kBN + 16;                      // epilogue LDS pitch ≡ 16 (mod 32)

__device__ __forceinline__ void glds16(const void* src, void* dst) {
  typedef const __attribute__((address_space(1))) void* gptr_t;
  typedef __attribute__((address_space(3))) void* lptr_t;
  __builtin_amdgcn_global_load_lds((gptr_t)src, (lptr_t)dst, 16, 0, 0);
}

constexpr int waitcnt_vm_lgkm0(int n) { return (n & 15) | ((n >> 4) << 14) | (7 << 4); }

// eight f32 (k order) → bf16 h / m / l with a = h + m + l exactly (round-to-nearest parts)
__device__ __forceinline__ void split3_8(const float (&v)[8], bf16x8& h, bf16x8& m, bf16x8& l) {
  u32x4 H, M, L;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
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
  h = __builtin_bit_cast(bf16x8, H);
  m = __builtin_bit_cast(bf16x8, M);
  l = __builtin_bit_cast(bf16x8, L);
}

// (tm, tn) of workgroup bid: full grid in groups of 4 tile rows; triangle (tm ≤ tn) row-major
// over 4 × 4 super-tiles (the gemm_ks order: consecutive ids share operand panels in one XCD)
template <int MODE>
__device__ __forceinline__ void sq_tile(int bid, int tiles_m, int tiles_n, int& tm, int& tn) {
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
  const int T = tiles_m, S = (T + G - 1) / G;
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

// Operand stage image in LDS (4 KB):
//   KC (element (row, k) at p[row·ld + k]): [64 rows][4 chunks of 4 k], chunk c of row r at slot
//     c ^ ((r >> 2) & 3) — the MFMA fragment reads (lane row r, chunks 2h, 2h + 1) are then
//     conflict-free ds_read_b128;
//   RC (element (row, k) at p[k·ld + row]): [16 k][64 rows] (k-rows of 256 B).
// One-KiB wave copy `piece` (0..3) of the operand: lane l moves 16 B.
template <bool KC>
__device__ __forceinline__ const float* piece_src(const float* __restrict__ base, int64_t ld, int row0, int nrows, int k0, int K,
                                                  int piece, int lane) {
  if (KC) {
    const int row = 16 * piece + (lane >> 2);
    const int slot = lane & 3, chunk = slot ^ ((row >> 2) & 3);
    const int grow = min(row0 + row, nrows - 1);  // rows past the edge: a valid row, never stored
    const int k = k0 + 4 * chunk;
    return base + (int64_t)grow * ld + (k < K ? k : 0);  // k past K: a valid address, zeroed at use
  }
  const int kr = 4 * piece + (lane >> 4);
  const int k = min(k0 + kr, K - 1);
  const int col = min(row0 + 4 * (lane & 15), nrows - 4);  // nrows % 4 == 0
  return base + (int64_t)k * ld + col;
}

// lane (r, h) of a 32-row block starting at row rb: k = 8h … 8h + 7 of its row from the stage image
template <bool KC>
__device__ __forceinline__ void read_frag(const unsigned char* img, int rb, int r, int h, float (&v)[8]) {
  const int row = rb + r;
  if (KC) {
    const int sw = (row >> 2) & 3;
    const float4 x = *reinterpret_cast<const float4*>(img + row * 64 + ((2 * h) ^ sw) * 16);
    const float4 y = *reinterpret_cast<const float4*>(img + row * 64 + ((2 * h + 1) ^ sw) * 16);
    v[0] = x.x; v[1] = x.y; v[2] = x.z; v[3] = x.w;
    v[4] = y.x; v[5] = y.y; v[6] = y.z; v[7] = y.w;
  } else {
    const float* f = reinterpret_cast<const float*>(img);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = f[(8 * h + j) * 64 + row];
  }
}

template <bool AKC, bool BKC, int MODE, int NS>
__global__ void __launch_bounds__(64 * kNW) gemm_sq_kernel(EvxGemmKs p) {
  static_assert(kPiecesPerWave * (NS - 2) <= 63, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) unsigned char lds[NS * kStageBytes];
  __shared__ __attribute__((aligned(16))) float red[kBM * kP];
  if (p.skip && *p.skip) return;
  if (p.sel && *p.sel) {
    if (p.A2) p.A = p.A2;
    p.alpha = p.alpha2;
    if (p.C2) p.C = p.C2;
  }
  int tm, tn;
  sq_tile<MODE>(evx::xcd_remap(blockIdx.x, gridDim.x), p.tiles_m, p.tiles_n, tm, tn);
  const int m0 = tm * kBM, n0 = tn * kBN;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w >> 1, wn = w & 1;
  const int r = lane & 31, h = lane >> 5;
  const int K = p.K, KB = (K + kStageK - 1) / kStageK;

  // the wave's two copies of a stage: piece w of A, piece w of B
  auto issue = [&](int kb, int buf) {
    unsigned char* dst = lds + buf * kStageBytes;
    const int k0 = kb * kStageK;
    glds16(piece_src<AKC>(p.A, p.lda, m0, p.M, k0, K, w, lane), dst + w * 1024);
    glds16(piece_src<BKC>(p.B, p.ldb, n0, p.N, k0, K, w, lane), dst + kOpBytes + w * 1024);
  };
  auto sync_stage = [&](int t) {
    // stage t landed (this wave's copies; later stages' stay in flight) and this wave's reads
    // of the buffer refilled next are done — then every wave's, at the barrier
    const int after = min(NS - 2, KB - 1 - t);
    switch (after) {
      case 0: __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(0)); break;
      case 1: __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(kPiecesPerWave)); break;
      case 2: __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(2 * kPiecesPerWave)); break;
      case 3: __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(3 * kPiecesPerWave)); break;
      case 4: __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(4 * kPiecesPerWave)); break;
      default: __builtin_amdgcn_s_waitcnt(waitcnt_vm_lgkm0(5 * kPiecesPerWave)); break;
    }
    asm volatile("s_barrier" ::: "memory");
  };
  static_assert(NS - 2 <= 5, "sync_stage waits cover NS ≤ 7");

  struct Frag {
    float a[8], b[8];
  };
  auto load_frag = [&](Frag& f, int buf, int t) {
    const unsigned char* img = lds + buf * kStageBytes;
    read_frag<AKC>(img, wm * 32, r, h, f.a);
    read_frag<BKC>(img + kOpBytes, wn * 32, r, h, f.b);
    const int kl = K - (t * kStageK + 8 * h);  // valid k of this lane's 8 (tail stage only)
    if (kl < 8) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (j >= kl) {
          f.a[j] = 0.f;
          f.b[j] = 0.f;
        }
    }
  };
  f32x16 acc_b, acc_s;
#pragma unroll
  for (int e = 0; e < 16; ++e) acc_b[e] = acc_s[e] = 0.f;
  auto mfma_frag = [&](const Frag& f) {
    bf16x8 ah, am, al, bh, bm, bl;
    split3_8(f.a, ah, am, al);
    split3_8(f.b, bh, bm, bl);
    // two chains: the three small-term products and the three large ones
    acc_s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, bh, acc_s, 0, 0, 0);
    acc_b = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bh, acc_b, 0, 0, 0);
    acc_s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bl, acc_s, 0, 0, 0);
    acc_b = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bm, acc_b, 0, 0, 0);
    acc_s = __builtin_amdgcn_mfma_f32_32x32x16_bf16(am, bm, acc_s, 0, 0, 0);
    acc_b = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, bh, acc_b, 0, 0, 0);
  };

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < KB) issue(s, s);
  Frag fr[2];
  int cur = 0, nxt = NS - 1;
  sync_stage(0);
  if (NS - 1 < KB) issue(NS - 1, nxt);
  load_frag(fr[0], cur, 0);
  cur = cur + 1 == NS ? 0 : cur + 1;
  nxt = nxt + 1 == NS ? 0 : nxt + 1;
  int t = 1;
  for (; t + 1 < KB; t += 2) {  // two stages per trip: the fragment sets swap roles statically
    sync_stage(t);
    if (t + NS - 1 < KB) issue(t + NS - 1, nxt);
    load_frag(fr[1], cur, t);
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(fr[0]);
    __builtin_amdgcn_sched_barrier(0);
    cur = cur + 1 == NS ? 0 : cur + 1;
    nxt = nxt + 1 == NS ? 0 : nxt + 1;
    sync_stage(t + 1);
    if (t + NS < KB) issue(t + NS, nxt);
    load_frag(fr[0], cur, t + 1);
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(fr[1]);
    __builtin_amdgcn_sched_barrier(0);
    cur = cur + 1 == NS ? 0 : cur + 1;
    nxt = nxt + 1 == NS ? 0 : nxt + 1;
  }
  if (t < KB) {
    sync_stage(t);
    load_frag(fr[1], cur, t);
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(fr[0]);
    __builtin_amdgcn_sched_barrier(0);
    mfma_frag(fr[1]);
  } else {
    mfma_frag(fr[0]);
  }

  // ---- epilogue (gemm_ks's, one partial tile): 32x32 map col = lane & 31,
  // row = (e & 3) + 8·(e >> 2) + 4·(lane >> 5)
#pragma unroll
  for (int e = 0; e < 16; ++e) {
    const int row = wm * 32 + (e & 3) + 8 * (e >> 2) + 4 * h;
    red[row * kP + wn * 32 + r] = acc_s[e] + acc_b[e];
  }
  __syncthreads();
  const float sc = p.alpha * (p.alpha_ptr ? p.alpha_ptr[0] : 1.f);
  double st_off = 0.0, st_dg = 0.0;
  float st_mn = FLT_MAX, st_mx = -FLT_MAX;
  constexpr int NV4 = kBM * kBN / 4;
  constexpr int PER = NV4 / (64 * kNW);
  float4 out[PER];
#pragma unroll
  for (int v = 0; v < PER; ++v) {
    const int e = threadIdx.x + 64 * kNW * v;
    const int row = e / (kBN / 4), c = (e % (kBN / 4)) * 4;
    float4 tt = *reinterpret_cast<const float4*>(&red[row * kP + c]);
    tt.x *= sc;
    tt.y *= sc;
    tt.z *= sc;
    tt.w *= sc;
    const int gr = m0 + row, gc = n0 + c;  // N % 4 == 0: the float4 is wholly in or out
    if (p.bias_n && gc < p.N) {
      const float4 bb = *reinterpret_cast<const float4*>(p.bias_n + gc);
      tt.x += bb.x;
      tt.y += bb.y;
      tt.z += bb.z;
      tt.w += bb.w;
    }
    if (gr < p.M && gc < p.N) {
      float* crow = p.C + (int64_t)gr * p.ldc;
      if (p.Cin) {
        const float4 ci = *reinterpret_cast<const float4*>(p.Cin + (int64_t)gr * p.ldcin + gc);
        tt.x += p.beta * ci.x;
        tt.y += p.beta * ci.y;
        tt.z += p.beta * ci.z;
        tt.w += p.beta * ci.w;
      }
      if (MODE != 0 && tm == tn) {
        // diagonal tile: only the upper triangle here (the mirror writes the lower one from it)
        const float vv[4] = {tt.x, tt.y, tt.z, tt.w};
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          const int cc = c + e2;
          if (row <= cc) crow[gc + e2] = (MODE == 2 && row == cc) ? 0.f : vv[e2];
        }
      } else {
        *reinterpret_cast<float4*>(crow + gc) = tt;
      }
      if (MODE == 1 && p.stat_part && (!p.stat_diag_only || tm == tn)) {
        const float vv[4] = {tt.x, tt.y, tt.z, tt.w};
#pragma unroll
        for (int e2 = 0; e2 < 4; ++e2) {
          const int cc = c + e2;
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
    out[v] = tt;
  }
  if (MODE == 1 && p.stat_part) {
    st_off = evx::wave_sum_d(st_off);
    st_dg = evx::wave_sum_d(st_dg);
    st_mn = evx::wave_min(st_mn);
    st_mx = evx::wave_max(st_mx);
    __shared__ double s_st[kNW][4];
    if (lane == 0) {
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
  // mirrored tile C[n0 + c][m0 + r] = ±v(r, c): consecutive threads on consecutive r
  __syncthreads();
#pragma unroll
  for (int v = 0; v < PER; ++v) {
    const int e = threadIdx.x + 64 * kNW * v;
    const int row = e / (kBN / 4), c = (e % (kBN / 4)) * 4;
    *reinterpret_cast<float4*>(&red[row * kP + c]) = out[v];
  }
  __syncthreads();
  const float sgn = MODE == 2 ? -1.f : 1.f;
  const bool diag = tm == tn;
  for (int e = threadIdx.x; e < kBM * kBN; e += 64 * kNW) {
    const int rr = e % kBM, cc = e / kBM;
    const int gr = n0 + cc, gc = m0 + rr;
    if (gr < p.N && gc < p.M && (!diag || rr < cc)) p.C[(int64_t)gr * p.ldc + gc] = sgn * red[rr * kP + cc];
  }
}

constexpr int kSqNS = 7;

template <int MODE>
void launch_sq(EvxGemmKs a, hipStream_t s) {
  a.tiles_m = (a.M + kBM - 1) / kBM;
  a.tiles_n = (a.N + kBN - 1) / kBN;
  const int tiles = MODE == 0 ? a.tiles_m * a.tiles_n : a.tiles_m * (a.tiles_m + 1) / 2;
  const dim3 grid(tiles), block(64 * kNW);
  if (a.a_kc && a.b_kc) gemm_sq_kernel<true, true, MODE, kSqNS><<<grid, block, 0, s>>>(a);
  else if (a.a_kc) gemm_sq_kernel<true, false, MODE, kSqNS><<<grid, block, 0, s>>>(a);
  else if (a.b_kc) gemm_sq_kernel<false, true, MODE, kSqNS><<<grid, block, 0, s>>>(a);
  else gemm_sq_kernel<false, false, MODE, kSqNS><<<grid, block, 0, s>>>(a);
}

bool al16(const void* q) { return q == nullptr || reinterpret_cast<uintptr_t>(q) % 16 == 0; }

}  // namespace

// Opt-in (EVOXMI_GEMM_SQ=1 or evx_gemm_sq_enable): measured SLOWER than gemm_ks on MI355X —
// 1000³ NT 41.5 vs 24.4 µs, TN 52.1 vs 22.4, the 1000 × 1000 × 5000 rank-μ product 166.5 vs
// 67.3 (profiles/r5_gemm_sq_ab.log).  Each 8 KB stage takes ≈0.65 µs: the LDS-DMA round trip
// under load (≈4 µs, the same as gemm_h3's 28 KB stages) over the 6 stages in flight — with
// 64 × 64 tiles the bytes in flight per CU are bounded by LDS, where gemm_ks's register-direct
// loads keep as many in the larger register file.  It also accumulates each output over the
// whole K in one chain (gemm_ks: four K-quarters), so long same-sign sums (a Gram diagonal over
// K = 5000) lose more to rounding: K is capped at 2048 here.
int g_sq_enabled = -1;

void evx_gemm_sq_enable(int on) { g_sq_enabled = on ? 1 : 0; }

bool evx_gemm_sq_shape(int M, int N, int mode) {
  if (g_sq_enabled < 0) {
    const char* e = getenv("EVOXMI_GEMM_SQ");
    g_sq_enabled = e ? atoi(e) : 0;
  }
  return g_sq_enabled && M % 4 == 0 && N % 4 == 0 && M >= 64 && N >= 64 && M <= 4096 && N <= 4096 && (mode == 0 || M == N);
}

int evx_gemm_sq_grid(int M, int N, int mode) {
  const int tm = (M + kBM - 1) / kBM, tn = (N + kBN - 1) / kBN;
  return mode == 0 ? tm * tn : tm * (tm + 1) / 2;
}

bool evx_gemm_sq_ok(const EvxGemmKs& a) {
  if (!evx_gemm_sq_shape(a.M, a.N, a.mode)) return false;
  if (a.K % 4 || a.K < 1 || a.K > 2048 || a.lda % 4 || a.ldb % 4 || a.ldc % 4 || (a.Cin && a.ldcin % 4)) return false;
  if (a.a_sub_k || a.row_terms || a.a_pl || a.b_pl || a.sub_cols) return false;
  return al16(a.A) && al16(a.A2) && al16(a.B) && al16(a.C) && al16(a.C2) && al16(a.Cin) && al16(a.bias_n);
}

void evx_gemm_sq(const EvxGemmKs& a, hipStream_t s) {
  switch (a.mode) {
    case 1: launch_sq<1>(a, s); break;
    case 2: launch_sq<2>(a, s); break;
    default: launch_sq<0>(a, s); break;
  }
}
