// f32 GEMM on CDNA4 matrix cores: v_mfma_f32_32x32x2_f32 (exact f32 fmaf chains).
//
//   C[M,N] = alpha * (*alpha_ptr) * Σ_k Ã[m,k] B̃[k,n] + bias_n[n] + beta * Cin[m,n]
//
// with fused operand prologues (K2/K3/K6 of SURVEY §2.10):
//   Ã[m,k] = (A[m,k] − a_sub[m|k]) * a_kscale[k] * a_kw[k]         (A may be row-gathered)
// Layout template parameters per operand:
//   KC = "K contiguous"  : element (r, k) at ptr[r*ld + k]       (row-major M×K / N×K)
//   RC = "row contiguous": element (r, k) at ptr[k*ld + r]       (row-major K×M / K×N)
//        RC operands may be K-row gathered: row k is taken from ptr[idx[k]*ld + r]
// Split-K: gridDim.z slices of K; slice z writes C + z*M*N (partial slabs, no atomics,
// deterministic — replicas on different ranks stay bit-identical).
//
// Tile 128x128x16, 256 threads = 4 waves in 2x2, each wave 64x64 = 2x2 MFMA 32x32 tiles
// (64 accumulator registers).  Operands are staged global → registers → LDS (k-major,
// row stride 132 floats to spread banks), double-buffered so the next K-tile's global
// loads are in flight during the current tile's 32 MFMAs per wave.  Block ids are
// remapped so consecutive tiles (sharing A/B panels) run on the same XCD's L2.
#include "evoxmi_common.h"
#include "evoxmi_launchers.h"

typedef float f32x16 __attribute__((ext_vector_type(16)));

namespace {

struct OperandDesc {
  const float* ptr;
  int64_t ld;
  const int32_t* gather;  // RC only: k -> source row
  const float* sub;       // subtracted vector (index space: sub_on_k ? k : r), may be null
  int sub_on_k;
  const float* kscale;    // per-k multiplier, may be null
  const float* kw;        // second per-k multiplier (weights), may be null
  const float* sscale;    // device scalar multiplier (e.g. 1/sigma), may be null
  int sscale_inv;         // 1: multiply by 1/(*sscale)
};

// K order inside a BK=32 tile: MFMA step s (0..15), lane half h → k = 16h + s.  Any
// permutation of k is valid as long as both operands use it; this one lets a lane read
// its 16 k-values of a K-contiguous row with 4 ds_read_b128.
// A TR-row × BK-k tile, staged through NV float4 registers per thread (256 threads).
//   KC: LDS [TR][32 + 4] (row stride 144 B: ds_read_b128 lane groups conflict-free)
//   RC: LDS [32][TR + 4]
template <bool RC, int TR, int BK>
struct Tile {
  static constexpr int HK = BK / 2;  // k-values per lane half
  static constexpr int NV = TR * BK / 1024;
  static constexpr int LDS_FLOATS = RC ? BK * (TR + 4) : TR * (BK + 4);
  float4 reg[NV];
  float4 pro[NV];  // prefetched per-k / per-r prologue factors

  __device__ __forceinline__ static void coords(int v, int& rl, int& kl) {
    const int t = threadIdx.x + 256 * v;
    if (!RC) { rl = t / (BK / 4); kl = (t % (BK / 4)) * 4; }  // float4 along k
    else { kl = t / (TR / 4); rl = (t % (TR / 4)) * 4; }      // float4 along r
  }

  template <bool PRO>
  __device__ __forceinline__ void load(const OperandDesc& d, int R, int K, int r0, int k0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int rl, kl;
      coords(v, rl, kl);
      const int r = r0 + rl, k = k0 + kl;
      float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
      if (!RC) {
        if (r < R) {
          const float* p = d.ptr + (int64_t)r * d.ld + k;
          if (k + 3 < K && ((((uintptr_t)p) & 15) == 0)) q = *reinterpret_cast<const float4*>(p);
          else {
            if (k < K) q.x = p[0];
            if (k + 1 < K) q.y = p[1];
            if (k + 2 < K) q.z = p[2];
            if (k + 3 < K) q.w = p[3];
          }
        }
        if (PRO) {  // per-k factors (kscale·kw) and per-k/r shift for this float4
          float4 f = make_float4(1.f, 1.f, 1.f, 1.f);
          if (d.kscale || d.kw) {
            float ff[4];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float x = 1.f;
              if (k + j < K) {
                if (d.kscale) x *= d.kscale[k + j];
                if (d.kw) x *= d.kw[k + j];
              }
              ff[j] = x;
            }
            f = make_float4(ff[0], ff[1], ff[2], ff[3]);
          }
          pro[v] = f;
        }
      } else {
        if (k < K) {
          const int64_t src = d.gather ? (int64_t)d.gather[k] : (int64_t)k;
          const float* p = d.ptr + src * d.ld + r;
          if (r + 3 < R && ((((uintptr_t)p) & 15) == 0)) q = *reinterpret_cast<const float4*>(p);
          else {
            if (r < R) q.x = p[0];
            if (r + 1 < R) q.y = p[1];
            if (r + 2 < R) q.z = p[2];
            if (r + 3 < R) q.w = p[3];
          }
        }
        if (PRO) {
          float x = 1.f;
          if (k < K) {
            if (d.kscale) x *= d.kscale[k];
            if (d.kw) x *= d.kw[k];
          }
          pro[v] = make_float4(x, x, x, x);
        }
      }
      reg[v] = q;
    }
  }

  // sub vector over r for RC operands is constant across K: loaded once
  template <bool PRO>
  __device__ __forceinline__ void store(const OperandDesc& d, int R, int K, int r0, int k0, float* lds, float sscale,
                                        const float4* rsub) const {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      int rl, kl;
      coords(v, rl, kl);
      float4 q = reg[v];
      if (PRO) {
        float x[4] = {q.x, q.y, q.z, q.w};
        const float f[4] = {pro[v].x, pro[v].y, pro[v].z, pro[v].w};
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = r0 + rl + (RC ? j : 0), k = k0 + kl + (RC ? 0 : j);
          float val = x[j];
          if (d.sub) {
            if (RC) val -= (&rsub[v].x)[j];
            else val -= d.sub_on_k ? (k < K ? d.sub[k] : 0.f) : (r < R ? d.sub[r] : 0.f);
          }
          val *= f[j] * sscale;
          x[j] = (r < R && k < K) ? val : 0.f;
        }
        q = make_float4(x[0], x[1], x[2], x[3]);
      }
      if (!RC) *reinterpret_cast<float4*>(&lds[rl * (BK + 4) + kl]) = q;
      else *reinterpret_cast<float4*>(&lds[kl * (TR + 4) + rl]) = q;
    }
  }

  // operand values for MFMA steps 4q..4q+3 of row `row` (lane half h): k = HK·h + step
  __device__ __forceinline__ static float4 frag(const float* lds, int row, int h, int q) {
    if (!RC) return *reinterpret_cast<const float4*>(&lds[row * (BK + 4) + HK * h + 4 * q]);
    const int k = HK * h + 4 * q;
    return make_float4(lds[k * (TR + 4) + row], lds[(k + 1) * (TR + 4) + row], lds[(k + 2) * (TR + 4) + row],
                       lds[(k + 3) * (TR + 4) + row]);
  }
};

template <bool A_RC, bool B_RC, int BM, int BN, int BK, bool PRO>
__global__ void __launch_bounds__(256, 2) gemm_f32_kernel(OperandDesc Ad, OperandDesc Bd, float* __restrict__ C, int64_t ldc,
                                                          int M, int N, int K, int k_per_split, float alpha,
                                                          const float* __restrict__ alpha_ptr,
                                                          const float* __restrict__ bias_n, float beta,
                                                          const float* __restrict__ Cin, int64_t ldcin) {
  constexpr int WGM = BM >= BN ? 2 : 1;
  constexpr int WGN = 4 / WGM;
  constexpr int WM = BM / WGM, WN = BN / WGN;
  constexpr int TM = WM / 32, TN = WN / 32;
  using TA = Tile<A_RC, BM, BK>;
  using TB = Tile<B_RC, BN, BK>;
  // BK = 32: double-buffered LDS (one barrier per K-tile);  BK = 64: single LDS buffer
  // with register prefetch (two barriers per K-tile, twice the MFMA work between the
  // global-load issue and its use — covers L2/MALL latency at 2 workgroups per CU).
  constexpr int NBUF = BK == 32 ? 2 : 1;
  __shared__ __attribute__((aligned(16))) float As[NBUF][TA::LDS_FLOATS];
  __shared__ __attribute__((aligned(16))) float Bs[NBUF][TB::LDS_FLOATS];

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nt = tiles_m * tiles_n;
  const int bid = evx::xcd_remap(blockIdx.x, nt);
  // N-fastest order: the tiles one XCD receives (consecutive ids after the remap) share
  // A row panels, so each XCD streams ~1/8 of A and the (small) B panel set once.
  const int tm = bid / tiles_n, tn = bid % tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kz0 = blockIdx.z * k_per_split;
  const int kz1 = min(K, kz0 + k_per_split);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid / WGN) * WM, wn = (wid % WGN) * WN;
  const int h = lane >> 5, c = lane & 31;

  float as = 1.f, bs = 1.f;
  float4 asub[TA::NV], bsub[TB::NV];
  if (PRO) {
    if (Ad.sscale) as = Ad.sscale_inv ? 1.f / Ad.sscale[0] : Ad.sscale[0];
    if (Bd.sscale) bs = Bd.sscale_inv ? 1.f / Bd.sscale[0] : Bd.sscale[0];
    // r-indexed shift vectors of RC operands are K-invariant: load once
#pragma unroll
    for (int v = 0; v < TA::NV; ++v) {
      int rl, kl;
      TA::coords(v, rl, kl);
      float x[4] = {0.f, 0.f, 0.f, 0.f};
      if (A_RC && Ad.sub && !Ad.sub_on_k)
        for (int j = 0; j < 4; ++j) x[j] = (m0 + rl + j < M) ? Ad.sub[m0 + rl + j] : 0.f;
      asub[v] = make_float4(x[0], x[1], x[2], x[3]);
    }
#pragma unroll
    for (int v = 0; v < TB::NV; ++v) {
      int rl, kl;
      TB::coords(v, rl, kl);
      float x[4] = {0.f, 0.f, 0.f, 0.f};
      if (B_RC && Bd.sub && !Bd.sub_on_k)
        for (int j = 0; j < 4; ++j) x[j] = (n0 + rl + j < N) ? Bd.sub[n0 + rl + j] : 0.f;
      bsub[v] = make_float4(x[0], x[1], x[2], x[3]);
    }
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  TA ta;
  TB tb;
  int buf = 0;
  if (kz0 < kz1) {
    ta.template load<PRO>(Ad, M, kz1, m0, kz0);
    tb.template load<PRO>(Bd, N, kz1, n0, kz0);
    ta.template store<PRO>(Ad, M, kz1, m0, kz0, As[0], as, asub);
    tb.template store<PRO>(Bd, N, kz1, n0, kz0, Bs[0], bs, bsub);
  }
  __syncthreads();

  for (int k0 = kz0; k0 < kz1; k0 += BK) {
    const bool more = (k0 + BK) < kz1;
    if (more) {
      ta.template load<PRO>(Ad, M, kz1, m0, k0 + BK);
      tb.template load<PRO>(Bd, N, kz1, n0, k0 + BK);
    }
    const float* as_ = As[buf];
    const float* bs_ = Bs[buf];
#pragma unroll
    for (int q = 0; q < BK / 8; ++q) {
      float4 a[TM], b[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) a[i] = TA::frag(as_, wm + 32 * i + c, h, q);
#pragma unroll
      for (int j = 0; j < TN; ++j) b[j] = TB::frag(bs_, wn + 32 * j + c, h, q);
#pragma unroll
      for (int e = 0; e < 4; ++e)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32((&a[i].x)[e], (&b[j].x)[e], acc[i][j], 0, 0, 0);
    }
    if (NBUF == 2) {
      if (more) {
        ta.template store<PRO>(Ad, M, kz1, m0, k0 + BK, As[buf ^ 1], as, asub);
        tb.template store<PRO>(Bd, N, kz1, n0, k0 + BK, Bs[buf ^ 1], bs, bsub);
      }
      __syncthreads();
      buf ^= 1;
    } else {
      __syncthreads();
      if (more) {
        ta.template store<PRO>(Ad, M, kz1, m0, k0 + BK, As[0], as, asub);
        tb.template store<PRO>(Bd, N, kz1, n0, k0 + BK, Bs[0], bs, bsub);
      }
      __syncthreads();
    }
  }

  // epilogue: C/D layout of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const float s = alpha * (alpha_ptr ? alpha_ptr[0] : 1.f);
  float* Cz = C + (int64_t)blockIdx.z * M * ldc;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = n0 + wn + 32 * j + c;
      if (col >= N) continue;
      const float bn = bias_n ? bias_n[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (row < M) {
          float v = s * acc[i][j][r] + bn;
          if (Cin) v += beta * Cin[(int64_t)row * ldcin + col];
          Cz[(int64_t)row * ldc + col] = v;
        }
      }
    }
}

template <bool A_RC, bool B_RC, int BM, int BN, int BK>
void launch_cfg(const OperandDesc& Ad, const OperandDesc& Bd, bool pro, float* C, int64_t ldc, int M, int N, int K, int kps,
                int splits, float alpha, const float* alpha_ptr, const float* bias_n, float beta, const float* Cin,
                int64_t ldcin, hipStream_t s) {
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  dim3 grid(tiles, 1, splits);
  if (pro)
    gemm_f32_kernel<A_RC, B_RC, BM, BN, BK, true><<<grid, 256, 0, s>>>(Ad, Bd, C, ldc, M, N, K, kps, alpha, alpha_ptr, bias_n, beta, Cin, ldcin);
  else
    gemm_f32_kernel<A_RC, B_RC, BM, BN, BK, false><<<grid, 256, 0, s>>>(Ad, Bd, C, ldc, M, N, K, kps, alpha, alpha_ptr, bias_n, beta, Cin, ldcin);
}

int g_cfg_override = -1;

// tile choice: the fewest rounds of (tiles / (2 · 256 CUs)) with the larger tile on ties
template <bool A_RC, bool B_RC>
void launch_layout(const OperandDesc& Ad, const OperandDesc& Bd, bool pro, float* C, int64_t ldc, int M, int N, int K, int kps,
                   int splits, float alpha, const float* alpha_ptr, const float* bias_n, float beta, const float* Cin,
                   int64_t ldcin, hipStream_t s) {
  int cfg = g_cfg_override;
  if (cfg < 0) {
    // measured on MI355X (tools/bench_kernels.py): 64×64 tiles fill the 256 CUs best at
    // the framework's shapes; K-contiguous operands prefer BK = 64 (register prefetch),
    // row-gathered (RC) operands BK = 32 (double-buffered LDS)
    cfg = (A_RC || B_RC) ? 3 : 7;
  }
  switch (cfg) {
    case 4: launch_cfg<A_RC, B_RC, 128, 128, 64>(Ad, Bd, pro, C, ldc, M, N, K, kps, splits, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s); break;
    case 5: launch_cfg<A_RC, B_RC, 64, 128, 64>(Ad, Bd, pro, C, ldc, M, N, K, kps, splits, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s); break;
    case 6: launch_cfg<A_RC, B_RC, 128, 64, 64>(Ad, Bd, pro, C, ldc, M, N, K, kps, splits, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s); break;
    case 7: launch_cfg<A_RC, B_RC, 64, 64, 64>(Ad, Bd, pro, C, ldc, M, N, K, kps, splits, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s); break;
    case 0: launch_cfg<A_RC, B_RC, 128, 128, 32>(Ad, Bd, pro, C, ldc, M, N, K, kps, splits, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s); break;
    case 1: launch_cfg<A_RC, B_RC, 64, 128, 32>(Ad, Bd, pro, C, ldc, M, N, K, kps, splits, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s); break;
    case 2: launch_cfg<A_RC, B_RC, 128, 64, 32>(Ad, Bd, pro, C, ldc, M, N, K, kps, splits, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s); break;
    default: launch_cfg<A_RC, B_RC, 64, 64, 32>(Ad, Bd, pro, C, ldc, M, N, K, kps, splits, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s); break;
  }
}

}  // namespace

void evx_gemm_set_config(int cfg) { g_cfg_override = cfg; }

void evx_gemm_f32(EvxOperand a, EvxOperand b, float* C, int64_t ldc, int M, int N, int K, int splits, float alpha,
                  const float* alpha_ptr, const float* bias_n, float beta, const float* Cin, int64_t ldcin, hipStream_t s) {
  OperandDesc Ad{a.ptr, a.ld, a.gather, a.sub, a.sub_on_k, a.kscale, a.kw, a.sscale, a.sscale_inv};
  OperandDesc Bd{b.ptr, b.ld, b.gather, b.sub, b.sub_on_k, b.kscale, b.kw, b.sscale, b.sscale_inv};
  const bool pro = a.sub || a.kscale || a.kw || a.sscale || b.sub || b.kscale || b.kw || b.sscale;
  const int sp = evx_gemm_splits_used(K, splits);
  int kps = (K + sp - 1) / sp;
  kps = (kps + 63) / 64 * 64;
  if (!a.rc && !b.rc) launch_layout<false, false>(Ad, Bd, pro, C, ldc, M, N, K, kps, sp, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s);
  else if (!a.rc && b.rc) launch_layout<false, true>(Ad, Bd, pro, C, ldc, M, N, K, kps, sp, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s);
  else if (a.rc && !b.rc) launch_layout<true, false>(Ad, Bd, pro, C, ldc, M, N, K, kps, sp, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s);
  else launch_layout<true, true>(Ad, Bd, pro, C, ldc, M, N, K, kps, sp, alpha, alpha_ptr, bias_n, beta, Cin, ldcin, s);
}

int evx_gemm_splits_used(int K, int splits) {
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = (kps + 63) / 64 * 64;
  int sp = (K + kps - 1) / kps;
  return sp < 1 ? 1 : sp;
}
