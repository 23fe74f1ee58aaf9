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

constexpr int BM = 128, BN = 128, BK = 16, LDS_STRIDE = BM + 4;

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

template <bool RC>
__device__ __forceinline__ void load_tile(const OperandDesc& d, int R, int K, int r0, int k0, float (&reg)[8]) {
  const int t = threadIdx.x;
  if (!RC) {
    // 128 rows x 16 k: thread -> (row = t>>2 (+64), kq = t&3) float4 along k
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int r = r0 + (t >> 2) + 64 * h;
      int k = k0 + (t & 3) * 4;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (r < R) {
        const float* p = d.ptr + (int64_t)r * d.ld + k;
        if (k + 3 < K && ((((uintptr_t)p) & 15) == 0)) {
          float4 q = *reinterpret_cast<const float4*>(p);
          v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) if (k + j < K) v[j] = p[j];
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) reg[4 * h + j] = v[j];
    }
  } else {
    // 16 k-rows x 128 r: thread -> (k = t>>5 (+8), rq = t&31) float4 along r
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      int k = k0 + (t >> 5) + 8 * h;
      int r = r0 + (t & 31) * 4;
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      if (k < K) {
        int64_t src = d.gather ? (int64_t)d.gather[k] : (int64_t)k;
        const float* p = d.ptr + src * d.ld + r;
        if (r + 3 < R && ((((uintptr_t)p) & 15) == 0)) {
          float4 q = *reinterpret_cast<const float4*>(p);
          v[0] = q.x; v[1] = q.y; v[2] = q.z; v[3] = q.w;
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) if (r + j < R) v[j] = p[j];
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) reg[4 * h + j] = v[j];
    }
  }
}

// apply the prologue transform and store into the k-major LDS tile
template <bool RC>
__device__ __forceinline__ void store_tile(const OperandDesc& d, int R, int K, int r0, int k0, const float (&reg)[8],
                                           float* lds, float sscale) {
  const int t = threadIdx.x;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int rl, kl;
      if (!RC) { rl = (t >> 2) + 64 * h; kl = (t & 3) * 4 + j; }
      else { kl = (t >> 5) + 8 * h; rl = (t & 31) * 4 + j; }
      int r = r0 + rl, k = k0 + kl;
      float v = reg[4 * h + j];
      if (r < R && k < K) {
        if (d.sub) v -= d.sub_on_k ? d.sub[k] : d.sub[r];
        if (d.kscale) v *= d.kscale[k];
        if (d.kw) v *= d.kw[k];
        v *= sscale;
      } else {
        v = 0.f;
      }
      lds[kl * LDS_STRIDE + rl] = v;
    }
  }
}

template <bool A_RC, bool B_RC>
__global__ void __launch_bounds__(256, 2) gemm_f32_kernel(OperandDesc Ad, OperandDesc Bd, float* __restrict__ C, int64_t ldc,
                                                          int M, int N, int K, int k_per_split, float alpha,
                                                          const float* __restrict__ alpha_ptr,
                                                          const float* __restrict__ bias_n, float beta,
                                                          const float* __restrict__ Cin, int64_t ldcin) {
  __shared__ float As[2][BK * LDS_STRIDE];
  __shared__ float Bs[2][BK * LDS_STRIDE];

  const int tiles_m = (M + BM - 1) / BM, tiles_n = (N + BN - 1) / BN;
  const int nt = tiles_m * tiles_n;
  const int bid = evx::xcd_remap(blockIdx.x, nt);
  // column-major tile order: consecutive tiles share the B (N) panel
  const int tm = bid % tiles_m, tn = bid / tiles_m;
  const int m0 = tm * BM, n0 = tn * BN;
  const int kz0 = blockIdx.z * k_per_split;
  const int kz1 = min(K, kz0 + k_per_split);

  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int wm = (wid >> 1) * 64, wn = (wid & 1) * 64;

  float as = 1.f, bs = 1.f;
  if (Ad.sscale) as = Ad.sscale_inv ? 1.f / Ad.sscale[0] : Ad.sscale[0];
  if (Bd.sscale) bs = Bd.sscale_inv ? 1.f / Bd.sscale[0] : Bd.sscale[0];

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  float ra[8], rb[8];
  int buf = 0;
  if (kz0 < kz1) {
    load_tile<A_RC>(Ad, M, kz1, m0, kz0, ra);
    load_tile<B_RC>(Bd, N, kz1, n0, kz0, rb);
    store_tile<A_RC>(Ad, M, kz1, m0, kz0, ra, As[0], as);
    store_tile<B_RC>(Bd, N, kz1, n0, kz0, rb, Bs[0], bs);
  }
  __syncthreads();

  for (int k0 = kz0; k0 < kz1; k0 += BK) {
    const bool more = (k0 + BK) < kz1;
    if (more) {  // issue next tile's global loads before the MFMAs
      load_tile<A_RC>(Ad, M, kz1, m0, k0 + BK, ra);
      load_tile<B_RC>(Bd, N, kz1, n0, k0 + BK, rb);
    }
    const float* as_ = As[buf];
    const float* bs_ = Bs[buf];
#pragma unroll
    for (int kk = 0; kk < BK; kk += 2) {
      const int kr = kk + (lane >> 5);
      float a0 = as_[kr * LDS_STRIDE + wm + (lane & 31)];
      float a1 = as_[kr * LDS_STRIDE + wm + 32 + (lane & 31)];
      float b0 = bs_[kr * LDS_STRIDE + wn + (lane & 31)];
      float b1 = bs_[kr * LDS_STRIDE + wn + 32 + (lane & 31)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (more) {
      store_tile<A_RC>(Ad, M, kz1, m0, k0 + BK, ra, As[buf ^ 1], as);
      store_tile<B_RC>(Bd, N, kz1, n0, k0 + BK, rb, Bs[buf ^ 1], bs);
    }
    __syncthreads();
    buf ^= 1;
  }

  // epilogue: C/D layout of 32x32: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
  const float s = alpha * (alpha_ptr ? alpha_ptr[0] : 1.f);
  float* Cz = C + (int64_t)blockIdx.z * M * ldc;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = n0 + wn + 32 * j + (lane & 31);
      if (col >= N) continue;
      const float bn = bias_n ? bias_n[col] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = m0 + wm + 32 * i + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (row < M) {
          float v = s * acc[i][j][r] + bn;
          if (Cin) v += beta * Cin[(int64_t)row * ldcin + col];
          Cz[(int64_t)row * ldc + col] = v;
        }
      }
    }
}

}  // namespace



void evx_gemm_f32(EvxOperand a, EvxOperand b, float* C, int64_t ldc, int M, int N, int K, int splits, float alpha,
                  const float* alpha_ptr, const float* bias_n, float beta, const float* Cin, int64_t ldcin, hipStream_t s) {
  OperandDesc Ad{a.ptr, a.ld, a.gather, a.sub, a.sub_on_k, a.kscale, a.kw, a.sscale, a.sscale_inv};
  OperandDesc Bd{b.ptr, b.ld, b.gather, b.sub, b.sub_on_k, b.kscale, b.kw, b.sscale, b.sscale_inv};
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  splits = (K + kps - 1) / kps;
  if (splits < 1) splits = 1;
  dim3 grid(tiles, 1, splits);
  if (!a.rc && !b.rc)
    gemm_f32_kernel<false, false><<<grid, 256, 0, s>>>(Ad, Bd, C, ldc, M, N, K, kps, alpha, alpha_ptr, bias_n, beta, Cin, ldcin);
  else if (!a.rc && b.rc)
    gemm_f32_kernel<false, true><<<grid, 256, 0, s>>>(Ad, Bd, C, ldc, M, N, K, kps, alpha, alpha_ptr, bias_n, beta, Cin, ldcin);
  else if (a.rc && !b.rc)
    gemm_f32_kernel<true, false><<<grid, 256, 0, s>>>(Ad, Bd, C, ldc, M, N, K, kps, alpha, alpha_ptr, bias_n, beta, Cin, ldcin);
  else
    gemm_f32_kernel<true, true><<<grid, 256, 0, s>>>(Ad, Bd, C, ldc, M, N, K, kps, alpha, alpha_ptr, bias_n, beta, Cin, ldcin);
}

int evx_gemm_splits_used(int K, int splits) {
  if (splits < 1) splits = 1;
  int kps = (K + splits - 1) / splits;
  kps = (kps + BK - 1) / BK * BK;
  int s = (K + kps - 1) / kps;
  return s < 1 ? 1 : s;
}
