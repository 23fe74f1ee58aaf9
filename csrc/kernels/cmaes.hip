// CMA-ES tell epilogue (K3 of SURVEY §2.10; reference es_variants/cma_es.py:162-198).
//
// After the rank-μ product S and the weighted mean shift dm are formed, the reference
// performs ~40 small vector/matrix ops per generation (mean, evolution paths, hσ, σ,
// covariance blend, symmetrisation, identity padding for the eigensolver, eigenbasis
// extraction).  On MI355X each of those is a ~2–5 µs launch, so they are fused into four
// kernels:
//   1. delta_gemv : δ = (m + c_m·dm) − m,  y = invsqrtC·δ   (one wave per row, float4)
//   2. paths      : p_σ, ‖p_σ‖, hσ, p_c, σ and the covariance blend factor a — one
//                   workgroup, every scalar stays on the device (graph-capturable)
//   3. cov_pad    : C' = a·C + c1·p_c p_cᵀ + cμ·S (written as the new state), the padded
//                   symmetric eigensolver input Cp = sym_upper(C') ⊕ I and the padded
//                   warm start Bp = B_prev ⊕ I, by 32×32 tiles (LDS transpose for the
//                   lower tiles, coalesced reads and writes everywhere)
//   4. eig_out    : B = Bp[:d, :d], D = sqrt(max(w, 1e-30)), B∘D⁻¹ (for invsqrtC = (B/D)Bᵀ)
#include "evoxmi_common.h"

namespace {
using namespace evx;

__global__ void __launch_bounds__(256) delta_gemv_kernel(const float* __restrict__ M, const float* __restrict__ mean,
                                                         const float* __restrict__ dm, float cm, int d, float* __restrict__ mean_out,
                                                         float* __restrict__ delta, float* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= d) return;
  const float* row = M + (int64_t)r * d;
  float acc = 0.f;
  if ((d & 3) == 0) {
    for (int c = lane * 4; c < d; c += 256) {
      const float4 m4 = *reinterpret_cast<const float4*>(row + c);
      const float4 mu = *reinterpret_cast<const float4*>(mean + c);
      const float4 g = *reinterpret_cast<const float4*>(dm + c);
      acc += m4.x * ((mu.x + cm * g.x) - mu.x) + m4.y * ((mu.y + cm * g.y) - mu.y) + m4.z * ((mu.z + cm * g.z) - mu.z) +
             m4.w * ((mu.w + cm * g.w) - mu.w);
    }
  } else {
    for (int c = lane; c < d; c += 64) acc += row[c] * ((mean[c] + cm * dm[c]) - mean[c]);
  }
  acc = wave_sum(acc);
  if (lane == 0) {
    y[r] = acc;
    const float mn = mean[r] + cm * dm[r];
    mean_out[r] = mn;
    delta[r] = mn - mean[r];
  }
}

struct PathConsts {
  float cs, c_ps, cc, c_pc, chiN, damps, c1, cmu, hs_thresh;
};

// scal: [0] sigma (in), outputs: sigma_out, a_out, hsig_out (device scalars)
__global__ void __launch_bounds__(1024) paths_kernel(const float* __restrict__ ps, const float* __restrict__ pc,
                                                     const float* __restrict__ y, const float* __restrict__ delta,
                                                     const float* __restrict__ sigma, const int64_t* __restrict__ count_iter, int d,
                                                     PathConsts k, float* __restrict__ ps_out, float* __restrict__ pc_out,
                                                     float* __restrict__ sigma_out, float* __restrict__ a_out, float* __restrict__ hsig_out,
                                                     const int64_t* __restrict__ count_eigen, int64_t* __restrict__ count_iter_out,
                                                     int64_t* __restrict__ count_eigen_out) {
  __shared__ float scratch[16];
  const float s = sigma[0];
  const float inv_s = 1.f / s;
  float nrm2 = 0.f;
  for (int i = threadIdx.x; i < d; i += blockDim.x) {
    const float v = (1.f - k.cs) * ps[i] + k.c_ps * y[i] * inv_s;
    ps_out[i] = v;
    nrm2 += v * v;
  }
  const float nrm = sqrtf(block_sum(nrm2, scratch));
  // with count_iter_out the generation counters advance here (count_iter + 1 used for this
  // generation, as the reference's ask would have left it; count_eigen + 1): two one-element add
  // launches fewer per captured generation
  const int64_t cnt = count_iter[0] + (count_iter_out ? 1 : 0);
  const float count = (float)cnt;
  const float hs = (nrm / sqrtf(1.f - powf(1.f - k.cs, 2.f * count)) < k.hs_thresh) ? 1.f : 0.f;
  for (int i = threadIdx.x; i < d; i += blockDim.x) pc_out[i] = (1.f - k.cc) * pc[i] + hs * k.c_pc * delta[i] * inv_s;
  if (threadIdx.x == 0) {
    sigma_out[0] = s * expf((k.cs / k.damps) * (nrm / k.chiN - 1.f));
    a_out[0] = (1.f - k.c1 - k.cmu) + k.c1 * (1.f - hs) * k.cc * (2.f - k.cc);
    hsig_out[0] = hs;
    if (count_iter_out) {
      count_iter_out[0] = cnt;
      count_eigen_out[0] = count_eigen[0] + 1;
    }
  }
}

constexpr int TS = 32;

// grid (np/32, np/32), 256 threads: tile (ti, tj); each thread handles 4 rows of the tile.
// Every element of C is read only by the thread that writes its C' (Cn may alias C: the
// captured generation updates the state's covariance in place): a strictly upper tile also
// writes its transpose into Cp's lower tile, so no workgroup reads another tile of C.
// Bp (the padded warm-start basis) is optional: the device eigensolver reads B unpadded.
__global__ void __launch_bounds__(256) cov_pad_kernel(const float* C, const float* __restrict__ S, int64_t lds,
                                                      const float* __restrict__ pc, const float* __restrict__ a_ptr, float c1, float cmu,
                                                      const float* __restrict__ Bprev, int d, int np, float* Cn,
                                                      float* __restrict__ Cp, float* __restrict__ Bp) {
  __shared__ float T[TS][TS + 1];
  const int ti = blockIdx.y, tj = blockIdx.x;
  const int c = threadIdx.x & 31, r0 = threadIdx.x >> 5;  // 8 row groups
  const float a = a_ptr[0];
  // own tile: C' (state), Bp, and the upper / diagonal tiles of Cp
#pragma unroll
  for (int rr = 0; rr < TS; rr += 8) {
    const int i = ti * TS + r0 + rr, j = tj * TS + c;
    float v = (i == j) ? 1.f : 0.f, b = v;
    if (i < d && j < d) {
      v = a * C[(int64_t)i * d + j] + c1 * pc[i] * pc[j] + cmu * S[(int64_t)i * lds + j];
      Cn[(int64_t)i * d + j] = v;
      if (Bp) b = Bprev[(int64_t)i * d + j];
    }
    if (Bp) Bp[(int64_t)i * np + j] = b;
    if (ti < tj) Cp[(int64_t)i * np + j] = v;  // strictly upper tile: as is
    if (ti <= tj) T[r0 + rr][c] = v;           // staged for the diagonal / transposed writes
  }
  if (ti > tj) return;  // strictly lower tiles of Cp come from the upper tile (tj, ti)
  __syncthreads();
#pragma unroll
  for (int rr = 0; rr < TS; rr += 8) {
    const int li = r0 + rr, lj = c;
    if (ti == tj) {  // diagonal tile: symmetrise from its upper half
      Cp[(int64_t)(ti * TS + li) * np + tj * TS + lj] = li <= lj ? T[li][lj] : T[lj][li];
    } else {  // Cp(tj, ti) = C'(ti, tj)ᵀ
      Cp[(int64_t)(tj * TS + li) * np + ti * TS + lj] = T[lj][li];
    }
  }
}

// keep (device eigensolver, round 6): while *keep == 0 the solve diverged or ran no iteration and
// the basis is the warm start Balt (d × d; may be the output buffer B itself — each element is
// read and written by the same thread) — the solver's own restore-copy launch is gone.  Rows over
// the grid, columns over the threads (no per-element 64-bit division).
__global__ void __launch_bounds__(256) eig_out_kernel(const float* __restrict__ Bp, const float* __restrict__ w, int d, int np,
                                                      float* B, float* __restrict__ D, float* __restrict__ BdivD,
                                                      const float* Balt, const int* __restrict__ keep) {
  const bool alt = Balt && keep && *keep == 0;
  const float* src = alt ? Balt : Bp;
  const int64_t lds = alt ? d : np;
  for (int i = blockIdx.x; i < d; i += gridDim.x) {
    for (int j = threadIdx.x; j < d; j += blockDim.x) {
      const float dj = sqrtf(fmaxf(w[j], 1e-30f));
      const float b = src[(int64_t)i * lds + j];
      const int64_t e = (int64_t)i * d + j;
      B[e] = b;
      BdivD[e] = b / dj;
      if (i == 0) D[j] = dj;
    }
  }
}


// Rank-μ operand: Yw[i, :] = (pop[rows[i], :] − mean) · sqrt(w_i) / σ, so Σ wᵢ yᵢ yᵢᵀ = Ywᵀ Yw
// is one plain GEMM (gather, centring, scaling in one pass instead of 4 library kernels).
// One workgroup per selected row, float4 along d.
// aug: the row also gets y[d] = σ·sqrt(wᵢ) and zeros up to ldy — the rank-μ product of these
// rows then carries Σ wᵢ (xᵢ − m) = the weighted mean shift in its last row (round 6: the
// separate weighted row sum and its column reduction, two launches, are gone)
__global__ void __launch_bounds__(256) center_rows_kernel(const float* __restrict__ pop, int64_t ldp, const int32_t* __restrict__ rows,
                                                          const float* __restrict__ mean, const float* __restrict__ sigma,
                                                          const float* __restrict__ w, int d, float* __restrict__ Y, int64_t ldy,
                                                          int aug) {
  const int i = blockIdx.x;
  const int64_t src = rows ? rows[i] : i;
  const float sw = sqrtf(w[i]), sc = sw / sigma[0];
  const float* x = pop + src * ldp;
  float* y = Y + (int64_t)i * ldy;
  if (aug)
    for (int c = d + (int)threadIdx.x; c < ldy; c += blockDim.x) y[c] = c == d ? sw * sigma[0] : 0.f;
  if ((d & 3) == 0 && (ldp & 3) == 0 && (ldy & 3) == 0) {
    for (int c = threadIdx.x * 4; c < d; c += blockDim.x * 4) {
      const float4 a = *(const float4*)(x + c), m = *(const float4*)(mean + c);
      *(float4*)(y + c) = make_float4((a.x - m.x) * sc, (a.y - m.y) * sc, (a.z - m.z) * sc, (a.w - m.w) * sc);
    }
  } else {
    for (int c = threadIdx.x; c < d; c += blockDim.x) y[c] = (x[c] - mean[c]) * sc;
  }
}

// Sharded tell (round 6): this rank's rows among the global top μ, compacted in global-rank
// order — rows_out[k] = local index, w_out[k] = its recombination weight, for k < count; the
// slots [count, K) get row 0 with weight 0, so the rank-μ partial sum keeps the static
// K = min(μ, local rows) a hipGraph needs.  One workgroup: a ballot / popcount scan over
// order[0, μ) in chunks of 1024.  Replaces a second (local) argsort, an index_copy_ and an
// index_select of the round-5 sharded tell.
__global__ void __launch_bounds__(1024) local_select_kernel(const int32_t* __restrict__ order, int mu, const float* __restrict__ w,
                                                            int start, int size, int K, int32_t* __restrict__ rows_out,
                                                            float* __restrict__ w_out) {
  __shared__ int wave_tot[16];
  __shared__ int base_s;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) base_s = 0;
  __syncthreads();
  for (int c0 = 0; c0 < mu; c0 += 1024) {
    const int i = c0 + tid;
    int g = -1;
    if (i < mu) g = order[i] - start;
    const bool p = g >= 0 && g < size;
    const unsigned long long b = __ballot(p);
    const int pre = __popcll(b & ((1ull << lane) - 1ull));
    if (lane == 0) wave_tot[wv] = __popcll(b);
    __syncthreads();
    int off = base_s;
    for (int k = 0; k < wv; ++k) off += wave_tot[k];
    if (p && off + pre < K) {
      rows_out[off + pre] = g;
      w_out[off + pre] = w[i];
    }
    __syncthreads();
    if (tid == 0) {
      int t = 0;
      for (int k = 0; k < 16; ++k) t += wave_tot[k];
      base_s += t;
    }
    __syncthreads();
  }
  for (int k = base_s + tid; k < K; k += 1024) {
    rows_out[k] = 0;
    w_out[k] = 0.f;
  }
}

// Symmetric d × d ↔ packed upper triangle (row i holds columns i..d−1 at i·d − i(i−1)/2): the
// sharded tell all-reduces the rank-μ partial sums in this form — d(d+1)/2 + d floats, half the
// bytes of the full matrix on the wire.  One workgroup per row.
__device__ __forceinline__ int64_t packed_off(int64_t i, int64_t d) { return i * d - i * (i - 1) / 2; }

__global__ void __launch_bounds__(256) sym_pack_kernel(const float* __restrict__ S, int64_t lds, int d, float* __restrict__ P) {
  const int i = blockIdx.x;
  const float* row = S + (int64_t)i * lds;
  float* o = P + packed_off(i, d) - i;
  for (int j = i + threadIdx.x; j < d; j += blockDim.x) o[j] = row[j];
}

__global__ void __launch_bounds__(256) sym_unpack_kernel(const float* __restrict__ P, int d, float* __restrict__ S, int64_t lds) {
  const int i = blockIdx.x;
  const float* o = P + packed_off(i, d) - i;
  for (int j = i + threadIdx.x; j < d; j += blockDim.x) {
    const float v = o[j];
    S[(int64_t)i * lds + j] = v;
    S[(int64_t)j * lds + i] = v;
  }
}

}  // namespace

void evx_cma_local_select(const int32_t* order, int mu, const float* w, int start, int size, int K, int32_t* rows, float* wk,
                          hipStream_t s) {
  local_select_kernel<<<1, 1024, 0, s>>>(order, mu, w, start, size, K, rows, wk);
}

void evx_sym_pack(const float* S, int64_t lds, int d, float* P, hipStream_t s) {
  if (d > 0) sym_pack_kernel<<<d, 256, 0, s>>>(S, lds, d, P);
}

void evx_sym_unpack(const float* P, int d, float* S, int64_t lds, hipStream_t s) {
  if (d > 0) sym_unpack_kernel<<<d, 256, 0, s>>>(P, d, S, lds);
}

void evx_cma_delta_gemv(const float* M, const float* mean, const float* dm, float cm, int d, float* mean_out, float* delta, float* y,
                        hipStream_t s) {
  delta_gemv_kernel<<<(d + 3) / 4, 256, 0, s>>>(M, mean, dm, cm, d, mean_out, delta, y);
}

void evx_cma_paths(const float* ps, const float* pc, const float* y, const float* delta, const float* sigma, const int64_t* count_iter,
                   int d, const float* consts, float* ps_out, float* pc_out, float* sigma_out, float* a_out, float* hsig_out,
                   hipStream_t s, const int64_t* count_eigen, int64_t* count_iter_out, int64_t* count_eigen_out) {
  PathConsts k{consts[0], consts[1], consts[2], consts[3], consts[4], consts[5], consts[6], consts[7], consts[8]};
  paths_kernel<<<1, 1024, 0, s>>>(ps, pc, y, delta, sigma, count_iter, d, k, ps_out, pc_out, sigma_out, a_out, hsig_out, count_eigen,
                                  count_iter_out, count_eigen_out);
}

void evx_cma_cov_pad(const float* C, const float* S, const float* pc, const float* a, float c1, float cmu, const float* Bprev, int d,
                     int np, float* Cn, float* Cp, float* Bp, hipStream_t s, int64_t lds) {
  dim3 grid(np / TS, np / TS);
  cov_pad_kernel<<<grid, 256, 0, s>>>(C, S, lds > 0 ? lds : d, pc, a, c1, cmu, Bprev, d, np, Cn, Cp, Bp);
}

void evx_cma_eig_out(const float* Bp, const float* w, int d, int np, float* B, float* D, float* BdivD, hipStream_t s, const float* Balt,
                     const int* keep) {
  const int g = d < 4096 ? d : 4096;
  if (g > 0) eig_out_kernel<<<g, 256, 0, s>>>(Bp, w, d, np, B, D, BdivD, Balt, keep);
}

void evx_cma_center_rows(const float* pop, int64_t ldp, const int32_t* rows, const float* mean, const float* sigma, const float* w, int K,
                         int d, float* Y, hipStream_t s, int64_t ldy, int aug) {
  if (ldy <= 0) ldy = d;
  if (K > 0) center_rows_kernel<<<K, 256, 0, s>>>(pop, ldp, rows, mean, sigma, w, d, Y, ldy, aug);
}
