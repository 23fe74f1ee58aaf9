// Variation operators as fused elementwise kernels (K11): PlatEMO SBX and polynomial
// mutation.  Random numbers are regenerated in-register from Philox counters with the
// same element indexing as evoxmi.ops.random (uniform → u24 of word i%4 of block i/4,
// randint(0,2) → top bit), so GPU and CPU draw identical streams.
#include "evoxmi_common.h"

namespace {

__device__ __forceinline__ uint32_t word_at(uint64_t i, uint32_t k0, uint32_t k1) {
  evx::u4 w = evx::philox_block(i >> 2, k0, k1);
  const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
  return ws[i & 3];
}

// keys: split(key, 2) → per-gene word (μ = top 24 bits, bit 0 = sign of β, bit 1 = skip),
// per-pair rate uniform.  One thread per 4 consecutive genes when they share a Philox
// block, else one gene per thread.  Column block (decision-axis state sharding): x / out
// hold columns [col0, col0 + d) of a dtot-dimensional population and every gene word is
// drawn at its global counter i·dtot + col0 + j, so a block equals those columns of the
// unsharded offspring.
__device__ __forceinline__ float sbx_beta(uint32_t w, float e) {
  const float mu = evx::u24(w);
  float beta = mu <= 0.5f ? exp2f(e * __log2f(2.f * mu)) : exp2f(-e * __log2f(2.f - 2.f * mu));
  if (w & 1u) beta = -beta;
  if (w & 2u) beta = 1.f;
  return beta;
}

__global__ void __launch_bounds__(256) sbx_kernel(const float* __restrict__ x, float* __restrict__ out, int n, int d,
                                                  const int64_t* __restrict__ keys, float pro_c, float dis_c, int type, int col0,
                                                  int dtot) {
  const int np = n / 2;
  const uint32_t kg0 = (uint32_t)keys[0], kg1 = (uint32_t)keys[1];
  const uint32_t kp0 = (uint32_t)keys[2], kp1 = (uint32_t)keys[3];
  const float e = 1.f / (dis_c + 1.f);
  const int vec = ((d | col0 | dtot) & 3) == 0 ? 4 : 1;
  const int64_t total = (int64_t)np * d / vec;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g0 = t * vec;
    const int i = (int)(g0 / d), j0 = (int)(g0 - (int64_t)i * d);
    const uint64_t gg = (uint64_t)i * dtot + col0 + j0;  // global gene counter
    const bool no_x = evx::u24(word_at((uint64_t)i, kp0, kp1)) > pro_c;
    uint32_t ws[4];
    if (vec == 4) {
      const evx::u4 w = evx::philox_block(gg >> 2, kg0, kg1);
      ws[0] = w.x; ws[1] = w.y; ws[2] = w.z; ws[3] = w.w;
    } else {
      ws[0] = word_at(gg, kg0, kg1);
    }
    for (int v = 0; v < vec; ++v) {
      const int j = j0 + v;
      const float p1 = x[(int64_t)i * d + j], p2 = x[(int64_t)(np + i) * d + j];
      const float beta = no_x ? 1.f : sbx_beta(ws[v], e);
      const float mid = 0.5f * (p1 + p2), half = 0.5f * (p1 - p2);
      out[(int64_t)i * d + j] = mid + beta * half;
      if (type == 1) out[(int64_t)(np + i) * d + j] = mid - beta * half;
    }
  }
  if (type == 1 && (n & 1)) {  // odd population: last parent passes through
    for (int j = blockIdx.x * blockDim.x + threadIdx.x; j < d; j += gridDim.x * blockDim.x)
      out[(int64_t)(2 * np) * d + j] = x[(int64_t)(n - 1) * d + j];
  }
}

// keys: split(key, 2) → site, mu.  Rows beyond the even prefix pass through.
__global__ void __launch_bounds__(256) pm_kernel(const float* __restrict__ x, float* __restrict__ out, int n, int d, int nm,
                                                 const float* __restrict__ lb, const float* __restrict__ ub,
                                                 const int64_t* __restrict__ keys, float pro_m, float dis_m, int col0, int dtot) {
  // column block: lb / ub are the block's, site probability and counters use the global column
  const int64_t total = (int64_t)n * d;
  uint32_t ks0 = (uint32_t)keys[0], ks1 = (uint32_t)keys[1];
  uint32_t ku0 = (uint32_t)keys[2], ku1 = (uint32_t)keys[3];
  const float e1 = dis_m + 1.f, inv = 1.f / (dis_m + 1.f);
  const float pr = pro_m / dtot;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(t / d), j = (int)(t - (int64_t)i * d);
    const uint64_t tg = (uint64_t)i * dtot + col0 + j;
    float v = x[t];
    if (i < nm) {
      const float lo = lb[j], hi = ub[j], span = hi - lo;
      v = fmaxf(fminf(v, hi), lo);
      const bool site = evx::u24(word_at(tg, ks0, ks1)) < pr;
      if (site) {
        const float mu = evx::u24(word_at(tg, ku0, ku1));  // drawn only at mutation sites
        if (mu <= 0.5f) {
          const float nrm = (v - lo) / span;
          v = v + span * (powf(2.f * mu + (1.f - 2.f * mu) * powf(1.f - nrm, e1), inv) - 1.f);
        } else {
          const float nrm = (hi - v) / span;
          v = v + span * (1.f - powf(2.f * (1.f - mu) + 2.f * (mu - 0.5f) * powf(1.f - nrm, e1), inv));
        }
      }
    }
    out[t] = v;
  }
}

int grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  return (int)(g > 8192 ? 8192 : (g < 1 ? 1 : g));
}


// Fused DE trial-vector generation (K10) for every DE variant of the zoo.
// Row i of the output:
//   m_j   = Σ_k coef[i,k] · P[idx[i,k], j]            (base + F·(sec−prim) + F·Σ±diffs)
//   x_j   = P[cur[i], j]
//   t_j   = bin:   (u(i,j) < CR_i || j == jr_i) ? m_j : x_j
//           exp:   ((j − jr_i) mod d) < L_i     ? m_j : x_j
//           arith: x_j + CR_i·(m_j − x_j)
//   repair: clip to [lb, ub] or LSHADE midpoint ((x + bound)/2)
// u(i,j) is regenerated from the Philox counter i·d + j (same stream as uniform(key,(R,d))).
// One thread per element, rows laid out contiguously; coef/idx/row params are broadcast
// loads that stay in L1/L2.  K ≤ 16.
__global__ void __launch_bounds__(256) de_trial_kernel(const float* __restrict__ P, const int32_t* __restrict__ idx,
                                                       const float* __restrict__ coef, int K, const int32_t* __restrict__ cur,
                                                       const int32_t* __restrict__ mode, const float* __restrict__ CR,
                                                       const int32_t* __restrict__ jr, const int32_t* __restrict__ L,
                                                       const int64_t* __restrict__ key, const float* __restrict__ lb,
                                                       const float* __restrict__ ub, int repair, float* __restrict__ out, int R,
                                                       int d, int rows, int* __restrict__ err, int col0, int dtot) {
  // column block (decision-axis state sharding): P / out hold columns [col0, col0 + d) of a
  // dtot-dimensional population; the Philox word, j_rand and the exponential window use the
  // global column, so every block equals the same columns of the unsharded trials
  // batched runs: grid.y = run b; its R trial rows, P rows and key are run-local
  const int64_t b = blockIdx.y;
  P += b * rows * (int64_t)d;
  idx += b * R * (int64_t)K;
  coef += b * R * (int64_t)K;
  cur += b * R; mode += b * R; CR += b * R; jr += b * R; L += b * R;
  key += 2 * b;
  out += b * R * (int64_t)d;
  const uint32_t k0 = (uint32_t)key[0], k1 = (uint32_t)key[1];
  const int64_t total = (int64_t)R * d;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int i = (int)(t / d), j = (int)(t - (int64_t)i * d), jg = col0 + j;
    float m = 0.f;
    for (int k = 0; k < K; ++k) {
      const float c = coef[i * K + k];
      const int r = idx[i * K + k];
      if ((unsigned)r >= (unsigned)rows) {  // never dereference a bad row: flag it and skip
        if (j == 0) atomicOr(err, 1);
        continue;
      }
      if (c != 0.f) m = fmaf(c, P[(int64_t)r * d + j], m);
    }
    int rc = cur[i];
    if ((unsigned)rc >= (unsigned)rows) {
      if (j == 0) atomicOr(err, 2);
      rc = 0;
    }
    const float x = P[(int64_t)rc * d + j];
    const int md = mode[i];
    float v;
    if (md == 0) {
      const float u = evx::u24(word_at((uint64_t)i * dtot + jg, k0, k1));
      v = (u < CR[i] || jg == jr[i]) ? m : x;
    } else if (md == 1) {
      int pos = jg - jr[i];
      if (pos < 0) pos += dtot;
      v = pos < L[i] ? m : x;
    } else {
      v = x + CR[i] * (m - x);
    }
    if (repair == 1) {
      v = fminf(fmaxf(v, lb[j]), ub[j]);
    } else if (repair == 2) {
      if (v < lb[j]) v = 0.5f * (x + lb[j]);
      if (v > ub[j]) v = 0.5f * (x + ub[j]);
    }
    out[t] = v;
  }
}

}  // namespace

void evx_sbx(const float* x, float* out, int n, int d, const int64_t* keys, float pro_c, float dis_c, int type, hipStream_t s, int col0,
             int dtot) {
  sbx_kernel<<<grid_for((int64_t)(n / 2) * d), 256, 0, s>>>(x, out, n, d, keys, pro_c, dis_c, type, col0, dtot > 0 ? dtot : d);
}

void evx_pm(const float* x, float* out, int n, int d, int nm, const float* lb, const float* ub, const int64_t* keys, float pro_m,
            float dis_m, hipStream_t s, int col0, int dtot) {
  pm_kernel<<<grid_for((int64_t)n * d), 256, 0, s>>>(x, out, n, d, nm, lb, ub, keys, pro_m, dis_m, col0, dtot > 0 ? dtot : d);
}

void evx_de_trial(const float* P, const int32_t* idx, const float* coef, int K, const int32_t* cur, const int32_t* mode,
                  const float* CR, const int32_t* jr, const int32_t* L, const int64_t* key, const float* lb, const float* ub,
                  int repair, float* out, int R, int d, int rows, int* err, hipStream_t s, int batch, int col0, int dtot) {
  const int64_t total = (int64_t)R * d;
  const dim3 grid((int)std::min<int64_t>((total + 255) / 256, 8192), batch);
  de_trial_kernel<<<grid, 256, 0, s>>>(P, idx, coef, K, cur, mode, CR, jr, L, key, lb, ub, repair, out, R, d, rows, err, col0,
                                       dtot > 0 ? dtot : d);
}
