// Philox4x32-10 bulk generation (uniform / normal) — K1 of SURVEY §2.10.
// One thread = one Philox block = 4 outputs, stored as one 16-B float4 (coalesced
// 1 KiB per wave-instruction).  The key is read from device memory so the launch
// is hipGraph-capturable (no host round-trip for the key).
#include "evoxmi_common.h"

namespace {

template <int DIST>
__global__ void __launch_bounds__(256) philox_fill_kernel(float* __restrict__ out, int64_t n,
                                                          const int64_t* __restrict__ key, int64_t block_offset) {
  // batched runs (BatchedRuns): grid.y indexes the key / output row
  key += 2 * (int64_t)blockIdx.y;
  out += n * (int64_t)blockIdx.y;
  uint32_t k0, k1;
  evx::load_key(key, k0, k1);
  const int64_t nb = (n + 3) >> 2;
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nb; b += (int64_t)gridDim.x * blockDim.x) {
    evx::u4 w = evx::philox_block((uint64_t)(b + block_offset), k0, k1);
    float4 v;
    if (DIST == 0) {
      v = make_float4(evx::u24(w.x), evx::u24(w.y), evx::u24(w.z), evx::u24(w.w));
    } else {
      v = evx::normal4(w);
    }
    const int64_t i = b << 2;
    if (i + 3 < n) {
      *reinterpret_cast<float4*>(out + i) = v;
    } else {
      float t[4] = {v.x, v.y, v.z, v.w};
      for (int j = 0; j < 4 && i + j < n; ++j) out[i + j] = t[j];
    }
  }
}

}  // namespace

void evx_philox_fill(float* out, int64_t n, const int64_t* key, int dist, int64_t elem_offset, hipStream_t s, int batch) {
  const int64_t nb = (n + 3) >> 2;
  int gx = (int)((nb + 255) / 256);
  if (gx > 4096) gx = 4096;
  if (gx < 1) gx = 1;
  const dim3 grid(gx, batch);
  if (dist == 0)
    philox_fill_kernel<0><<<grid, 256, 0, s>>>(out, n, key, elem_offset >> 2);
  else
    philox_fill_kernel<1><<<grid, 256, 0, s>>>(out, n, key, elem_offset >> 2);
}

// A column window of a Philox matrix: out[i][c] = element (row0 + i)·dtot + col0 + c of the
// uniform (DIST 0) / normal (DIST 1) stream — the block a decision-axis-sharded rank owns,
// bitwise equal to those columns of philox_fill over the whole (·, dtot) matrix.  One thread
// per 4 outputs; 16-B loads of the Philox block when the window is 4-aligned.
namespace {
template <int DIST>
__global__ void __launch_bounds__(256) philox_window_kernel(float* __restrict__ out, const int64_t* __restrict__ key, int64_t rows,
                                                            int64_t dtot, int64_t col0, int64_t own, int64_t row0) {
  uint32_t k0, k1;
  evx::load_key(key, k0, k1);
  const bool v4 = (own & 3) == 0 && (col0 & 3) == 0 && (dtot & 3) == 0;
  const int64_t per_row = v4 ? own >> 2 : own;
  const int64_t total = rows * per_row;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / per_row, c = t - i * per_row;
    if (v4) {
      const int64_t j = c << 2;
      const evx::u4 w = evx::philox_block((uint64_t)(((row0 + i) * dtot + col0 + j) >> 2), k0, k1);
      const float4 v = DIST == 0 ? make_float4(evx::u24(w.x), evx::u24(w.y), evx::u24(w.z), evx::u24(w.w)) : evx::normal4(w);
      *reinterpret_cast<float4*>(out + i * own + j) = v;
    } else {
      const uint64_t e = (uint64_t)((row0 + i) * dtot + col0 + c);
      const evx::u4 w = evx::philox_block(e >> 2, k0, k1);
      const int q = (int)(e & 3);
      float v;
      if (DIST == 0) {
        v = evx::u24(q == 0 ? w.x : (q == 1 ? w.y : (q == 2 ? w.z : w.w)));
      } else {
        const float4 n4 = evx::normal4(w);
        v = q == 0 ? n4.x : (q == 1 ? n4.y : (q == 2 ? n4.z : n4.w));
      }
      out[i * own + c] = v;
    }
  }
}
}  // namespace

void evx_philox_window(float* out, const int64_t* key, int64_t rows, int64_t dtot, int64_t col0, int64_t own, int64_t row0, int dist,
                       hipStream_t s) {
  const bool v4 = (own & 3) == 0 && (col0 & 3) == 0 && (dtot & 3) == 0;
  const int64_t total = rows * (v4 ? own >> 2 : own);
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  if (dist == 0)
    philox_window_kernel<0><<<(unsigned)g, 256, 0, s>>>(out, key, rows, dtot, col0, own, row0);
  else
    philox_window_kernel<1><<<(unsigned)g, 256, 0, s>>>(out, key, rows, dtot, col0, own, row0);
}

// Raw Philox words for small key-management ops (split / fold_in / bits): one launch
// instead of ~80 int64 elementwise kernels.  out[b][w] = word w of block (offset + b)
// with counter (b_lo, b_hi, 0, domain).  Words are stored as int64 (uint32 values).
namespace {
// W = words kept per block (4, or 2 for key splits: the (num, 2) keys written directly)
template <int W>
__global__ void philox_words_kernel(const int64_t* __restrict__ key, int64_t nblocks, uint32_t domain, int64_t offset,
                                    int64_t* __restrict__ out) {
  key += 2 * (int64_t)blockIdx.y;
  out += W * nblocks * (int64_t)blockIdx.y;
  uint32_t k0, k1;
  evx::load_key(key, k0, k1);
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nblocks; b += (int64_t)gridDim.x * blockDim.x) {
    uint64_t c = (uint64_t)(b + offset);
    evx::u4 w = evx::philox4x32_10(evx::u4{(uint32_t)c, (uint32_t)(c >> 32), 0u, domain}, k0, k1);
    out[W * b + 0] = w.x;
    out[W * b + 1] = w.y;
    if (W == 4) {
      out[W * b + 2] = w.z;
      out[W * b + 3] = w.w;
    }
  }
}
}  // namespace

void evx_philox_words(const int64_t* key, int64_t nblocks, uint32_t domain, int64_t offset, int64_t* out, hipStream_t s,
                      int batch, int words) {
  int gx = (int)((nblocks + 255) / 256);
  if (gx > 1024) gx = 1024;
  if (gx < 1) gx = 1;
  const dim3 grid(gx, batch);
  if (words == 2)
    philox_words_kernel<2><<<grid, 256, 0, s>>>(key, nblocks, domain, offset, out);
  else
    philox_words_kernel<4><<<grid, 256, 0, s>>>(key, nblocks, domain, offset, out);
}

// ---------------------------------------------------------------------------------------
// OpenES gradient with regenerated noise: partial[c][j] = Σ_{i in chunk c}
// w[i] · ε(i, j), with ε(i, j) = normal(key, element (row0 + i)·d + j) — exactly the value
// `normal(key, (rows, d), offset=row0·d)[i, j]` that `ask` drew — so `tell` never stores
// the N×P noise matrix.  One column per thread, chunks of rows per grid.y (partials summed
// in a fixed order on the host side: deterministic).
namespace {
// (col0, dtot): the column window [col0, col0 + d) of a (·, dtot) noise matrix (decision-axis
// sharding: each rank reduces only its own columns)
__global__ void __launch_bounds__(256) es_noise_grad_kernel(const int64_t* __restrict__ key, const float* __restrict__ w, int64_t rows,
                                                            int64_t d, int64_t row0, int64_t per, float* __restrict__ partial,
                                                            int64_t col0, int64_t dtot) {
  uint32_t k0, k1;
  evx::load_key(key, k0, k1);
  const int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  const int64_t c = blockIdx.y;
  if (j >= d) return;
  const int64_t i0 = c * per, i1 = min(rows, i0 + per);
  float acc = 0.f;
  for (int64_t i = i0; i < i1; ++i) {
    const uint64_t e = (uint64_t)((row0 + i) * dtot + col0 + j);
    const evx::u4 b = evx::philox_block(e >> 2, k0, k1);
    // the Box–Muller pair of element e only (same operations as evx::normal4)
    const int q = (int)(e & 3);
    const float r = sqrtf(-2.0f * logf(evx::u24(q < 2 ? b.x : b.z)));
    float sn, cs;
    sincosf(6.283185307179586f * evx::u24(q < 2 ? b.y : b.w), &sn, &cs);
    acc = fmaf(w[i], r * ((q & 1) ? sn : cs), acc);
  }
  partial[c * d + j] = acc;
}
}  // namespace

void evx_es_noise_grad(const int64_t* key, const float* w, int64_t rows, int64_t d, int64_t row0, int chunks, float* partial,
                       hipStream_t s, int64_t col0, int64_t dtot) {
  const int64_t per = (rows + chunks - 1) / chunks;
  const dim3 grid((unsigned)((d + 255) / 256), (unsigned)chunks);
  es_noise_grad_kernel<<<grid, 256, 0, s>>>(key, w, rows, d, row0, per, partial, col0, dtot > 0 ? dtot : d);
}

// ---------------------------------------------------------------------------------------
// OpenES population rows [row0, row0 + rows) in one pass: x(g, j) = c(j) + s·σ·ε(r, j) with
// (mirrored sampling, h = pop / 2) r = g mod h and s = +1 for g < h, −1 after; ε(r, j) =
// normal(key, element r·d + j) — the noise `tell` regenerates (es_noise_grad_kernel).  The
// f32 noise matrix, its mirrored copy and their concatenation are never written.  The sum is
// c + (s·σ)·ε with two roundings: bitwise the torch expression it replaces.
namespace {
// (col0, dtot): columns [col0, col0 + d) of the (·, dtot) rows, center holding those d columns
__global__ void __launch_bounds__(256) es_population_kernel(const int64_t* __restrict__ key, const float* __restrict__ center, float sigma,
                                                            int64_t rows, int64_t d, int64_t half, int64_t row0, float* __restrict__ out,
                                                            int64_t col0, int64_t dtot) {
  // two roundings (σ·ε, then + c) like the torch expression: no FMA contraction in this scope
  // (plain operators: the pragma does not reach the __fmul_rn / __fadd_rn header definitions)
#pragma clang fp contract(off)
  uint32_t k0, k1;
  evx::load_key(key, k0, k1);
  const bool v4 = (d & 3) == 0 && (col0 & 3) == 0 && (dtot & 3) == 0;
  const int64_t per_row = v4 ? d >> 2 : d;
  const int64_t total = rows * per_row;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = t / per_row, c = t - i * per_row;
    const int64_t g = row0 + i;
    const bool neg = half > 0 && g >= half;
    const int64_t r = neg ? g - half : g;
    const float ss = neg ? -sigma : sigma;
    if (v4) {
      const int64_t j = c << 2;
      const float4 n = evx::normal4(evx::philox_block((uint64_t)((r * dtot + col0 + j) >> 2), k0, k1));
      const float4 ce = *reinterpret_cast<const float4*>(center + j);
      float4 o;
      o.x = ce.x + ss * n.x;
      o.y = ce.y + ss * n.y;
      o.z = ce.z + ss * n.z;
      o.w = ce.w + ss * n.w;
      *reinterpret_cast<float4*>(out + i * d + j) = o;
    } else {
      const uint64_t e = (uint64_t)(r * dtot + col0 + c);
      const evx::u4 b = evx::philox_block(e >> 2, k0, k1);
      const float4 n4 = evx::normal4(b);
      const int q = (int)(e & 3);
      const float n = q == 0 ? n4.x : (q == 1 ? n4.y : (q == 2 ? n4.z : n4.w));
      out[i * d + c] = center[c] + ss * n;
    }
  }
}
}  // namespace

void evx_es_population(const int64_t* key, const float* center, float sigma, int64_t rows, int64_t d, int64_t half, int64_t row0, float* out,
                       hipStream_t s, int64_t col0, int64_t dtot) {
  if (dtot <= 0) dtot = d;
  const bool v4 = (d & 3) == 0 && (col0 & 3) == 0 && (dtot & 3) == 0;
  const int64_t total = rows * (v4 ? d >> 2 : d);
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  es_population_kernel<<<(unsigned)g, 256, 0, s>>>(key, center, sigma, rows, d, half, row0, out, col0, dtot);
}
