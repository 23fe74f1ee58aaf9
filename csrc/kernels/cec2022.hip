// CEC2022 basic functions as one wave64-per-row reduction kernel (K6 epilogue stage).
//
// z_eff(j) = (Z[row, idx(j)] − sub[idx(j)]) · scale,   idx(j) = perm ? perm[start + j] : start + j
// for j in [0, L).  Functions that need neighbours (Rosenbrock, Levy, expanded
// Griewank-Rosenbrock, expanded Schaffer, Schaffer F7) re-read z_eff(j ± 1) — the row
// is L1/L2 resident, so each element is fetched from HBM once.  The f < 1e-8 clamp and
// composition weights are applied by the caller.  Function ids match
// evoxmi/problems/numerical/cec2022.py.
#include "evoxmi_common.h"
#include "evoxmi_launchers.h"

namespace {

constexpr float PI_F = 3.14159265358979323846f;

enum { ZAKHAROV = 0, ROSENBROCK, SCHAFFERF7, RASTRIGIN, LEVY, BENTCIGAR, HGBAT, KATSUURA, ACKLEY, SCHWEFEL, HAPPYCAT,
       ELLIPTIC, DISCUS, EXPSCHAFFER, EXPGRIEROSEN, GRIEWANK, SPHERE };

// PERM / SUB are template flags (not per-element pointer tests): with a runtime test in the
// unrolled row loop the compiler kept every load behind its own vmcnt(0) wait (one memory
// latency per element); specialised, a lane's 16 loads issue together
template <bool PERM, bool SUB>
struct RowViewT {
  const float* z;
  const int32_t* perm;
  const float* sub;
  int start;
  float scale;
  __device__ __forceinline__ float operator()(int j) const {
    const int i = PERM ? perm[start + j] : start + j;
    float v = z[i];
    if (SUB) v -= sub[i];
    return v * scale;
  }
};

// f of one row (wave64: every lane returns the same value).  SCHAFFERF7's y pairs come from Y
// (a separate row), the permuted Z row (yperm) or z itself.
// the row loop of a basic function: lanes stride the row by 64.  The iterations in which every
// lane is in range run without a guard, unrolled by 8, so a lane's loads of a chunk issue
// together (behind a per-element `j < L` test the compiler kept each load behind its own
// vmcnt(0) wait: one memory latency per element); the ragged last iteration is guarded
template <class F>
__device__ __forceinline__ void for_row(int L, int lane, F&& f) {
  const int full = L >> 6;
  int q = 0;
#pragma unroll 8
  for (; q < full; ++q) f(lane + 64 * q);
  const int j = lane + 64 * full;
  if (j < L) f(j);
}

template <class RowView>
__device__ __forceinline__ float basic_row(const RowView& z, int fid, int L, int lane, const float* __restrict__ yr,
                                           const float* __restrict__ zrow, const int32_t* __restrict__ perm, int yperm) {
  float a = 0.f, b = 0.f, p = 1.f;
  const float fL = (float)L;
  switch (fid) {
    case ZAKHAROV:
      for_row(L, lane, [&](int j) { float v = z(j); a += v * v; b += 0.5f * (float)(j + 1) * v; });
      break;
    case ROSENBROCK:
      for_row(L - 1, lane, [&](int j) {
        float v = z(j) + 1.f, w = z(j + 1) + 1.f;
        float t = v * v - w, u = 1.f - v;
        a += 100.f * t * t + u * u;
      });
      break;
    case SCHAFFERF7:
      for_row(L - 1, lane, [&](int j) {
        float y0, y1;
        if (yr) { y0 = yr[j]; y1 = yr[j + 1]; }
        else if (yperm) { y0 = zrow[perm[j]]; y1 = zrow[perm[j + 1]]; }
        else { y0 = z(j); y1 = z(j + 1); }
        float s = sqrtf(y0 * y0 + y1 * y1);
        float t = sinf(50.f * powf(s, 0.2f));
        float r = sqrtf(s);
        a += r + r * t * t;
      });
      break;
    case RASTRIGIN:
      for_row(L, lane, [&](int j) { float v = z(j) * 0.0512f; a += v * v - 10.f * cosf(2.f * PI_F * v) + 10.f; });
      break;
    case LEVY:
      for_row(L, lane, [&](int j) {
        float w = 1.f + z(j) * 0.25f;
        if (j == 0) { float s0 = sinf(PI_F * w); a += s0 * s0; }
        if (j < L - 1) { float s = sinf(PI_F * w + 1.f); a += (w - 1.f) * (w - 1.f) * (1.f + 10.f * s * s); }
        else { float s = sinf(2.f * PI_F * w); a += (w - 1.f) * (w - 1.f) * (1.f + s * s); }
      });
      break;
    case BENTCIGAR:
      for_row(L, lane, [&](int j) { float v = z(j); a += (j == 0 ? 1.f : 1e6f) * v * v; });
      break;
    case HGBAT:
    case HAPPYCAT:
      for_row(L, lane, [&](int j) { float v = z(j) * 0.05f - 1.f; a += v * v; b += v; });
      break;
    case KATSUURA: {
      const float ex = 10.f / powf(fL, 1.2f);
      for_row(L, lane, [&](int j) {
        float v = z(j) * 0.05f, temp = 0.f, t1 = 1.f;
        for (int k = 1; k <= 32; ++k) {
          t1 *= 2.f;
          float t2 = t1 * v;
          temp += fabsf(t2 - floorf(t2 + 0.5f)) / t1;
        }
        p *= powf(1.f + (float)(j + 1) * temp, ex);
      });
      break;
    }
    case ACKLEY:
      for_row(L, lane, [&](int j) { float v = z(j); a += v * v; b += cosf(2.f * PI_F * v); });
      break;
    case SCHWEFEL:
      for_row(L, lane, [&](int j) {
        float v = z(j) * 10.f + 4.209687462275036e2f;
        if (v > 500.f) {
          float m = 500.f - fmodf(v, 500.f);
          float t = (v - 500.f) / 100.f;
          a += -m * sinf(sqrtf(m)) + t * t / fL;
        } else if (v < -500.f) {
          float m = fmodf(fabsf(v), 500.f);
          float t = (v + 500.f) / 100.f;
          a += -(-500.f + m) * sinf(sqrtf(500.f - m)) + t * t / fL;
        } else {
          a += -v * sinf(sqrtf(fabsf(v)));
        }
      });
      break;
    case ELLIPTIC:
      // 10^(6j/(L−1)) as exp2 (powf's special-case handling is most of the loop's instructions)
      for_row(L, lane, [&](int j) { float v = z(j); a += exp2f(6.f * (float)j / (fL - 1.f) * 3.3219280948873623f) * v * v; });
      break;
    case DISCUS:
      for_row(L, lane, [&](int j) { float v = z(j); a += (j == 0 ? 1e6f : 1.f) * v * v; });
      break;
    case EXPSCHAFFER:
      for_row(L, lane, [&](int j) {
        float v = z(j), u = z(j == 0 ? L - 1 : j - 1);
        float sq = v * v + u * u;
        float s = sinf(sqrtf(sq));
        float d = 1.f + 0.001f * sq;
        a += 0.5f + (s * s - 0.5f) / (d * d);
      });
      break;
    case EXPGRIEROSEN:
      for_row(L, lane, [&](int j) {
        float v = z(j) * 0.05f + 1.f, w = z(j == L - 1 ? 0 : j + 1) * 0.05f + 1.f;
        float t1 = v * v - w, t2 = v - 1.f;
        float temp = 100.f * t1 * t1 + t2 * t2;
        a += temp * temp / 4000.f - cosf(temp) + 1.f;
      });
      break;
    case GRIEWANK:
      for_row(L, lane, [&](int j) { float v = z(j); a += v * v; p *= cosf(v / sqrtf((float)(j + 1))); });
      break;
    default:  // SPHERE
      for_row(L, lane, [&](int j) { float v = z(j); a += v * v; });
      break;
  }
  a = evx::wave_sum(a);
  b = evx::wave_sum(b);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) p *= __shfl_xor(p, o, 64);
  switch (fid) {
    case ZAKHAROV: return a + b * b + b * b * b * b;
    case SCHAFFERF7: return a * a / (fL - 1.f) / (fL - 1.f);
    case HGBAT: return sqrtf(fabsf(a * a - b * b)) + (0.5f * a + b) / fL + 0.5f;
    case HAPPYCAT: return powf(fabsf(a - fL), 0.25f) + (0.5f * a + b) / fL + 0.5f;
    case KATSUURA: { float c = 10.f / fL / fL; return p * c - c; }
    case ACKLEY: return -20.f * expf(-0.2f * sqrtf(a / fL)) - expf(b / fL) + 20.f + 2.718281828459045f;
    case SCHWEFEL: return a + 4.189828872724338e2f * fL;
    case GRIEWANK: return a / 4000.f - p + 1.f;
    default: return a;
  }
}

__global__ void __launch_bounds__(256) cec_basic_kernel(const float* __restrict__ Z, int64_t ld, int N, int fid,
                                                        const int32_t* __restrict__ perm, int start, int L,
                                                        const float* __restrict__ sub, float scale,
                                                        const float* __restrict__ Y, int64_t ldy, int ystart, int yperm,
                                                        float* __restrict__ out, float clamp) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= N) return;
  const float* zrow = Z + (int64_t)row * ld;
  const float* yr = Y ? Y + (int64_t)row * ldy + ystart : nullptr;
  float f;
  if (perm) {
    if (sub) f = basic_row(RowViewT<true, true>{zrow, perm, sub, start, scale}, fid, L, lane, yr, zrow, perm, yperm);
    else f = basic_row(RowViewT<true, false>{zrow, perm, sub, start, scale}, fid, L, lane, yr, zrow, perm, yperm);
  } else {
    if (sub) f = basic_row(RowViewT<false, true>{zrow, perm, sub, start, scale}, fid, L, lane, yr, zrow, perm, yperm);
    else f = basic_row(RowViewT<false, false>{zrow, perm, sub, start, scale}, fid, L, lane, yr, zrow, perm, yperm);
  }
  if (lane == 0) out[row] = (clamp > 0.f && f < clamp) ? 0.f : f;  // the CEC'22 f < 1e-8 -> 0 clamp when clamp > 0 (NaN stays NaN)
}

// Composition functions (F9–F12) in two launches instead of 2n + ~15: (1) wave (row, part i) —
// grid.y = part — computes the component's basic function from its block of the stacked rotation
// GEMM output (zcol ≥ 0) or from x − o (zcol < 0), and ‖x − o_i‖² from the same pass over the x
// row, writing (λ_i f_i + bias_i, d_i²); (2) one thread per row forms the weights
// w_i = exp(−d_i²/(2 D σ_i²)) / d_i (a zero distance selects its component(s)), the weighted sum
// and the f < thr → 0 clamp.  The part index is uniform per workgroup, so each wave runs one
// case of the basic-function switch at full occupancy (a per-row loop over parts in one kernel
// held 76-189 VGPRs and ran at 2-4 waves per SIMD: 238 µs at F9, 10 000 × 1000).
__global__ void __launch_bounds__(256) cec_compose_parts_kernel(const float* __restrict__ Z, int64_t ldz, const float* __restrict__ X,
                                                                int64_t ldx, int N, int D, EvxCecCompose c, float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int i = blockIdx.y;
  if (row >= N) return;
  const float* xrow = X + (int64_t)row * ldx;
  const float* o = c.os + (int64_t)i * c.ldo;
  float a = 0.f;
  for_row(D, lane, [&](int j) {
    const float t = xrow[j] - o[j];
    a = fmaf(t, t, a);
  });
  a = evx::wave_sum(a);
  const bool rot = c.zcol[i] >= 0;  // uniform per workgroup
  const float f = rot ? basic_row(RowViewT<false, false>{Z + (int64_t)row * ldz + c.zcol[i], nullptr, nullptr, 0, c.scale[i]}, c.fid[i], D,
                                  lane, nullptr, nullptr, nullptr, 0)
                      : basic_row(RowViewT<false, true>{xrow, nullptr, c.os + (int64_t)c.comp[i] * c.ldo, 0, c.scale[i]}, c.fid[i], D,
                                  lane, nullptr, nullptr, nullptr, 0);
  if (lane == 0) *reinterpret_cast<float2*>(part + ((int64_t)row * c.n + i) * 2) = make_float2(c.lamb[i] * f + c.bias[i], a);
}

__global__ void __launch_bounds__(256) cec_compose_final_kernel(const float* __restrict__ part, int N, int D, EvxCecCompose c,
                                                                float* __restrict__ out) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= N) return;
  const float2* pr = reinterpret_cast<const float2*>(part) + (int64_t)row * c.n;
  float wsum = 0.f, zsum = 0.f, fsum = 0.f;
  int nzero = 0;
  for (int i = 0; i < c.n; ++i) {
    const float2 gd = pr[i];
    const float t1 = 1.f / sqrtf(gd.y);
    if (!isfinite(t1)) {
      ++nzero;
      zsum += gd.x;
    }
    wsum += t1 * expf(-0.5f * gd.y / (c.sigma[i] * c.sigma[i] * (float)D));
  }
  float f;
  if (nzero > 0) {
    f = zsum / (float)nzero;
  } else {
    for (int i = 0; i < c.n; ++i) {
      const float2 gd = pr[i];
      const float wi = (1.f / sqrtf(gd.y)) * expf(-0.5f * gd.y / (c.sigma[i] * c.sigma[i] * (float)D));
      fsum += (wi / wsum) * gd.x;
    }
    f = fsum;
  }
  out[row] = f < c.thr ? 0.f : f;
}

}  // namespace

void evx_cec_basic(const float* Z, int64_t ld, int N, int fid, const int32_t* perm, int start, int L, const float* sub,
                   float scale, const float* Y, int64_t ldy, int ystart, int yperm, float* out, hipStream_t s, float clamp) {
  dim3 grid((N + 3) / 4);
  cec_basic_kernel<<<grid, 256, 0, s>>>(Z, ld, N, fid, perm, start, L, sub, scale, Y, ldy, ystart, yperm, out, clamp);
}

namespace {
// f of every row from the per-column-tile additive terms of the fused rotation GEMM
// (gemm_ks row-terms epilogue), summed in tile order (deterministic); the < 1e-8 clamp of
// the CEC'22 evaluation is applied here
__global__ void cec_rowterms_final_kernel(const float* __restrict__ parts, int tiles_n, int M, int fid, float* __restrict__ out) {
  const int row = blockIdx.x * blockDim.x + threadIdx.x;
  if (row >= M) return;
  float a = 0.f, b = 0.f;
  for (int t = 0; t < tiles_n; ++t) {
    const float2 v = *reinterpret_cast<const float2*>(parts + ((int64_t)t * M + row) * 2);
    a += v.x;
    b += v.y;
  }
  const float f = fid == 0 ? a + b * b + b * b * b * b : a;
  out[row] = f < 1e-8f ? 0.f : f;
}
}  // namespace

void evx_cec_compose(const float* Z, int64_t ldz, const float* X, int64_t ldx, int N, int D, const EvxCecCompose& c, float* part,
                     float* out, hipStream_t s) {
  if (N <= 0) return;
  cec_compose_parts_kernel<<<dim3((N + 3) / 4, c.n), 256, 0, s>>>(Z, ldz, X, ldx, N, D, c, part);
  cec_compose_final_kernel<<<(N + 255) / 256, 256, 0, s>>>(part, N, D, c, out);
}

void evx_cec_rowterms_final(const float* parts, int tiles_n, int M, int fid, float* out, hipStream_t s) {
  cec_rowterms_final_kernel<<<(M + 255) / 256, 256, 0, s>>>(parts, tiles_n, M, fid, out);
}
