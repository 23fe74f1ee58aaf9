// Fused DTLZ1–4 evaluation: one wave64 per population row.
//
// The distance function g is a row reduction over x[m-1:] (lanes stride the tail,
// reduced with xor-shuffles); then lanes 0..m-1 each build one objective
//   f_j = s·(1+g) · prod_{i < m-1-j} h(x_i) · (j > 0 ? t(x_{m-1-j}) : 1)
// directly (m ≤ 16, so the m-1 term product per lane is cheap) and write it, so the
// (n, m) output is produced in one pass over X with no intermediate tensors.
// Reference semantics: problems/numerical/dtlz.py:8-200.
#include "evoxmi_common.h"

namespace {
using namespace evx;

constexpr float PI_F = 3.14159265358979323846f;

template <int V>
__global__ void __launch_bounds__(256) dtlz_kernel(const float* __restrict__ X, float* __restrict__ F, int N, int D, int M) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= N) return;
  const float* x = X + (int64_t)row * D;
  float s = 0.f;
  for (int j = M - 1 + lane; j < D; j += 64) {
    const float y = x[j] - 0.5f;
    if (V == 1 || V == 3)
      s += y * y - cosf(20.f * PI_F * y);
    else
      s += y * y;
  }
  s = wave_sum(s);
  const float g = (V == 1 || V == 3) ? 100.f * ((float)(D - M + 1) + s) : s;
  if (lane < M) {
    const int j = lane;
    float f = (V == 1 ? 0.5f : 1.f) * (1.f + g);
    const int np = M - 1 - j;
    for (int i = 0; i < np; ++i) {
      float xi = x[i];
      if (V == 4) xi = powf(xi, 100.f);
      f *= (V == 1) ? xi : fmaxf(cosf(xi * PI_F * 0.5f), 0.f);
    }
    if (j > 0) {
      float xi = x[np];
      if (V == 4) xi = powf(xi, 100.f);
      f *= (V == 1) ? (1.f - xi) : sinf(xi * PI_F * 0.5f);
    }
    F[(int64_t)row * M + j] = f;
  }
}

// ---------------------------------------------------------------- LSMOP1–9 distance terms (K14)
// One wave64 per row computes g_k for every objective group k straight from the RAW
// decision row: the linkage x̃_c = (1 + t_c)·x_c − 10·x_0 (t_c = (c+1)/d, or
// cos(π(c+1)/(2d)) for LSMOP5–9) is applied in-register, each of the nk subcomponent
// segments is reduced by the wave (sum / second sum / product / max as the inner
// function needs), and g_k = Σ_sub f(segment) / (sublen_k · nk).  The (n, d) matrix is
// read once; the linked copy and the 15 strided segment copies of the eager path vanish.
constexpr int LS_MAXG = 16;
struct LsmopGroups {
  int start[LS_MAXG], sublen[LS_MAXG], func[LS_MAXG];
  int ng, nk, cosine;
};

__device__ __forceinline__ float wave_reduce(float v, int op) {  // op 0 sum, 1 prod, 2 max
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o, 64);
    v = op == 0 ? v + u : (op == 1 ? v * u : fmaxf(v, u));
  }
  return v;
}

// one segment's partial terms for inner function FN (a: sum / max, b: product / second sum),
// this lane's elements i = lane, lane + 64, …; four loads in flight per lane (the loop body is
// straight-line, the function chosen at compile time) — one load per iteration left the kernel
// waiting on HBM latency 79 % of its cycles
template <int FN>
__device__ __forceinline__ void seg_terms(const float* __restrict__ x, int s0, int L, int lane, float x0, float invd, int cosine,
                                          float& a, float& b) {
  auto link = [&](int c) {
    const float t = cosine ? cosf((float)(c + 1) * invd * (PI_F * 0.5f)) : (float)(c + 1) * invd;
    return (1.f + t) * x[c] - 10.f * x0;
  };
  auto acc = [&](int i, float z) {
    if (FN == 0) a += z * z;                                                                  // sphere
    else if (FN == 1) { a += z * z; b *= cosf(z * rsqrtf((float)(i + 1))); }                 // griewank
    else if (FN == 2) {                                                                       // rosenbrock
      if (i + 1 < L) { const float zn = link(s0 + i + 1), u = zn - z * z; a += 100.f * u * u + (z - 1.f) * (z - 1.f); }
    } else if (FN == 3) { a += z * z; b += cosf(2.f * PI_F * z); }                          // ackley
    else if (FN == 4) a = fmaxf(a, fabsf(z));                                                // schwefel (max |z|)
    else a += z * z - 10.f * cosf(2.f * PI_F * z) + 10.f;                                     // rastrigin
  };
  int i = lane;
  for (; i + 192 < L; i += 256) {
    const float z0 = link(s0 + i), z1 = link(s0 + i + 64), z2 = link(s0 + i + 128), z3 = link(s0 + i + 192);
    acc(i, z0);
    acc(i + 64, z1);
    acc(i + 128, z2);
    acc(i + 192, z3);
  }
  for (; i < L; i += 64) acc(i, link(s0 + i));
}

// one wave64 per row (no block barriers: every reduction is a 6-step xor butterfly)
__global__ void __launch_bounds__(256) lsmop_g_kernel(const float* __restrict__ X, float* __restrict__ G, int N, int D, LsmopGroups gr) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= N) return;
  const float* x = X + (int64_t)row * D;
  const float x0 = x[0];
  const float invd = 1.f / (float)D;
  float gout = 0.f;
  for (int k = 0; k < gr.ng; ++k) {
    const int L = gr.sublen[k], fn = gr.func[k];
    float gk = 0.f;
    for (int sub = 0; sub < gr.nk; ++sub) {
      const int s0 = gr.start[k] + sub * L;
      float a = 0.f, b = (fn == 1) ? 1.f : 0.f;
      switch (fn) {
        case 0: seg_terms<0>(x, s0, L, lane, x0, invd, gr.cosine, a, b); break;
        case 1: seg_terms<1>(x, s0, L, lane, x0, invd, gr.cosine, a, b); break;
        case 2: seg_terms<2>(x, s0, L, lane, x0, invd, gr.cosine, a, b); break;
        case 3: seg_terms<3>(x, s0, L, lane, x0, invd, gr.cosine, a, b); break;
        case 4: seg_terms<4>(x, s0, L, lane, x0, invd, gr.cosine, a, b); break;
        default: seg_terms<5>(x, s0, L, lane, x0, invd, gr.cosine, a, b); break;
      }
      float v;
      if (fn == 4) {
        v = wave_reduce(a, 2);
      } else if (fn == 1) {
        v = wave_reduce(a, 0) / 4000.f - wave_reduce(b, 1) + 1.f;
      } else if (fn == 3) {
        const float sa = wave_reduce(a, 0), sb = wave_reduce(b, 0);
        v = -20.f * expf(-0.2f * sqrtf(sa / (float)L)) - expf(sb / (float)L) + 20.f + 2.718281828459045f;
      } else {
        v = wave_reduce(a, 0);
      }
      gk += v;
    }
    if (lane == k) gout = gk / (float)(L * gr.nk);
  }
  if (lane < gr.ng) G[(int64_t)row * gr.ng + lane] = gout;
}

}  // namespace

void evx_lsmop_g(const float* X, float* G, int N, int D, int ng, int nk, int cosine, const int* start, const int* sublen, const int* func,
                 hipStream_t s) {
  LsmopGroups gr;
  gr.ng = ng;
  gr.nk = nk;
  gr.cosine = cosine;
  for (int k = 0; k < ng && k < LS_MAXG; ++k) {
    gr.start[k] = start[k];
    gr.sublen[k] = sublen[k];
    gr.func[k] = func[k];
  }
  lsmop_g_kernel<<<(N + 3) / 4, 256, 0, s>>>(X, G, N, D, gr);
}

void evx_dtlz(const float* X, float* F, int N, int D, int M, int variant, hipStream_t s) {
  const dim3 block(256), grid((N + 3) / 4);
  switch (variant) {
    case 1: dtlz_kernel<1><<<grid, block, 0, s>>>(X, F, N, D, M); break;
    case 2: dtlz_kernel<2><<<grid, block, 0, s>>>(X, F, N, D, M); break;
    case 3: dtlz_kernel<3><<<grid, block, 0, s>>>(X, F, N, D, M); break;
    default: dtlz_kernel<4><<<grid, block, 0, s>>>(X, F, N, D, M); break;
  }
}
