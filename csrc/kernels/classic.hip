// Fused row-reduction evaluation of the classic benchmark functions (K5).
// One wave64 per row; lanes stride the row with 16-B loads when d % 4 == 0, the
// per-lane partials are reduced with DPP/shuffle, lane 0 writes the fitness.
// Memory-bound: (N·d·4) bytes read once, N·4 written.
#include "evoxmi_common.h"

namespace {

constexpr float PI_F = 3.14159265358979323846f;

// per-element accumulate for function F; acc0/acc1 = running sums (or product)
template <int F>
__device__ __forceinline__ void accum(float x, float xn, int j, float c, float& s0, float& s1) {
  if (F == 0) {  // sphere
    s0 += x * x;
  } else if (F == 1) {  // ackley: mean(x^2), mean(cos(c x))
    s0 += x * x;
    s1 += cosf(c * x);
  } else if (F == 2) {  // rastrigin
    s0 += x * x - 10.f * cosf(2.f * PI_F * x);
  } else if (F == 4) {  // griewank: sum and log|prod| via product in s1
    s0 += x * x;
    s1 *= cosf(x / sqrtf((float)(j + 1)));
  } else if (F == 5) {  // schwefel
    s0 += x * sinf(sqrtf(fabsf(x)));
  } else if (F == 6) {  // ellipsoid
    s0 += (float)(j + 1) * x * x;
  }
}

template <int F>
__global__ void __launch_bounds__(256) classic_kernel(const float* __restrict__ X, float* __restrict__ out, int N, int D,
                                                      float a, float b, float c) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  if (row >= N) return;
  const float* x = X + (int64_t)row * D;
  float s0 = 0.f, s1 = (F == 4) ? 1.f : 0.f;
  if (F == 3) {  // rosenbrock needs neighbours
    for (int j = lane; j < D - 1; j += 64) {
      float xi = x[j], xn = x[j + 1];
      float t = xn - xi * xi, u = xi - 1.f;
      s0 += 100.f * t * t + u * u;
    }
  } else if ((D & 3) == 0) {
    const float4* x4 = reinterpret_cast<const float4*>(x);
    for (int q = lane; q < (D >> 2); q += 64) {
      float4 v = x4[q];
      int j = q << 2;
      accum<F>(v.x, 0.f, j, c, s0, s1);
      accum<F>(v.y, 0.f, j + 1, c, s0, s1);
      accum<F>(v.z, 0.f, j + 2, c, s0, s1);
      accum<F>(v.w, 0.f, j + 3, c, s0, s1);
    }
  } else {
    for (int j = lane; j < D; j += 64) accum<F>(x[j], 0.f, j, c, s0, s1);
  }
  s0 = evx::wave_sum(s0);
  if (F == 1) s1 = evx::wave_sum(s1);
  if (F == 4) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) s1 *= __shfl_xor(s1, o, 64);
  }
  if (lane == 0) {
    float f;
    if (F == 0 || F == 3 || F == 6) f = s0;
    else if (F == 1) f = -a * expf(-b * sqrtf(s0 / D)) - expf(s1 / D) + a + 2.718281828459045f;
    else if (F == 2) f = 10.f * D + s0;
    else if (F == 4) f = s0 / 4000.f - s1 + 1.f;
    else f = 418.9828872724338f * D - s0;  // schwefel
    out[row] = f;
  }
}

}  // namespace

void evx_classic_eval(const float* X, float* out, int N, int D, int func, float a, float b, float c, hipStream_t s) {
  dim3 block(256);
  dim3 grid((N + 3) / 4);
  switch (func) {
    case 0: classic_kernel<0><<<grid, block, 0, s>>>(X, out, N, D, a, b, c); break;
    case 1: classic_kernel<1><<<grid, block, 0, s>>>(X, out, N, D, a, b, c); break;
    case 2: classic_kernel<2><<<grid, block, 0, s>>>(X, out, N, D, a, b, c); break;
    case 3: classic_kernel<3><<<grid, block, 0, s>>>(X, out, N, D, a, b, c); break;
    case 4: classic_kernel<4><<<grid, block, 0, s>>>(X, out, N, D, a, b, c); break;
    case 5: classic_kernel<5><<<grid, block, 0, s>>>(X, out, N, D, a, b, c); break;
    default: classic_kernel<6><<<grid, block, 0, s>>>(X, out, N, D, a, b, c); break;
  }
}
