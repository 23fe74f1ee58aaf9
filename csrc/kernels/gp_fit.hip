// Batched hyper-parameter fit of linear-kernel GP regressions (IM-MOEA inverse models).
//
// IM-MOEA (reference algorithms/mo/im_moea.py:284-330) fits, per partition × objective ×
// decision variable, a GP x_d = GP(f_m) with kernel k(f, f') = v·f·f' and Gaussian noise of
// standard deviation s, by 250 Adam steps (lr 1e-3) on the negative marginal likelihood of
// softplus-unconstrained (v, s) from v = s = 1.  With a rank-one kernel the likelihood is
// closed form in four sufficient statistics (a = Σf², b = Σf·x, c = Σx², n):
//   nll = ½(c − v b²/D)/s² + ½(n − 1) log s² + ½ log D + const,   D = s² + v a,
// so every model's optimisation is a scalar recurrence: one thread per model runs all 250
// steps in registers (float64), thousands of models in one launch.
// evoxmi/algorithms/mo/im_moea.py:linear_gp_fit holds the torch reference.
#include "evoxmi_common.h"

namespace {

__device__ __forceinline__ double softplus(double u) { return u > 30.0 ? u : log1p(exp(u)); }
__device__ __forceinline__ double sigmoid(double u) { return 1.0 / (1.0 + exp(-u)); }

__global__ void __launch_bounds__(256) linear_gp_fit_kernel(const double* __restrict__ a, const double* __restrict__ b,
                                                            const double* __restrict__ c, const double* __restrict__ n, int64_t models,
                                                            int steps, double lr, float* __restrict__ v_out, float* __restrict__ s2_out) {
  const int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x;
  if (i >= models) return;
  const double A = a[i], Bb = b[i], Cc = c[i], N = n[i];
  const double u0 = 0.5413248546129181;  // softplus⁻¹(1)
  double uv = u0, us = u0, mv = 0.0, ms = 0.0, vv = 0.0, vs = 0.0, b1t = 1.0, b2t = 1.0;
  for (int t = 0; t < steps; ++t) {
    const double v = softplus(uv), s = softplus(us), s2 = s * s;
    const double D = s2 + v * A;
    const double gv = -0.5 * Bb * Bb / (D * D) + 0.5 * A / D;
    const double gs2 = -0.5 * Cc / (s2 * s2) + 0.5 * v * Bb * Bb * (s2 + D) / (D * D * s2 * s2) + 0.5 * (N - 1.0) / s2 + 0.5 / D;
    const double g_uv = gv * sigmoid(uv), g_us = gs2 * 2.0 * s * sigmoid(us);
    b1t *= 0.9;
    b2t *= 0.999;
    mv = 0.9 * mv + 0.1 * g_uv;
    ms = 0.9 * ms + 0.1 * g_us;
    vv = 0.999 * vv + 0.001 * g_uv * g_uv;
    vs = 0.999 * vs + 0.001 * g_us * g_us;
    uv -= lr * (mv / (1.0 - b1t)) / (sqrt(vv / (1.0 - b2t)) + 1e-8);
    us -= lr * (ms / (1.0 - b1t)) / (sqrt(vs / (1.0 - b2t)) + 1e-8);
  }
  const double s = softplus(us);
  v_out[i] = (float)softplus(uv);
  s2_out[i] = (float)(s * s);
}

}  // namespace

void evx_linear_gp_fit(const double* a, const double* b, const double* c, const double* n, int64_t models, int steps, double lr,
                       float* v, float* s2, hipStream_t s) {
  if (models > 0) linear_gp_fit_kernel<<<(int)((models + 255) / 256), 256, 0, s>>>(a, b, c, n, models, steps, lr, v, s2);
}
