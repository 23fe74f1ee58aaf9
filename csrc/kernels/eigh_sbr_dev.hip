// Device-controlled schedule of the sorted-block-refinement eigensolver (K4, round 3).
//
// The host-driven solver (evoxmi/ops/sbr.py:eigh_warm) reads the convergence statistics
// back after every iteration (or once per planned solve) to choose the next iteration's
// variant — Newton–Schulz or not, damping, far step, Taylor order, local threshold — and
// when to stop.  That split every CMA-ES generation into graph segments around a host
// phase.  Here the same decisions run on the device: the solve is a fixed schedule of K
// iterations captured once into the generation's graph, every kernel of an iteration reads
// a control word and returns at once when its variant is off (or the solve has converged),
// and one single-workgroup kernel per iteration (sbr_dev_ctrl_kernel) reduces the stats
// partials that the Bᵀ C B GEMM wrote in its epilogue and writes the next iteration's
// control words.  No host read, no plan, nothing outside the checkpointed state.
//
// Control words per iteration j (int32[8]):
//   0 skip_all   1 skip_far   2 skip_damp   3 skip_x3 (order 4)   4 sel6 (order 6)
//   5 skip_ns    6 sel_ns (Bq·V lands in the Newton–Schulz input)   7 skip_copy (near-only: Bq → B)
// Persistent words st[8]: 0 stopped, 1 fallback (diverged), 2 refinement iterations run,
//   3 last_far, 4 theta sticky, 5 keep (0 ⇒ restore the warm-start basis), 6 converged.
#include "evoxmi_common.h"
#include "evoxmi_sbr.h"
#include <float.h>
#include <math.h>

namespace {

struct SbrDevParams {
  float tol, ns_kappa, damp_kappa, t4_kappa, near_only;
  float theta0;  // local far threshold factor once κ ≤ theta_kappa (0: only after a stall)
  float theta_kappa;
  int ns_iters;
  int lean_from;  // slots ≥ lean_from carry no damping / Newton–Schulz / X³ kernels (order 4, undamped)
};

__device__ __forceinline__ void rel_kappa(const double* h, double& r, double& k) {
  const double off = fmax(h[0], 0.0), dg = h[1], mn = h[2], mx = h[3];
  r = dg > 0.0 ? sqrt(off / dg) : (double)NAN;
  k = mx > mn ? sqrt(off) / (mx - mn) : (double)INFINITY;
}

// Taylor operands of exp(αX) for the order the control word selects (sel6), with M of
// exp(−αX) (the transposed product, ops/sbr.py:expm_t_device).  V2 != null: when this
// iteration's damping ran (ctrl[2] == 0) every workgroup forms α from its power-step vectors
// itself and workgroup 0 stores it — the damping's own single-workgroup final launch is gone.
__global__ void __launch_bounds__(256) sbr_dev_prep_kernel(const float* __restrict__ X, const float* __restrict__ X2,
                                                           const float* __restrict__ X3, int n, float* __restrict__ alpha,
                                                           float* __restrict__ P, float* __restrict__ MT, const int* __restrict__ ctrl,
                                                           const float* __restrict__ V2, const float* __restrict__ V3, float tau) {
  if (ctrl[1]) return;
  const bool six = ctrl[4] != 0;
  float a;
  if (V2 && ctrl[2] == 0) {
    a = evx_sbr_damping_alpha(V2, V3, n, tau);
    if (blockIdx.x == 0 && threadIdx.x == 0) alpha[0] = a;
  } else {
    a = alpha[0];
  }
  const float a2 = a * a, a3 = a2 * a;
  // rows over the grid, columns over the threads (float4 when n % 4 == 0): no per-element
  // 64-bit division (the flat-index form spent most of its time in the i = e / n expansion)
  const bool v4 = (n & 3) == 0;
  const int nc = v4 ? n >> 2 : n;
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const int64_t r = (int64_t)i * n;
    for (int c = threadIdx.x; c < nc; c += blockDim.x) {
      const int w = v4 ? 4 : 1;
      float xs[4] = {}, x2s[4] = {}, x3s[4] = {};
      if (v4) {
        const float4 x = reinterpret_cast<const float4*>(X + r)[c], y = reinterpret_cast<const float4*>(X2 + r)[c];
        xs[0] = x.x; xs[1] = x.y; xs[2] = x.z; xs[3] = x.w;
        x2s[0] = y.x; x2s[1] = y.y; x2s[2] = y.z; x2s[3] = y.w;
        if (six) {
          const float4 z = reinterpret_cast<const float4*>(X3 + r)[c];
          x3s[0] = z.x; x3s[1] = z.y; x3s[2] = z.z; x3s[3] = z.w;
        }
      } else {
        xs[0] = X[r + c];
        x2s[0] = X2[r + c];
        if (six) x3s[0] = X3[r + c];
      }
      float ps[4], ms[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int j = c * w + q;
        const float x = a * xs[q], x2 = a2 * x2s[q];
        const float id = i == j ? 1.f : 0.f;
        if (six) {
          const float x3 = a3 * x3s[q];
          ps[q] = a3 * (x * (1.f / 24.f) + x2 * (1.f / 120.f) + x3 * (1.f / 720.f));
          ms[q] = id - x + 0.5f * x2 - x3 * (1.f / 6.f);
        } else {
          ps[q] = a2 * (x * (1.f / 6.f) + x2 * (1.f / 24.f));
          ms[q] = id - x + 0.5f * x2;
        }
      }
      if (v4) {
        reinterpret_cast<float4*>(P + r)[c] = make_float4(ps[0], ps[1], ps[2], ps[3]);
        reinterpret_cast<float4*>(MT + r)[c] = make_float4(ms[0], ms[1], ms[2], ms[3]);
      } else {
        P[r + c] = ps[0];
        MT[r + c] = ms[0];
      }
    }
  }
}

__global__ void __launch_bounds__(256) sbr_dev_copy_kernel(const float* __restrict__ src, float* __restrict__ dst, int64_t n,
                                                           const int* __restrict__ skip) {
  if (skip && *skip) return;
  const int64_t n4 = n / 4;
  const float4* s4 = reinterpret_cast<const float4*>(src);
  float4* d4 = reinterpret_cast<float4*>(dst);
  const int64_t g = blockIdx.x * (int64_t)blockDim.x + threadIdx.x, stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = g; e < n4; e += stride) d4[e] = s4[e];
  for (int64_t e = 4 * n4 + g; e < n; e += stride) dst[e] = src[e];
}

// j = −1: the initial Bᵀ C B; j ≥ 0: after iteration j.  One workgroup.
__global__ void __launch_bounds__(256) sbr_dev_ctrl_kernel(const double* __restrict__ part, int nparts, int j, int K,
                                                           double* __restrict__ hist, float* __restrict__ alpha,
                                                           float* __restrict__ theta, int* __restrict__ ctrl, int* __restrict__ st,
                                                           SbrDevParams prm, const float* __restrict__ A, int64_t lda, int n,
                                                           float* __restrict__ w_out, double* __restrict__ eig_stats,
                                                           float* __restrict__ w_init, double* __restrict__ log, int log_len,
                                                           int* __restrict__ log_count) {
  __shared__ double s[4][4];
  __shared__ int s_keep;
  const int t = threadIdx.x;
  const bool executed = j < 0 || ctrl[8 * j] == 0;
  double* hj1 = hist + 4 * (j + 1);
  if (executed) {
    double off = 0.0, dg = 0.0, mn = DBL_MAX, mx = -DBL_MAX;
    for (int i = t; i < nparts; i += 256) {
      off += part[4 * i];
      dg += part[4 * i + 1];
      mn = fmin(mn, part[4 * i + 2]);
      mx = fmax(mx, part[4 * i + 3]);
    }
    // wave reductions (no barrier), then the four wave results through LDS: one barrier
    // instead of the eight of a 256-wide tree (this kernel sits on the schedule's serial path)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      off += __shfl_xor(off, o);
      dg += __shfl_xor(dg, o);
      mn = fmin(mn, __shfl_xor(mn, o));
      mx = fmax(mx, __shfl_xor(mx, o));
    }
    if ((t & 63) == 0) {
      s[0][t >> 6] = off;
      s[1][t >> 6] = dg;
      s[2][t >> 6] = mn;
      s[3][t >> 6] = mx;
    }
    __syncthreads();
    if (t == 0) {
      hj1[0] = (s[0][0] + s[0][1]) + (s[0][2] + s[0][3]);
      hj1[1] = (s[1][0] + s[1][1]) + (s[1][2] + s[1][3]);
      hj1[2] = fmin(fmin(s[2][0], s[2][1]), fmin(s[2][2], s[2][3]));
      hj1[3] = fmax(fmax(s[3][0], s[3][1]), fmax(s[3][2], s[3][3]));
    }
  } else if (t < 4) {
    hj1[t] = hist[4 * j + t];
  }
  if (j < 0) {  // the warm-start diagonal: the result if the refinement has to be abandoned
    for (int i = t; i < n; i += 256) w_init[i] = A[(int64_t)i * lda + i];
  }
  __syncthreads();
  if (t == 0) {
    if (j < 0) {
      st[0] = 0;  // stopped
      st[1] = 0;  // fallback
      st[2] = 0;  // iterations run
      st[3] = 1;  // last_far
      st[4] = 0;  // theta sticky
      st[6] = 0;  // converged
      alpha[0] = 1.f;
    }
    double r, k;
    rel_kappa(hj1, r, k);
    if (j >= 0 && executed && !st[0]) {
      st[2] = j + 1;
      double rp, kp;
      rel_kappa(hist + 4 * j, rp, kp);
      const bool far_j = ctrl[8 * j + 1] == 0;
      if (!isfinite(r) || r > 1.5 * rp) {
        st[0] = 1;  // diverged: stop, restore the warm-start basis at the end
        st[1] = 1;
      } else {
        // an undamped far iteration close to the tolerance that barely helped: pairs in a
        // cluster denser than the global threshold assumes — local threshold from now on
        if (far_j && alpha[j + 1] >= 1.f && r < 100.0 * prm.tol && r > 0.6 * rp) st[4] = 1;
        st[3] = far_j ? 1 : 0;
      }
    }
    if (!st[0] && r <= prm.tol) {
      st[0] = 1;
      st[6] = 1;
    }
    const int nx = j + 1;
    if (nx < K) {
      int* c = ctrl + 8 * nx;
      if (st[0]) {
        c[0] = 1; c[1] = 1; c[2] = 1; c[3] = 1; c[4] = 0; c[5] = 1; c[6] = 0; c[7] = 1;
      } else {
        const float a_prev = alpha[nx];  // step size of the iteration just run (1 at the start)
        const bool lean = nx >= prm.lean_from;
        const bool ns = !lean && (nx < prm.ns_iters || a_prev < 1.f || k > prm.ns_kappa);
        const bool damp = !lean && (nx == 0 || k > prm.damp_kappa);
        const bool far = !(nx > 0 && r <= prm.near_only * prm.tol && st[3]);
        const bool six = !lean && !(k < prm.t4_kappa);
        c[0] = 0;
        c[1] = far ? 0 : 1;
        c[2] = (far && damp) ? 0 : 1;
        c[3] = (far && six) ? 0 : 1;
        c[4] = six ? 1 : 0;
        c[5] = (far && ns) ? 0 : 1;
        c[6] = ns ? 1 : 0;
        c[7] = far ? 1 : 0;
        // local far threshold: sticky after a stalled far iteration, or (theta0) once the far
        // step is small (κ ≤ theta_kappa: with larger steps the extra strongly coupled far pairs
        // rotated at once can make a cold-start iteration diverge)
        const bool th = st[4] || (prm.theta0 > 0.f && k <= prm.theta_kappa);
        theta[nx] = th ? (prm.theta0 > 0.f ? prm.theta0 : 1.f) : 0.f;
        alpha[nx + 1] = 1.f;  // the damping kernel of iteration nx overwrites it when it runs
      }
    }
    if (nx == K) {
      const bool fb = st[1] != 0;
      double rf, kf;
      rel_kappa(fb ? hist : hist + 4 * K, rf, kf);
      eig_stats[0] = rf;
      eig_stats[1] = 0.0;
      eig_stats[2] = (double)st[2];
      eig_stats[3] = fb ? 1.0 : 0.0;
      st[5] = fb ? 0 : 1;  // keep: the restore copy is skipped unless the refinement diverged
      if (log && log_len > 0) {  // per-solve history ring (read by benches after the timed loop)
        const int c = *log_count;
        double* o = log + 4 * (int64_t)(c % log_len);
        o[0] = eig_stats[0];
        o[1] = eig_stats[1];
        o[2] = eig_stats[2];
        o[3] = eig_stats[3];
        *log_count = c + 1;
      }
    }
    s_keep = st[1] ? 0 : 1;
  }
  __syncthreads();
  if (j + 1 == K) {
    const bool keep = s_keep != 0;
    for (int i = t; i < n; i += 256) w_out[i] = keep ? A[(int64_t)i * lda + i] : w_init[i];
  }
}

}  // namespace

void evx_sbr_dev_prep(const float* X, const float* X2, const float* X3, int n, float* alpha, float* P, float* MT, const int* ctrl,
                      hipStream_t s, const float* V2, const float* V3, float tau) {
  // a grid-stride loop over 256 workgroups: the schedule skips this kernel in most
  // iterations, and an empty launch costs in proportion to its workgroup count
  const int64_t total = (int64_t)n * n;
  int g = (int)((total + 255) / 256);
  if (g > 256) g = 256;
  sbr_dev_prep_kernel<<<g, 256, 0, s>>>(X, X2, X3, n, alpha, P, MT, ctrl, V2, V3, tau);
}

void evx_sbr_dev_copy(const float* src, float* dst, int64_t n, const int* skip, hipStream_t s) {
  int g = (int)((n / 4 + 255) / 256);
  if (g < 1) g = 1;
  if (g > 256) g = 256;  // mostly skipped: keep the empty launch small
  sbr_dev_copy_kernel<<<g, 256, 0, s>>>(src, dst, n, skip);
}

void evx_sbr_dev_ctrl(const double* part, int nparts, int j, int K, double* hist, float* alpha, float* theta, int* ctrl, int* st,
                      const float* prm6, int ns_iters, const float* A, int64_t lda, int n, float* w_out, double* eig_stats, float* w_init,
                      double* log, int log_len, int* log_count, hipStream_t s, int lean_from) {
  SbrDevParams p{prm6[0], prm6[1], prm6[2], prm6[3], prm6[4], prm6[5], prm6[6], ns_iters, lean_from};
  sbr_dev_ctrl_kernel<<<1, 256, 0, s>>>(part, nparts, j, K, hist, alpha, theta, ctrl, st, p, A, lda, n, w_out, eig_stats, w_init, log,
                                        log_len, log_count);
}
