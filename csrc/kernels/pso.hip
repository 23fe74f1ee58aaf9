// Fused PSO tell (K7): pbest select + velocity/position update + clip in one pass.
// rp / rg are regenerated from Philox counters (element index = row*d + col, the
// same words evoxmi.ops.random.uniform produces), so no (N, d) noise is stored.
// Each thread owns 4 consecutive elements = one Philox block per key.
#include "evoxmi_common.h"

namespace {

// one element's update, shared by both kernels so the column-block variant rounds exactly
// like the unsharded one
__device__ __forceinline__ void pso_elem(int64_t i, int r, int c, uint32_t up, uint32_t ug, const float* __restrict__ pop,
                                         const float* __restrict__ vel, const float* __restrict__ lbl,
                                         const float* __restrict__ lbf, const float* __restrict__ fit,
                                         const float* __restrict__ gbl, float w, float phip, float phig,
                                         const float* __restrict__ lb, const float* __restrict__ ub, float* __restrict__ opop,
                                         float* __restrict__ ovel, float* __restrict__ olbl, float* __restrict__ olbf) {
  // explicit FMA order, no compiler contraction: the same rounding in every kernel that inlines it
#pragma clang fp contract(off)
  const float x = pop[i];
  const bool better = lbf[r] > fit[r];
  const float lb_loc = better ? x : lbl[i];
  const float social = (phig * evx::u24(ug)) * (gbl[c] - x);
  const float v = fmaf(w, vel[i], fmaf(phip * evx::u24(up), lb_loc - x, social));
  opop[i] = fminf(fmaxf(x + v, lb[c]), ub[c]);
  ovel[i] = v;
  olbl[i] = lb_loc;
  if (c == 0) olbf[r] = fminf(lbf[r], fit[r]);
}

__global__ void __launch_bounds__(256) pso_kernel(const float* __restrict__ pop, const float* __restrict__ vel,
                                                  const float* __restrict__ lbl, const float* __restrict__ lbf,
                                                  const float* __restrict__ fit, const float* __restrict__ gbl,
                                                  const int64_t* __restrict__ kp, const int64_t* __restrict__ kg,
                                                  float w, float phip, float phig, const float* __restrict__ lb,
                                                  const float* __restrict__ ub, float* __restrict__ opop,
                                                  float* __restrict__ ovel, float* __restrict__ olbl,
                                                  float* __restrict__ olbf, int N, int D) {
  uint32_t p0, p1, g0, g1;
  evx::load_key(kp, p0, p1);
  evx::load_key(kg, g0, g1);
  const int64_t total = (int64_t)N * D;
  const int64_t nb = (total + 3) >> 2;
  for (int64_t b = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; b < nb; b += (int64_t)gridDim.x * blockDim.x) {
    evx::u4 wp = evx::philox_block((uint64_t)b, p0, p1);
    evx::u4 wg = evx::philox_block((uint64_t)b, g0, g1);
    uint32_t rpw[4] = {wp.x, wp.y, wp.z, wp.w};
    uint32_t rgw[4] = {wg.x, wg.y, wg.z, wg.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      int64_t i = (b << 2) + j;
      if (i >= total) break;
      int r = (int)(i / D), c = (int)(i - (int64_t)r * D);
      pso_elem(i, r, c, rpw[j], rgw[j], pop, vel, lbl, lbf, fit, gbl, w, phip, phig, lb, ub, opop, ovel, olbl, olbf);
    }
  }
}

// Column-block variant (decision-axis state sharding, P2): this rank holds columns
// [col0, col0 + D) of a D_tot-dimensional swarm; element (r, c) draws the Philox word of global
// index r·D_tot + col0 + c, so every rank updates its block exactly as the unsharded swarm.
__global__ void __launch_bounds__(256) pso_cols_kernel(const float* __restrict__ pop, const float* __restrict__ vel,
                                                       const float* __restrict__ lbl, const float* __restrict__ lbf,
                                                       const float* __restrict__ fit, const float* __restrict__ gbl,
                                                       const int64_t* __restrict__ kp, const int64_t* __restrict__ kg,
                                                       float w, float phip, float phig, const float* __restrict__ lb,
                                                       const float* __restrict__ ub, float* __restrict__ opop,
                                                       float* __restrict__ ovel, float* __restrict__ olbl,
                                                       float* __restrict__ olbf, int N, int D, int col0, int Dtot) {
  uint32_t p0, p1, g0, g1;
  evx::load_key(kp, p0, p1);
  evx::load_key(kg, g0, g1);
  const int64_t total = (int64_t)N * D;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / D), c = (int)(i - (int64_t)r * D);
    const uint64_t gi = (uint64_t)r * Dtot + col0 + c;
    const evx::u4 wp = evx::philox_block(gi >> 2, p0, p1), wg = evx::philox_block(gi >> 2, g0, g1);
    const int j = (int)(gi & 3);
    const uint32_t up = j == 0 ? wp.x : (j == 1 ? wp.y : (j == 2 ? wp.z : wp.w));
    const uint32_t ug = j == 0 ? wg.x : (j == 1 ? wg.y : (j == 2 ? wg.z : wg.w));
    pso_elem(i, r, c, up, ug, pop, vel, lbl, lbf, fit, gbl, w, phip, phig, lb, ub, opop, ovel, olbl, olbf);
  }
}

}  // namespace

void evx_pso_update_cols(const float* pop, const float* vel, const float* lbl, const float* lbf, const float* fit,
                         const float* gbl, const int64_t* kp, const int64_t* kg, float w, float phip, float phig,
                         const float* lb, const float* ub, float* opop, float* ovel, float* olbl, float* olbf, int N, int D,
                         int col0, int Dtot, hipStream_t s) {
  int64_t total = (int64_t)N * D;
  int grid = (int)((total + 255) / 256);
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  pso_cols_kernel<<<grid, 256, 0, s>>>(pop, vel, lbl, lbf, fit, gbl, kp, kg, w, phip, phig, lb, ub, opop, ovel, olbl, olbf, N, D, col0,
                                       Dtot);
}

void evx_pso_update(const float* pop, const float* vel, const float* lbl, const float* lbf, const float* fit,
                    const float* gbl, const int64_t* kp, const int64_t* kg, float w, float phip, float phig,
                    const float* lb, const float* ub, float* opop, float* ovel, float* olbl, float* olbf, int N, int D,
                    hipStream_t s) {
  int64_t nb = ((int64_t)N * D + 3) / 4;
  int grid = (int)((nb + 255) / 256);
  if (grid > 8192) grid = 8192;
  if (grid < 1) grid = 1;
  pso_kernel<<<grid, 256, 0, s>>>(pop, vel, lbl, lbf, fit, gbl, kp, kg, w, phip, phig, lb, ub, opop, ovel, olbl, olbf, N, D);
}
