// K15 experiment: can the MFMA pipe speed up the per-individual policy mat-vec of the Ant rollout?
//
// The rollout (csrc/kernels/neuro.hip, ant_rollout_reg_kernel) runs one individual per wave; its layer 2 is
// a 64x64 mat-vec with per-individual weights (OpenES: W_i = W_c + sigma E_i, no operand shared between
// waves), so every matrix-core form has to pad a dimension.  This probe times one wave's dependent chain
// of L layer-2 steps  a <- tanh(W a)  three ways, on the same register-resident weights:
//   0  VALU: lane j owns column j of W; a broadcast through LDS (16 ds_read_b128) + 64 v_fma (the kernel's code)
//   1  v_mfma_f32_4x4x1_16b_f32: block b = rows 4b..4b+3, B = a[k] in all four columns (3/4 of every
//      instruction is redundant, result taken from c[lane & 3], layout-agnostic), 64 MFMAs, 4 chains
//   2  v_mfma_f32_16x16x4_f32: four 16-row tiles x 16 k-groups, B = a[k] in all 16 columns (15/16 padding),
//      64 MFMAs, results scattered back through LDS
//   3  split: k < KS on the MFMA pipe (form 1), k >= KS on the VALU, issued interleaved from the same wave
// and checks every form against a float64 host reference.
//
// build: hipcc --offload-arch=gfx950 -O3 -o tools/k15_mfma_probe tools/k15_mfma_probe.hip
// run:   tools/k15_mfma_probe [waves]   (prints one JSON line per form)
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                   \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));    \
      exit(1);                                                                     \
    }                                                                              \
  } while (0)

constexpr int WAVES = 4;  // waves per workgroup, one per SIMD (as in the rollout)

__device__ __forceinline__ float fast_tanh(float x) {
  const float e = __expf(-2.f * fabsf(x));
  return copysignf((1.f - e) / (1.f + e), x);
}

template <int FORM, int KS = 0>  // form 3: k < KS on the MFMA pipe
__global__ void __launch_bounds__(64 * WAVES) probe(const float* __restrict__ W, const float* __restrict__ a0, int L,
                                                    float* __restrict__ out, unsigned long long* __restrict__ cyc) {
  __shared__ __attribute__((aligned(16))) float buf_all[WAVES][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ind = blockIdx.x * WAVES + wv;
  float* buf = buf_all[wv];
  const float* Wi = W + (size_t)ind * 64 * 64;  // row-major W[out][in]
  float w[64];
  if (FORM == 2) {
    // tile m, k-group g: lane holds A[row = l % 16][k = l / 16] of W[16m + row][4g + k]
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int g = 0; g < 16; ++g) w[m * 16 + g] = Wi[(16 * m + (lane & 15)) * 64 + 4 * g + (lane >> 4)];
  } else {
#pragma unroll
    for (int k = 0; k < 64; ++k) w[k] = Wi[lane * 64 + k];  // lane = output row
  }
  float a = a0[(size_t)ind * 64 + lane];
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int t = 0; t < L; ++t) {
    buf[lane] = a;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float y;
    if (FORM == 0) {
      float c[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float4 v = reinterpret_cast<const float4*>(buf)[i];
        c[0] = fmaf(v.x, w[4 * i], c[0]);
        c[1] = fmaf(v.y, w[4 * i + 1], c[1]);
        c[2] = fmaf(v.z, w[4 * i + 2], c[2]);
        c[3] = fmaf(v.w, w[4 * i + 3], c[3]);
      }
      y = (c[0] + c[1]) + (c[2] + c[3]);
    } else if (FORM == 1) {
      f4 c[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float4 v = reinterpret_cast<const float4*>(buf)[i];
        c[0] = __builtin_amdgcn_mfma_f32_4x4x1f32(w[4 * i], v.x, c[0], 0, 0, 0);
        c[1] = __builtin_amdgcn_mfma_f32_4x4x1f32(w[4 * i + 1], v.y, c[1], 0, 0, 0);
        c[2] = __builtin_amdgcn_mfma_f32_4x4x1f32(w[4 * i + 2], v.z, c[2], 0, 0, 0);
        c[3] = __builtin_amdgcn_mfma_f32_4x4x1f32(w[4 * i + 3], v.w, c[3], 0, 0, 0);
      }
      const int r = lane & 3;
      y = (c[0][r] + c[1][r]) + (c[2][r] + c[3][r]);
    } else if (FORM == 2) {
      f4 c[4] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
#pragma unroll
      for (int g = 0; g < 16; ++g) {
        const float b = buf[4 * g + (lane >> 4)];
#pragma unroll
        for (int m = 0; m < 4; ++m) c[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(w[m * 16 + g], b, c[m], 0, 0, 0);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      // tile m: lane l holds rows 4 (l / 16) + v of every column (all columns equal)
      if ((lane & 15) == 0) {
#pragma unroll
        for (int m = 0; m < 4; ++m)
#pragma unroll
          for (int v = 0; v < 4; ++v) buf[16 * m + 4 * (lane >> 4) + v] = c[m][v];
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
      y = buf[lane];
      __builtin_amdgcn_wave_barrier();
    } else {
      f4 c[2] = {{0.f, 0.f, 0.f, 0.f}, {0.f, 0.f, 0.f, 0.f}};
      float d[2] = {0.f, 0.f};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float4 v = reinterpret_cast<const float4*>(buf)[i];
        const float vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = 4 * i + q;
          if (k < KS)
            c[q & 1] = __builtin_amdgcn_mfma_f32_4x4x1f32(w[k], vv[q], c[q & 1], 0, 0, 0);
          else
            d[q & 1] = fmaf(vv[q], w[k], d[q & 1]);
        }
      }
      const int r = lane & 3;
      y = (c[0][r] + c[1][r]) + (d[0] + d[1]);
    }
    a = fast_tanh(y);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[(size_t)ind * 64 + lane] = a;
  if (lane == 0) cyc[ind] = t1 - t0;
}

template <int FORM, int KS = 0>
static void run(const char* name, int nw, int L, int Lc, const float* dW, const float* da0, float* dout,
                unsigned long long* dcyc, const std::vector<double>& ref) {
  const int grid = nw / WAVES;
  hipLaunchKernelGGL((probe<FORM, KS>), dim3(grid), dim3(64 * WAVES), 0, 0, dW, da0, Lc, dout, dcyc);  // check + warm-up
  CHECK(hipDeviceSynchronize());
  std::vector<float> chk((size_t)nw * 64);
  CHECK(hipMemcpy(chk.data(), dout, chk.size() * 4, hipMemcpyDeviceToHost));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((probe<FORM, KS>), dim3(grid), dim3(64 * WAVES), 0, 0, dW, da0, L, dout, dcyc);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<unsigned long long> cyc(nw);
  CHECK(hipMemcpy(cyc.data(), dcyc, cyc.size() * 8, hipMemcpyDeviceToHost));
  double err = 0.0, cmax = 0.0;
  for (size_t i = 0; i < ref.size(); ++i) err = fmax(err, fabs(chk[i] - ref[i]));
  for (int i = 0; i < nw; ++i) cmax = fmax(cmax, (double)cyc[i]);
  printf("{\"form\": \"%s\", \"waves\": %d, \"steps\": %d, \"ns_per_step\": %.2f, \"memtime_ticks_per_step\": %.1f, "
         "\"max_abs_err_%d_steps\": %.3g}\n",
         name, nw, L, ms * 1e6 / L, cmax / L, Lc, err);
}

int main(int argc, char** argv) {
  const int nw = argc > 1 ? atoi(argv[1]) : 64;
  const int L = 2000, Lc = 6;
  if (nw % WAVES) return 1;
  std::vector<float> W((size_t)nw * 4096), a0((size_t)nw * 64);
  unsigned s = 12345u;
  auto rnd = [&]() { s = s * 1664525u + 1013904223u; return ((s >> 8) * (1.f / 16777216.f)) * 2.f - 1.f; };
  for (auto& x : W) x = rnd() * 0.3f;
  for (auto& x : a0) x = rnd();
  // float64 reference of the same chain
  const int nref = nw < 64 ? nw : 64;  // the host reference covers the first 64 waves
  std::vector<double> ref((size_t)nref * 64);
  for (int n = 0; n < nref; ++n) {
    std::vector<double> a(64), y(64);
    for (int j = 0; j < 64; ++j) a[j] = a0[(size_t)n * 64 + j];
    for (int t = 0; t < Lc; ++t) {
      for (int i = 0; i < 64; ++i) {
        double acc = 0.0;
        for (int k = 0; k < 64; ++k) acc += (double)W[(size_t)n * 4096 + i * 64 + k] * a[k];
        y[i] = acc;
      }
      for (int i = 0; i < 64; ++i) a[i] = std::tanh(y[i]);
    }
    for (int j = 0; j < 64; ++j) ref[(size_t)n * 64 + j] = a[j];
  }
  float *dW, *da0, *dout;
  unsigned long long* dcyc;
  CHECK(hipMalloc(&dW, W.size() * 4));
  CHECK(hipMalloc(&da0, a0.size() * 4));
  CHECK(hipMalloc(&dout, a0.size() * 4));
  CHECK(hipMalloc(&dcyc, nw * 8));
  CHECK(hipMemcpy(dW, W.data(), W.size() * 4, hipMemcpyHostToDevice));
  CHECK(hipMemcpy(da0, a0.data(), a0.size() * 4, hipMemcpyHostToDevice));
  run<0>("valu", nw, L, Lc, dW, da0, dout, dcyc, ref);
  run<1>("mfma_4x4x1_16b", nw, L, Lc, dW, da0, dout, dcyc, ref);
  run<2>("mfma_16x16x4", nw, L, Lc, dW, da0, dout, dcyc, ref);
  run<3, 16>("split_mfma16_valu48", nw, L, Lc, dW, da0, dout, dcyc, ref);
  run<3, 24>("split_mfma24_valu40", nw, L, Lc, dW, da0, dout, dcyc, ref);
  run<3, 32>("split_mfma32_valu32", nw, L, Lc, dW, da0, dout, dcyc, ref);
  return 0;
}
