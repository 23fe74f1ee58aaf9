// MFMA throughput / shader-clock probe: f32 16x16x4 MFMA chains (no memory traffic) on
// 1 or 256 workgroups, with s_memtime (shader clock) / s_memrealtime (100 MHz) deltas.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ void __launch_bounds__(256) mfma_loop(int iters, float* out, unsigned long long* clk) {
  f32x4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float a = threadIdx.x * 1e-3f, b = 1e-3f;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * 256 + threadIdx.x] = s;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main() {
  float* out;
  unsigned long long* clk;
  (void)hipMalloc(&out, 4096 * 256 * 4);
  (void)hipMalloc(&clk, 4096 * 16);
  const int iters = 20000;
  for (int grid : {1, 256, 512, 1024}) {
    for (int rep = 0; rep < 2; ++rep) {
      hipEvent_t e0, e1;
      (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
      (void)hipEventRecord(e0);
      mfma_loop<16><<<grid, 256>>>(iters, out, clk);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      unsigned long long h[2];
      (void)hipMemcpy(h, clk, 16, hipMemcpyDeviceToHost);
      const double flops = 2048.0 * 16 * iters * 4 * grid;  // per wave per MFMA 2048 FLOP, 4 waves/WG
      const double mhz = (double)h[0] / ((double)h[1] / 100.0);
      const double cyc_per_mfma = (double)h[0] / (16.0 * iters);
      printf("grid %5d: %8.3f ms  %7.1f TF/s  shader clk %6.0f MHz  %.1f clk per MFMA per wave\n", grid, ms, flops / ms / 1e9,
             mhz, cyc_per_mfma);
    }
  }
  return 0;
}
