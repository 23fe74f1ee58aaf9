// Lone-wave VALU issue probe: is a packed f32 FMA (v_pk_fma_f32, two FMAs per lane) as cheap to
// issue as a scalar v_fma_f32 when one wave owns its SIMD?  That is the regime of the Ant rollout
// (ant_rollout_reg_kernel: one wave per SIMD at pop 1024, issue-bound at ~4.4 cycles per VALU
// instruction, profiles/NOTES.md "lone-wave latency").  One 64-lane wave, s_memtime around a loop
// of 32 instructions per trip; prints cycles per instruction for each mode.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/probe_pk tools/probe_pk_f32.hip && /tmp/probe_pk
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ void __launch_bounds__(64) probe(float* out, unsigned long long* cyc, int iters) {
  const float l = (float)threadIdx.x * 1e-3f;
  f2 a[8], b = {1.0001f, 0.9999f}, c = {1e-4f, -1e-4f};
  float s[8], sb = 1.0001f, sc = 1e-4f;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    a[i] = f2{l + i, l - i};
    s[i] = l + i;
  }
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        if constexpr (MODE == 0) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[i]) : "v"(sb), "v"(sc));
        if constexpr (MODE == 1) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        if constexpr (MODE == 2) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a[i]) : "v"(b));
        if constexpr (MODE == 3) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[0]) : "v"(sb), "v"(sc));
        if constexpr (MODE == 4) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(a[0]) : "v"(b), "v"(c));
        // op_sel_hi:[1,0,1]: src1's low dword feeds both halves (a lane scalar broadcast into the pair)
        if constexpr (MODE == 5) asm volatile("v_pk_fma_f32 %0, %0, %1, %2 op_sel_hi:[1,0,1]" : "+v"(a[i]) : "v"(b), "v"(c));
        if constexpr (MODE == 6) asm volatile("v_add_f32 %0, %0, %1" : "+v"(s[i]) : "v"(sc));
        if constexpr (MODE == 7) asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a[i]) : "v"(c));
        // dependent scalar chain with two interleaved chains (latency vs issue)
        if constexpr (MODE == 8) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(s[i & 1]) : "v"(sb), "v"(sc));
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) acc += a[i].x + a[i].y + s[i];
  out[threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

template <int MODE>
static double run(float* out, unsigned long long* cyc, int iters) {
  unsigned long long h = 0;
  probe<MODE><<<1, 64>>>(out, cyc, iters);  // warm
  probe<MODE><<<1, 64>>>(out, cyc, iters);
  (void)hipMemcpy(&h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  return (double)h / (iters * 32.0);
}

int main() {
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 64 * sizeof(float));
  (void)hipMalloc(&cyc, sizeof(unsigned long long));
  const int it = 20000;
  // s_memtime ticks at the shader clock on gfx950 (MI355X_MICROARCH.md constants table)
  printf("v_fma_f32 x8 independent      %.2f cyc/instr\n", run<0>(out, cyc, it));
  printf("v_pk_fma_f32 x8 independent   %.2f cyc/instr\n", run<1>(out, cyc, it));
  printf("v_pk_mul_f32 x8 independent   %.2f cyc/instr\n", run<2>(out, cyc, it));
  printf("v_fma_f32 one dependent chain %.2f cyc/instr\n", run<3>(out, cyc, it));
  printf("v_pk_fma_f32 one chain        %.2f cyc/instr\n", run<4>(out, cyc, it));
  printf("v_pk_fma_f32 broadcast src1   %.2f cyc/instr\n", run<5>(out, cyc, it));
  printf("v_add_f32 x8 independent      %.2f cyc/instr\n", run<6>(out, cyc, it));
  printf("v_pk_add_f32 x8 independent   %.2f cyc/instr\n", run<7>(out, cyc, it));
  printf("v_fma_f32 two chains          %.2f cyc/instr\n", run<8>(out, cyc, it));
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
