// Host-side launchers implemented in csrc/kernels/*.hip (no torch dependency).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

void evx_philox_fill(float* out, int64_t n, const int64_t* key, int dist, int64_t elem_offset, hipStream_t s);
void evx_classic_eval(const float* X, float* out, int N, int D, int func, float a, float b, float c, hipStream_t s);
void evx_pso_update(const float* pop, const float* vel, const float* lbl, const float* lbf, const float* fit,
                    const float* gbl, const int64_t* kp, const int64_t* kg, float w, float phip, float phig,
                    const float* lb, const float* ub, float* opop, float* ovel, float* olbl, float* olbf, int N, int D,
                    hipStream_t s);
