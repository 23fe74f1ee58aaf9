// Shared device helpers for evoxmi HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define EVX_WAVE 64

namespace evx {

// ---------------------------------------------------------------- Philox4x32-10
// Same constants / round structure as evoxmi/ops/random.py (bit-identical words).
struct u4 { uint32_t x, y, z, w; };

__device__ __forceinline__ u4 philox4x32_10(u4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    uint32_t hi0 = __umulhi(0xD2511F53u, c.x), lo0 = 0xD2511F53u * c.x;
    uint32_t hi1 = __umulhi(0xCD9E8D57u, c.z), lo1 = 0xCD9E8D57u * c.z;
    c = u4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// block b of the "bits" domain (counter = (b_lo, b_hi, 0, 0))
__device__ __forceinline__ u4 philox_block(uint64_t b, uint32_t k0, uint32_t k1) {
  return philox4x32_10(u4{(uint32_t)b, (uint32_t)(b >> 32), 0u, 0u}, k0, k1);
}

__device__ __forceinline__ float u24(uint32_t w) {
  return ((float)(w >> 8) + 0.5f) * (1.0f / 16777216.0f);
}

// 4 normals from one block, Box-Muller on (x,y) and (z,w) — matches random.normal
__device__ __forceinline__ float4 normal4(u4 w) {
  float r0 = sqrtf(-2.0f * logf(u24(w.x)));
  float r1 = sqrtf(-2.0f * logf(u24(w.z)));
  float s0, c0, s1, c1;
  sincosf(6.283185307179586f * u24(w.y), &s0, &c0);
  sincosf(6.283185307179586f * u24(w.w), &s1, &c1);
  return make_float4(r0 * c0, r0 * s0, r1 * c1, r1 * s1);
}

__device__ __forceinline__ void load_key(const int64_t* key, uint32_t& k0, uint32_t& k1) {
  k0 = (uint32_t)key[0];
  k1 = (uint32_t)key[1];
}

// ---------------------------------------------------------------- wave reductions
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// block-wide sum; `scratch` holds >= blockDim/64 floats; result broadcast to all
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += scratch[i];
  return t;
}

// XCD-aware bijective remap of a 1-D block id (MI355X: 8 XCDs, round-robin dispatch).
// Consecutive logical tiles land on the same XCD so they share its L2.
__device__ __forceinline__ int xcd_remap(int bid, int nblocks) {
  const int NX = 8;
  int q = nblocks / NX, r = nblocks % NX;
  int xcd = bid % NX, idx = bid / NX;
  int base = (xcd < r) ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + idx;
}

}  // namespace evx

#define EVX_CHECK_LAUNCH() (void)hipGetLastError()
