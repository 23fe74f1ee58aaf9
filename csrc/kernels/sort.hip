// Single-workgroup LDS bitonic argsort (K19) for populations up to 16384.
// Keys are f32 fitness values mapped to order-preserving u32 (NaN → +inf side, i.e.
// sorted last like torch.sort), packed with the 32-bit index into one u64 so that a
// single 64-bit compare orders by (key, index): deterministic and equal to a stable
// sort.  The whole array lives in LDS (16384 x 8 B = 128 KiB of the 160 KiB per CU);
// 1024 threads, one barrier per bitonic stage, stages with stride < 64 are done with
// wave shuffles... kept in LDS here for simplicity (≈105 stages at n=16384).
#include "evoxmi_common.h"

namespace {

__device__ __forceinline__ uint32_t f2ord(float f) {
  uint32_t u = __float_as_uint(f);
  if (f != f) return 0xFFFFFFFFu;  // NaN last
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float ord2f(uint32_t o) {
  uint32_t u = (o & 0x80000000u) ? (o & 0x7FFFFFFFu) : ~o;
  return __uint_as_float(u);
}

template <int LOGN>
__global__ void __launch_bounds__(1024) bitonic_argsort_kernel(const float* __restrict__ keys, int n, int descending,
                                                               float* __restrict__ out_keys, int32_t* __restrict__ out_idx) {
  constexpr int NP = 1 << LOGN;
  __shared__ unsigned long long s[NP];
  for (int i = threadIdx.x; i < NP; i += blockDim.x) {
    unsigned long long v;
    if (i < n) {
      float k = keys[i];
      // torch semantics: NaN is the largest value (last ascending, first descending)
      uint32_t o = (k != k) ? (descending ? 0u : 0xFFFFFFFFu) : f2ord(descending ? -k : k);
      v = ((unsigned long long)o << 32) | (uint32_t)i;
    } else {
      v = 0xFFFFFFFFFFFFFFFFull;  // padding sorts last
    }
    s[i] = v;
  }
  __syncthreads();
  for (int k = 2; k <= NP; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < NP / 2; t += blockDim.x) {
        int i = ((t & ~(j - 1)) << 1) | (t & (j - 1));  // lower element of the pair
        int p = i | j;
        bool up = ((i & k) == 0);
        unsigned long long a = s[i], b = s[p];
        if ((a > b) == up) {
          s[i] = b;
          s[p] = a;
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < n; i += blockDim.x) {
    unsigned long long v = s[i];
    const int32_t src = (int32_t)(v & 0xFFFFFFFFu);
    if (out_keys) out_keys[i] = keys[src];
    out_idx[i] = src;
  }
}

}  // namespace

int evx_argsort_max_n() { return 16384; }

void evx_argsort(const float* keys, int n, int descending, float* out_keys, int32_t* out_idx, hipStream_t s) {
  int logn = 10;
  while ((1 << logn) < n) ++logn;
  switch (logn) {
    case 10: bitonic_argsort_kernel<10><<<1, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
    case 11: bitonic_argsort_kernel<11><<<1, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
    case 12: bitonic_argsort_kernel<12><<<1, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
    case 13: bitonic_argsort_kernel<13><<<1, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
    default: bitonic_argsort_kernel<14><<<1, 1024, 0, s>>>(keys, n, descending, out_keys, out_idx); break;
  }
}
