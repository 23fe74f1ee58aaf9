// Standalone timing probe for gemm_ks.hip variants (compile-time macros EVX_KS_DEPTH,
// EVX_KS_FAKE_LOADS, EVX_KS_NO_LOADS): hipcc --offload-arch=gfx950 -O3 -I csrc/include [-D...] tools/gemm_ks_probe.cpp
// Every case runs in both precision modes (bf16x6 split products, f32 MFMA).
#include "../csrc/kernels/gemm_ks.hip"
#include <cstdio>
#include <vector>
#include <cstdlib>

static float* dev_rand(size_t n) {
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = (float)rand() / (float)RAND_MAX - 0.5f;
  float* d;
  (void)hipMalloc(&d, n * 4);
  (void)hipMemcpy(d, h.data(), n * 4, hipMemcpyHostToDevice);
  return d;
}

static double run(int M, int N, int K, int akc, int bkc, int mode, int tile, int reps) {
  float* A = dev_rand((size_t)M * K);
  float* B = dev_rand((size_t)N * K);
  float* C;
  (void)hipMalloc(&C, (size_t)M * N * 4);
  EvxGemmKs a{};
  a.A = A; a.lda = akc ? K : M;
  a.B = B; a.ldb = bkc ? K : N;
  a.C = C; a.ldc = N;
  a.M = M; a.N = N; a.K = K; a.a_kc = akc; a.b_kc = bkc; a.mode = mode; a.alpha = 1.f; a.c_vec4 = 1;
  evx_gemm_ks_set_tile(tile);
  hipStream_t s = 0;
  for (int i = 0; i < 10; ++i) evx_gemm_ks(a, s);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0, s);
  for (int i = 0; i < reps; ++i) evx_gemm_ks(a, s);
  (void)hipEventRecord(e1, s);
  (void)hipEventSynchronize(e1);
  float ms;
  (void)hipEventElapsedTime(&ms, e0, e1);
  (void)hipFree(A); (void)hipFree(B); (void)hipFree(C);
  return ms * 1e3 / reps;
}

int main() {
  struct Case { const char* name; int M, N, K, akc, bkc, mode, tile; };
  Case cs[] = {
    {"1000^3 NT full t4", 1000, 1000, 1000, 1, 1, 0, 4},
    {"1000^3 NT full t3", 1000, 1000, 1000, 1, 1, 0, 3},
    {"1000^3 NT full t2", 1000, 1000, 1000, 1, 1, 0, 2},
    {"1000^3 NT sym t3", 1000, 1000, 1000, 1, 1, 1, 3},
    {"1000^3 NT sym t2", 1000, 1000, 1000, 1, 1, 1, 2},
    {"1000^3 NN full t4", 1000, 1000, 1000, 1, 0, 0, 4},
    {"1000^3 TN sym t3", 1000, 1000, 1000, 0, 0, 1, 3},
    {"10000x1000x1000 NT t4", 10000, 1000, 1000, 1, 1, 0, 4},
    {"10000x1000x1000 NT t3", 10000, 1000, 1000, 1, 1, 0, 3},
    {"10000x1000x1000 NT t8", 10000, 1000, 1000, 1, 1, 0, 8},
    {"1000x1000x5000 TN sym t3", 1000, 1000, 5000, 0, 0, 1, 3},
    {"1000x1000x5000 NT sym t3", 1000, 1000, 5000, 1, 1, 1, 3},
    {"2048^3 NT full t4", 2048, 2048, 2048, 1, 1, 0, 4},
  };
  for (auto& c : cs) {
    for (int prec : {2, 1, 0}) {
      evx_gemm_ks_set_prec(prec);
      const double us = run(c.M, c.N, c.K, c.akc, c.bkc, c.mode, c.tile, 50);
      double flops = 2.0 * c.M * c.N * c.K;
      printf("%-26s %-3s %9.2f us  %7.1f TF/s (full-product equivalent)\n", c.name, prec == 2 ? "x6w" : prec ? "x6" : "f32", us, flops / us / 1e6);
    }
  }
  return 0;
}
