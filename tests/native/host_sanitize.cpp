// Host-code sanitizer harness: the framework's host-side C++ algorithms
// built alone with -fsanitize=address,undefined and driven by tests/test_native_sanitize.py.
// Input on stdin:  "sr n pc" then n values of I1, n of I2, n-1 uniforms; output: the ranks.
//                  "tile M N mode override": the GEMM tile code, workgroups and column tiles.
#include <cstdio>
#include <cstring>
#include <vector>

#include "../../csrc/host/gemm_tiles.h"
#include "../../csrc/host/stochastic_ranking.h"

int main() {
  char cmd[16];
  while (std::scanf("%15s", cmd) == 1) {
    if (std::strcmp(cmd, "sr") == 0) {
      long n;
      float pc;
      if (std::scanf("%ld %f", &n, &pc) != 2 || n < 0) return 2;
      std::vector<float> a(n), b(n), u(n > 0 ? n - 1 : 0);
      for (auto& v : a) if (std::scanf("%f", &v) != 1) return 3;
      for (auto& v : b) if (std::scanf("%f", &v) != 1) return 3;
      for (auto& v : u) if (std::scanf("%f", &v) != 1) return 3;
      std::vector<int64_t> r(n);
      evx_host::stochastic_ranking(a.data(), b.data(), u.data(), pc, (int64_t)n, r.data());
      for (long i = 0; i < n; ++i) std::printf("%lld ", (long long)r[i]);
      std::printf("\n");
    } else if (std::strcmp(cmd, "tile") == 0) {  // "tile M N mode override" → tile grid tiles_n
      long long M, N;
      int mode, ov;
      if (std::scanf("%lld %lld %d %d", &M, &N, &mode, &ov) != 4) return 5;
      std::printf("%d %lld %lld\n", evx_host::gemm_ks_tile(M, N, mode, ov), (long long)evx_host::gemm_ks_grid(M, N, mode, ov),
                  (long long)evx_host::gemm_ks_tiles_n(M, N, mode, ov));
    } else {
      return 4;
    }
  }
  return 0;
}
