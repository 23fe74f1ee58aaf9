// Host-side stochastic ranking (Runarsson & Yao 2000) used by SRA (reference
// algorithms/mo/sra.py:22-85): bubble-sort sweeps in which each adjacent comparison uses
// indicator I1 with probability pc (else I2), larger value first, stopping after
// ⌈n/2⌉ sweeps or a sweep without swaps.  Inherently sequential and tiny (n ≤ 2N), so it
// runs on the host; header-only so the sanitizer harness (tests/native) builds it alone.
#pragma once
#include <stdint.h>

#include <utility>

namespace evx_host {

// a, b: indicator values per individual; u: n−1 uniforms (one per adjacent position);
// rank: output permutation (rank[0] = best), initialised to the identity here.
inline void stochastic_ranking(const float* a, const float* b, const float* u, float pc, int64_t n, int64_t* rank) {
  for (int64_t i = 0; i < n; ++i) rank[i] = i;
  const int64_t sweeps = (n + 1) / 2;
  bool swapped = true;
  for (int64_t it = 0; it < sweeps && swapped; ++it) {
    swapped = false;
    for (int64_t j = 0; j + 1 < n; ++j) {
      const float* key = (u[j] < pc) ? a : b;
      if (key[rank[j]] < key[rank[j + 1]]) {
        std::swap(rank[j], rank[j + 1]);
        swapped = true;
      }
    }
  }
}

}  // namespace evx_host
