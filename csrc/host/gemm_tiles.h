// Host-side tile selection of the K-split f32 MFMA GEMM (gemm_ks.hip): which output tile a
// launch uses and how many workgroups / column tiles it has.  Pure integer logic shared by
// every GEMM launch (and by the bindings that size per-workgroup partial buffers), kept
// header-only so the host sanitizer harness (tests/native) builds it alone.
#pragma once
#include <stdint.h>

namespace evx_host {

// tile code t: output tile 16t × 16t, except t = 8: 128 × 64 (tall full products).  (A
// 128 × 128 tile on the 32x32x16 bf16x6 form spills 85 registers: measured slower, dropped.)
inline int gemm_ks_tile(int64_t M, int64_t N, int mode, int override_tile = 0) {
  if (override_tile) return (override_tile == 8 && mode != 0) ? 4 : override_tile;
  // tall full products (sampling / CEC rotation, 10 000 × 1000 × 1000): 128 × 64 tiles —
  // half the B-panel reloads per output of 64 × 64 (tools/gemm_ks_probe.cpp: 210 vs 317 µs)
  if (mode == 0 && M >= 2048 && N >= 64) return 8;
  // fewest workgroup rounds over the 256 CUs × tile work, larger tile on ties
  int best = 4;
  double best_cost = 1e300;
  for (int t : {4, 3, 2}) {
    const int64_t b = 16 * t;
    const int64_t tm = (M + b - 1) / b, tn = (N + b - 1) / b;
    const int64_t tiles = mode == 0 ? tm * tn : tm * (tm + 1) / 2;
    const double cost = (double)((tiles + 255) / 256) * (double)(b * b);
    if (cost < best_cost * 0.999) {
      best_cost = cost;
      best = t;
    }
  }
  return best;
}

inline int64_t gemm_ks_tile_rows(int t) { return 16 * (int64_t)t; }
inline int64_t gemm_ks_tile_cols(int t) { return t == 8 ? 64 : 16 * (int64_t)t; }

// workgroups of a launch: full grid, or the upper-triangle tiles of a (skew-)symmetric output
inline int64_t gemm_ks_grid(int64_t M, int64_t N, int mode, int override_tile = 0) {
  const int t = gemm_ks_tile(M, N, mode, override_tile);
  const int64_t bm = gemm_ks_tile_rows(t), bn = gemm_ks_tile_cols(t);
  const int64_t tm = (M + bm - 1) / bm, tn = (N + bn - 1) / bn;
  return mode == 0 ? tm * tn : tm * (tm + 1) / 2;
}

inline int64_t gemm_ks_tiles_n(int64_t M, int64_t N, int mode, int override_tile = 0) {
  const int t = gemm_ks_tile(M, N, mode, override_tile);
  const int64_t bn = gemm_ks_tile_cols(t);
  return (N + bn - 1) / bn;
}

}  // namespace evx_host
