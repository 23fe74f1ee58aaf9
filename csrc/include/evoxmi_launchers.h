// Host-side launchers implemented in csrc/kernels/*.hip (no torch dependency).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

void evx_philox_fill(float* out, int64_t n, const int64_t* key, int dist, int64_t elem_offset, hipStream_t s, int batch = 1);
void evx_philox_window(float* out, const int64_t* key, int64_t rows, int64_t dtot, int64_t col0, int64_t own, int64_t row0, int dist,
                       hipStream_t s);
void evx_classic_eval(const float* X, float* out, int N, int D, int func, float a, float b, float c, hipStream_t s);
void evx_pso_update(const float* pop, const float* vel, const float* lbl, const float* lbf, const float* fit,
                    const float* gbl, const int64_t* kp, const int64_t* kg, float w, float phip, float phig,
                    const float* lb, const float* ub, float* opop, float* ovel, float* olbl, float* olbf, int N, int D,
                    hipStream_t s);
void evx_pso_update_cols(const float* pop, const float* vel, const float* lbl, const float* lbf, const float* fit,
                         const float* gbl, const int64_t* kp, const int64_t* kg, float w, float phip, float phig,
                         const float* lb, const float* ub, float* opop, float* ovel, float* olbl, float* olbf, int N, int D,
                         int col0, int Dtot, hipStream_t s);

struct EvxOperand {
  const float* ptr;
  int64_t ld;
  int rc;
  const int32_t* gather;
  const float* sub;
  int sub_on_k;
  const float* kscale;
  const float* kw;
  const float* sscale;
  int sscale_inv;
};
void evx_gemm_f32(EvxOperand a, EvxOperand b, float* C, int64_t ldc, int M, int N, int K, int splits, float alpha,
                  const float* alpha_ptr, const float* bias_n, float beta, const float* Cin, int64_t ldcin, hipStream_t s);
int evx_gemm_splits_used(int K, int splits);
// K-split register-direct f32 GEMM (gemm_ks.hip): C = s·A·B (+ bias_n) (+ beta·Cin), s = alpha·(*alpha_ptr)
// a_kc: A(m, k) at A[m·lda + k] (else A[k·lda + m]);  b_kc: B(k, n) at B[n·ldb + k] (else B[k·ldb + n])
// mode 0: full; 1: symmetric output (tiles tm ≤ tn computed, mirrored); 2: skew-symmetric output
struct EvxGemmKs {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  float* C;
  int64_t ldc;
  int M, N, K;
  int a_kc, b_kc, mode;
  float alpha;
  const float* alpha_ptr;
  const float* bias_n;
  float beta;
  const float* Cin;
  int64_t ldcin;
  const int32_t* skip;
  const float* a_sub_k;  // A(m, k) − a_sub_k[k] before the product (K-contiguous A only), may be null
  // device-selected variant: when *sel != 0 the kernel uses A2 (if non-null), alpha2 and C2 (if
  // non-null) instead of A, alpha, C (the eigensolver's fixed schedule picks Taylor order /
  // Newton–Schulz output on the device)
  const int32_t* sel;
  const float* A2;
  float alpha2;
  float* C2;
  // symmetric mode: per-workgroup stats partials [Σ offdiag², Σ diag², min diag, max diag]
  // (double[4] per workgroup, sbr_stats_final layout), may be null
  double* stat_part;
  int stat_diag_only;  // stats of the diagonal only ([0, Σ diag², min, max]: the X² bounds of the eigensolver)
  int c_vec4;
  int tiles_m, tiles_n;  // set by the launcher
  // row-terms epilogue (MODE 0, CEC'22 F1 / F4 on the rotated population): C is not written;
  // per output tile and row the additive terms of the basic function over the tile's columns
  // go to row_terms[(tn · M + row) · 2 + {0, 1}] (Zakharov: Σ z², Σ ½(j+1) z; Rastrigin:
  // Σ y² − 10 cos 2πy + 10 with y = 0.0512 z, 0), finished by evx_cec_rowterms_final
  float* row_terms;
  int row_fid;
  // bf16x6 only: operands pre-split into fragment planes (evx_split_planes / evx_philox_normal_planes):
  // uint16 [3][rows][kp] (h, m, l), kp = K rounded up to 32, each 32-k group in fragment order —
  // the operand's f32 pointer is then not read (a K-contiguous operand of the same shape)
  const uint16_t* a_pl;
  const uint16_t* b_pl;
  int64_t a_pl_rows, b_pl_rows, pl_kp;
  // per-column-block A shift (stacked products sharing A, e.g. the CEC'22 composition
  // rotations): output columns [c·sub_cols, (c+1)·sub_cols) use a_sub_k + c·sub_ld
  // (sub_cols a multiple of the tile width; 0: one shift for all columns)
  int sub_cols;
  int64_t sub_ld;
  int force_tile;  // tile code for this launch (0: the shape heuristic)
  // 0: the process-wide precision (evx_gemm_ks_set_prec); 3: bf16x3 (hh + hm + mh, ≈16-bit
  // products — the eigensolver's correction products, gemm_ks.hip split2)
  int prec;
  // added to the diagonal of the result (after alpha / Cin): Bᵀ B − I for Newton–Schulz
  float diag_add;
};
void evx_gemm_ks(const EvxGemmKs& a, hipStream_t s);
// LDS-staged bf16x6 GEMM on "blocked planes" (gemm_blk.hip): an f32 matrix rows × K stored as
// bf16 [ceil(K/16)][Rp][3][16] (Rp = evx_blk_rows(rows); the buffer carries kEvxBlkSlackRows
// spare 96-byte records after the last block, read only for output rows / columns past M / N)
constexpr int kEvxBlkSlackRows = 512;
struct EvxGemmBlk {
  const uint16_t* A;  // blocked planes of the M × K operand
  int64_t a_rows;     // Rp of A
  const uint16_t* B;  // blocked planes of the N × K operand (C = A·Bᵀ)
  int64_t b_rows;
  int KB;             // 16-k blocks
  int M, N;
  float* C;
  int64_t ldc;
  float alpha;
  const float* alpha_ptr;
  const float* bias_n;
  const int32_t* skip;
  int tiles_m, tiles_n;  // set by the launcher
  const float* a_rinv;   // f16x3 only: per-row inverse scales of A (M) and B (N)
  const float* b_rinv;
  int sub_cols;           // f16x3 stacked operands: output column block c·sub_cols reads A's plane
  int64_t a_comp_stride;  // set c (a_comp_stride uint16 elements and a_rows row scales apart)
  // f16x3 row-terms epilogue (CEC'22 F1 Zakharov fid 0 / F4 Rastrigin fid 3): C is not written;
  // per 128-column tile and row the basic function's two additive terms go to
  // row_terms[(tn · M + row) · 2 + {0, 1}] (finished by evx_cec_rowterms_final)
  float* row_terms;
  int row_fid;
};
void evx_gemm_blk(const EvxGemmBlk& a, hipStream_t s);
int evx_gemm_blk_tile_m();
int evx_gemm_blk_tile_n();
int evx_gemm_h3_tiles_n(int N);  // 128-column tiles of gemm_h3 (row-terms partial count)
int64_t evx_blk_rows(int64_t rows);
int64_t evx_blk_elems(int64_t rows, int K);  // uint16 elements of a blocked-planes buffer
// blocked planes of (X[r][k] − sub_k[k])·colscale[k] (sub_k / colscale may be null)
void evx_split_blk(const float* X, int64_t ld, int64_t rows, int K, const float* sub_k, const float* colscale, uint16_t* out,
                   hipStream_t s);
// f16x3 planes (gemm_blk.hip): f16 [ceil(K/16)][Rp][2][16] + per-row inverse scales rinv[Rp]
int64_t evx_h3_elems(int64_t rows, int K);
void evx_split_h3(const float* X, int64_t ld, int64_t rows, int K, const float* sub_k, const float* colscale, uint16_t* out,
                  float* rinv, hipStream_t s, int ncomp = 1, int64_t sub_ld = 0);
void evx_philox_h3(const int64_t* key, int64_t rows, int d, int64_t row0, uint16_t* out, float* rinv, hipStream_t s);
void evx_gemm_h3(const EvxGemmBlk& a, hipStream_t s);
// blocked planes of rows [row0, row0 + rows) of normal(key, (·, d)) (d % 4 == 0)
void evx_philox_blk(const int64_t* key, int64_t rows, int d, int64_t row0, uint16_t* out, hipStream_t s);
// fragment planes of X (rows × K, K-contiguous, row stride ld), X[r][k]·colscale[k] when colscale
// fragment planes of rows [row0, row0 + rows) of the virtual normal matrix normal(key, (·, d)) (d % 4 == 0)
int evx_gemm_ks_tiles_n(int M, int N, int mode);  // column tiles of a launch (row-terms partial count)
void evx_cec_rowterms_final(const float* parts, int tiles_n, int M, int fid, float* out, hipStream_t s);
// composition (F9–F12) in two launches: per part i the basic function fid[i] on z = Z[:, zcol[i] : +D]·scale[i]
// (zcol ≥ 0, the stacked rotation GEMM's block) or (x − os[comp[i]])·scale[i] (zcol < 0), the distance
// ‖x − os[i]‖², weights from sigma, f = Σ w̃ (lamb·f_i + bias), clamped below thr
constexpr int kEvxCecMaxParts = 8;
struct EvxCecCompose {
  int n;
  int fid[kEvxCecMaxParts], zcol[kEvxCecMaxParts], comp[kEvxCecMaxParts];
  float scale[kEvxCecMaxParts], sigma[kEvxCecMaxParts], lamb[kEvxCecMaxParts], bias[kEvxCecMaxParts];
  const float* os;  // shift rows (≥ n rows, ldo apart)
  int64_t ldo;
  float thr;
};
void evx_cec_compose(const float* Z, int64_t ldz, const float* X, int64_t ldx, int N, int D, const EvxCecCompose& c, float* part,
                     float* out, hipStream_t s);  // part: float[N · n · 2] scratch
int evx_gemm_ks_grid(int M, int N, int mode);  // workgroups of a launch (stat_part length)
int evx_gemm_ks_tile(int M, int N, int mode);
void evx_gemm_ks_set_tile(int t);
// 1: bf16x6 split products on the bf16 matrix pipe (default), 0: f32 MFMA
void evx_gemm_ks_set_prec(int prec);
void evx_gemm_ks_set_nw8(int tiles);  // 8-wave workgroups for grids of at most this many tiles
int evx_gemm_ks_prec();
void evx_cma_local_select(const int32_t* order, int mu, const float* w, int start, int size, int K, int32_t* rows, float* wk,
                          hipStream_t s);
void evx_sym_pack(const float* S, int64_t lds, int d, float* P, hipStream_t s);
void evx_sym_unpack(const float* P, int d, float* S, int64_t lds, hipStream_t s);
void evx_cma_center_rows(const float* pop, int64_t ldp, const int32_t* rows, const float* mean, const float* sigma, const float* w, int K,
                         int d, float* Y, hipStream_t s, int64_t ldy = 0, int aug = 0);
void evx_radix_argsort(const float* keys, int n, int descending, float* out_keys, int32_t* out_idx, hipStream_t s, int batch);
int evx_argsort_max_n();
void evx_argsort(const float* keys, int n, int descending, float* out_keys, int32_t* out_idx, hipStream_t s, int batch = 1);
void evx_cec_basic(const float* Z, int64_t ld, int N, int fid, const int32_t* perm, int start, int L, const float* sub,
                   float scale, const float* Y, int64_t ldy, int ystart, int yperm, float* out, hipStream_t s, float clamp = 0.f);
// outer round `round` of a sweep (0: within-block pairing, ≥1: circle-method rounds; the
// pairing is computed in-kernel and equals jacobi.py:_schedule_cpu row `round`)
void evx_jacobi_round(float* A, float* B, int np, int round, float* Vbuf, const int* flag, float inner_tol, int max_inner,
                      hipStream_t s);
// one sweep (nb rounds) with round t−1's B update inside round t's solve launch (V0/V1:
// npairs·32·32 floats each, alternated by round parity); all of B is updated on return
void evx_jacobi_sweep_overlapB(float* A, float* B, int np, float* V0, float* V1, const int* flag, float inner_tol,
                               int max_inner, hipStream_t s);
void evx_jacobi_solve(const float* A, int np, const int* sched_t, float* Vbuf, const int* flag, float inner_tol, int max_inner,
                      int mode, hipStream_t s);
// round t's apply; with sched_next != nullptr the same launch also solves round t+1's
// subproblems into Vnext (counters: npairs ints, zeroed, private to this round)
void evx_jacobi_apply_solve(float* A, float* B, int np, const int* sched_t, const float* Vcur, const int* flag,
                            const int* sched_next, int mode_next, float* Vnext, int* counters, float inner_tol, int max_inner,
                            hipStream_t s);
void evx_jacobi_check(const float* A, int np, double* part, int* flag, double tol2, double* last_off, hipStream_t s);
int evx_jacobi_parts();
void evx_es_population(const int64_t* key, const float* center, float sigma, int64_t rows, int64_t d, int64_t half, int64_t row0, float* out,
                       hipStream_t s, int64_t col0 = 0, int64_t dtot = 0);
void evx_es_noise_grad(const int64_t* key, const float* w, int64_t rows, int64_t d, int64_t row0, int chunks, float* partial,
                       hipStream_t s, int64_t col0 = 0, int64_t dtot = 0);
void evx_philox_words(const int64_t* key, int64_t nblocks, uint32_t domain, int64_t offset, int64_t* out, hipStream_t s,
                      int batch = 1, int words = 4);
void evx_colsum(const float* partial, int chunks, int D, float* out, hipStream_t s);
void evx_weighted_rowsum(const float* X, int64_t ldx, const int32_t* idx, const float* w, const float* sub, int K, int D,
                         float* partial, int chunks, hipStream_t s);
void evx_gemm_set_config(int cfg);
void evx_sbx(const float* x, float* out, int n, int d, const int64_t* keys, float pro_c, float dis_c, int type, hipStream_t s, int col0 = 0,
             int dtot = 0);
void evx_pm(const float* x, float* out, int n, int d, int nm, const float* lb, const float* ub, const int64_t* keys, float pro_m,
            float dis_m, hipStream_t s, int col0 = 0, int dtot = 0);
void evx_dtlz(const float* X, float* F, int N, int D, int M, int variant, hipStream_t s);
void evx_de_trial(const float* P, const int32_t* idx, const float* coef, int K, const int32_t* cur, const int32_t* mode,
                  const float* CR, const int32_t* jr, const int32_t* L, const int64_t* key, const float* lb, const float* ub,
                  int repair, float* out, int R, int d, int rows, int* err, hipStream_t s, int batch = 1, int col0 = 0, int dtot = 0);
void evx_moead_scan(float* objs, const float* off_objs, const int32_t* P, const float* W, float* z, int32_t* owner, int N, int R,
                    int T, int M, int func, int nr, int update_z, hipStream_t s);
void evx_ant_rollout(const float* W, int64_t P, int N, int h1, int h2, const float* init, int cap, float* ret, int* steps, hipStream_t s);
size_t evx_nds_workspace_words(int n);
int evx_nds_peel_blocks(int n);
void evx_nds(const float* f, int n, int m, int limit, uint32_t* DW, int32_t* rank, uint32_t* ws, int32_t* err, int blocks,
             hipStream_t s);

// moead.hip
void evx_moead_parents(const int64_t* nb, int N, int T, const int64_t* key, int32_t* p0, int32_t* p1, hipStream_t s, int row0 = 0);
void evx_moead_variation(const float* pop, const int32_t* p0, const int32_t* p1, float* out, int N, int d, const int64_t* kx,
                         const int64_t* km, const float* lb, const float* ub, float pro_c, float dis_c, float pro_m, float dis_m,
                         int nm, hipStream_t s, int row0 = 0, const int32_t* win = nullptr);
void evx_moead_replace(const float* pop_obj, const float* off_obj, const float* W, const float* z, const float* zmax,
                       const int32_t* rowptr, const int32_t* owner, int N, int M, int func, int32_t* win, float* new_obj,
                       hipStream_t s);
void evx_moead_select_rows(const float* pop, const float* off, const int32_t* win, float* out, int N, int d, hipStream_t s);
void evx_moead_select_rows_inplace(float* pop, const float* off, const int32_t* win, int N, int d, hipStream_t s);
void evx_lsmop_g(const float* X, float* G, int N, int D, int ng, int nk, int cosine, const int* start, const int* sublen, const int* func,
                 hipStream_t s);

// cmaes.hip
void evx_cma_delta_gemv(const float* M, const float* mean, const float* dm, float cm, int d, float* mean_out, float* delta, float* y,
                        hipStream_t s);
void evx_cma_paths(const float* ps, const float* pc, const float* y, const float* delta, const float* sigma, const int64_t* count_iter,
                   int d, const float* consts, float* ps_out, float* pc_out, float* sigma_out, float* a_out, float* hsig_out,
                   hipStream_t s,
                   const int64_t* count_eigen = nullptr, int64_t* count_iter_out = nullptr, int64_t* count_eigen_out = nullptr);
void evx_cma_cov_pad(const float* C, const float* S, const float* pc, const float* a, float c1, float cmu, const float* Bprev, int d,
                     int np, float* Cn, float* Cp, float* Bp, hipStream_t s, int64_t lds = 0);
void evx_cma_eig_out(const float* Bp, const float* w, int d, int np, float* B, float* D, float* BdivD, hipStream_t s,
                     const float* Balt = nullptr, const int* keep = nullptr);

// nsga_select.hip
void evx_nsga_select(const int32_t* rank, const float* f, int n, int m, int N, int mask_pos, int64_t* keep, hipStream_t s);
// sorted-block refinement of a warm-started eigendecomposition (eigh_sbr.hip, evoxmi/ops/sbr.py)
int evx_sbr_nblocks(int n, int off);
int evx_sbr_stat_parts();
void evx_sbr_stats(const float* A, int n, int64_t lda, double* part, double* out, hipStream_t s);
void evx_sbr_block(const float* A, int n, int64_t lda, int off, int sweeps, int* perm, float* Q, float* dq, hipStream_t s,
                   long long* dbg = nullptr);
void evx_sbr_far(const float* A, int n, int64_t lda, int off, const int* perm, const float* Q, const float* dq,
                 const double* stats, float thr_fac, float* X, int64_t ldx, hipStream_t s);
void evx_sbr_bq(const float* B, int rows, int n, int64_t ldb, int off, const int* perm, const float* Q, float* Bq, int64_t ldq,
                hipStream_t s);
int evx_sbr_symstats_parts(int n);
// 16-wide blocks in a shifted sorted order (eigh_sbr16.hip)
int evx_sbr16_nblocks(int n, int sb);
int evx_sbr16_max_n();
void evx_sbr_taylor4_prep(const float* X, const float* X2, int n, const float* alpha, float* P, float* M, hipStream_t s, int mt = 0);
void evx_sbr_damping(const float* X2, int n, int64_t ldx, const float* V, float* work, float tau, float* alpha, hipStream_t s,
                     const int* skip = nullptr, int no_final = 0, const double* xpart = nullptr, int nparts = 0);
void evx_sbr16_block(const float* A, int n, int64_t lda, int shift, int sweeps, int* perm, float* Q, float* dq, int sb, hipStream_t s,
                     const int* skip = nullptr, float skip_tol = 0.f);
void evx_sbr16_far(const float* A, int n, int64_t lda, const int* perm, const float* Q, const float* dq, const double* stats,
                   float thr_fac, float theta, float* X, int64_t ldx, int sb, hipStream_t s,
                   const float* theta_ptr = nullptr, const int* skip = nullptr);
void evx_sbr16_bq(const float* B, int rows, int n, int64_t ldb, const int* perm, const float* Q, float* Bq, int64_t ldq, int sb,
                  hipStream_t s,
                     const int* skip = nullptr);
void evx_sbr_symstats(const float* T, int n, int64_t ldt, float* A, int64_t lda, double* part, double* out, hipStream_t s);
void evx_sbr_taylor_prep(const float* X, const float* X2, const float* X3, int n, const float* alpha, float* P, float* M,
                         hipStream_t s, int mt = 0);

// mo_geom.hip (K17 k-nearest rows, K18 Monte-Carlo hypervolume)
int evx_knn_max_t();
int evx_knn_max_m();
void evx_knn(const float* X, const float* Y, int N, int M, int m, int T, float* out_d, int32_t* out_i, hipStream_t s);
int evx_hv_max_m();
void evx_hv_count(const float* S, const float* P, int ns, int np, int m, int strict, int32_t* count, hipStream_t s);
void evx_hv_contrib(const float* S, const float* P, const int32_t* count, const float* alpha, int ns, int np, int m, float* f,
                    hipStream_t s);

// batched linear-kernel GP hyper-parameter fits (gp_fit.hip, IM-MOEA)
void evx_linear_gp_fit(const double* a, const double* b, const double* c, const double* n, int64_t models, int steps, double lr,
                       float* v, float* s2, hipStream_t s);

// device-controlled SBR schedule (eigh_sbr_dev.hip)
void evx_sbr_dev_prep(const float* X, const float* X2, const float* X3, int n, float* alpha, float* P, float* MT, int* ctrl,
                      hipStream_t s, const float* V2 = nullptr, const float* V3 = nullptr,
                      float tau = 1.f, const double* xpart = nullptr, int nparts = 0, const float* copy_src = nullptr, float* copy_dst = nullptr, int minus_id = 0);
void evx_sbr_dev_copy(const float* src, float* dst, int64_t n, const int* skip, hipStream_t s);
void evx_sbr_dev_ctrl(const double* part, int nparts, int j, int K, double* hist, float* alpha, float* theta, int* ctrl, int* st,
                      const float* prm6, int ns_iters, const float* A, int64_t lda, int n, float* w_out, double* eig_stats, float* w_init,
                      double* log, int log_len, int* log_count, hipStream_t s, int lean_from = 1 << 30, int recover = 0, int lean_guard = 0, int xgate = 0, int damp_from = -1, int* rep_seq = nullptr, double* rep_ring = nullptr, int rep_len = 0);
// far generator + Bq in one launch (skip_far / skip_bq: their control words)
void evx_sbr16_far_bq(const float* A, int n, int64_t lda, const int* perm, const float* Q, const float* dq, const double* stats,
                      float thr_fac, const float* theta_ptr, float* X, int64_t ldx, const float* B, int rows, int64_t ldb, float* Bq,
                      int64_t ldq, int sb, hipStream_t s, const int* skip_far, const int* skip_bq, bool pre = false);

// owner-computes MOEA/D (moead.hip)
void evx_moead_halo_replace(float* obj, const float* off_obj, const float* W, const float* z, const float* zmax, const int32_t* rowptr,
                            const int32_t* owner, const int32_t* slots, int H, int M, int func, int32_t* win_h, hipStream_t s);
void evx_peer_release(hipStream_t s);
void evx_moead_halo_gather(float* pop, const int32_t* slots, const int32_t* win_h, int H, const int64_t* peer, const int32_t* starts,
                           int world, int d, hipStream_t s, int32_t* first = nullptr,
                           int N = 0);

// rank-by-counting stable argsort in one launch (sort.hip), n ≤ evx_rank_argsort_max_n()
int evx_rank_argsort_max_n();
void evx_rank_argsort(const float* keys, int n, int descending, float* out_keys, int32_t* out_idx, hipStream_t s, int batch);
// two-pass stable argsort for n ≤ evx_merge_argsort_max_n(): rank inside 4096-key chunks, then co-rank
// merge by lockstep binary searches; ws_keys / ws_idx hold batch * n entries each
int evx_merge_argsort_max_n();
void evx_merge_argsort(const float* keys, int n, int descending, float* out_keys, int32_t* out_idx, uint32_t* ws_keys,
                       int32_t* ws_idx, hipStream_t s, int batch);
