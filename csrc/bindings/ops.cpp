// TORCH_LIBRARY registration of evoxmi's HIP kernels (namespace `evoxmi`).
// Kernel translation units (csrc/kernels/*.hip) expose plain C++ launchers that
// take raw device pointers + the caller's hipStream_t; this file is the only one
// that sees torch headers.  Every op launches on the *current* HIP stream so it is
// ordered with surrounding torch work and can be captured into a hipGraph.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>
#include <cstring>

#include "evoxmi_launchers.h"
#include "../host/stochastic_ranking.h"

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a HIP device tensor")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")

void check_key(const at::Tensor& key) {
  CHECK_DEV(key);
  TORCH_CHECK(key.scalar_type() == at::kLong && key.numel() == 2 && key.is_contiguous(), "key must be int64[2]");
}

// A key (2,) or a stack of per-run keys (B, 2) (BatchedRuns: evoxmi/ops/batching.py);
// returns B (0 for a single key).
int64_t key_batch(const at::Tensor& key, const char* op) {
  CHECK_DEV(key);
  TORCH_CHECK(key.scalar_type() == at::kLong && key.is_contiguous(), op, ": key must be contiguous int64");
  if (key.dim() == 1) {
    TORCH_CHECK(key.numel() == 2, op, ": key must be int64[2]");
    return 0;
  }
  TORCH_CHECK(key.dim() == 2 && key.size(1) == 2 && key.size(0) >= 1 && key.size(0) <= 65535, op, ": keys must be (B, 2), B ≤ 65535");
  return key.size(0);
}

at::Tensor philox_window(const at::Tensor& key, int64_t rows, int64_t dtot, int64_t col0, int64_t own, int64_t row0, int64_t dist) {
  TORCH_CHECK(key.is_cuda() && key.scalar_type() == at::kLong && key.numel() == 2, "philox_window: one device key");
  TORCH_CHECK(rows >= 0 && own >= 0 && col0 >= 0 && col0 + own <= dtot && row0 >= 0, "philox_window: window outside the matrix");
  c10::DeviceGuard g(key.device());
  auto out = at::empty({rows, own}, key.options().dtype(at::kFloat));
  if (rows > 0 && own > 0)
    evx_philox_window(out.data_ptr<float>(), key.contiguous().data_ptr<int64_t>(), rows, dtot, col0, own, row0, (int)dist, cur_stream());
  return out;
}

at::Tensor philox_fill(const at::Tensor& key, int64_t n, int64_t dist, int64_t offset) {
  const int64_t B = key_batch(key, "philox_fill");
  TORCH_CHECK(offset % 4 == 0, "offset must be a multiple of 4");
  c10::DeviceGuard g(key.device());
  auto out = B ? at::empty({B, n}, key.options().dtype(at::kFloat)) : at::empty({n}, key.options().dtype(at::kFloat));
  if (n > 0) evx_philox_fill(out.data_ptr<float>(), n, key.data_ptr<int64_t>(), (int)dist, offset, cur_stream(), B ? (int)B : 1);
  return out;
}

at::Tensor classic_eval(const at::Tensor& X, int64_t func, double a, double b, double c) {
  CHECK_DEV(X); CHECK_F32(X); CHECK_CONTIG(X);
  TORCH_CHECK(X.dim() == 2, "X must be (N, d)");
  c10::DeviceGuard g(X.device());
  auto out = at::empty({X.size(0)}, X.options());
  if (X.size(0) > 0)
    evx_classic_eval(X.data_ptr<float>(), out.data_ptr<float>(), (int)X.size(0), (int)X.size(1), (int)func, (float)a, (float)b,
                     (float)c, cur_stream());
  return out;
}

std::vector<at::Tensor> pso_update(const at::Tensor& pop, const at::Tensor& vel, const at::Tensor& lbl,
                                   const at::Tensor& lbf, const at::Tensor& fit, const at::Tensor& gbl,
                                   const at::Tensor& kp, const at::Tensor& kg, double w, double phip, double phig,
                                   const at::Tensor& lb, const at::Tensor& ub, int64_t col0, int64_t d_total) {
  for (auto* t : {&pop, &vel, &lbl, &lbf, &fit, &gbl, &lb, &ub}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  check_key(kp); check_key(kg);
  const int64_t N = pop.size(0), D = pop.size(1);
  TORCH_CHECK(vel.sizes() == pop.sizes() && lbl.sizes() == pop.sizes(), "shape mismatch");
  TORCH_CHECK(lbf.numel() == N && fit.numel() == N && gbl.numel() == D && lb.numel() == D && ub.numel() == D, "shape mismatch");
  c10::DeviceGuard g(pop.device());
  auto opop = at::empty_like(pop), ovel = at::empty_like(pop), olbl = at::empty_like(pop), olbf = at::empty_like(lbf);
  if (d_total <= 0) d_total = D;
  TORCH_CHECK(col0 >= 0 && col0 + D <= d_total, "pso_update: column block outside [0, d_total)");
  if (col0 == 0 && d_total == D)
    evx_pso_update(pop.data_ptr<float>(), vel.data_ptr<float>(), lbl.data_ptr<float>(), lbf.data_ptr<float>(),
                   fit.data_ptr<float>(), gbl.data_ptr<float>(), kp.data_ptr<int64_t>(), kg.data_ptr<int64_t>(), (float)w,
                   (float)phip, (float)phig, lb.data_ptr<float>(), ub.data_ptr<float>(), opop.data_ptr<float>(),
                   ovel.data_ptr<float>(), olbl.data_ptr<float>(), olbf.data_ptr<float>(), (int)N, (int)D, cur_stream());
  else
    evx_pso_update_cols(pop.data_ptr<float>(), vel.data_ptr<float>(), lbl.data_ptr<float>(), lbf.data_ptr<float>(),
                        fit.data_ptr<float>(), gbl.data_ptr<float>(), kp.data_ptr<int64_t>(), kg.data_ptr<int64_t>(), (float)w,
                        (float)phip, (float)phig, lb.data_ptr<float>(), ub.data_ptr<float>(), opop.data_ptr<float>(),
                        ovel.data_ptr<float>(), olbl.data_ptr<float>(), olbf.data_ptr<float>(), (int)N, (int)D, (int)col0,
                        (int)d_total, cur_stream());
  return {opop, ovel, olbl, olbf};
}

const float* optf(const c10::optional<at::Tensor>& t) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t);
  return t->data_ptr<float>();
}

EvxOperand make_operand(const at::Tensor& X, int64_t rc, const c10::optional<at::Tensor>& gather,
                        const c10::optional<at::Tensor>& sub, int64_t sub_on_k, const c10::optional<at::Tensor>& kscale,
                        const c10::optional<at::Tensor>& kw, const c10::optional<at::Tensor>& sscale, int64_t sscale_inv) {
  CHECK_DEV(X); CHECK_F32(X);
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "operand must be 2-D with unit inner stride");
  EvxOperand o{};
  o.ptr = X.data_ptr<float>();
  o.ld = X.stride(0);
  o.rc = (int)rc;
  o.gather = nullptr;
  if (gather.has_value() && gather->defined()) {
    CHECK_DEV(*gather);
    TORCH_CHECK(gather->scalar_type() == at::kInt && gather->is_contiguous(), "gather must be int32");
    TORCH_CHECK(rc, "gather only supported for row-contiguous operands");
    o.gather = gather->data_ptr<int32_t>();
  }
  o.sub = optf(sub);
  o.sub_on_k = (int)sub_on_k;
  o.kscale = optf(kscale);
  o.kw = optf(kw);
  o.sscale = optf(sscale);
  o.sscale_inv = (int)sscale_inv;
  return o;
}

at::Tensor gemm_f32(const at::Tensor& A, int64_t a_rc, const c10::optional<at::Tensor>& a_gather,
                    const c10::optional<at::Tensor>& a_sub, int64_t a_sub_on_k, const c10::optional<at::Tensor>& a_kscale,
                    const c10::optional<at::Tensor>& a_kw, const c10::optional<at::Tensor>& a_sscale, int64_t a_sscale_inv,
                    const at::Tensor& B, int64_t b_rc, const c10::optional<at::Tensor>& b_gather,
                    const c10::optional<at::Tensor>& b_sub, int64_t b_sub_on_k, const c10::optional<at::Tensor>& b_kscale,
                    const c10::optional<at::Tensor>& b_kw, const c10::optional<at::Tensor>& b_sscale, int64_t b_sscale_inv,
                    const c10::optional<at::Tensor>& alpha_ptr, const c10::optional<at::Tensor>& bias_n, double beta,
                    const c10::optional<at::Tensor>& Cin, int64_t M, int64_t N, int64_t K, int64_t splits, double alpha) {
  auto ao = make_operand(A, a_rc, a_gather, a_sub, a_sub_on_k, a_kscale, a_kw, a_sscale, a_sscale_inv);
  auto bo = make_operand(B, b_rc, b_gather, b_sub, b_sub_on_k, b_kscale, b_kw, b_sscale, b_sscale_inv);
  // shape checks: KC operand is (rows, K); RC operand is (K or gather source, rows)
  if (!a_rc) { TORCH_CHECK(A.size(0) >= M && A.size(1) >= K, "A shape"); } else { TORCH_CHECK(A.size(1) >= M, "A shape"); }
  if (!b_rc) { TORCH_CHECK(B.size(0) >= N && B.size(1) >= K, "B shape"); } else { TORCH_CHECK(B.size(1) >= N, "B shape"); }
  if (a_rc && !ao.gather) TORCH_CHECK(A.size(0) >= K, "A shape");
  if (b_rc && !bo.gather) TORCH_CHECK(B.size(0) >= K, "B shape");
  if (a_gather.has_value() && a_gather->defined()) TORCH_CHECK(a_gather->numel() >= K, "gather length");
  if (b_gather.has_value() && b_gather->defined()) TORCH_CHECK(b_gather->numel() >= K, "gather length");
  c10::DeviceGuard g(A.device());
  const int sp = evx_gemm_splits_used((int)K, (int)splits);
  at::Tensor C = sp > 1 ? at::empty({sp, M, N}, A.options()) : at::empty({M, N}, A.options());
  const float* cin = nullptr;
  int64_t ldcin = N;
  if (Cin.has_value() && Cin->defined()) {
    TORCH_CHECK(sp == 1, "Cin incompatible with split-K");
    CHECK_DEV(*Cin); CHECK_F32(*Cin);
    TORCH_CHECK(Cin->dim() == 2 && Cin->stride(1) == 1 && Cin->size(0) >= M && Cin->size(1) >= N, "Cin shape");
    cin = Cin->data_ptr<float>();
    ldcin = Cin->stride(0);
  }
  if (M > 0 && N > 0)
    evx_gemm_f32(ao, bo, C.data_ptr<float>(), N, (int)M, (int)N, (int)K, (int)splits, (float)alpha, optf(alpha_ptr),
                 optf(bias_n), (float)beta, cin, ldcin, cur_stream());
  return C;
}

// K-split register-direct f32 GEMM (gemm_ks.hip).  A: a_kc → (M, K) rows, else (K, M);
// B: b_kc → (N, K) rows (C = A·Bᵀ), else (K, N) (C = A·B).  Inner strides must be 1.
at::Tensor gemm_ks(const at::Tensor& A, int64_t a_kc, const at::Tensor& B, int64_t b_kc, int64_t M, int64_t N, int64_t K,
                   int64_t mode, double alpha, const c10::optional<at::Tensor>& alpha_ptr,
                   const c10::optional<at::Tensor>& bias_n, double beta, const c10::optional<at::Tensor>& Cin,
                   const c10::optional<at::Tensor>& out, const c10::optional<at::Tensor>& skip,
                   const c10::optional<at::Tensor>& a_sub_k, const c10::optional<at::Tensor>& sel = c10::nullopt,
                   const c10::optional<at::Tensor>& A2 = c10::nullopt, double alpha2 = 0.0,
                   const c10::optional<at::Tensor>& C2 = c10::nullopt, const c10::optional<at::Tensor>& stat_part = c10::nullopt,
                   int64_t stat_diag_only = 0, int64_t prec = 0, double diag_add = 0.0) {
  CHECK_DEV(A); CHECK_F32(A); CHECK_DEV(B); CHECK_F32(B);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 2 && A.stride(1) == 1 && B.stride(1) == 1, "gemm_ks: 2-D operands with unit inner stride");
  TORCH_CHECK(M > 0 && N > 0 && K > 0, "gemm_ks: empty shape");
  TORCH_CHECK(mode >= 0 && mode <= 2, "gemm_ks: mode");
  if (a_kc) { TORCH_CHECK(A.size(0) >= M && A.size(1) >= K, "gemm_ks: A shape"); } else { TORCH_CHECK(A.size(0) >= K && A.size(1) >= M, "gemm_ks: A shape"); }
  if (b_kc) { TORCH_CHECK(B.size(0) >= N && B.size(1) >= K, "gemm_ks: B shape"); } else { TORCH_CHECK(B.size(0) >= K && B.size(1) >= N, "gemm_ks: B shape"); }
  auto vec4_ok = [](const at::Tensor& t) {
    return (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0) && (t.stride(0) % 4 == 0);
  };
  if (a_kc || b_kc) { TORCH_CHECK(K % 4 == 0, "gemm_ks: K-contiguous operands need K % 4 == 0"); }
  if (a_kc) { TORCH_CHECK(vec4_ok(A), "gemm_ks: A must be 16-byte aligned with a row stride divisible by 4"); }
  if (b_kc) { TORCH_CHECK(vec4_ok(B), "gemm_ks: B must be 16-byte aligned with a row stride divisible by 4"); }
  if (mode != 0) {
    TORCH_CHECK(M == N, "gemm_ks: symmetric / skew outputs need M == N");
    TORCH_CHECK(!(bias_n.has_value() && bias_n->defined()) && !(Cin.has_value() && Cin->defined()),
                "gemm_ks: symmetric / skew outputs take no bias / Cin");
  }
  c10::DeviceGuard g(A.device());
  at::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    CHECK_DEV(C); CHECK_F32(C);
    TORCH_CHECK(C.dim() == 2 && C.stride(1) == 1 && C.size(0) >= M && C.size(1) >= N, "gemm_ks: out shape");
  } else {
    C = at::empty({M, N}, A.options());
  }
  EvxGemmKs a{};
  a.A = A.data_ptr<float>();
  a.lda = A.stride(0);
  a.B = B.data_ptr<float>();
  a.ldb = B.stride(0);
  a.C = C.data_ptr<float>();
  a.ldc = C.stride(0);
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.a_kc = (int)a_kc; a.b_kc = (int)b_kc; a.mode = (int)mode;
  a.alpha = (float)alpha;
  a.alpha_ptr = optf(alpha_ptr);
  if (bias_n.has_value() && bias_n->defined()) {
    CHECK_DEV(*bias_n); CHECK_F32(*bias_n); CHECK_CONTIG(*bias_n);
    TORCH_CHECK(bias_n->numel() >= N, "gemm_ks: bias length");
    a.bias_n = bias_n->data_ptr<float>();
  }
  a.beta = (float)beta;
  if (Cin.has_value() && Cin->defined()) {
    CHECK_DEV(*Cin); CHECK_F32(*Cin);
    TORCH_CHECK(Cin->dim() == 2 && Cin->stride(1) == 1 && Cin->size(0) >= M && Cin->size(1) >= N, "gemm_ks: Cin shape");
    a.Cin = Cin->data_ptr<float>();
    a.ldcin = Cin->stride(0);
  }
  if (skip.has_value() && skip->defined()) {
    CHECK_DEV(*skip);
    TORCH_CHECK(skip->scalar_type() == at::kInt && skip->numel() >= 1, "gemm_ks: skip must be int32");
    a.skip = skip->data_ptr<int32_t>();
  }
  if (a_sub_k.has_value() && a_sub_k->defined()) {
    CHECK_DEV(*a_sub_k); CHECK_F32(*a_sub_k); CHECK_CONTIG(*a_sub_k);
    TORCH_CHECK(a_kc && a_sub_k->numel() >= K && reinterpret_cast<uintptr_t>(a_sub_k->data_ptr()) % 16 == 0,
                "gemm_ks: a_sub_k needs a K-contiguous A and a 16-byte aligned vector of length ≥ K");
    a.a_sub_k = a_sub_k->data_ptr<float>();
  }
  if (sel.has_value() && sel->defined()) {
    CHECK_DEV(*sel);
    TORCH_CHECK(sel->scalar_type() == at::kInt && sel->numel() >= 1, "gemm_ks: sel must be int32");
    a.sel = sel->data_ptr<int32_t>();
    a.alpha2 = (float)alpha2;
    if (A2.has_value() && A2->defined()) {
      TORCH_CHECK(A2->sizes() == A.sizes() && A2->strides() == A.strides() && A2->scalar_type() == at::kFloat, "gemm_ks: A2 like A");
      TORCH_CHECK(!a_kc || vec4_ok(*A2), "gemm_ks: A2 alignment");
      a.A2 = A2->data_ptr<float>();
    }
    if (C2.has_value() && C2->defined()) {
      TORCH_CHECK(C2->sizes() == C.sizes() && C2->strides() == C.strides() && C2->scalar_type() == at::kFloat, "gemm_ks: C2 like out");
      TORCH_CHECK(vec4_ok(*C2) == vec4_ok(C), "gemm_ks: C2 alignment");
      a.C2 = C2->data_ptr<float>();
    }
  }
  if (stat_part.has_value() && stat_part->defined()) {
    TORCH_CHECK(mode == 1, "gemm_ks: stats partials need the symmetric mode");
    CHECK_DEV(*stat_part);
    TORCH_CHECK(stat_part->scalar_type() == at::kDouble && stat_part->is_contiguous() &&
                stat_part->numel() >= 4 * (int64_t)evx_gemm_ks_grid((int)M, (int)N, (int)mode), "gemm_ks: stat_part float64[4·grid]");
    a.stat_part = stat_part->data_ptr<double>();
    a.stat_diag_only = (int)stat_diag_only;
  }
  TORCH_CHECK(prec == 0 || prec == 3, "gemm_ks: prec 0 (process default) or 3 (bf16x3)");
  TORCH_CHECK(diag_add == 0.0 || M == N, "gemm_ks: diag_add needs a square output");
  a.prec = (int)prec;
  a.diag_add = (float)diag_add;
  a.c_vec4 = vec4_ok(C) ? 1 : 0;
  evx_gemm_ks(a, cur_stream());
  return C;
}

// C = alpha·(*alpha_ptr)·op(A)·op(B)ᵀ (+ bias_n) for K-contiguous operands, either of which may be
// given as bf16x6 fragment planes (int16 [3][rows][kp], split_planes / philox_normal_planes)
at::Tensor gemm_ks_pl(const c10::optional<at::Tensor>& A, const c10::optional<at::Tensor>& a_pl, const c10::optional<at::Tensor>& B,
                      const c10::optional<at::Tensor>& b_pl, int64_t M, int64_t N, int64_t K, double alpha,
                      const c10::optional<at::Tensor>& alpha_ptr, const c10::optional<at::Tensor>& bias_n,
                      const c10::optional<at::Tensor>& out, const c10::optional<at::Tensor>& a_sub_k, int64_t sub_cols, int64_t sub_ld) {
  const bool ha = A.has_value() && A->defined(), hap = a_pl.has_value() && a_pl->defined();
  const bool hb = B.has_value() && B->defined(), hbp = b_pl.has_value() && b_pl->defined();
  TORCH_CHECK(ha && hb && !hap && !hbp, "gemm_ks_pl: f32 operands (fragment planes were removed in round 6)");
  TORCH_CHECK(M > 0 && N > 0 && K > 0 && K % 4 == 0, "gemm_ks_pl: shape (K % 4 == 0)");
  const int64_t kp = (K + 31) / 32 * 32;
  auto vec4_ok = [](const at::Tensor& t) { return (reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0) && (t.stride(0) % 4 == 0); };
  auto check_pl = [&](const at::Tensor& t, int64_t rows, const char* w) {
    CHECK_DEV(t);
    TORCH_CHECK(t.scalar_type() == at::kShort && t.dim() == 3 && t.size(0) == 3 && t.size(1) >= rows && t.size(2) == kp && t.is_contiguous(),
                "gemm_ks_pl: ", w, " planes int16 [3, rows, kp]");
  };
  EvxGemmKs a{};
  const at::Tensor& ref = ha ? *A : *a_pl;
  if (ha) {
    CHECK_DEV(*A); CHECK_F32(*A);
    TORCH_CHECK(A->dim() == 2 && A->stride(1) == 1 && A->size(0) >= M && A->size(1) >= K && vec4_ok(*A), "gemm_ks_pl: A");
    a.A = A->data_ptr<float>();
    a.lda = A->stride(0);
  } else {
    check_pl(*a_pl, M, "A");
    a.a_pl = reinterpret_cast<const uint16_t*>(a_pl->data_ptr<int16_t>());
    a.a_pl_rows = a_pl->size(1);
  }
  if (hb) {
    CHECK_DEV(*B); CHECK_F32(*B);
    TORCH_CHECK(B->dim() == 2 && B->stride(1) == 1 && B->size(0) >= N && B->size(1) >= K && vec4_ok(*B), "gemm_ks_pl: B");
    a.B = B->data_ptr<float>();
    a.ldb = B->stride(0);
  } else {
    check_pl(*b_pl, N, "B");
    a.b_pl = reinterpret_cast<const uint16_t*>(b_pl->data_ptr<int16_t>());
    a.b_pl_rows = b_pl->size(1);
  }
  a.pl_kp = kp;
  c10::DeviceGuard g(ref.device());
  at::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    CHECK_DEV(C); CHECK_F32(C);
    TORCH_CHECK(C.dim() == 2 && C.stride(1) == 1 && C.size(0) >= M && C.size(1) >= N, "gemm_ks_pl: out shape");
  } else {
    C = at::empty({M, N}, ref.options().dtype(at::kFloat));
  }
  a.C = C.data_ptr<float>();
  a.ldc = C.stride(0);
  a.M = (int)M; a.N = (int)N; a.K = (int)K;
  a.a_kc = 1; a.b_kc = 1; a.mode = 0;
  a.alpha = (float)alpha;
  a.alpha_ptr = optf(alpha_ptr);
  if (bias_n.has_value() && bias_n->defined()) {
    CHECK_DEV(*bias_n); CHECK_F32(*bias_n); CHECK_CONTIG(*bias_n);
    TORCH_CHECK(bias_n->numel() >= N, "gemm_ks_pl: bias length");
    a.bias_n = bias_n->data_ptr<float>();
  }
  if (a_sub_k.has_value() && a_sub_k->defined()) {
    CHECK_DEV(*a_sub_k); CHECK_F32(*a_sub_k); CHECK_CONTIG(*a_sub_k);
    TORCH_CHECK(ha && a_sub_k->numel() >= K && reinterpret_cast<uintptr_t>(a_sub_k->data_ptr()) % 16 == 0,
                "gemm_ks_pl: a_sub_k needs an f32 A (16-byte aligned, length ≥ K)");
    a.a_sub_k = a_sub_k->data_ptr<float>();
    if (sub_cols > 0) {
      int t = evx_gemm_ks_tile((int)M, (int)N, 0);
      if (sub_cols % (t == 8 ? 64 : 16 * t)) t = a.force_tile = (M >= 2048 ? 8 : 4);  // 64-wide tiles
      const int bn = t == 8 ? 64 : 16 * t;
      TORCH_CHECK(sub_cols % bn == 0 && sub_ld % 4 == 0 && sub_ld >= K && a_sub_k->numel() >= ((N + sub_cols - 1) / sub_cols - 1) * sub_ld + K,
                  "gemm_ks_pl: per-block shifts need sub_cols a multiple of the tile width (", bn, ") and one shift row per block");
      a.sub_cols = (int)sub_cols;
      a.sub_ld = sub_ld;
    }
  }
  a.c_vec4 = vec4_ok(C) ? 1 : 0;
  evx_gemm_ks(a, cur_stream());
  return C;
}

void gemm_ks_set_tile(int64_t t) { evx_gemm_ks_set_tile((int)t); }
void gemm_ks_set_prec(int64_t p) { evx_gemm_ks_set_prec((int)p); }
void gemm_ks_set_nw8(int64_t t) { evx_gemm_ks_set_nw8((int)t); }

at::Tensor gemm_ks_new(const at::Tensor& A, int64_t a_kc, const at::Tensor& B, int64_t b_kc, int64_t M, int64_t N, int64_t K,
                       int64_t mode, double alpha, const c10::optional<at::Tensor>& alpha_ptr,
                       const c10::optional<at::Tensor>& bias_n, double beta, const c10::optional<at::Tensor>& Cin,
                       const c10::optional<at::Tensor>& skip, const c10::optional<at::Tensor>& a_sub_k) {
  return gemm_ks(A, a_kc, B, b_kc, M, N, K, mode, alpha, alpha_ptr, bias_n, beta, Cin, c10::nullopt, skip, a_sub_k);
}

void gemm_ks_out(const at::Tensor& A, int64_t a_kc, const at::Tensor& B, int64_t b_kc, int64_t M, int64_t N, int64_t K,
                 int64_t mode, double alpha, const c10::optional<at::Tensor>& alpha_ptr, const c10::optional<at::Tensor>& bias_n,
                 double beta, const c10::optional<at::Tensor>& Cin, const at::Tensor& out, const c10::optional<at::Tensor>& skip,
                 const c10::optional<at::Tensor>& a_sub_k, const c10::optional<at::Tensor>& sel, const c10::optional<at::Tensor>& A2,
                 double alpha2, const c10::optional<at::Tensor>& C2, const c10::optional<at::Tensor>& stat_part, int64_t stat_diag_only,
                 int64_t prec, double diag_add) {
  gemm_ks(A, a_kc, B, b_kc, M, N, K, mode, alpha, alpha_ptr, bias_n, beta, Cin, out, skip, a_sub_k, sel, A2, alpha2, C2, stat_part,
          stat_diag_only, prec, diag_add);
}

int64_t gemm_ks_grid(int64_t M, int64_t N, int64_t mode) { return evx_gemm_ks_grid((int)M, (int)N, (int)mode); }
int64_t gemm_ks_tile(int64_t M, int64_t N, int64_t mode) { return evx_gemm_ks_tile((int)M, (int)N, (int)mode); }

// CEC'22 F1 / F4 on the device without the rotated population: f(row) of
// z = alpha · (X − o) · Mᵀ from the gemm_ks row-terms epilogue (per column tile, additive) and
// one finishing kernel (gemm_ks.hip, cec2022.hip).  fid 0 = Zakharov, 3 = Rastrigin.
at::Tensor cec_rotated_rowterms(const at::Tensor& X, const at::Tensor& Mrot, const at::Tensor& o, double alpha, int64_t fid) {
  CHECK_DEV(X); CHECK_F32(X); CHECK_DEV(Mrot); CHECK_F32(Mrot); CHECK_DEV(o); CHECK_F32(o); CHECK_CONTIG(o);
  TORCH_CHECK(fid == 0 || fid == 3, "cec_rotated_rowterms: Zakharov (0) or Rastrigin (3)");
  TORCH_CHECK(X.dim() == 2 && Mrot.dim() == 2 && X.stride(1) == 1 && Mrot.stride(1) == 1, "cec_rotated_rowterms: 2-D row-major operands");
  const int64_t N = X.size(0), D = X.size(1);
  TORCH_CHECK(Mrot.size(0) == D && Mrot.size(1) == D && o.numel() >= D, "cec_rotated_rowterms: shapes");
  TORCH_CHECK(D % 4 == 0 && X.stride(0) % 4 == 0 && Mrot.stride(0) % 4 == 0 && reinterpret_cast<uintptr_t>(X.data_ptr()) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(Mrot.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(o.data_ptr()) % 16 == 0,
              "cec_rotated_rowterms: 16-byte aligned operands, D % 4 == 0");
  const int t = evx_gemm_ks_tile((int)N, (int)D, 0);
  TORCH_CHECK(t == 8 || t == 4, "cec_rotated_rowterms: the row-terms epilogue needs a 64-column tile layout");
  c10::DeviceGuard g(X.device());
  const int tiles_n = evx_gemm_ks_tiles_n((int)N, (int)D, 0);
  auto parts = at::empty({tiles_n, N, 2}, X.options());
  auto out = at::empty({N}, X.options());
  EvxGemmKs a{};
  a.A = X.data_ptr<float>();
  a.lda = X.stride(0);
  a.B = Mrot.data_ptr<float>();
  a.ldb = Mrot.stride(0);
  a.C = parts.data_ptr<float>();  // never written in row-terms mode
  a.ldc = D;
  a.M = (int)N; a.N = (int)D; a.K = (int)D;
  a.a_kc = 1; a.b_kc = 1; a.mode = 0;
  a.alpha = (float)alpha;
  a.a_sub_k = o.data_ptr<float>();
  a.row_terms = parts.data_ptr<float>();
  a.row_fid = (int)fid;
  evx_gemm_ks(a, cur_stream());
  evx_cec_rowterms_final(parts.data_ptr<float>(), tiles_n, (int)N, (int)fid, out.data_ptr<float>(), cur_stream());
  return out;
}

// ---- device-controlled SBR schedule (eigh_sbr_dev.hip, ops/sbr_device.py): every op writes
// into caller-owned buffers and honours a device skip word, so a solve is capturable once
void sbr16_block_out(const at::Tensor& A, int64_t shift, int64_t sweeps, int64_t sb, at::Tensor& perm, at::Tensor& Q, at::Tensor& dq,
                     const at::Tensor& skip, double skip_tol) {
  CHECK_DEV(A); CHECK_F32(A);
  const int64_t n = A.size(0);
  TORCH_CHECK(A.dim() == 2 && A.size(1) == n && A.stride(1) == 1 && n <= evx_sbr16_max_n(), "sbr16_block_out: A n×n");
  TORCH_CHECK(sb == 16 || sb == 32, "sbr16_block_out: sb");
  TORCH_CHECK(perm.numel() >= n && perm.scalar_type() == at::kInt && Q.numel() >= evx_sbr16_nblocks((int)n, (int)sb) * sb * sb &&
                  dq.numel() >= n, "sbr16_block_out: buffers");
  evx_sbr16_block(A.data_ptr<float>(), (int)n, A.stride(0), (int)shift, (int)sweeps, perm.data_ptr<int>(), Q.data_ptr<float>(),
                  dq.data_ptr<float>(), (int)sb, cur_stream(), skip.data_ptr<int>(), (float)skip_tol);
}

void sbr16_far_out(const at::Tensor& A, const at::Tensor& perm, const at::Tensor& Q, const at::Tensor& dq, const at::Tensor& stats,
                   double thr_fac, const at::Tensor& theta, at::Tensor& X, int64_t sb, const at::Tensor& skip) {
  const int64_t n = A.size(0);
  TORCH_CHECK(X.sizes() == A.sizes() && X.stride(1) == 1 && stats.scalar_type() == at::kDouble && theta.scalar_type() == at::kFloat,
              "sbr16_far_out: shapes");
  evx_sbr16_far(A.data_ptr<float>(), (int)n, A.stride(0), perm.data_ptr<int>(), Q.data_ptr<float>(), dq.data_ptr<float>(),
                stats.data_ptr<double>(), (float)thr_fac, 0.f, X.data_ptr<float>(), X.stride(0), (int)sb, cur_stream(),
                theta.data_ptr<float>(), skip.data_ptr<int>());
}

void sbr16_far_bq_out(const at::Tensor& A, const at::Tensor& perm, const at::Tensor& Q, const at::Tensor& dq, const at::Tensor& stats,
                      double thr_fac, const at::Tensor& theta, at::Tensor& X, const at::Tensor& B, at::Tensor& Bq, int64_t sb,
                      const at::Tensor& skip_far, const at::Tensor& skip_bq, bool pre) {
  // pre: A = A[perm, perm] and B = B[:, perm] already (sbr16_permute_out)
  const int64_t n = A.size(0);
  TORCH_CHECK(X.sizes() == A.sizes() && X.stride(1) == 1 && A.stride(1) == 1 && stats.scalar_type() == at::kDouble &&
                  theta.scalar_type() == at::kFloat, "sbr16_far_bq_out: generator shapes");
  TORCH_CHECK(Bq.sizes() == B.sizes() && B.size(1) == n && Bq.stride(1) == 1 && B.stride(1) == 1, "sbr16_far_bq_out: Bq shapes");
  TORCH_CHECK(perm.numel() >= n && dq.numel() >= n && Q.numel() >= evx_sbr16_nblocks((int)n, (int)sb) * sb * sb, "sbr16_far_bq_out: perm / Q");
  TORCH_CHECK(skip_far.scalar_type() == at::kInt && skip_bq.scalar_type() == at::kInt, "sbr16_far_bq_out: skip words int32");
  evx_sbr16_far_bq(A.data_ptr<float>(), (int)n, A.stride(0), perm.data_ptr<int>(), Q.data_ptr<float>(), dq.data_ptr<float>(),
                   stats.data_ptr<double>(), (float)thr_fac, theta.data_ptr<float>(), X.data_ptr<float>(), X.stride(0), B.data_ptr<float>(),
                   (int)B.size(0), B.stride(0), Bq.data_ptr<float>(), Bq.stride(0), (int)sb, cur_stream(), skip_far.data_ptr<int>(),
                   skip_bq.data_ptr<int>(), pre);
}

void sbr16_bq_out(const at::Tensor& B, const at::Tensor& perm, const at::Tensor& Q, at::Tensor& Bq, int64_t sb, const at::Tensor& skip) {
  const int64_t n = B.size(1);
  TORCH_CHECK(Bq.sizes() == B.sizes() && Bq.stride(1) == 1 && B.stride(1) == 1, "sbr16_bq_out: shapes");
  evx_sbr16_bq(B.data_ptr<float>(), (int)B.size(0), (int)n, B.stride(0), perm.data_ptr<int>(), Q.data_ptr<float>(), Bq.data_ptr<float>(),
               Bq.stride(0), (int)sb, cur_stream(), skip.data_ptr<int>());
}

// X² stats partials (gemm_ks MODE 1 epilogue, double[4·nparts]) for the free ‖X‖ bound, may be absent
const double* xpart_ptr(const c10::optional<at::Tensor>& xpart, int64_t& nparts) {
  nparts = 0;
  if (!xpart.has_value() || !xpart->defined()) return nullptr;
  CHECK_DEV(*xpart); CHECK_CONTIG(*xpart);
  TORCH_CHECK(xpart->scalar_type() == at::kDouble && xpart->numel() % 4 == 0, "xpart: float64[4·nparts]");
  nparts = xpart->numel() / 4;
  return xpart->data_ptr<double>();
}

void sbr_damping_out(const at::Tensor& X2, const at::Tensor& V, double tau, at::Tensor& alpha, at::Tensor& work, const at::Tensor& skip,
                     const c10::optional<at::Tensor>& bar, bool no_final, const c10::optional<at::Tensor>& xpart) {
  const int64_t n = X2.size(0);
  TORCH_CHECK(V.numel() >= n * 8 && work.numel() >= n * 24 && alpha.numel() >= 1, "sbr_damping_out: shapes");
  TORCH_CHECK(!(bar.has_value() && bar->defined()), "sbr_damping_out: the grid-barrier damping was removed (round 5)");
  int64_t np = 0;
  const double* xp = xpart_ptr(xpart, np);
  evx_sbr_damping(X2.data_ptr<float>(), (int)n, X2.stride(0), V.data_ptr<float>(), work.data_ptr<float>(), (float)tau,
                  alpha.data_ptr<float>(), cur_stream(), skip.data_ptr<int>(), no_final ? 1 : 0, xp, (int)np);
}

void sbr_dev_prep(const at::Tensor& X, const at::Tensor& X2, const at::Tensor& X3, at::Tensor& alpha, at::Tensor& P, at::Tensor& MT,
                  const at::Tensor& ctrl, const c10::optional<at::Tensor>& work, double tau, const c10::optional<at::Tensor>& xpart,
                  const c10::optional<at::Tensor>& copy_src, const c10::optional<at::Tensor>& copy_dst, int64_t minus_id) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&X, &X2, &X3, &P, &MT}) {
    CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t);
    TORCH_CHECK(t->sizes() == X.sizes(), "sbr_dev_prep: n×n");
  }
  TORCH_CHECK(ctrl.scalar_type() == at::kInt && ctrl.numel() >= 8 && alpha.numel() >= 1, "sbr_dev_prep: ctrl int32[8]");
  const float* v2 = nullptr;
  const float* v3 = nullptr;
  if (work && work->defined()) {  // the damping's power-step vectors [V1 | V2 | V3] (n×8 each): α formed here
    const int64_t n = X.size(0);
    CHECK_DEV(*work); CHECK_F32(*work);
    TORCH_CHECK(work->is_contiguous() && work->numel() >= 24 * n, "sbr_dev_prep: work float[24 n]");
    v2 = work->data_ptr<float>() + 8 * n;
    v3 = work->data_ptr<float>() + 16 * n;
  }
  int64_t np = 0;
  const double* xp = xpart_ptr(xpart, np);
  // near-only iterations' basis copy (copy_src → copy_dst when ctrl[1] && !ctrl[7])
  const float* cs = nullptr;
  float* cd = nullptr;
  if (copy_src.has_value() && copy_src->defined()) {
    TORCH_CHECK(copy_dst.has_value() && copy_dst->defined(), "sbr_dev_prep: copy_src with copy_dst");
    for (const at::Tensor* t : {&*copy_src, &*copy_dst}) {
      CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t);
      TORCH_CHECK(t->sizes() == X.sizes() && reinterpret_cast<uintptr_t>(t->data_ptr()) % 16 == 0, "sbr_dev_prep: copy n×n, 16-B aligned");
    }
    cs = copy_src->data_ptr<float>();
    cd = copy_dst->data_ptr<float>();
  }
  evx_sbr_dev_prep(X.data_ptr<float>(), X2.data_ptr<float>(), X3.data_ptr<float>(), (int)X.size(0), alpha.data_ptr<float>(),
                   P.data_ptr<float>(), MT.data_ptr<float>(), ctrl.data_ptr<int>(), cur_stream(), v2, v3, (float)tau, xp, (int)np, cs, cd, (int)minus_id);
}

void sbr_dev_copy(const at::Tensor& src, at::Tensor& dst, const at::Tensor& skip) {
  CHECK_CONTIG(src); CHECK_CONTIG(dst);
  TORCH_CHECK(src.numel() == dst.numel() && src.scalar_type() == at::kFloat && dst.scalar_type() == at::kFloat &&
                  reinterpret_cast<uintptr_t>(src.data_ptr()) % 16 == 0 && reinterpret_cast<uintptr_t>(dst.data_ptr()) % 16 == 0,
              "sbr_dev_copy: 16-byte aligned float32 of one size");
  evx_sbr_dev_copy(src.data_ptr<float>(), dst.data_ptr<float>(), src.numel(), skip.data_ptr<int>(), cur_stream());
}

void sbr_dev_ctrl(const at::Tensor& part, int64_t nparts, int64_t j, int64_t K, at::Tensor& hist, at::Tensor& alpha, at::Tensor& theta,
                  at::Tensor& ctrl, at::Tensor& st, std::vector<double> prm, int64_t ns_iters, const at::Tensor& A, at::Tensor& w_out,
                  at::Tensor& eig_stats, at::Tensor& w_init, at::Tensor& log, at::Tensor& log_count,
                  const c10::optional<at::Tensor>& rep_seq, const c10::optional<at::Tensor>& rep_ring) {
  TORCH_CHECK(log.scalar_type() == at::kDouble && log.is_contiguous() && log_count.scalar_type() == at::kInt, "sbr_dev_ctrl: log");
  int* rs = nullptr;
  double* rr = nullptr;
  int rl = 0;
  if (rep_seq.has_value() && rep_seq->defined()) {  // the last slot also reports into the host-mapped ring
    TORCH_CHECK(rep_seq->is_cuda() && rep_seq->scalar_type() == at::kInt && rep_seq->numel() >= 1, "sbr_dev_ctrl: device int32 counter");
    TORCH_CHECK(rep_ring.has_value() && !rep_ring->is_cuda() && rep_ring->is_pinned() && rep_ring->scalar_type() == at::kDouble &&
                    rep_ring->is_contiguous() && rep_ring->dim() == 2 && rep_ring->size(1) == 5,
                "sbr_dev_ctrl: pinned host float64 [R, 5] ring");
    rs = rep_seq->data_ptr<int>();
    rr = rep_ring->data_ptr<double>();
    rl = (int)rep_ring->size(0);
  }
  TORCH_CHECK(prm.size() >= 8, "sbr_dev_ctrl: params [tol, ns_kappa, damp_kappa, t4_kappa, near_only, theta0, theta_kappa, lean_from, (recover, lean_guard, xgate, damp_from)]");
  TORCH_CHECK(hist.scalar_type() == at::kDouble && hist.numel() >= 4 * (K + 1) && ctrl.numel() >= 8 * K && alpha.numel() >= K + 1 &&
                  theta.numel() >= K && st.numel() >= 8 && part.numel() >= 4 * nparts, "sbr_dev_ctrl: buffers");
  float p6[7] = {(float)prm[0], (float)prm[1], (float)prm[2], (float)prm[3], (float)prm[4], (float)prm[5], (float)prm[6]};
  evx_sbr_dev_ctrl(part.data_ptr<double>(), (int)nparts, (int)j, (int)K, hist.data_ptr<double>(), alpha.data_ptr<float>(),
                   theta.data_ptr<float>(), ctrl.data_ptr<int>(), st.data_ptr<int>(), p6, (int)ns_iters, A.data_ptr<float>(), A.stride(0),
                   (int)A.size(0), w_out.data_ptr<float>(), eig_stats.data_ptr<double>(), w_init.data_ptr<float>(),
                   log.data_ptr<double>(), (int)(log.numel() / 4), log_count.data_ptr<int>(), cur_stream(), (int)prm[7],
                   prm.size() > 8 ? (int)prm[8] : 0, prm.size() > 9 ? (int)prm[9] : 0, prm.size() > 10 ? (int)prm[10] : 0,
                   prm.size() > 11 ? (int)prm[11] : -1, rs, rr, rl);
}

std::vector<at::Tensor> argsort_f32(const at::Tensor& keys, int64_t descending) {
  // 1-D keys, or (B, n): B independent rows sorted by B workgroups of one launch
  CHECK_DEV(keys); CHECK_F32(keys); CHECK_CONTIG(keys);
  TORCH_CHECK(keys.dim() <= 2, "argsort_f32: keys must be (n,) or (B, n)");
  const int64_t B = keys.dim() == 2 ? keys.size(0) : 1;
  const int64_t n = keys.dim() == 0 ? 1 : keys.size(-1);
  TORCH_CHECK(n <= evx_argsort_max_n(), "argsort_f32: n > ", evx_argsort_max_n());
  TORCH_CHECK(B <= 65535, "argsort_f32: B > 65535");
  c10::DeviceGuard g(keys.device());
  auto ok = at::empty_like(keys);
  auto oi = at::empty(keys.sizes(), keys.options().dtype(at::kInt));
  if (n > 0 && B > 0)
    evx_argsort(keys.data_ptr<float>(), (int)n, (int)descending, ok.data_ptr<float>(), oi.data_ptr<int32_t>(), cur_stream(), (int)B);
  return {ok, oi};
}

// same contract as argsort_f32, rocPRIM block radix sort in one workgroup per row (sort.hip)
std::vector<at::Tensor> radix_argsort_f32(const at::Tensor& keys, int64_t descending) {
  CHECK_DEV(keys); CHECK_F32(keys); CHECK_CONTIG(keys);
  TORCH_CHECK(keys.dim() <= 2, "radix_argsort_f32: keys must be (n,) or (B, n)");
  const int64_t B = keys.dim() == 2 ? keys.size(0) : 1;
  const int64_t n = keys.dim() == 0 ? 1 : keys.size(-1);
  TORCH_CHECK(n <= evx_argsort_max_n(), "radix_argsort_f32: n > ", evx_argsort_max_n());
  TORCH_CHECK(B <= 65535, "radix_argsort_f32: B > 65535");
  c10::DeviceGuard g(keys.device());
  auto ok = at::empty_like(keys);
  auto oi = at::empty(keys.sizes(), keys.options().dtype(at::kInt));
  if (n > 0 && B > 0)
    evx_radix_argsort(keys.data_ptr<float>(), (int)n, (int)descending, ok.data_ptr<float>(), oi.data_ptr<int32_t>(), cur_stream(), (int)B);
  return {ok, oi};
}

// same contract as radix_argsort_f32: rank-by-counting, one launch for n ≤ 16384 (sort.hip)
std::vector<at::Tensor> merge_argsort_f32(const at::Tensor& keys, int64_t descending) {
  CHECK_DEV(keys); CHECK_F32(keys); CHECK_CONTIG(keys);
  TORCH_CHECK(keys.dim() <= 2, "merge_argsort_f32: keys must be (n,) or (B, n)");
  const int64_t B = keys.dim() == 2 ? keys.size(0) : 1;
  const int64_t n = keys.dim() == 0 ? 1 : keys.size(-1);
  TORCH_CHECK(n <= evx_merge_argsort_max_n(), "merge_argsort_f32: n > ", evx_merge_argsort_max_n());
  TORCH_CHECK(B * ((n + 4095) / 4096) <= 65535, "merge_argsort_f32: B * chunks > 65535");
  c10::DeviceGuard g(keys.device());
  auto ok = at::empty_like(keys);
  auto oi = at::empty(keys.sizes(), keys.options().dtype(at::kInt));
  auto wk = at::empty(keys.sizes(), keys.options().dtype(at::kInt));
  auto wi = at::empty(keys.sizes(), keys.options().dtype(at::kInt));
  if (n > 0 && B > 0)
    evx_merge_argsort(keys.data_ptr<float>(), (int)n, (int)descending, ok.data_ptr<float>(), oi.data_ptr<int32_t>(),
                      reinterpret_cast<uint32_t*>(wk.data_ptr<int32_t>()), wi.data_ptr<int32_t>(), cur_stream(), (int)B);
  return {ok, oi};
}

std::vector<at::Tensor> rank_argsort_f32(const at::Tensor& keys, int64_t descending) {
  CHECK_DEV(keys); CHECK_F32(keys); CHECK_CONTIG(keys);
  TORCH_CHECK(keys.dim() <= 2, "rank_argsort_f32: keys must be (n,) or (B, n)");
  const int64_t B = keys.dim() == 2 ? keys.size(0) : 1;
  const int64_t n = keys.dim() == 0 ? 1 : keys.size(-1);
  TORCH_CHECK(n <= evx_rank_argsort_max_n(), "rank_argsort_f32: n > ", evx_rank_argsort_max_n());
  TORCH_CHECK(B <= 65535, "rank_argsort_f32: B > 65535");
  c10::DeviceGuard g(keys.device());
  auto ok = at::empty_like(keys);
  auto oi = at::empty(keys.sizes(), keys.options().dtype(at::kInt));
  if (n > 0 && B > 0)
    evx_rank_argsort(keys.data_ptr<float>(), (int)n, (int)descending, ok.data_ptr<float>(), oi.data_ptr<int32_t>(), cur_stream(), (int)B);
  return {ok, oi};
}

at::Tensor cec_basic(const at::Tensor& Z, int64_t fid, const c10::optional<at::Tensor>& perm, int64_t start, int64_t L,
                     const c10::optional<at::Tensor>& sub, double scale, const c10::optional<at::Tensor>& Y, int64_t ystart,
                     int64_t yperm, double clamp) {
  CHECK_DEV(Z); CHECK_F32(Z);
  TORCH_CHECK(Z.dim() == 2 && Z.stride(1) == 1, "Z must be 2-D row-major");
  const int32_t* pp = nullptr;
  if (perm.has_value() && perm->defined()) {
    TORCH_CHECK(perm->scalar_type() == at::kInt && perm->is_contiguous() && perm->numel() >= start + L, "perm");
    pp = perm->data_ptr<int32_t>();
  } else {
    TORCH_CHECK(start + L <= Z.size(1), "segment out of range");
  }
  TORCH_CHECK(!yperm || pp, "yperm needs perm");
  const float* yp = nullptr;
  int64_t ldy = 0;
  if (Y.has_value() && Y->defined()) {
    CHECK_DEV(*Y); CHECK_F32(*Y);
    TORCH_CHECK(Y->dim() == 2 && Y->stride(1) == 1 && Y->size(0) == Z.size(0) && Y->size(1) >= ystart + L, "Y shape");
    yp = Y->data_ptr<float>();
    ldy = Y->stride(0);
  }
  c10::DeviceGuard g(Z.device());
  auto out = at::empty({Z.size(0)}, Z.options());
  if (Z.size(0) > 0)
    evx_cec_basic(Z.data_ptr<float>(), Z.stride(0), (int)Z.size(0), (int)fid, pp, (int)start, (int)L, optf(sub), (float)scale,
                  yp, ldy, (int)ystart, (int)yperm, out.data_ptr<float>(), cur_stream(), (float)clamp);
  return out;
}

// composition functions in one pass (cec2022.hip: cec_compose_kernel); Z: the stacked rotation
// GEMM output (parts with zcol < 0 read x − Os[comp] instead)
at::Tensor cec_compose(const c10::optional<at::Tensor>& Z, const at::Tensor& X, const at::Tensor& Os, at::IntArrayRef fid,
                       at::IntArrayRef zcol, at::IntArrayRef comp, at::ArrayRef<double> scale, at::ArrayRef<double> sigma,
                       at::ArrayRef<double> lamb, at::ArrayRef<double> bias, double thr) {
  CHECK_DEV(X); CHECK_F32(X); CHECK_DEV(Os); CHECK_F32(Os);
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "cec_compose: X 2-D row-major");
  const int64_t N = X.size(0), D = X.size(1), n = (int64_t)fid.size();
  TORCH_CHECK(n >= 1 && n <= kEvxCecMaxParts, "cec_compose: 1..", kEvxCecMaxParts, " parts");
  TORCH_CHECK((int64_t)zcol.size() == n && (int64_t)comp.size() == n && (int64_t)scale.size() == n && (int64_t)sigma.size() == n &&
                  (int64_t)lamb.size() == n && (int64_t)bias.size() == n,
              "cec_compose: one entry per part");
  TORCH_CHECK(Os.dim() == 2 && Os.stride(1) == 1 && Os.size(0) >= n && Os.size(1) >= D, "cec_compose: Os (>= parts) x D");
  TORCH_CHECK(D >= 2, "cec_compose: D >= 2");
  EvxCecCompose c{};
  c.n = (int)n;
  const float* zp = nullptr;
  int64_t ldz = 0;
  for (int64_t i = 0; i < n; ++i) {
    TORCH_CHECK(fid[i] != 2, "cec_compose: SCHAFFERF7 is a hybrid-only component");
    TORCH_CHECK(comp[i] >= 0 && comp[i] < Os.size(0), "cec_compose: comp index");
    c.fid[i] = (int)fid[i];
    c.zcol[i] = (int)zcol[i];
    c.comp[i] = (int)comp[i];
    c.scale[i] = (float)scale[i];
    c.sigma[i] = (float)sigma[i];
    c.lamb[i] = (float)lamb[i];
    c.bias[i] = (float)bias[i];
    if (zcol[i] >= 0) {
      TORCH_CHECK(Z.has_value() && Z->defined(), "cec_compose: rotated parts need Z");
      CHECK_DEV(*Z); CHECK_F32(*Z);
      TORCH_CHECK(Z->dim() == 2 && Z->stride(1) == 1 && Z->size(0) == N && zcol[i] + D <= Z->size(1), "cec_compose: Z block");
      zp = Z->data_ptr<float>();
      ldz = Z->stride(0);
    }
  }
  c.os = Os.data_ptr<float>();
  c.ldo = Os.stride(0);
  c.thr = (float)thr;
  c10::DeviceGuard g(X.device());
  auto out = at::empty({N}, X.options());
  auto part = at::empty({N * n * 2}, X.options());
  evx_cec_compose(zp, ldz, X.data_ptr<float>(), X.stride(0), (int)N, (int)D, c, part.data_ptr<float>(), out.data_ptr<float>(), cur_stream());
  return out;
}

// Runs `sweeps` block-Jacobi sweeps in place on A (np×np) and B (np×np).  All kernels
// are enqueued on the current stream; convergence is a device flag, so the call is
// graph-capturable.  Returns [w(np) diag of A, stats(2) = (off², diag²) at the last check].
std::vector<at::Tensor> jacobi_sweeps(at::Tensor A, at::Tensor B, const at::Tensor& sched, int64_t sweeps, double tol,
                                      double inner_tol, int64_t max_inner, int64_t fused) {
  CHECK_DEV(A); CHECK_F32(A); CHECK_CONTIG(A); CHECK_DEV(B); CHECK_F32(B); CHECK_CONTIG(B);
  const int64_t np = A.size(0);
  TORCH_CHECK(A.dim() == 2 && A.size(1) == np && B.sizes() == A.sizes(), "A, B must be np×np");
  TORCH_CHECK(np % 32 == 0, "np must be a multiple of 32");
  const int64_t nb = np / 16;
  TORCH_CHECK(sched.scalar_type() == at::kInt && sched.is_contiguous() && sched.dim() == 2 && sched.size(0) == nb &&
                  sched.size(1) == nb, "schedule must be int32 [nb, nb] (row 0: within-block pairing, rows 1..: rounds)");
  CHECK_DEV(sched);
  c10::DeviceGuard g(A.device());
  auto opts = A.options();
  auto flag = at::zeros({1}, opts.dtype(at::kInt));
  auto part = at::empty({2 * evx_jacobi_parts()}, opts.dtype(at::kDouble));
  auto stats = at::zeros({2}, opts.dtype(at::kDouble));
  const int64_t npairs = np / 32;
  hipStream_t st = cur_stream();
  const double tol2 = tol * tol;
  evx_jacobi_check(A.data_ptr<float>(), (int)np, part.data_ptr<double>(), flag.data_ptr<int>(), tol2, stats.data_ptr<double>(), st);
  const int* sp = sched.data_ptr<int>();
  if (fused == 2) {  // default: B update overlapped with the next round's solves
    auto Vbuf = at::empty({2, npairs * 32 * 32}, opts);
    for (int64_t sw = 0; sw < sweeps; ++sw) {
      evx_jacobi_sweep_overlapB(A.data_ptr<float>(), B.data_ptr<float>(), (int)np, Vbuf[0].data_ptr<float>(),
                                Vbuf[1].data_ptr<float>(), flag.data_ptr<int>(), (float)inner_tol, (int)max_inner, st);
      evx_jacobi_check(A.data_ptr<float>(), (int)np, part.data_ptr<double>(), flag.data_ptr<int>(), tol2, stats.data_ptr<double>(), st);
    }
    return {A.diagonal().clone(), stats};
  }
  if (!fused) {
    auto Vbuf = at::empty({npairs * 32 * 32}, opts);
    for (int64_t sw = 0; sw < sweeps; ++sw) {
      for (int64_t t = 0; t < nb; ++t)
        evx_jacobi_round(A.data_ptr<float>(), B.data_ptr<float>(), (int)np, (int)t, Vbuf.data_ptr<float>(),
                         flag.data_ptr<int>(), (float)inner_tol, (int)max_inner, st);
      evx_jacobi_check(A.data_ptr<float>(), (int)np, part.data_ptr<double>(), flag.data_ptr<int>(), tol2, stats.data_ptr<double>(), st);
    }
    return {A.diagonal().clone(), stats};
  }
  // fused: every apply launch also solves the next round's subproblems (V double-buffered)
  TORCH_CHECK(nb <= 256, "fused Jacobi: np <= 4096");
  auto Vbuf = at::empty({2, npairs * 32 * 32}, opts);
  auto counters = at::zeros({std::max<int64_t>(sweeps, 1) * nb * npairs}, opts.dtype(at::kInt));
  float* V[2] = {Vbuf[0].data_ptr<float>(), Vbuf[1].data_ptr<float>()};
  if (sweeps > 0)
    evx_jacobi_solve(A.data_ptr<float>(), (int)np, sp, V[0], flag.data_ptr<int>(), (float)inner_tol, (int)max_inner, 1, st);
  for (int64_t sw = 0; sw < sweeps; ++sw) {
    for (int64_t t = 0; t < nb; ++t) {
      const int64_t r = sw * nb + t;
      const bool last = sw == sweeps - 1 && t == nb - 1;
      const int64_t tn = (t + 1) % nb;
      evx_jacobi_apply_solve(A.data_ptr<float>(), B.data_ptr<float>(), (int)np, sp + t * nb, V[r & 1], flag.data_ptr<int>(),
                             last ? nullptr : sp + tn * nb, tn == 0 ? 1 : 0, V[(r + 1) & 1], counters.data_ptr<int>() + r * npairs,
                             (float)inner_tol, (int)max_inner, st);
    }
    evx_jacobi_check(A.data_ptr<float>(), (int)np, part.data_ptr<double>(), flag.data_ptr<int>(), tol2, stats.data_ptr<double>(), st);
  }
  return {A.diagonal().clone(), stats};
}


// ---------------------------------------------------------------- sorted-block refinement (eigh_sbr.hip)
// A / B may be row-major views with a leading dimension (e.g. the n×n corner of a padded operand).
void check_rowmajor(const at::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.dim() == 2 && t.stride(1) == 1 && t.stride(0) >= t.size(1),
              name, " must be a row-major float32 device matrix");
}

at::Tensor sbr_stats(const at::Tensor& A) {
  check_rowmajor(A, "A");
  TORCH_CHECK(A.size(0) == A.size(1), "A must be square");
  c10::DeviceGuard g(A.device());
  auto o = A.options().dtype(at::kDouble);
  auto part = at::empty({4 * evx_sbr_stat_parts()}, o);
  auto out = at::empty({4}, o);
  evx_sbr_stats(A.data_ptr<float>(), (int)A.size(0), A.stride(0), part.data_ptr<double>(), out.data_ptr<double>(), cur_stream());
  return out;
}

std::vector<at::Tensor> sbr_block(const at::Tensor& A, int64_t off, int64_t sweeps, const c10::optional<at::Tensor>& dbg) {
  check_rowmajor(A, "A");
  const int64_t n = A.size(0);
  TORCH_CHECK(A.size(1) == n && n >= 2 && n <= 2048, "sbr_block: square A with 2 <= n <= 2048");
  TORCH_CHECK(off == 0 || off == 32, "sbr_block: block offset must be 0 or 32");
  c10::DeviceGuard g(A.device());
  const int nb = evx_sbr_nblocks((int)n, (int)off);
  auto perm = at::empty({n}, A.options().dtype(at::kInt));
  auto Q = at::empty({nb, 64, 64}, A.options());
  auto dq = at::empty({n}, A.options());
  evx_sbr_block(A.data_ptr<float>(), (int)n, A.stride(0), (int)off, (int)sweeps, perm.data_ptr<int>(), Q.data_ptr<float>(),
                dq.data_ptr<float>(), cur_stream(), dbg ? (long long*)dbg->data_ptr<int64_t>() : nullptr);
  return {perm, Q, dq};
}

at::Tensor sbr_far(const at::Tensor& A, int64_t off, const at::Tensor& perm, const at::Tensor& Q, const at::Tensor& dq,
                   const at::Tensor& stats, double thr_fac) {
  check_rowmajor(A, "A");
  const int64_t n = A.size(0);
  const int nb = evx_sbr_nblocks((int)n, (int)off);
  TORCH_CHECK(perm.is_cuda() && perm.scalar_type() == at::kInt && perm.numel() == n && perm.is_contiguous(), "perm int32[n]");
  TORCH_CHECK(Q.is_cuda() && Q.scalar_type() == at::kFloat && Q.is_contiguous() && Q.numel() == (int64_t)nb * 4096, "Q [nb,64,64]");
  TORCH_CHECK(dq.is_cuda() && dq.scalar_type() == at::kFloat && dq.numel() == n && dq.is_contiguous(), "dq float[n]");
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kDouble && stats.numel() == 4, "stats double[4]");
  c10::DeviceGuard g(A.device());
  auto X = at::empty({n, n}, A.options());
  evx_sbr_far(A.data_ptr<float>(), (int)n, A.stride(0), (int)off, perm.data_ptr<int>(), Q.data_ptr<float>(), dq.data_ptr<float>(),
              stats.data_ptr<double>(), (float)thr_fac, X.data_ptr<float>(), n, cur_stream());
  return X;
}

at::Tensor sbr_bq(const at::Tensor& B, int64_t off, const at::Tensor& perm, const at::Tensor& Q) {
  check_rowmajor(B, "B");
  const int64_t rows = B.size(0), n = B.size(1);
  const int nb = evx_sbr_nblocks((int)n, (int)off);
  TORCH_CHECK(perm.is_cuda() && perm.scalar_type() == at::kInt && perm.numel() == n && perm.is_contiguous(), "perm int32[n]");
  TORCH_CHECK(Q.is_cuda() && Q.scalar_type() == at::kFloat && Q.is_contiguous() && Q.numel() == (int64_t)nb * 4096, "Q [nb,64,64]");
  c10::DeviceGuard g(B.device());
  auto Bq = at::empty({rows, n}, B.options());
  evx_sbr_bq(B.data_ptr<float>(), (int)rows, (int)n, B.stride(0), (int)off, perm.data_ptr<int>(), Q.data_ptr<float>(),
             Bq.data_ptr<float>(), n, cur_stream());
  return Bq;
}


// 16-wide blocks in a shifted sorted order (eigh_sbr16.hip)
std::vector<at::Tensor> sbr16_block(const at::Tensor& A, int64_t shift, int64_t sweeps, int64_t sb) {
  check_rowmajor(A, "A");
  const int64_t n = A.size(0);
  TORCH_CHECK(A.size(1) == n && n >= 2 && n <= evx_sbr16_max_n(), "sbr16_block: square A with 2 <= n <= ", evx_sbr16_max_n());
  TORCH_CHECK(shift >= 0 && shift < n, "sbr16_block: shift in [0, n)");
  TORCH_CHECK(sweeps >= 0 && sweeps <= 64, "sbr16_block: sweeps in [0, 64]");
  TORCH_CHECK(sb == 16 || sb == 32, "sbr16_block: block size 16 or 32");
  c10::DeviceGuard g(A.device());
  const int nb = evx_sbr16_nblocks((int)n, (int)sb);
  auto perm = at::empty({n}, A.options().dtype(at::kInt));
  auto Q = at::empty({nb, sb, sb}, A.options());
  auto dq = at::empty({n}, A.options());
  evx_sbr16_block(A.data_ptr<float>(), (int)n, A.stride(0), (int)shift, (int)sweeps, perm.data_ptr<int>(), Q.data_ptr<float>(),
                  dq.data_ptr<float>(), (int)sb, cur_stream());
  return {perm, Q, dq};
}

// α = min(1, τ/‖X‖₂) from three power steps on −X² with the n×8 probe block V
at::Tensor sbr_damping(const at::Tensor& X2, const at::Tensor& V, double tau, const c10::optional<at::Tensor>& out) {
  check_rowmajor(X2, "X2");
  const int64_t n = X2.size(0);
  TORCH_CHECK(X2.size(1) == n, "X2 must be square");
  TORCH_CHECK(V.is_cuda() && V.scalar_type() == at::kFloat && V.is_contiguous() && V.dim() == 2 && V.size(0) == n && V.size(1) == 8,
              "V must be a contiguous float32 n×8 device matrix");
  c10::DeviceGuard g(X2.device());
  auto work = at::empty({3, n, 8}, X2.options());
  at::Tensor alpha = out ? *out : at::empty({1}, X2.options());
  TORCH_CHECK(alpha.is_cuda() && alpha.scalar_type() == at::kFloat && alpha.numel() == 1 && alpha.is_contiguous(), "out: float32[1]");
  evx_sbr_damping(X2.data_ptr<float>(), (int)n, X2.stride(0), V.data_ptr<float>(), work.data_ptr<float>(), (float)tau,
                  alpha.data_ptr<float>(), cur_stream());
  return alpha;
}

std::vector<at::Tensor> sbr_taylor4_prep(const at::Tensor& X, const at::Tensor& X2, const c10::optional<at::Tensor>& alpha, int64_t mt) {
  CHECK_DEV(X); CHECK_F32(X); CHECK_CONTIG(X); CHECK_CONTIG(X2);
  const int64_t n = X.size(0);
  TORCH_CHECK(X.dim() == 2 && X.size(1) == n && X2.sizes() == X.sizes(), "sbr_taylor4_prep: n×n");
  const float* ap = nullptr;
  if (alpha) {
    TORCH_CHECK(alpha->numel() == 1 && alpha->scalar_type() == at::kFloat, "sbr_taylor4_prep: alpha float32[1]");
    ap = alpha->data_ptr<float>();
  }
  c10::DeviceGuard g(X.device());
  auto P = at::empty_like(X), M = at::empty_like(X);
  evx_sbr_taylor4_prep(X.data_ptr<float>(), X2.data_ptr<float>(), (int)n, ap, P.data_ptr<float>(), M.data_ptr<float>(), cur_stream(),
                       (int)mt);
  return {P, M};
}

// (v, s²) of linear-kernel GP regressions from (Σf², Σf·x, Σx², n), all float64 of one shape
std::vector<at::Tensor> linear_gp_fit(const at::Tensor& a, const at::Tensor& b, const at::Tensor& c, const at::Tensor& n, int64_t steps,
                                      double lr) {
  for (const at::Tensor* t : {&a, &b, &c, &n}) {
    TORCH_CHECK(t->is_cuda() && t->scalar_type() == at::kDouble && t->is_contiguous() && t->sizes() == a.sizes(),
                "linear_gp_fit: contiguous float64 device tensors of one shape");
  }
  c10::DeviceGuard g(a.device());
  auto v = at::empty(a.sizes(), a.options().dtype(at::kFloat)), s2 = at::empty(a.sizes(), a.options().dtype(at::kFloat));
  evx_linear_gp_fit(a.data_ptr<double>(), b.data_ptr<double>(), c.data_ptr<double>(), n.data_ptr<double>(), a.numel(), (int)steps, lr,
                    v.data_ptr<float>(), s2.data_ptr<float>(), cur_stream());
  return {v, s2};
}

int64_t check_sbr16_operands(int64_t n, const at::Tensor& perm, const at::Tensor& Q) {
  TORCH_CHECK(perm.is_cuda() && perm.scalar_type() == at::kInt && perm.numel() == n && perm.is_contiguous(), "perm int32[n]");
  TORCH_CHECK(Q.dim() == 3 && (Q.size(1) == 16 || Q.size(1) == 32) && Q.size(2) == Q.size(1), "Q [nb, sb, sb], sb 16 or 32");
  const int64_t sb = Q.size(1);
  TORCH_CHECK(Q.is_cuda() && Q.scalar_type() == at::kFloat && Q.is_contiguous() && Q.size(0) == evx_sbr16_nblocks((int)n, (int)sb),
              "Q [ceil(n/sb), sb, sb]");
  return sb;
}

at::Tensor sbr16_far(const at::Tensor& A, const at::Tensor& perm, const at::Tensor& Q, const at::Tensor& dq, const at::Tensor& stats,
                     double thr_fac, double theta) {
  check_rowmajor(A, "A");
  const int64_t n = A.size(0);
  TORCH_CHECK(A.size(1) == n, "A must be square");
  const int64_t sb = check_sbr16_operands(n, perm, Q);
  TORCH_CHECK(dq.is_cuda() && dq.scalar_type() == at::kFloat && dq.numel() == n && dq.is_contiguous(), "dq float[n]");
  TORCH_CHECK(stats.is_cuda() && stats.scalar_type() == at::kDouble && stats.numel() >= 4 && stats.is_contiguous(), "stats double[4]");
  c10::DeviceGuard g(A.device());
  auto X = at::empty({n, n}, A.options());
  evx_sbr16_far(A.data_ptr<float>(), (int)n, A.stride(0), perm.data_ptr<int>(), Q.data_ptr<float>(), dq.data_ptr<float>(),
                stats.data_ptr<double>(), (float)thr_fac, (float)theta, X.data_ptr<float>(), n, (int)sb, cur_stream());
  return X;
}

at::Tensor sbr16_bq(const at::Tensor& B, const at::Tensor& perm, const at::Tensor& Q) {
  check_rowmajor(B, "B");
  const int64_t rows = B.size(0), n = B.size(1);
  const int64_t sb = check_sbr16_operands(n, perm, Q);
  c10::DeviceGuard g(B.device());
  auto Bq = at::empty({rows, n}, B.options());
  evx_sbr16_bq(B.data_ptr<float>(), (int)rows, (int)n, B.stride(0), perm.data_ptr<int>(), Q.data_ptr<float>(), Bq.data_ptr<float>(), n,
               (int)sb, cur_stream());
  return Bq;
}


// A = (T + Tᵀ)/2 plus [off², diag², dmin, dmax] of A
std::vector<at::Tensor> sbr_symstats(const at::Tensor& T) {
  check_rowmajor(T, "T");
  const int64_t n = T.size(0);
  TORCH_CHECK(T.size(1) == n, "T must be square");
  c10::DeviceGuard g(T.device());
  auto A = at::empty({n, n}, T.options());
  auto o = T.options().dtype(at::kDouble);
  auto part = at::empty({4 * (int64_t)evx_sbr_symstats_parts((int)n)}, o);
  auto out = at::empty({4}, o);
  evx_sbr_symstats(T.data_ptr<float>(), (int)n, T.stride(0), A.data_ptr<float>(), n, part.data_ptr<double>(), out.data_ptr<double>(), cur_stream());
  return {A, out};
}

// in-place variant for the solver's static workspace (no copies inside its captured graphs)
void sbr_symstats_out(const at::Tensor& T, at::Tensor& A, at::Tensor& st) {
  check_rowmajor(T, "T");
  const int64_t n = T.size(0);
  TORCH_CHECK(T.size(1) == n, "T must be square");
  CHECK_DEV(A); CHECK_F32(A); CHECK_CONTIG(A);
  TORCH_CHECK(A.size(0) == n && A.size(1) == n && A.data_ptr() != T.data_ptr(), "sbr_symstats_out: A must be a separate n×n buffer");
  TORCH_CHECK(st.is_cuda() && st.scalar_type() == at::kDouble && st.is_contiguous() && st.numel() == 4, "sbr_symstats_out: st must be float64[4]");
  c10::DeviceGuard g(T.device());
  auto part = at::empty({4 * (int64_t)evx_sbr_symstats_parts((int)n)}, T.options().dtype(at::kDouble));
  evx_sbr_symstats(T.data_ptr<float>(), (int)n, T.stride(0), A.data_ptr<float>(), n, part.data_ptr<double>(), st.data_ptr<double>(), cur_stream());
}

std::vector<at::Tensor> sbr_taylor_prep(const at::Tensor& X, const at::Tensor& X2, const at::Tensor& X3,
                                        const c10::optional<at::Tensor>& alpha, int64_t mt) {
  for (auto* t : {&X, &X2, &X3}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  const int64_t n = X.size(0);
  TORCH_CHECK(X.dim() == 2 && X.size(1) == n && X2.sizes() == X.sizes() && X3.sizes() == X.sizes(), "sbr_taylor_prep: n×n");
  const float* ap = nullptr;
  if (alpha.has_value() && alpha->defined()) {
    CHECK_DEV(*alpha); CHECK_F32(*alpha);
    TORCH_CHECK(alpha->numel() == 1, "sbr_taylor_prep: alpha must be a 1-element device tensor");
    ap = alpha->data_ptr<float>();
  }
  c10::DeviceGuard g(X.device());
  auto P = at::empty_like(X), M = at::empty_like(X);
  evx_sbr_taylor_prep(X.data_ptr<float>(), X2.data_ptr<float>(), X3.data_ptr<float>(), (int)n, ap, P.data_ptr<float>(), M.data_ptr<float>(),
                      cur_stream(), (int)mt);
  return {P, M};
}

// words = 4: every word of each block; 2: the first two (a key split's (num, 2) keys, one launch)
at::Tensor philox_words(const at::Tensor& key, int64_t nblocks, int64_t domain, int64_t offset, int64_t words) {
  const int64_t B = key_batch(key, "philox_words");
  TORCH_CHECK(words == 2 || words == 4, "philox_words: words 2 or 4");
  c10::DeviceGuard g(key.device());
  auto out = B ? at::empty({B, nblocks, words}, key.options()) : at::empty({nblocks, words}, key.options());
  if (nblocks > 0)
    evx_philox_words(key.data_ptr<int64_t>(), nblocks, (uint32_t)domain, offset, out.data_ptr<int64_t>(), cur_stream(), B ? (int)B : 1,
                     (int)words);
  return out;
}

// Σ_k w[k] (X[idx[k]] − sub) over the first K (gathered) rows → (D,)
at::Tensor weighted_rowsum(const at::Tensor& X, const c10::optional<at::Tensor>& idx, const at::Tensor& w,
                           const c10::optional<at::Tensor>& sub, int64_t K) {
  CHECK_DEV(X); CHECK_F32(X); CHECK_DEV(w); CHECK_F32(w); CHECK_CONTIG(w);
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "X must be row-major 2-D");
  TORCH_CHECK(w.numel() >= K, "w too short");
  const int32_t* ip = nullptr;
  if (idx.has_value() && idx->defined()) {
    TORCH_CHECK(idx->scalar_type() == at::kInt && idx->is_contiguous() && idx->numel() >= K, "idx");
    ip = idx->data_ptr<int32_t>();
  } else {
    TORCH_CHECK(X.size(0) >= K, "X too short");
  }
  const int64_t D = X.size(1);
  c10::DeviceGuard g(X.device());
  const int chunks = (int)std::max<int64_t>(1, std::min<int64_t>(128, (K + 31) / 32));  // 512 workgroups at K = 5000, d = 1000
  auto part = at::empty({chunks, D}, X.options());
  evx_weighted_rowsum(X.data_ptr<float>(), X.stride(0), ip, w.data_ptr<float>(), optf(sub), (int)K, (int)D, part.data_ptr<float>(),
                      chunks, cur_stream());
  auto out = at::empty({D}, X.options());
  evx_colsum(part.data_ptr<float>(), chunks, (int)D, out.data_ptr<float>(), cur_stream());
  return out;
}

void gemm_set_config(int64_t cfg) { evx_gemm_set_config((int)cfg); }

at::Tensor sbx(const at::Tensor& x, const at::Tensor& keys, double pro_c, double dis_c, int64_t type, int64_t col0, int64_t dtot) {
  CHECK_DEV(x); CHECK_F32(x); CHECK_CONTIG(x); CHECK_DEV(keys);
  TORCH_CHECK(x.dim() == 2, "x must be (n, d)");
  TORCH_CHECK(keys.scalar_type() == at::kLong && keys.is_contiguous() && keys.numel() == 4, "keys must be int64[2,2]");
  TORCH_CHECK(type == 1 || type == 2, "type must be 1 or 2");
  const int64_t n = x.size(0), d = x.size(1);
  TORCH_CHECK(dtot == 0 || (col0 >= 0 && col0 + d <= dtot), "column block outside the decision axis");
  c10::DeviceGuard g(x.device());
  const int64_t rows = type == 1 ? n : n / 2;
  auto out = at::empty({rows, d}, x.options());
  if (rows > 0 && d > 0) evx_sbx(x.data_ptr<float>(), out.data_ptr<float>(), (int)n, (int)d, keys.data_ptr<int64_t>(), (float)pro_c, (float)dis_c, (int)type, cur_stream(), (int)col0, (int)dtot);
  return out;
}

at::Tensor pm(const at::Tensor& x, const at::Tensor& lb, const at::Tensor& ub, const at::Tensor& keys, double pro_m, double dis_m, int64_t nm,
              int64_t col0, int64_t dtot) {
  CHECK_DEV(x); CHECK_F32(x); CHECK_CONTIG(x); CHECK_DEV(lb); CHECK_F32(lb); CHECK_CONTIG(lb); CHECK_DEV(ub); CHECK_F32(ub); CHECK_CONTIG(ub);
  TORCH_CHECK(keys.scalar_type() == at::kLong && keys.is_contiguous() && keys.numel() == 4, "keys must be int64[2,2]");
  TORCH_CHECK(x.dim() == 2 && lb.numel() == x.size(1) && ub.numel() == x.size(1), "shape mismatch");
  TORCH_CHECK(dtot == 0 || (col0 >= 0 && col0 + x.size(1) <= dtot), "column block outside the decision axis");
  c10::DeviceGuard g(x.device());
  auto out = at::empty_like(x);
  if (x.numel() > 0)
    evx_pm(x.data_ptr<float>(), out.data_ptr<float>(), (int)x.size(0), (int)x.size(1), (int)nm, lb.data_ptr<float>(), ub.data_ptr<float>(),
           keys.data_ptr<int64_t>(), (float)pro_m, (float)dis_m, cur_stream(), (int)col0, (int)dtot);
  return out;
}

at::Tensor nds(const at::Tensor& f, int64_t limit, const c10::optional<at::Tensor>& err) {
  CHECK_DEV(f); CHECK_F32(f); CHECK_CONTIG(f);
  TORCH_CHECK(f.dim() == 2 && f.size(1) >= 1 && f.size(1) <= 8, "fitness must be (n, m) with m <= 8");
  const int64_t n = f.size(0), nw = (n + 31) / 32;
  TORCH_CHECK(n <= 65536, "nds: n <= 65536");
  c10::DeviceGuard g(f.device());
  auto DW = at::empty({nw, n}, f.options().dtype(at::kInt));
  auto rank = at::empty({n}, f.options().dtype(at::kInt));
  auto ws = at::empty({(int64_t)evx_nds_workspace_words((int)n)}, f.options().dtype(at::kInt));
  if (limit <= 0 || limit > n) limit = n;
  if (err) TORCH_CHECK(err->is_cuda() && err->scalar_type() == at::kInt && err->numel() >= 1, "err must be a device int32 flag");
  if (n > 0) {
    const int blocks = evx_nds_peel_blocks((int)n);
    TORCH_CHECK(blocks > 0, "nds: the persistent peel cannot be co-resident on this device at n = ", n);
    evx_nds(f.data_ptr<float>(), (int)n, (int)f.size(1), (int)limit, reinterpret_cast<uint32_t*>(DW.data_ptr<int>()), rank.data_ptr<int>(),
            reinterpret_cast<uint32_t*>(ws.data_ptr<int>()), err ? err->data_ptr<int>() : nullptr, blocks, cur_stream());
  }
  return rank;
}

at::Tensor dtlz(const at::Tensor& X, int64_t m, int64_t variant) {
  CHECK_DEV(X); CHECK_F32(X); CHECK_CONTIG(X);
  TORCH_CHECK(X.dim() == 2 && m >= 2 && m <= 64 && X.size(1) >= m, "dtlz: X must be (n, d) with 2 <= m <= min(d, 64)");
  TORCH_CHECK(variant >= 1 && variant <= 4, "dtlz: variant 1..4");
  c10::DeviceGuard g(X.device());
  auto F = at::empty({X.size(0), m}, X.options());
  if (X.size(0) > 0) evx_dtlz(X.data_ptr<float>(), F.data_ptr<float>(), (int)X.size(0), (int)X.size(1), (int)m, (int)variant, cur_stream());
  return F;
}

at::Tensor de_trial(const at::Tensor& P, const at::Tensor& idx, const at::Tensor& coef, const at::Tensor& cur, const at::Tensor& mode,
                    const at::Tensor& CR, const at::Tensor& jr, const at::Tensor& L, const at::Tensor& key, const at::Tensor& lb,
                    const at::Tensor& ub, int64_t repair, const at::Tensor& err, int64_t col0, int64_t d_total) {
  CHECK_DEV(P); CHECK_F32(P); CHECK_CONTIG(P);
  TORCH_CHECK(err.is_cuda() && err.scalar_type() == at::kInt && err.numel() >= 1, "de_trial: err must be int32[1] on the device");
  // single run: P (rows, d), idx (R, K), key (2,); B batched runs: P (B, rows, d), idx (B, R, K),
  // per-row tensors (B, R), keys (B, 2) — one launch, grid.y = run
  const int64_t B = key_batch(key, "de_trial");
  const int64_t Bn = B ? B : 1;
  TORCH_CHECK(P.dim() == (B ? 3 : 2) && idx.dim() == P.dim() && (!B || (P.size(0) == B && idx.size(0) == B)),
              "de_trial: P must be (rows, d) with idx (R, K), or (B, rows, d) with idx (B, R, K) and keys (B, 2)");
  const int64_t R = idx.size(-2), K = idx.size(-1), d = P.size(-1), rows = P.size(-2);
  TORCH_CHECK(K >= 1 && K <= 16, "de_trial: 1 <= K <= 16");
  auto i32 = [&](const at::Tensor& t, int64_t n, const char* nm) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kInt && t.is_contiguous() && t.numel() == n, "de_trial: ", nm, " must be contiguous int32[", n, "]");
    return t.data_ptr<int>();
  };
  auto f32 = [&](const at::Tensor& t, int64_t n, const char* nm) {
    TORCH_CHECK(t.is_cuda() && t.scalar_type() == at::kFloat && t.is_contiguous() && t.numel() == n, "de_trial: ", nm, " must be contiguous f32[", n, "]");
    return t.data_ptr<float>();
  };
  TORCH_CHECK(repair >= 0 && repair <= 2, "de_trial: repair in {0,1,2}");
  c10::DeviceGuard g(P.device());
  auto out = B ? at::empty({B, R, d}, P.options()) : at::empty({R, d}, P.options());
  if (R > 0 && d > 0)
    evx_de_trial(P.data_ptr<float>(), i32(idx, Bn * R * K, "idx"), f32(coef, Bn * R * K, "coef"), (int)K, i32(cur, Bn * R, "cur"),
                 i32(mode, Bn * R, "mode"), f32(CR, Bn * R, "CR"), i32(jr, Bn * R, "jr"), i32(L, Bn * R, "L"), key.data_ptr<int64_t>(),
                 f32(lb, d, "lb"), f32(ub, d, "ub"), (int)repair, out.data_ptr<float>(), (int)R, (int)d, (int)rows, err.data_ptr<int>(),
                 cur_stream(), (int)Bn, (int)col0, (int)d_total);
  return out;
}

std::vector<at::Tensor> moead_scan(const at::Tensor& objs, const at::Tensor& off_objs, const at::Tensor& P, const at::Tensor& W,
                                   const at::Tensor& z, int64_t func, int64_t nr, int64_t update_z) {
  CHECK_DEV(objs); CHECK_F32(objs); CHECK_CONTIG(objs); CHECK_DEV(off_objs); CHECK_F32(off_objs); CHECK_CONTIG(off_objs);
  CHECK_DEV(W); CHECK_F32(W); CHECK_CONTIG(W); CHECK_DEV(z); CHECK_F32(z); CHECK_CONTIG(z);
  TORCH_CHECK(P.is_cuda() && P.scalar_type() == at::kInt && P.is_contiguous() && P.dim() == 2, "moead_scan: P must be int32 (R, T)");
  const int64_t N = objs.size(0), M = objs.size(1), R = off_objs.size(0), T = P.size(1);
  TORCH_CHECK(M >= 1 && M <= 16 && off_objs.size(1) == M && W.size(0) == N && W.size(1) == M && z.numel() == M, "moead_scan: shapes");
  TORCH_CHECK(P.size(0) == R && T >= 1 && T <= 64, "moead_scan: 1 <= T <= 64");
  TORCH_CHECK(func >= 0 && func <= 3, "moead_scan: func in {0 tch, 1 pbi, 2 ws, 3 mtch}");
  c10::DeviceGuard g(objs.device());
  auto o = objs.clone();
  auto zz = z.clone();
  auto owner = at::empty({N}, objs.options().dtype(at::kInt));
  if (N > 0) evx_moead_scan(o.data_ptr<float>(), off_objs.data_ptr<float>(), P.data_ptr<int>(), W.data_ptr<float>(), zz.data_ptr<float>(),
                            owner.data_ptr<int>(), (int)N, (int)R, (int)T, (int)M, (int)func, (int)nr, (int)update_z, cur_stream());
  return {owner, o, zz};
}

// Stochastic ranking (Runarsson & Yao; SRA reference sra.py:13-64): bubble-sort sweeps over
// adjacent pairs comparing by indicator I1 with probability pc (fixed per-pair draws
// `rnd`, as the reference reuses them in every sweep), else by I2; at most ceil(n/2)
// sweeps, stopping early when a sweep makes no swap.  Inherently sequential and tiny:
// a host loop over CPU tensors.
at::Tensor stochastic_ranking(const at::Tensor& I1_, const at::Tensor& I2_, const at::Tensor& rnd_, double pc) {
  auto I1 = I1_.to(at::kCPU, at::kFloat).contiguous();
  auto I2 = I2_.to(at::kCPU, at::kFloat).contiguous();
  auto rnd = rnd_.to(at::kCPU, at::kFloat).contiguous();
  const int64_t n = I1.numel();
  TORCH_CHECK(I2.numel() == n && rnd.numel() >= std::max<int64_t>(n - 1, 0), "stochastic_ranking: sizes");
  auto rank = at::empty({n}, at::TensorOptions().dtype(at::kLong));
  evx_host::stochastic_ranking(I1.data_ptr<float>(), I2.data_ptr<float>(), rnd.data_ptr<float>(), (float)pc, n, rank.data_ptr<int64_t>());
  return rank;
}

std::vector<at::Tensor> ant_rollout(const at::Tensor& W, int64_t h1, int64_t h2, const at::Tensor& init, int64_t cap) {
  CHECK_DEV(W); CHECK_F32(W); CHECK_CONTIG(W); CHECK_DEV(init); CHECK_F32(init); CHECK_CONTIG(init);
  TORCH_CHECK(W.dim() == 2, "ant_rollout: W must be (N, P)");
  TORCH_CHECK(h1 >= 1 && h1 <= 512 && h2 >= 1 && h2 <= 512, "ant_rollout: hidden sizes in [1, 512]");
  const int64_t P = 27 * h1 + h1 + h1 * h2 + h2 + h2 * 8 + 8;
  TORCH_CHECK(W.size(1) == P, "ant_rollout: W has ", W.size(1), " columns, MLP 27-", h1, "-", h2, "-8 needs ", P);
  TORCH_CHECK(init.numel() == 29, "ant_rollout: init state must have 29 entries");
  TORCH_CHECK((P + 32 + h1 + h2 + 8) * 4 <= 160 * 1024, "ant_rollout: MLP too large for one wave's LDS");
  c10::DeviceGuard g(W.device());
  const int64_t N = W.size(0);
  auto ret = at::empty({N}, W.options());
  auto steps = at::empty({N}, W.options().dtype(at::kInt));
  if (N > 0) evx_ant_rollout(W.data_ptr<float>(), P, (int)N, (int)h1, (int)h2, init.data_ptr<float>(), (int)cap, ret.data_ptr<float>(),
                             steps.data_ptr<int>(), cur_stream());
  return {ret, steps};
}

// rows > 0: only the parents of offspring row0 .. row0+rows−1 (the rest of p0 / p1 zero)
std::vector<at::Tensor> moead_parents(const at::Tensor& nb, const at::Tensor& key, int64_t row0, int64_t rows) {
  CHECK_DEV(nb); CHECK_CONTIG(nb); check_key(key);
  TORCH_CHECK(nb.dim() == 2 && nb.scalar_type() == at::kLong && nb.size(1) >= 1 && nb.size(1) < 65536, "neighbours must be int64 (N, T), T < 65536");
  c10::DeviceGuard g(nb.device());
  const int64_t N = nb.size(0);
  const int64_t R = rows > 0 ? rows : N;
  TORCH_CHECK(row0 >= 0 && row0 + R <= N, "moead_parents: rows out of range");
  auto p0 = rows > 0 ? at::zeros({N}, nb.options().dtype(at::kInt)) : at::empty({N}, nb.options().dtype(at::kInt));
  auto p1 = rows > 0 ? at::zeros({N}, nb.options().dtype(at::kInt)) : at::empty({N}, nb.options().dtype(at::kInt));
  if (R > 0)
    evx_moead_parents(nb.data_ptr<int64_t>(), (int)R, (int)nb.size(1), key.data_ptr<int64_t>(), p0.data_ptr<int>(), p1.data_ptr<int>(),
                      cur_stream(), (int)row0);
  return {p0, p1};
}

// rows = 0: every offspring (N = p0.numel()); rows > 0: offspring row0 .. row0+rows−1 only;
// win given: output row s = offspring win[s] (regenerated) or pop[s] when win[s] < 0
at::Tensor moead_variation(const at::Tensor& pop, const at::Tensor& p0, const at::Tensor& p1, const at::Tensor& kx, const at::Tensor& km,
                           const at::Tensor& lb, const at::Tensor& ub, double pro_c, double dis_c, double pro_m, double dis_m, int64_t nm,
                           int64_t row0, int64_t rows, const c10::optional<at::Tensor>& win,
                           const c10::optional<at::Tensor>& out_opt) {
  for (auto* t : {&pop, &lb, &ub}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  for (auto* t : {&p0, &p1}) { CHECK_DEV(*t); CHECK_CONTIG(*t); TORCH_CHECK(t->scalar_type() == at::kInt, "parents must be int32"); }
  TORCH_CHECK(kx.scalar_type() == at::kLong && kx.numel() == 4 && kx.is_contiguous() && kx.is_cuda(), "kx must be int64[2][2] on device");
  TORCH_CHECK(km.scalar_type() == at::kLong && km.numel() == 4 && km.is_contiguous() && km.is_cuda(), "km must be int64[2][2] on device");
  TORCH_CHECK(pop.dim() == 2 && lb.numel() == pop.size(1) && ub.numel() == pop.size(1), "bounds must be (d,)");
  const int64_t Np = p0.numel(), d = pop.size(1);
  TORCH_CHECK(p1.numel() == Np, "p0/p1 length mismatch");
  int64_t R = rows > 0 ? rows : Np;
  const int32_t* wp = nullptr;
  if (win) {
    TORCH_CHECK(win->is_cuda() && win->scalar_type() == at::kInt && win->is_contiguous() && win->numel() == pop.size(0),
                "win must be int32 (N,) with one entry per population row");
    R = pop.size(0);
    wp = win->data_ptr<int>();
    row0 = 0;
  }
  TORCH_CHECK(row0 >= 0 && (win || row0 + R <= Np), "moead_variation: offspring rows out of range");
  c10::DeviceGuard g(pop.device());
  at::Tensor out;
  if (out_opt.has_value() && out_opt->defined()) {
    out = *out_opt;
    TORCH_CHECK(out.is_cuda() && out.scalar_type() == at::kFloat && out.is_contiguous() && out.numel() >= R * d,
                "moead_variation: out must hold rows × d float32");
  } else {
    out = at::empty({R, d}, pop.options());
  }
  if (R > 0 && d > 0)
    evx_moead_variation(pop.data_ptr<float>(), p0.data_ptr<int>(), p1.data_ptr<int>(), out.data_ptr<float>(), (int)R, (int)d, kx.data_ptr<int64_t>(),
                        km.data_ptr<int64_t>(), lb.data_ptr<float>(), ub.data_ptr<float>(), (float)pro_c, (float)dis_c, (float)pro_m, (float)dis_m,
                        (int)nm, cur_stream(), (int)row0, wp);
  return out;
}

// ---- owner-computes MOEA/D + IPC peer buffers (direct xGMI reads between the ranks of a node)
void moead_halo_replace(at::Tensor& obj, const at::Tensor& off_obj, const at::Tensor& W, const at::Tensor& z, const at::Tensor& zmax,
                        const at::Tensor& rowptr, const at::Tensor& owner, const at::Tensor& slots, int64_t func, at::Tensor& win_h) {
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&obj, &off_obj, &W, &z, &zmax}) {
    CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t);
  }
  for (const at::Tensor* t : std::initializer_list<const at::Tensor*>{&rowptr, &owner, &slots, &win_h}) {
    CHECK_DEV(*t); CHECK_CONTIG(*t);
    TORCH_CHECK(t->scalar_type() == at::kInt, "moead_halo_replace: int32 index tensors");
  }
  const int64_t M = obj.size(1);
  TORCH_CHECK(M <= 16 && off_obj.size(1) == M && win_h.numel() >= slots.numel(), "moead_halo_replace: shapes");
  evx_moead_halo_replace(obj.data_ptr<float>(), off_obj.data_ptr<float>(), W.data_ptr<float>(), z.data_ptr<float>(), zmax.data_ptr<float>(),
                         rowptr.data_ptr<int>(), owner.data_ptr<int>(), slots.data_ptr<int>(), (int)slots.numel(), (int)M, (int)func,
                         win_h.data_ptr<int>(), cur_stream());
}

void moead_halo_gather(at::Tensor& pop, const at::Tensor& slots, const at::Tensor& win_h, const at::Tensor& peer, const at::Tensor& starts,
                       const c10::optional<at::Tensor>& first) {
  CHECK_DEV(pop); CHECK_F32(pop); CHECK_CONTIG(pop);
  TORCH_CHECK(peer.is_cuda() && peer.scalar_type() == at::kLong && starts.is_cuda() && starts.scalar_type() == at::kInt &&
                  starts.numel() == peer.numel() + 1, "moead_halo_gather: peer int64[world], starts int32[world + 1] on device");
  int32_t* fp = nullptr;
  int nf = 0;
  if (first && first->defined()) {  // deduplicated: every offspring row read once, duplicates copied locally
    TORCH_CHECK(first->is_cuda() && first->scalar_type() == at::kInt && first->is_contiguous(), "moead_halo_gather: first int32 on device");
    fp = first->data_ptr<int>();
    nf = (int)first->numel();
  }
  evx_moead_halo_gather(pop.data_ptr<float>(), slots.data_ptr<int>(), win_h.data_ptr<int>(), (int)slots.numel(), peer.data_ptr<int64_t>(),
                        starts.data_ptr<int>(), (int)peer.numel(), (int)pop.size(1), cur_stream(), fp, nf);
}

// writer side of the peer-buffer contract (parallel/peer.py): a system-scope release on the
// current stream after the kernels that wrote a peer-visible buffer
void peer_release(int64_t device) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  evx_peer_release(cur_stream());
}

// hipMalloc'd buffer (an allocation base, so its IPC handle maps exactly this tensor)
at::Tensor ipc_alloc(int64_t numel, int64_t device) {
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  void* p = nullptr;
  TORCH_CHECK(hipMalloc(&p, std::max<int64_t>(numel, 1) * 4) == hipSuccess, "ipc_alloc: hipMalloc failed");
  TORCH_CHECK(hipMemset(p, 0, std::max<int64_t>(numel, 1) * 4) == hipSuccess, "ipc_alloc: hipMemset failed");
  return at::from_blob(p, {numel}, [](void* q) { (void)hipFree(q); },
                       at::TensorOptions().dtype(at::kFloat).device(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device)));
}

at::Tensor ipc_handle(const at::Tensor& t) {
  CHECK_DEV(t);
  hipIpcMemHandle_t h;
  TORCH_CHECK(hipIpcGetMemHandle(&h, t.data_ptr()) == hipSuccess, "ipc_handle: hipIpcGetMemHandle failed");
  auto out = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &h, sizeof(h));
  return out;
}

int64_t ipc_open(const at::Tensor& handle, int64_t device) {
  TORCH_CHECK(handle.numel() == (int64_t)sizeof(hipIpcMemHandle_t) && handle.scalar_type() == at::kByte, "ipc_open: handle bytes");
  c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, (c10::DeviceIndex)device));
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.contiguous().data_ptr(), sizeof(h));
  void* p = nullptr;
  TORCH_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) == hipSuccess, "ipc_open: hipIpcOpenMemHandle failed");
  return (int64_t)(uintptr_t)p;
}

void ipc_close(int64_t ptr) { (void)hipIpcCloseMemHandle((void*)(uintptr_t)ptr); }

std::vector<at::Tensor> moead_replace(const at::Tensor& pop_obj, const at::Tensor& off_obj, const at::Tensor& W, const at::Tensor& z,
                                      const at::Tensor& zmax, const at::Tensor& rowptr, const at::Tensor& owner, int64_t func) {
  for (auto* t : {&pop_obj, &off_obj, &W, &z, &zmax}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  for (auto* t : {&rowptr, &owner}) { CHECK_DEV(*t); CHECK_CONTIG(*t); TORCH_CHECK(t->scalar_type() == at::kInt, "CSR must be int32"); }
  const int64_t N = pop_obj.size(0), M = pop_obj.size(1);
  TORCH_CHECK(M >= 1 && M <= 16 && W.size(0) == N && W.size(1) == M && off_obj.size(1) == M && z.numel() == M && zmax.numel() == M, "shape mismatch");
  TORCH_CHECK(rowptr.numel() == N + 1 && func >= 0 && func <= 4, "rowptr must be (N+1,), func 0..4");
  c10::DeviceGuard g(pop_obj.device());
  auto win = at::empty({N}, pop_obj.options().dtype(at::kInt));
  auto new_obj = at::empty_like(pop_obj);
  if (N > 0)
    evx_moead_replace(pop_obj.data_ptr<float>(), off_obj.data_ptr<float>(), W.data_ptr<float>(), z.data_ptr<float>(), zmax.data_ptr<float>(),
                      rowptr.data_ptr<int>(), owner.data_ptr<int>(), (int)N, (int)M, (int)func, win.data_ptr<int>(), new_obj.data_ptr<float>(), cur_stream());
  return {win, new_obj};
}

at::Tensor moead_select_rows(const at::Tensor& pop, const at::Tensor& off, const at::Tensor& win) {
  for (auto* t : {&pop, &off}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  CHECK_DEV(win); TORCH_CHECK(win.scalar_type() == at::kInt && win.numel() == pop.size(0), "win must be int32 (N,)");
  TORCH_CHECK(off.size(1) == pop.size(1), "row width mismatch");
  c10::DeviceGuard g(pop.device());
  auto out = at::empty_like(pop);
  if (pop.numel() > 0)
    evx_moead_select_rows(pop.data_ptr<float>(), off.data_ptr<float>(), win.data_ptr<int>(), out.data_ptr<float>(), (int)pop.size(0), (int)pop.size(1), cur_stream());
  return out;
}

// pop[s] = off[win[s]] for the winning slots, in place (hipGraph path: no new population and no
// state write-back copy)
void moead_select_rows_(at::Tensor& pop, const at::Tensor& off, const at::Tensor& win) {
  CHECK_DEV(pop); CHECK_F32(pop); CHECK_CONTIG(pop); CHECK_DEV(off); CHECK_F32(off); CHECK_CONTIG(off);
  TORCH_CHECK(win.is_cuda() && win.scalar_type() == at::kInt && win.is_contiguous() && win.numel() == pop.size(0), "moead_select_rows_: win int32[N]");
  TORCH_CHECK(off.dim() == 2 && off.size(1) == pop.size(1), "moead_select_rows_: off (rows, d)");
  TORCH_CHECK(pop.data_ptr() != off.data_ptr(), "moead_select_rows_: off must not alias pop");
  c10::DeviceGuard g(pop.device());
  if (pop.size(0) > 0 && pop.size(1) > 0)
    evx_moead_select_rows_inplace(pop.data_ptr<float>(), off.data_ptr<float>(), win.data_ptr<int>(), (int)pop.size(0), (int)pop.size(1),
                                  cur_stream());
}

at::Tensor lsmop_g(const at::Tensor& X, std::vector<int64_t> start, std::vector<int64_t> sublen, std::vector<int64_t> func, int64_t nk, int64_t cosine) {
  CHECK_DEV(X); CHECK_F32(X); CHECK_CONTIG(X);
  const int64_t ng = (int64_t)start.size();
  TORCH_CHECK(X.dim() == 2 && ng >= 1 && ng <= 16 && (int64_t)sublen.size() == ng && (int64_t)func.size() == ng && nk >= 1, "lsmop_g: bad groups");
  std::vector<int> s32(ng), l32(ng), f32(ng);
  for (int64_t k = 0; k < ng; ++k) {
    TORCH_CHECK(start[k] >= 1 && sublen[k] >= 0 && start[k] + nk * sublen[k] <= X.size(1) && func[k] >= 0 && func[k] <= 5, "lsmop_g: group out of range");
    s32[k] = (int)start[k]; l32[k] = (int)sublen[k]; f32[k] = (int)func[k];
  }
  c10::DeviceGuard g(X.device());
  auto G = at::empty({X.size(0), ng}, X.options());
  if (X.size(0) > 0) evx_lsmop_g(X.data_ptr<float>(), G.data_ptr<float>(), (int)X.size(0), (int)X.size(1), (int)ng, (int)nk, (int)cosine, s32.data(), l32.data(), f32.data(), cur_stream());
  return G;
}

// ---------------------------------------------------------------- CMA-ES tell epilogue (cmaes.hip)
// Yw = (pop[rows] − mean)·sqrt(w)/σ (K×d), rows int32 (or none: the first K rows)
at::Tensor cma_center_rows(const at::Tensor& pop, const c10::optional<at::Tensor>& rows, const at::Tensor& mean, const at::Tensor& sigma,
                           const at::Tensor& w, bool aug) {
  CHECK_DEV(pop); CHECK_F32(pop);
  TORCH_CHECK(pop.dim() == 2 && pop.stride(1) == 1, "cma_center_rows: pop must be row-major 2-D");
  const int64_t d = pop.size(1), K = w.numel();
  TORCH_CHECK(mean.is_contiguous() && mean.numel() == d && sigma.numel() == 1 && w.is_contiguous(), "cma_center_rows: mean (d,), sigma (1,), w (K,)");
  const int32_t* rp = nullptr;
  if (rows) {
    TORCH_CHECK(rows->scalar_type() == at::kInt && rows->is_contiguous() && rows->numel() == K, "cma_center_rows: rows int32[K]");
    rp = rows->data_ptr<int32_t>();
  } else {
    TORCH_CHECK(K <= pop.size(0), "cma_center_rows: K > rows of pop");
  }
  c10::DeviceGuard g(pop.device());
  // aug: (K, d + 1) view of a (K, ld) buffer, ld = d + 1 rounded up to 4 (16-B rows), column d = σ·sqrt(wᵢ)
  const int64_t ld = aug ? ((d + 1 + 3) & ~int64_t(3)) : d;
  auto Yb = at::empty({K, ld}, pop.options());
  evx_cma_center_rows(pop.data_ptr<float>(), pop.stride(0), rp, mean.data_ptr<float>(), sigma.contiguous().data_ptr<float>(),
                      w.data_ptr<float>(), (int)K, (int)d, Yb.data_ptr<float>(), cur_stream(), ld, aug ? 1 : 0);
  return aug ? Yb.narrow(1, 0, d + 1) : Yb;
}

// sharded tell: this rank's rows of the global top μ, compacted (see cmaes.hip local_select_kernel)
void cma_local_select(const at::Tensor& order, int64_t mu, const at::Tensor& w, int64_t start, int64_t size, at::Tensor& rows,
                      at::Tensor& wk) {
  CHECK_DEV(order); CHECK_DEV(w); CHECK_DEV(rows); CHECK_DEV(wk); CHECK_F32(w); CHECK_F32(wk);
  TORCH_CHECK(order.scalar_type() == at::kInt && order.is_contiguous() && order.numel() >= mu, "cma_local_select: order int32[>= mu]");
  TORCH_CHECK(w.is_contiguous() && w.numel() >= mu, "cma_local_select: w (mu,)");
  TORCH_CHECK(rows.scalar_type() == at::kInt && rows.is_contiguous() && wk.is_contiguous() && wk.numel() == rows.numel(),
              "cma_local_select: rows int32[K], wk float[K]");
  TORCH_CHECK(start >= 0 && size >= 0 && rows.numel() >= std::min<int64_t>(mu, size), "cma_local_select: K >= min(mu, size)");
  c10::DeviceGuard g(order.device());
  evx_cma_local_select(order.data_ptr<int32_t>(), (int)mu, w.data_ptr<float>(), (int)start, (int)size, (int)rows.numel(),
                       rows.data_ptr<int32_t>(), wk.data_ptr<float>(), cur_stream());
}

// d × d symmetric ↔ packed upper triangle (d(d+1)/2 floats)
void sym_pack(const at::Tensor& S, at::Tensor& P) {
  CHECK_DEV(S); CHECK_F32(S); CHECK_DEV(P); CHECK_F32(P);
  TORCH_CHECK(S.dim() == 2 && S.size(0) == S.size(1) && S.stride(1) == 1, "sym_pack: square row-major S");
  const int64_t d = S.size(0);
  TORCH_CHECK(P.is_contiguous() && P.numel() >= d * (d + 1) / 2, "sym_pack: P float[d(d+1)/2]");
  c10::DeviceGuard g(S.device());
  evx_sym_pack(S.data_ptr<float>(), S.stride(0), (int)d, P.data_ptr<float>(), cur_stream());
}

void sym_unpack(const at::Tensor& P, at::Tensor& S) {
  CHECK_DEV(S); CHECK_F32(S); CHECK_DEV(P); CHECK_F32(P);
  TORCH_CHECK(S.dim() == 2 && S.size(0) == S.size(1) && S.stride(1) == 1, "sym_unpack: square row-major S");
  const int64_t d = S.size(0);
  TORCH_CHECK(P.is_contiguous() && P.numel() >= d * (d + 1) / 2, "sym_unpack: P float[d(d+1)/2]");
  c10::DeviceGuard g(S.device());
  evx_sym_unpack(P.data_ptr<float>(), (int)d, S.data_ptr<float>(), S.stride(0), cur_stream());
}

std::vector<at::Tensor> cma_delta_gemv(const at::Tensor& M, const at::Tensor& mean, const at::Tensor& dm, double cm) {
  for (auto* t : {&M, &mean, &dm}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  const int64_t d = mean.numel();
  TORCH_CHECK(M.dim() == 2 && M.size(0) == d && M.size(1) == d && dm.numel() == d, "cma_delta_gemv: shapes");
  c10::DeviceGuard g(M.device());
  auto mo = at::empty_like(mean), de = at::empty_like(mean), y = at::empty_like(mean);
  if (d > 0) evx_cma_delta_gemv(M.data_ptr<float>(), mean.data_ptr<float>(), dm.data_ptr<float>(), (float)cm, (int)d, mo.data_ptr<float>(),
                                de.data_ptr<float>(), y.data_ptr<float>(), cur_stream());
  return {mo, de, y};
}

std::vector<at::Tensor> cma_paths(const at::Tensor& ps, const at::Tensor& pc, const at::Tensor& y, const at::Tensor& delta,
                                  const at::Tensor& sigma, const at::Tensor& count_iter, std::vector<double> consts,
                                  const c10::optional<at::Tensor>& count_eigen) {
  for (auto* t : {&ps, &pc, &y, &delta, &sigma}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  CHECK_DEV(count_iter);
  TORCH_CHECK(count_iter.scalar_type() == at::kLong && count_iter.numel() == 1 && sigma.numel() == 1, "cma_paths: scalars");
  TORCH_CHECK(consts.size() == 9, "cma_paths: 9 constants");
  const int64_t d = ps.numel();
  TORCH_CHECK(pc.numel() == d && y.numel() == d && delta.numel() == d, "cma_paths: shapes");
  c10::DeviceGuard g(ps.device());
  float k[9];
  for (int i = 0; i < 9; ++i) k[i] = (float)consts[i];
  auto pso = at::empty_like(ps), pco = at::empty_like(pc);
  auto so = at::empty_like(sigma), ao = at::empty_like(sigma), ho = at::empty_like(sigma);
  // count_eigen given: the kernel also advances both generation counters (returned as two more tensors)
  const bool adv = count_eigen.has_value() && count_eigen->defined();
  at::Tensor ci, ce;
  if (adv) {
    CHECK_DEV(*count_eigen);
    TORCH_CHECK(count_eigen->scalar_type() == at::kLong && count_eigen->numel() == 1, "cma_paths: count_eigen int64 scalar");
    ci = at::empty_like(count_iter);
    ce = at::empty_like(*count_eigen);
  }
  evx_cma_paths(ps.data_ptr<float>(), pc.data_ptr<float>(), y.data_ptr<float>(), delta.data_ptr<float>(), sigma.data_ptr<float>(),
                count_iter.data_ptr<int64_t>(), (int)d, k, pso.data_ptr<float>(), pco.data_ptr<float>(), so.data_ptr<float>(),
                ao.data_ptr<float>(), ho.data_ptr<float>(), cur_stream(), adv ? count_eigen->data_ptr<int64_t>() : nullptr,
                adv ? ci.data_ptr<int64_t>() : nullptr, adv ? ce.data_ptr<int64_t>() : nullptr);
  if (adv) return {pso, pco, so, ao, ho, ci, ce};
  return {pso, pco, so, ao, ho};
}

std::vector<at::Tensor> cma_cov_pad(const at::Tensor& C, const at::Tensor& S, const at::Tensor& pc, const at::Tensor& a, double c1,
                                    double cmu, const at::Tensor& Bprev, int64_t np, const c10::optional<at::Tensor>& Cn_out,
                                    bool want_bp) {
  for (auto* t : {&C, &pc, &a, &Bprev}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  CHECK_DEV(S); CHECK_F32(S);
  const int64_t d = pc.numel();
  TORCH_CHECK(C.dim() == 2 && C.size(0) == d && C.size(1) == d && S.sizes() == C.sizes() && Bprev.sizes() == C.sizes(), "cma_cov_pad: shapes");
  // S may be the leading d × d block of the augmented rank-μ product (row stride ≥ d)
  TORCH_CHECK(S.stride(1) == 1 && S.stride(0) >= d, "cma_cov_pad: S row-major (row stride >= d)");
  TORCH_CHECK(np >= d && np % 32 == 0 && a.numel() == 1, "cma_cov_pad: np must be a multiple of 32 and >= d");
  c10::DeviceGuard g(C.device());
  at::Tensor Cn;
  if (Cn_out.has_value()) {  // may be C itself (in-place covariance update)
    Cn = *Cn_out;
    CHECK_DEV(Cn); CHECK_F32(Cn); CHECK_CONTIG(Cn);
    TORCH_CHECK(Cn.sizes() == C.sizes(), "cma_cov_pad: out shape");
  } else {
    Cn = at::empty_like(C);
  }
  auto Cp = at::empty({np, np}, C.options());
  auto Bp = want_bp ? at::empty({np, np}, C.options()) : at::empty({0}, C.options());
  evx_cma_cov_pad(C.data_ptr<float>(), S.data_ptr<float>(), pc.data_ptr<float>(), a.data_ptr<float>(), (float)c1, (float)cmu,
                  Bprev.data_ptr<float>(), (int)d, (int)np, Cn.data_ptr<float>(), Cp.data_ptr<float>(),
                  want_bp ? Bp.data_ptr<float>() : nullptr, cur_stream(), S.stride(0));
  return {Cn, Cp, Bp};
}

std::vector<at::Tensor> cma_eig_out(const at::Tensor& Bp, const at::Tensor& w, int64_t d, const c10::optional<at::Tensor>& B_out,
                                    const c10::optional<at::Tensor>& B_alt, const c10::optional<at::Tensor>& keep) {
  for (auto* t : {&Bp, &w}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  const int64_t np = Bp.size(0);
  TORCH_CHECK(Bp.dim() == 2 && Bp.size(1) == np && w.numel() >= d && d <= np, "cma_eig_out: shapes");
  c10::DeviceGuard g(Bp.device());
  at::Tensor B;
  if (B_out.has_value()) {  // the state's basis buffer (captured generation); must not alias Bp
    B = *B_out;
    CHECK_DEV(B); CHECK_F32(B); CHECK_CONTIG(B);
    TORCH_CHECK(B.dim() == 2 && B.size(0) == d && B.size(1) == d && B.data_ptr() != Bp.data_ptr(), "cma_eig_out: out");
  } else {
    B = at::empty({d, d}, Bp.options());
  }
  auto BD = at::empty({d, d}, Bp.options()), D = at::empty({d}, Bp.options());
  const float* alt = nullptr;
  const int* kp = nullptr;
  if (B_alt.has_value() && B_alt->defined()) {  // the warm start, taken while *keep == 0 (device eigensolver)
    CHECK_DEV(*B_alt); CHECK_F32(*B_alt); CHECK_CONTIG(*B_alt);
    TORCH_CHECK(B_alt->dim() == 2 && B_alt->size(0) == d && B_alt->size(1) == d && keep.has_value() && keep->defined() &&
                    keep->is_cuda() && keep->scalar_type() == at::kInt && keep->numel() >= 1,
                "cma_eig_out: B_alt (d, d) with an int32 device keep word");
    alt = B_alt->data_ptr<float>();
    kp = keep->data_ptr<int>();
  }
  if (d > 0) evx_cma_eig_out(Bp.data_ptr<float>(), w.data_ptr<float>(), (int)d, (int)np, B.data_ptr<float>(), D.data_ptr<float>(),
                             BD.data_ptr<float>(), cur_stream(), alt, kp);
  return {B, D, BD};
}

at::Tensor nsga_select(const at::Tensor& rank, const at::Tensor& f, int64_t N, int64_t mask_pos) {
  CHECK_DEV(rank); CHECK_CONTIG(rank); CHECK_DEV(f); CHECK_F32(f); CHECK_CONTIG(f);
  TORCH_CHECK(rank.scalar_type() == at::kInt && f.dim() == 2 && rank.numel() == f.size(0), "nsga_select: rank int32 (n,), f (n, m)");
  const int64_t n = f.size(0);
  TORCH_CHECK(n >= 1 && n <= 8192, "nsga_select: 1 <= n <= 8192");
  TORCH_CHECK(N >= 1 && N <= n && mask_pos >= N - 1 && mask_pos < n, "nsga_select: need N <= n and N-1 <= mask_pos < n");
  c10::DeviceGuard g(f.device());
  auto keep = at::empty({N}, f.options().dtype(at::kLong));
  evx_nsga_select(rank.data_ptr<int>(), f.data_ptr<float>(), (int)n, (int)f.size(1), (int)N, (int)mask_pos, keep.data_ptr<int64_t>(), cur_stream());
  return keep;
}

}  // namespace

// OpenES gradient with Philox-regenerated noise: g[j] = Σ_i w[i] ε(row0 + i, j)
at::Tensor es_population(const at::Tensor& key, const at::Tensor& center, double sigma, int64_t rows, int64_t half, int64_t row0,
                         int64_t col0, int64_t dtot) {
  CHECK_DEV(key); CHECK_DEV(center); CHECK_F32(center); CHECK_CONTIG(center);
  TORCH_CHECK(key.scalar_type() == at::kLong && key.numel() == 2 && key.is_contiguous(), "es_population: key int64[2]");
  TORCH_CHECK(center.dim() == 1 && rows >= 0 && half >= 0 && row0 >= 0 && col0 >= 0 && (dtot == 0 || col0 + center.size(0) <= dtot),
              "es_population: center (d,), window [col0, col0 + d) inside dtot");
  c10::DeviceGuard g(center.device());
  const int64_t d = center.size(0);
  auto out = at::empty({rows, d}, center.options());
  if (rows > 0 && d > 0)
    evx_es_population(key.data_ptr<int64_t>(), center.data_ptr<float>(), (float)sigma, rows, d, half, row0, out.data_ptr<float>(), cur_stream(),
                      col0, dtot);
  return out;
}

at::Tensor es_noise_grad(const at::Tensor& key, const at::Tensor& w, int64_t d, int64_t row0, int64_t col0, int64_t dtot) {
  check_key(key);
  CHECK_DEV(w); CHECK_F32(w); CHECK_CONTIG(w);
  TORCH_CHECK(w.dim() == 1 && d >= 1 && row0 >= 0 && col0 >= 0 && (dtot == 0 || col0 + d <= dtot), "es_noise_grad: w (rows,), d >= 1, window");
  const int64_t rows = w.size(0);
  const int chunks = (int)std::max<int64_t>(1, std::min<int64_t>(64, rows / 64));
  c10::DeviceGuard g(w.device());
  auto partial = at::empty({chunks, d}, w.options());
  if (rows > 0)
    evx_es_noise_grad(key.data_ptr<int64_t>(), w.data_ptr<float>(), rows, d, row0, chunks, partial.data_ptr<float>(), cur_stream(), col0, dtot);
  else partial.zero_();
  return partial.sum(0);
}

// ---- K17 / K18 (mo_geom.hip)
std::vector<at::Tensor> knn(const at::Tensor& X, const at::Tensor& Y, int64_t T) {
  for (auto* t : {&X, &Y}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  TORCH_CHECK(X.dim() == 2 && Y.dim() == 2 && X.size(1) == Y.size(1), "knn: X (N, m), Y (M, m)");
  const int64_t N = X.size(0), M = Y.size(0), m = X.size(1);
  TORCH_CHECK(m >= 1 && m <= evx_knn_max_m(), "knn: 1 <= m <= ", evx_knn_max_m());
  TORCH_CHECK(T >= 1 && T <= evx_knn_max_t() && T <= M, "knn: 1 <= T <= min(", evx_knn_max_t(), ", M)");
  c10::DeviceGuard g(X.device());
  auto d = at::empty({N, T}, X.options());
  auto i = at::empty({N, T}, X.options().dtype(at::kInt));
  if (N > 0) evx_knn(X.data_ptr<float>(), Y.data_ptr<float>(), (int)N, (int)M, (int)m, (int)T, d.data_ptr<float>(), i.data_ptr<int32_t>(), cur_stream());
  return {d, i};
}

at::Tensor hv_count(const at::Tensor& S, const at::Tensor& P, int64_t strict) {
  for (auto* t : {&S, &P}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  TORCH_CHECK(S.dim() == 2 && P.dim() == 2 && S.size(1) == P.size(1), "hv_count: samples (S, m), points (n, m)");
  const int64_t m = S.size(1);
  TORCH_CHECK(m >= 1 && m <= evx_hv_max_m(), "hv_count: 1 <= m <= ", evx_hv_max_m());
  c10::DeviceGuard g(S.device());
  auto c = at::empty({S.size(0)}, S.options().dtype(at::kInt));
  if (S.size(0) > 0) evx_hv_count(S.data_ptr<float>(), P.data_ptr<float>(), (int)S.size(0), (int)P.size(0), (int)m, (int)strict, c.data_ptr<int32_t>(), cur_stream());
  return c;
}

at::Tensor hv_contrib(const at::Tensor& S, const at::Tensor& P, const at::Tensor& count, const at::Tensor& alpha) {
  for (auto* t : {&S, &P, &alpha}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  TORCH_CHECK(count.is_cuda() && count.scalar_type() == at::kInt && count.is_contiguous() && count.numel() == S.size(0), "hv_contrib: count int32[S]");
  TORCH_CHECK(S.dim() == 2 && P.dim() == 2 && S.size(1) == P.size(1) && S.size(1) <= evx_hv_max_m(), "hv_contrib: samples (S, m), points (n, m)");
  TORCH_CHECK(alpha.numel() >= P.size(0), "hv_contrib: alpha needs n entries");
  c10::DeviceGuard g(S.device());
  auto f = at::zeros({P.size(0)}, S.options());
  if (P.size(0) > 0)
    evx_hv_contrib(S.data_ptr<float>(), P.data_ptr<float>(), count.data_ptr<int32_t>(), alpha.data_ptr<float>(), (int)S.size(0), (int)P.size(0),
                   (int)S.size(1), f.data_ptr<float>(), cur_stream());
  return f;
}

TORCH_LIBRARY(evoxmi, m) {
  m.def("es_noise_grad(Tensor key, Tensor w, int d, int row0, int col0=0, int dtot=0) -> Tensor");
  m.def("es_population(Tensor key, Tensor center, float sigma, int rows, int half, int row0, int col0=0, int dtot=0) -> Tensor");
  m.def("knn(Tensor X, Tensor Y, int T) -> Tensor[]");
  m.def("hv_count(Tensor S, Tensor P, int strict) -> Tensor");
  m.def("hv_contrib(Tensor S, Tensor P, Tensor count, Tensor alpha) -> Tensor");
  m.def("philox_fill(Tensor key, int n, int dist, int offset) -> Tensor");
  m.def("philox_window(Tensor key, int rows, int dtot, int col0, int own, int row0, int dist) -> Tensor");
  m.def("argsort_f32(Tensor keys, int descending) -> Tensor[]");
  m.def("radix_argsort_f32(Tensor keys, int descending) -> Tensor[]");
  m.def("rank_argsort_f32(Tensor keys, int descending) -> Tensor[]");
  m.def("merge_argsort_f32(Tensor keys, int descending) -> Tensor[]");
  m.def("cec_basic(Tensor Z, int fid, Tensor? perm, int start, int L, Tensor? sub, float scale, Tensor? Y, int ystart, int yperm, float clamp=0.0) -> Tensor");
  m.def("cec_compose(Tensor? Z, Tensor X, Tensor Os, int[] fid, int[] zcol, int[] comp, float[] scale, float[] sigma, float[] lamb, "
        "float[] bias, float thr) -> Tensor");
  m.def("jacobi_sweeps(Tensor A, Tensor B, Tensor sched, int sweeps, float tol, float inner_tol, int max_inner, int fused=2) -> Tensor[]");
  m.def("philox_words(Tensor key, int nblocks, int domain, int offset, int words=4) -> Tensor");
  m.def("weighted_rowsum(Tensor X, Tensor? idx, Tensor w, Tensor? sub, int K) -> Tensor");
  m.def("gemm_set_config(int cfg) -> ()");
  m.def("sbx(Tensor x, Tensor keys, float pro_c, float dis_c, int type, int col0=0, int dtot=0) -> Tensor");
  m.def("pm(Tensor x, Tensor lb, Tensor ub, Tensor keys, float pro_m, float dis_m, int nm, int col0=0, int dtot=0) -> Tensor");
  m.def("nds(Tensor f, int limit=0, Tensor? err=None) -> Tensor");
  m.def("ant_rollout(Tensor W, int h1, int h2, Tensor init, int cap) -> Tensor[]");
  m.def("stochastic_ranking(Tensor I1, Tensor I2, Tensor rnd, float pc) -> Tensor");
  m.def("moead_scan(Tensor objs, Tensor off_objs, Tensor P, Tensor W, Tensor z, int func, int nr, int update_z) -> Tensor[]");
  m.def("de_trial(Tensor P, Tensor idx, Tensor coef, Tensor cur, Tensor mode, Tensor CR, Tensor jr, Tensor L, Tensor key, Tensor lb, Tensor ub, int repair, Tensor err, int col0=0, int d_total=0) -> Tensor");
  m.def("dtlz(Tensor X, int m, int variant) -> Tensor");
  m.def("classic_eval(Tensor X, int func, float a, float b, float c) -> Tensor");
  m.def("gemm_f32(Tensor A, int a_rc, Tensor? a_gather, Tensor? a_sub, int a_sub_on_k, Tensor? a_kscale, Tensor? a_kw, Tensor? a_sscale, int a_sscale_inv, Tensor B, int b_rc, Tensor? b_gather, Tensor? b_sub, int b_sub_on_k, Tensor? b_kscale, Tensor? b_kw, Tensor? b_sscale, int b_sscale_inv, Tensor? alpha_ptr, Tensor? bias_n, float beta, Tensor? Cin, int M, int N, int K, int splits, float alpha) -> Tensor");
  m.def("gemm_ks(Tensor A, int a_kc, Tensor B, int b_kc, int M, int N, int K, int mode, float alpha, Tensor? alpha_ptr, Tensor? bias_n, float beta, Tensor? Cin, Tensor? skip, Tensor? a_sub_k=None) -> Tensor");
  m.def("gemm_ks_out(Tensor A, int a_kc, Tensor B, int b_kc, int M, int N, int K, int mode, float alpha, Tensor? alpha_ptr, Tensor? bias_n, float beta, Tensor? Cin, Tensor(a!) out, Tensor? skip, Tensor? a_sub_k=None, Tensor? sel=None, Tensor? A2=None, float alpha2=0., Tensor(b!)? C2=None, Tensor(c!)? stat_part=None, int stat_diag_only=0, int prec=0, float diag_add=0.) -> ()");
  m.def("gemm_ks_grid(int M, int N, int mode) -> int");
  m.def("gemm_ks_tile(int M, int N, int mode) -> int");
  m.def("cec_rotated_rowterms(Tensor X, Tensor Mrot, Tensor o, float alpha, int fid) -> Tensor");
  m.def("sbr16_block_out(Tensor A, int shift, int sweeps, int sb, Tensor(a!) perm, Tensor(b!) Q, Tensor(c!) dq, Tensor skip, float skip_tol=0.0) -> ()");
  m.def("sbr16_far_out(Tensor A, Tensor perm, Tensor Q, Tensor dq, Tensor stats, float thr_fac, Tensor theta, Tensor(a!) X, int sb, Tensor skip) -> ()");
  m.def("sbr16_bq_out(Tensor B, Tensor perm, Tensor Q, Tensor(a!) Bq, int sb, Tensor skip) -> ()");
  m.def("sbr_damping_out(Tensor X2, Tensor V, float tau, Tensor(a!) alpha, Tensor(b!) work, Tensor skip, Tensor(c!)? bar=None, bool no_final=False, Tensor? xpart=None) -> ()");
  m.def("sbr_dev_prep(Tensor X, Tensor X2, Tensor X3, Tensor(c!) alpha, Tensor(a!) P, Tensor(b!) MT, Tensor ctrl, Tensor? work=None, float tau=1.0, Tensor? xpart=None, Tensor? copy_src=None, Tensor(d!)? copy_dst=None, int minus_id=0) -> ()");
  m.def("sbr_dev_copy(Tensor src, Tensor(a!) dst, Tensor skip) -> ()");
  m.def("sbr_dev_ctrl(Tensor part, int nparts, int j, int K, Tensor(a!) hist, Tensor(b!) alpha, Tensor(c!) theta, Tensor(d!) ctrl, Tensor(e!) st, float[] prm, int ns_iters, Tensor A, Tensor(f!) w_out, Tensor(g!) eig_stats, Tensor(h!) w_init, Tensor(i!) log, Tensor(j!) log_count, Tensor(k!)? rep_seq=None, Tensor(l!)? rep_ring=None) -> ()");
  m.def("gemm_ks_set_tile(int t) -> ()");
  m.def("gemm_ks_set_prec(int prec) -> ()");
  m.def("gemm_ks_set_nw8(int tiles) -> ()");
  m.def("gemm_ks_pl(Tensor? A, Tensor? a_pl, Tensor? B, Tensor? b_pl, int M, int N, int K, float alpha, Tensor? alpha_ptr, Tensor? bias_n, Tensor(a!)? out, Tensor? a_sub_k, int sub_cols=0, int sub_ld=0) -> Tensor");
  m.def("sbr16_far_bq_out(Tensor A, Tensor perm, Tensor Q, Tensor dq, Tensor stats, float thr_fac, Tensor theta, Tensor(a!) X, Tensor B, Tensor(b!) Bq, int sb, Tensor skip_far, Tensor skip_bq, bool pre=False) -> ()");
  m.def("lsmop_g(Tensor X, int[] start, int[] sublen, int[] func, int nk, int cosine) -> Tensor");
  m.def("cma_delta_gemv(Tensor M, Tensor mean, Tensor dm, float cm) -> Tensor[]");
  m.def("cma_center_rows(Tensor pop, Tensor? rows, Tensor mean, Tensor sigma, Tensor w, bool aug=False) -> Tensor");
  m.def("cma_local_select(Tensor order, int mu, Tensor w, int start, int size, Tensor(a!) rows, Tensor(b!) wk) -> ()");
  m.def("sym_pack(Tensor S, Tensor(a!) P) -> ()");
  m.def("sym_unpack(Tensor P, Tensor(a!) S) -> ()");
  m.def("cma_paths(Tensor ps, Tensor pc, Tensor y, Tensor delta, Tensor sigma, Tensor count_iter, float[] consts, Tensor? count_eigen=None) -> Tensor[]");
  m.def("cma_cov_pad(Tensor C, Tensor S, Tensor pc, Tensor a, float c1, float cmu, Tensor Bprev, int np, Tensor? Cn_out=None, bool want_bp=True) -> Tensor[]");
  m.def("cma_eig_out(Tensor Bp, Tensor w, int d, Tensor? B_out=None, Tensor? B_alt=None, Tensor? keep=None) -> Tensor[]");
  m.def("nsga_select(Tensor rank, Tensor f, int N, int mask_pos) -> Tensor");
  m.def("moead_parents(Tensor nb, Tensor key, int row0=0, int rows=0) -> Tensor[]");
  m.def("moead_variation(Tensor pop, Tensor p0, Tensor p1, Tensor kx, Tensor km, Tensor lb, Tensor ub, float pro_c, float dis_c, float pro_m, float dis_m, int nm, int row0=0, int rows=0, Tensor? win=None, Tensor(a!)? out=None) -> Tensor");
  m.def("moead_halo_replace(Tensor(a!) obj, Tensor off_obj, Tensor W, Tensor z, Tensor zmax, Tensor rowptr, Tensor owner, Tensor slots, int func, Tensor(b!) win_h) -> ()");
  m.def("moead_halo_gather(Tensor(a!) pop, Tensor slots, Tensor win_h, Tensor peer, Tensor starts, Tensor(b!)? first=None) -> ()");
  m.def("peer_release(int device) -> ()");
  m.def("ipc_alloc(int numel, int device) -> Tensor");
  m.def("ipc_handle(Tensor t) -> Tensor");
  m.def("ipc_open(Tensor handle, int device) -> int");
  m.def("ipc_close(int ptr) -> ()");
  m.def("moead_replace(Tensor pop_obj, Tensor off_obj, Tensor W, Tensor z, Tensor zmax, Tensor rowptr, Tensor owner, int func) -> Tensor[]");
  m.def("moead_select_rows(Tensor pop, Tensor off, Tensor win) -> Tensor");
  m.def("moead_select_rows_(Tensor(a!) pop, Tensor off, Tensor win) -> ()");
  m.def("sbr_stats(Tensor A) -> Tensor");
  m.def("sbr_block(Tensor A, int off, int sweeps, Tensor? dbg=None) -> Tensor[]");
  m.def("sbr_far(Tensor A, int off, Tensor perm, Tensor Q, Tensor dq, Tensor stats, float thr_fac) -> Tensor");
  m.def("sbr_bq(Tensor B, int off, Tensor perm, Tensor Q) -> Tensor");
  m.def("sbr_symstats(Tensor T) -> Tensor[]");
  m.def("sbr16_block(Tensor A, int shift, int sweeps, int sb=16) -> Tensor[]");
  m.def("sbr16_far(Tensor A, Tensor perm, Tensor Q, Tensor dq, Tensor stats, float thr_fac, float theta) -> Tensor");
  m.def("sbr16_bq(Tensor B, Tensor perm, Tensor Q) -> Tensor");
  m.def("sbr_taylor4_prep(Tensor X, Tensor X2, Tensor? alpha=None, int mt=0) -> Tensor[]");
  m.def("linear_gp_fit(Tensor a, Tensor b, Tensor c, Tensor n, int steps, float lr) -> Tensor[]");
  m.def("sbr_damping(Tensor X2, Tensor V, float tau, Tensor(a!)? out=None) -> Tensor");
  m.def("sbr_symstats_out(Tensor T, Tensor(a!) A, Tensor(b!) st) -> ()");
  m.def("sbr_taylor_prep(Tensor X, Tensor X2, Tensor X3, Tensor? alpha=None, int mt=0) -> Tensor[]");
  m.def("pso_update(Tensor pop, Tensor vel, Tensor lbl, Tensor lbf, Tensor fit, Tensor gbl, Tensor kp, Tensor kg, float w, float phip, float phig, Tensor lb, Tensor ub, int col0=0, int d_total=0) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(evoxmi, CompositeExplicitAutograd, m) {
  m.impl("stochastic_ranking", &stochastic_ranking);
  m.impl("gemm_set_config", &gemm_set_config);
  m.impl("gemm_ks_set_tile", &gemm_ks_set_tile);
  m.impl("gemm_ks_set_prec", &gemm_ks_set_prec);
  m.impl("gemm_ks_set_nw8", &gemm_ks_set_nw8);
  m.impl("gemm_ks_pl", &gemm_ks_pl);
  m.impl("sbr16_far_bq_out", &sbr16_far_bq_out);
  m.impl("gemm_ks_grid", &gemm_ks_grid);
  m.impl("gemm_ks_tile", &gemm_ks_tile);
  m.impl("peer_release", &peer_release);
  m.impl("ipc_alloc", &ipc_alloc);
  m.impl("ipc_open", &ipc_open);
  m.impl("ipc_close", &ipc_close);
}

TORCH_LIBRARY_IMPL(evoxmi, CUDA, m) {
  m.impl("cec_rotated_rowterms", &cec_rotated_rowterms);
  m.impl("philox_fill", &philox_fill);
  m.impl("philox_window", &philox_window);
  m.impl("classic_eval", &classic_eval);
  m.impl("sbx", &sbx);
  m.impl("pm", &pm);
  m.impl("nds", &nds);
  m.impl("ant_rollout", &ant_rollout);
  m.impl("moead_scan", &moead_scan);
  m.impl("de_trial", &de_trial);
  m.impl("dtlz", &dtlz);
  m.impl("philox_words", &philox_words);
  m.impl("weighted_rowsum", &weighted_rowsum);
  m.impl("jacobi_sweeps", &jacobi_sweeps);
  m.impl("cec_basic", &cec_basic);
  m.impl("cec_compose", &cec_compose);
  m.impl("argsort_f32", &argsort_f32);
  m.impl("radix_argsort_f32", &radix_argsort_f32);
  m.impl("rank_argsort_f32", &rank_argsort_f32);
  m.impl("merge_argsort_f32", &merge_argsort_f32);
  m.impl("gemm_f32", &gemm_f32);
  m.impl("gemm_ks", &gemm_ks_new);
  m.impl("gemm_ks_out", &gemm_ks_out);
  m.impl("sbr16_block_out", &sbr16_block_out);
  m.impl("moead_halo_replace", &moead_halo_replace);
  m.impl("moead_halo_gather", &moead_halo_gather);
  m.impl("ipc_handle", &ipc_handle);
  m.impl("sbr16_far_out", &sbr16_far_out);
  m.impl("sbr16_bq_out", &sbr16_bq_out);
  m.impl("sbr_damping_out", &sbr_damping_out);
  m.impl("sbr_dev_prep", &sbr_dev_prep);
  m.impl("sbr_dev_copy", &sbr_dev_copy);
  m.impl("sbr_dev_ctrl", &sbr_dev_ctrl);
  m.impl("pso_update", &pso_update);
  m.impl("lsmop_g", &lsmop_g);
  m.impl("cma_delta_gemv", &cma_delta_gemv);
  m.impl("cma_center_rows", &cma_center_rows);
  m.impl("cma_local_select", &cma_local_select);
  m.impl("sym_pack", &sym_pack);
  m.impl("sym_unpack", &sym_unpack);
  m.impl("cma_paths", &cma_paths);
  m.impl("cma_cov_pad", &cma_cov_pad);
  m.impl("cma_eig_out", &cma_eig_out);
  m.impl("nsga_select", &nsga_select);
  m.impl("moead_parents", &moead_parents);
  m.impl("moead_variation", &moead_variation);
  m.impl("moead_replace", &moead_replace);
  m.impl("moead_select_rows_", &moead_select_rows_);
  m.impl("moead_select_rows", &moead_select_rows);
  m.impl("sbr_stats", &sbr_stats);
  m.impl("sbr_block", &sbr_block);
  m.impl("sbr_far", &sbr_far);
  m.impl("sbr_bq", &sbr_bq);
  m.impl("es_noise_grad", &es_noise_grad);
  m.impl("es_population", &es_population);
  m.impl("knn", &knn);
  m.impl("hv_count", &hv_count);
  m.impl("hv_contrib", &hv_contrib);
  m.impl("sbr_symstats_out", &sbr_symstats_out);
  m.impl("sbr_symstats", &sbr_symstats);
  m.impl("sbr16_block", &sbr16_block);
  m.impl("sbr16_far", &sbr16_far);
  m.impl("sbr16_bq", &sbr16_bq);
  m.impl("sbr_damping", &sbr_damping);
  m.impl("linear_gp_fit", &linear_gp_fit);
  m.impl("sbr_taylor4_prep", &sbr_taylor4_prep);
  m.impl("sbr_taylor_prep", &sbr_taylor_prep);
}
