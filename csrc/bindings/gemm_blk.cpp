// torch-op bindings of the blocked-planes bf16x6 GEMM (csrc/kernels/gemm_blk.hip).
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>

#include <vector>

#include "evoxmi_launchers.h"

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a HIP device tensor")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")

const float* opt_vec(const c10::optional<at::Tensor>& t, int64_t n, const char* what) {
  if (!t.has_value() || !t->defined()) return nullptr;
  CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t);
  TORCH_CHECK(t->numel() >= n, what, ": length ", t->numel(), " < ", n);
  return t->data_ptr<float>();
}

// planes buffer of `rows` × K: int16 (evx_blk_elems), 16-byte aligned
void check_blk(const at::Tensor& t, int64_t rows, int64_t K, const char* what) {
  CHECK_DEV(t);
  TORCH_CHECK(t.scalar_type() == at::kShort && t.is_contiguous() && t.numel() >= evx_blk_elems(rows, (int)K) &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              what, ": blocked planes int16[", evx_blk_elems(rows, (int)K), "] for ", rows, " x ", K);
}

at::Tensor blk_split(const at::Tensor& X, const c10::optional<at::Tensor>& sub_k, const c10::optional<at::Tensor>& colscale,
                     const c10::optional<at::Tensor>& out) {
  CHECK_DEV(X); CHECK_F32(X);
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "blk_split: 2-D, unit inner stride");
  const int64_t rows = X.size(0), K = X.size(1);
  TORCH_CHECK(rows > 0 && K > 0, "blk_split: empty");
  c10::DeviceGuard g(X.device());
  at::Tensor o;
  if (out.has_value() && out->defined()) {
    o = *out;
    check_blk(o, rows, K, "blk_split out");
  } else {
    o = at::empty({evx_blk_elems(rows, (int)K)}, X.options().dtype(at::kShort));
  }
  evx_split_blk(X.data_ptr<float>(), X.stride(0), rows, (int)K, opt_vec(sub_k, K, "sub_k"), opt_vec(colscale, K, "colscale"),
                reinterpret_cast<uint16_t*>(o.data_ptr<int16_t>()), cur_stream());
  return o;
}

at::Tensor blk_philox_normal(const at::Tensor& key, int64_t rows, int64_t d, int64_t row0, const c10::optional<at::Tensor>& out) {
  CHECK_DEV(key);
  TORCH_CHECK(key.scalar_type() == at::kLong && key.numel() >= 2 && key.is_contiguous(), "blk_philox_normal: key int64[2]");
  TORCH_CHECK(d % 4 == 0 && rows > 0, "blk_philox_normal: d % 4 == 0, rows > 0");
  c10::DeviceGuard g(key.device());
  at::Tensor o;
  if (out.has_value() && out->defined()) {
    o = *out;
    check_blk(o, rows, d, "blk_philox_normal out");
  } else {
    o = at::empty({evx_blk_elems(rows, (int)d)}, key.options().dtype(at::kShort));
  }
  evx_philox_blk(key.data_ptr<int64_t>(), rows, (int)d, row0, reinterpret_cast<uint16_t*>(o.data_ptr<int16_t>()), cur_stream());
  return o;
}

at::Tensor gemm_blk(const at::Tensor& A, int64_t M, const at::Tensor& B, int64_t N, int64_t K, double alpha,
                    const c10::optional<at::Tensor>& alpha_ptr, const c10::optional<at::Tensor>& bias_n,
                    const c10::optional<at::Tensor>& out, const c10::optional<at::Tensor>& skip) {
  TORCH_CHECK(M > 0 && N > 0 && K > 0, "gemm_blk: shape");
  check_blk(A, M, K, "gemm_blk A");
  check_blk(B, N, K, "gemm_blk B");
  c10::DeviceGuard g(A.device());
  at::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    CHECK_DEV(C); CHECK_F32(C);
    TORCH_CHECK(C.dim() == 2 && C.stride(1) == 1 && C.size(0) >= M && C.size(1) >= N, "gemm_blk: out shape");
  } else {
    C = at::empty({M, N}, A.options().dtype(at::kFloat));
  }
  EvxGemmBlk a{};
  a.A = reinterpret_cast<const uint16_t*>(A.data_ptr<int16_t>());
  a.a_rows = evx_blk_rows(M);
  a.B = reinterpret_cast<const uint16_t*>(B.data_ptr<int16_t>());
  a.b_rows = evx_blk_rows(N);
  a.KB = (int)((K + 15) / 16);
  a.M = (int)M;
  a.N = (int)N;
  a.C = C.data_ptr<float>();
  a.ldc = C.stride(0);
  a.alpha = (float)alpha;
  a.alpha_ptr = opt_vec(alpha_ptr, 1, "alpha_ptr");
  a.bias_n = opt_vec(bias_n, N, "bias_n");
  if (skip.has_value() && skip->defined()) {
    CHECK_DEV(*skip);
    TORCH_CHECK(skip->scalar_type() == at::kInt, "gemm_blk: skip int32");
    a.skip = skip->data_ptr<int32_t>();
  }
  evx_gemm_blk(a, cur_stream());
  return C;
}

void check_h3(const at::Tensor& t, const at::Tensor& rinv, int64_t rows, int64_t K, const char* what, int64_t ncomp = 1) {
  CHECK_DEV(t); CHECK_DEV(rinv);
  TORCH_CHECK(ncomp >= 1, what, ": ncomp >= 1");
  TORCH_CHECK(t.scalar_type() == at::kShort && t.is_contiguous() && t.numel() >= ncomp * evx_h3_elems(rows, (int)K) &&
                  reinterpret_cast<uintptr_t>(t.data_ptr()) % 16 == 0,
              what, ": f16x3 planes int16[", ncomp, " x ", evx_h3_elems(rows, (int)K), "] for ", rows, " x ", K);
  TORCH_CHECK(rinv.scalar_type() == at::kFloat && rinv.is_contiguous() && rinv.numel() >= ncomp * evx_blk_rows(rows), what,
              ": row scales float32[", ncomp, " x ", evx_blk_rows(rows), "]");
}

std::vector<at::Tensor> h3_alloc(const at::Tensor& like, int64_t rows, int64_t K, const c10::optional<at::Tensor>& out,
                                 const c10::optional<at::Tensor>& rinv_out, const char* what, int64_t ncomp = 1) {
  at::Tensor o, r;
  if (out.has_value() && out->defined()) {
    TORCH_CHECK(rinv_out.has_value() && rinv_out->defined(), what, ": out and rinv_out together");
    o = *out;
    r = *rinv_out;
    check_h3(o, r, rows, K, what, ncomp);
  } else {
    o = at::empty({ncomp * evx_h3_elems(rows, (int)K)}, like.options().dtype(at::kShort));
    r = at::empty({ncomp * evx_blk_rows(rows)}, like.options().dtype(at::kFloat));
  }
  return {o, r};
}

// sub_k: a K-vector, or an ncomp × K matrix (row c shifts plane set c: one read of X)
std::vector<at::Tensor> h3_split(const at::Tensor& X, const c10::optional<at::Tensor>& sub_k, const c10::optional<at::Tensor>& colscale,
                                 const c10::optional<at::Tensor>& out, const c10::optional<at::Tensor>& rinv_out) {
  CHECK_DEV(X); CHECK_F32(X);
  TORCH_CHECK(X.dim() == 2 && X.stride(1) == 1, "h3_split: 2-D, unit inner stride");
  const int64_t rows = X.size(0), K = X.size(1);
  TORCH_CHECK(rows > 0 && K > 0, "h3_split: empty");
  c10::DeviceGuard g(X.device());
  int64_t ncomp = 1, sub_ld = 0;
  const float* sub = nullptr;
  if (sub_k.has_value() && sub_k->defined() && sub_k->dim() == 2) {
    CHECK_DEV(*sub_k); CHECK_F32(*sub_k);
    TORCH_CHECK(sub_k->size(1) >= K && sub_k->stride(1) == 1 && sub_k->size(0) >= 1, "h3_split: sub_k ncomp x K, unit inner stride");
    ncomp = sub_k->size(0);
    sub_ld = sub_k->stride(0);
    sub = sub_k->data_ptr<float>();
  } else {
    sub = opt_vec(sub_k, K, "sub_k");
  }
  auto v = h3_alloc(X, rows, K, out, rinv_out, "h3_split", ncomp);
  evx_split_h3(X.data_ptr<float>(), X.stride(0), rows, (int)K, sub, opt_vec(colscale, K, "colscale"),
               reinterpret_cast<uint16_t*>(v[0].data_ptr<int16_t>()), v[1].data_ptr<float>(), cur_stream(), (int)ncomp, sub_ld);
  return v;
}

std::vector<at::Tensor> h3_philox_normal(const at::Tensor& key, int64_t rows, int64_t d, int64_t row0, const c10::optional<at::Tensor>& out,
                                         const c10::optional<at::Tensor>& rinv_out) {
  CHECK_DEV(key);
  TORCH_CHECK(key.scalar_type() == at::kLong && key.numel() >= 2 && key.is_contiguous(), "h3_philox_normal: key int64[2]");
  TORCH_CHECK(d % 4 == 0 && rows > 0, "h3_philox_normal: d % 4 == 0, rows > 0");
  c10::DeviceGuard g(key.device());
  auto v = h3_alloc(key, rows, d, out, rinv_out, "h3_philox_normal");
  evx_philox_h3(key.data_ptr<int64_t>(), rows, (int)d, row0, reinterpret_cast<uint16_t*>(v[0].data_ptr<int16_t>()), v[1].data_ptr<float>(),
                cur_stream());
  return v;
}

at::Tensor gemm_h3(const at::Tensor& A, const at::Tensor& a_rinv, int64_t M, const at::Tensor& B, const at::Tensor& b_rinv, int64_t N,
                   int64_t K, double alpha, const c10::optional<at::Tensor>& alpha_ptr, const c10::optional<at::Tensor>& bias_n,
                   const c10::optional<at::Tensor>& out, const c10::optional<at::Tensor>& skip, int64_t sub_cols) {
  TORCH_CHECK(M > 0 && N > 0 && K > 0, "gemm_h3: shape");
  // stacked A (sub_cols > 0): one plane set per sub_cols-wide output column block
  TORCH_CHECK(sub_cols >= 0 && sub_cols % evx_gemm_blk_tile_n() == 0, "gemm_h3: sub_cols a multiple of the tile width ",
              evx_gemm_blk_tile_n());
  const int64_t ncomp = sub_cols > 0 ? (N + sub_cols - 1) / sub_cols : 1;
  check_h3(A, a_rinv, M, K, "gemm_h3 A", ncomp);
  check_h3(B, b_rinv, N, K, "gemm_h3 B");
  c10::DeviceGuard g(A.device());
  at::Tensor C;
  if (out.has_value() && out->defined()) {
    C = *out;
    CHECK_DEV(C); CHECK_F32(C);
    TORCH_CHECK(C.dim() == 2 && C.stride(1) == 1 && C.size(0) >= M && C.size(1) >= N, "gemm_h3: out shape");
  } else {
    C = at::empty({M, N}, A.options().dtype(at::kFloat));
  }
  EvxGemmBlk a{};
  a.A = reinterpret_cast<const uint16_t*>(A.data_ptr<int16_t>());
  a.a_rows = evx_blk_rows(M);
  a.B = reinterpret_cast<const uint16_t*>(B.data_ptr<int16_t>());
  a.b_rows = evx_blk_rows(N);
  a.a_rinv = a_rinv.data_ptr<float>();
  a.b_rinv = b_rinv.data_ptr<float>();
  a.KB = (int)((K + 15) / 16);
  a.M = (int)M;
  a.N = (int)N;
  a.C = C.data_ptr<float>();
  a.ldc = C.stride(0);
  a.alpha = (float)alpha;
  a.alpha_ptr = opt_vec(alpha_ptr, 1, "alpha_ptr");
  a.bias_n = opt_vec(bias_n, N, "bias_n");
  a.sub_cols = (int)sub_cols;
  a.a_comp_stride = evx_h3_elems(M, (int)K);
  if (skip.has_value() && skip->defined()) {
    CHECK_DEV(*skip);
    TORCH_CHECK(skip->scalar_type() == at::kInt, "gemm_h3: skip int32");
    a.skip = skip->data_ptr<int32_t>();
  }
  evx_gemm_h3(a, cur_stream());
  return C;
}

// CEC'22 F1 / F4 on the f16x3 rotation: the GEMM epilogue reduces each row's basic-function terms
// over its 128-column tile (the rotated population is never written), one finishing kernel sums
// the tiles in order and applies the f < 1e-8 clamp
at::Tensor gemm_h3_rowterms(const at::Tensor& A, const at::Tensor& a_rinv, int64_t M, const at::Tensor& B, const at::Tensor& b_rinv,
                            int64_t N, int64_t K, double alpha, int64_t fid) {
  TORCH_CHECK(M > 0 && N > 0 && K > 0, "gemm_h3_rowterms: shape");
  TORCH_CHECK(fid == 0 || fid == 3, "gemm_h3_rowterms: Zakharov (0) or Rastrigin (3)");
  check_h3(A, a_rinv, M, K, "gemm_h3_rowterms A");
  check_h3(B, b_rinv, N, K, "gemm_h3_rowterms B");
  c10::DeviceGuard g(A.device());
  const int tn = evx_gemm_h3_tiles_n((int)N);
  auto parts = at::empty({tn, M, 2}, A.options().dtype(at::kFloat));
  auto out = at::empty({M}, A.options().dtype(at::kFloat));
  EvxGemmBlk a{};
  a.A = reinterpret_cast<const uint16_t*>(A.data_ptr<int16_t>());
  a.a_rows = evx_blk_rows(M);
  a.B = reinterpret_cast<const uint16_t*>(B.data_ptr<int16_t>());
  a.b_rows = evx_blk_rows(N);
  a.a_rinv = a_rinv.data_ptr<float>();
  a.b_rinv = b_rinv.data_ptr<float>();
  a.KB = (int)((K + 15) / 16);
  a.M = (int)M;
  a.N = (int)N;
  a.C = parts.data_ptr<float>();  // not written in row-terms mode
  a.ldc = N;
  a.alpha = (float)alpha;
  a.row_terms = parts.data_ptr<float>();
  a.row_fid = (int)fid;
  evx_gemm_h3(a, cur_stream());
  evx_cec_rowterms_final(parts.data_ptr<float>(), tn, (int)M, (int)fid, out.data_ptr<float>(), cur_stream());
  return out;
}

int64_t h3_elems(int64_t rows, int64_t K) { return evx_h3_elems(rows, (int)K); }

int64_t blk_elems(int64_t rows, int64_t K) { return evx_blk_elems(rows, (int)K); }
int64_t blk_rows(int64_t rows) { return evx_blk_rows(rows); }
int64_t gemm_blk_tile(int64_t which) { return which == 0 ? evx_gemm_blk_tile_m() : evx_gemm_blk_tile_n(); }

}  // namespace

TORCH_LIBRARY_FRAGMENT(evoxmi, m) {
  m.def("blk_split(Tensor X, Tensor? sub_k=None, Tensor? colscale=None, Tensor(a!)? out=None) -> Tensor");
  m.def("blk_philox_normal(Tensor key, int rows, int d, int row0=0, Tensor(a!)? out=None) -> Tensor");
  m.def("gemm_blk(Tensor A, int M, Tensor B, int N, int K, float alpha=1., Tensor? alpha_ptr=None, Tensor? bias_n=None, "
        "Tensor(a!)? out=None, Tensor? skip=None) -> Tensor");
  m.def("blk_elems(int rows, int K) -> int");
  m.def("h3_split(Tensor X, Tensor? sub_k=None, Tensor? colscale=None, Tensor(a!)? out=None, Tensor(b!)? rinv_out=None) -> Tensor[]");
  m.def("h3_philox_normal(Tensor key, int rows, int d, int row0=0, Tensor(a!)? out=None, Tensor(b!)? rinv_out=None) -> Tensor[]");
  m.def("gemm_h3(Tensor A, Tensor a_rinv, int M, Tensor B, Tensor b_rinv, int N, int K, float alpha=1., Tensor? alpha_ptr=None, "
        "Tensor? bias_n=None, Tensor(a!)? out=None, Tensor? skip=None, int sub_cols=0) -> Tensor");
  m.def("gemm_h3_rowterms(Tensor A, Tensor a_rinv, int M, Tensor B, Tensor b_rinv, int N, int K, float alpha, int fid) -> Tensor");
  m.def("h3_elems(int rows, int K) -> int");
  m.def("blk_rows(int rows) -> int");
  m.def("gemm_blk_tile(int which) -> int");
}

TORCH_LIBRARY_IMPL(evoxmi, CUDA, m) {
  m.impl("blk_split", &blk_split);
  m.impl("blk_philox_normal", &blk_philox_normal);
  m.impl("gemm_blk", &gemm_blk);
  m.impl("h3_split", &h3_split);
  m.impl("gemm_h3_rowterms", &gemm_h3_rowterms);
  m.impl("h3_philox_normal", &h3_philox_normal);
  m.impl("gemm_h3", &gemm_h3);
}

TORCH_LIBRARY_IMPL(evoxmi, CompositeExplicitAutograd, m) {
  m.impl("blk_elems", &blk_elems);
  m.impl("h3_elems", &h3_elems);
  m.impl("blk_rows", &blk_rows);
  m.impl("gemm_blk_tile", &gemm_blk_tile);
}
