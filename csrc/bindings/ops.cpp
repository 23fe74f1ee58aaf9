// TORCH_LIBRARY registration of evoxmi's HIP kernels (namespace `evoxmi`).
// Kernel translation units (csrc/kernels/*.hip) expose plain C++ launchers that
// take raw device pointers + the caller's hipStream_t; this file is the only one
// that sees torch headers.  Every op launches on the *current* HIP stream so it is
// ordered with surrounding torch work and can be captured into a hipGraph.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/hip/HIPGuard.h>
#include <hip/hip_runtime.h>

#include "evoxmi_launchers.h"

namespace {

inline hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

#define CHECK_DEV(t) TORCH_CHECK((t).is_cuda(), #t " must be a HIP device tensor")
#define CHECK_F32(t) TORCH_CHECK((t).scalar_type() == at::kFloat, #t " must be float32")
#define CHECK_CONTIG(t) TORCH_CHECK((t).is_contiguous(), #t " must be contiguous")

void check_key(const at::Tensor& key) {
  CHECK_DEV(key);
  TORCH_CHECK(key.scalar_type() == at::kLong && key.numel() == 2 && key.is_contiguous(), "key must be int64[2]");
}

at::Tensor philox_fill(const at::Tensor& key, int64_t n, int64_t dist, int64_t offset) {
  check_key(key);
  TORCH_CHECK(offset % 4 == 0, "offset must be a multiple of 4");
  c10::hip::HIPGuard g(key.device());
  auto out = at::empty({n}, key.options().dtype(at::kFloat));
  if (n > 0) evx_philox_fill(out.data_ptr<float>(), n, key.data_ptr<int64_t>(), (int)dist, offset, cur_stream());
  return out;
}

at::Tensor classic_eval(const at::Tensor& X, int64_t func, double a, double b, double c) {
  CHECK_DEV(X); CHECK_F32(X); CHECK_CONTIG(X);
  TORCH_CHECK(X.dim() == 2, "X must be (N, d)");
  c10::hip::HIPGuard g(X.device());
  auto out = at::empty({X.size(0)}, X.options());
  if (X.size(0) > 0)
    evx_classic_eval(X.data_ptr<float>(), out.data_ptr<float>(), (int)X.size(0), (int)X.size(1), (int)func, (float)a, (float)b,
                     (float)c, cur_stream());
  return out;
}

std::vector<at::Tensor> pso_update(const at::Tensor& pop, const at::Tensor& vel, const at::Tensor& lbl,
                                   const at::Tensor& lbf, const at::Tensor& fit, const at::Tensor& gbl,
                                   const at::Tensor& kp, const at::Tensor& kg, double w, double phip, double phig,
                                   const at::Tensor& lb, const at::Tensor& ub) {
  for (auto* t : {&pop, &vel, &lbl, &lbf, &fit, &gbl, &lb, &ub}) { CHECK_DEV(*t); CHECK_F32(*t); CHECK_CONTIG(*t); }
  check_key(kp); check_key(kg);
  const int64_t N = pop.size(0), D = pop.size(1);
  TORCH_CHECK(vel.sizes() == pop.sizes() && lbl.sizes() == pop.sizes(), "shape mismatch");
  TORCH_CHECK(lbf.numel() == N && fit.numel() == N && gbl.numel() == D && lb.numel() == D && ub.numel() == D, "shape mismatch");
  c10::hip::HIPGuard g(pop.device());
  auto opop = at::empty_like(pop), ovel = at::empty_like(pop), olbl = at::empty_like(pop), olbf = at::empty_like(lbf);
  evx_pso_update(pop.data_ptr<float>(), vel.data_ptr<float>(), lbl.data_ptr<float>(), lbf.data_ptr<float>(),
                 fit.data_ptr<float>(), gbl.data_ptr<float>(), kp.data_ptr<int64_t>(), kg.data_ptr<int64_t>(), (float)w,
                 (float)phip, (float)phig, lb.data_ptr<float>(), ub.data_ptr<float>(), opop.data_ptr<float>(),
                 ovel.data_ptr<float>(), olbl.data_ptr<float>(), olbf.data_ptr<float>(), (int)N, (int)D, cur_stream());
  return {opop, ovel, olbl, olbf};
}

}  // namespace

TORCH_LIBRARY(evoxmi, m) {
  m.def("philox_fill(Tensor key, int n, int dist, int offset) -> Tensor");
  m.def("classic_eval(Tensor X, int func, float a, float b, float c) -> Tensor");
  m.def("pso_update(Tensor pop, Tensor vel, Tensor lbl, Tensor lbf, Tensor fit, Tensor gbl, Tensor kp, Tensor kg, float w, float phip, float phig, Tensor lb, Tensor ub) -> Tensor[]");
}

TORCH_LIBRARY_IMPL(evoxmi, CUDA, m) {
  m.impl("philox_fill", &philox_fill);
  m.impl("classic_eval", &classic_eval);
  m.impl("pso_update", &pso_update);
}
