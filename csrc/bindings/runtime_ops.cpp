// Small runtime ops (stream-ordered host transfers) for the framework's host-side control.
#include <torch/library.h>
#include <ATen/ATen.h>
#include <c10/hip/HIPStream.h>
#include <c10/core/DeviceGuard.h>
#include <hip/hip_runtime.h>

#include "evoxmi_launchers.h"

namespace {

// src (device) → dst (pinned host) on the current stream, no host wait: under a hipGraph
// capture this becomes a memcpy node that refreshes dst on every replay.  The caller learns
// that the copy landed from an event it records after the step (no synchronize).
void copy_d2h_async(const at::Tensor& src, at::Tensor& dst) {
  TORCH_CHECK(src.is_cuda() && src.is_contiguous(), "copy_d2h_async: contiguous device source");
  TORCH_CHECK(!dst.is_cuda() && dst.is_pinned() && dst.is_contiguous(), "copy_d2h_async: contiguous pinned host destination");
  TORCH_CHECK(src.scalar_type() == dst.scalar_type() && src.numel() <= dst.numel(), "copy_d2h_async: dtype / size");
  c10::DeviceGuard g(src.device());
  const auto st = hipMemcpyAsync(dst.data_ptr(), src.data_ptr(), src.numel() * src.element_size(), hipMemcpyDeviceToHost,
                                 c10::hip::getCurrentHIPStream().stream());
  TORCH_CHECK(st == hipSuccess, "copy_d2h_async: ", hipGetErrorString(st));
}


}  // namespace

TORCH_LIBRARY_FRAGMENT(evoxmi, m) {
  m.def("copy_d2h_async(Tensor src, Tensor(a!) dst) -> ()");
}

TORCH_LIBRARY_IMPL(evoxmi, CompositeExplicitAutograd, m) {
  m.impl("copy_d2h_async", &copy_d2h_async);
}
