// Per-step loss bookkeeping of the training loop in one launch.
//
// Replaces, per step, the host-side reductions of Trainer._train_epoch (common/trainer.py:183-193):
//   loss_tuple = tuple(per_loss.item() for per_loss in losses); total_loss += loss_tuple;
//   if self._check_nan(loss): ... (loss = sum(losses))
// which the engine keeps on the device (no host sync per step): the float64 running sums of every
// loss component and a sticky NaN flag read by the fused Adam (skip the update) and at epoch end.
// torch would issue ~8 small kernels for it (casts, stack, add, sum, isnan, or).
#include "fr_common.h"

namespace {

constexpr int kMaxParts = 8;

struct Parts {
  const float* p[kMaxParts];
  int n;
};

__global__ void step_book_kernel(Parts parts, double* __restrict__ acc, int accumulate, int32_t* __restrict__ nan_flag) {
  if (threadIdx.x != 0) return;
  float s = 0.f;  // sum(losses) in fp32, left to right, as Python's sum over fp32 tensors
  for (int i = 0; i < parts.n; ++i) {
    const float v = parts.p[i][0];
    acc[i] = accumulate ? acc[i] + (double)v : (double)v;
    s = i == 0 ? v : s + v;
  }
  if (s != s) nan_flag[0] |= 1;
}

}  // namespace

extern "C" int fr_step_book(const float* const* d_parts, int n, double* d_acc, int accumulate, int32_t* d_nan,
                            void* stream) {
  FR_REQUIRE(n >= 1 && n <= kMaxParts, "1..8 loss parts");
  FR_REQUIRE(d_parts && d_acc && d_nan, "null argument");
  Parts p{};
  for (int i = 0; i < n; ++i) {
    FR_REQUIRE(d_parts[i] != nullptr, "null loss part");
    p.p[i] = d_parts[i];
  }
  p.n = n;
  hipLaunchKernelGGL(step_book_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), p, d_acc,
                     accumulate, d_nan);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
