// Per-step loss bookkeeping of the training loop in one launch.
//
// Replaces, per step, the host-side reductions of Trainer._train_epoch (common/trainer.py:183-193):
//   loss_tuple = tuple(per_loss.item() for per_loss in losses); total_loss += loss_tuple;
//   if self._check_nan(loss): ... (loss = sum(losses))
// which the engine keeps on the device (no host sync per step): the float64 running sums of every
// loss component and a sticky NaN flag read by the fused Adam (skip the update) and at epoch end.
// torch would issue ~8 small kernels for it (casts, stack, add, sum, isnan, or).  The same launch
// advances the step's device counters (the fused encoder's dropout-hash step counters, the device
// feed's batch cursor): they are read earlier in the step and must move once per step.
#include "fr_common.h"

namespace {

constexpr int kMaxParts = 8;

constexpr int kMaxCounters = 8;

struct Parts {
  const float* p[kMaxParts];
  int n;
  int64_t* ctr[kMaxCounters];  // device step counters advanced by this step (dropout hash, batch cursor)
  int nc;
};

__global__ void step_book_kernel(Parts parts, double* __restrict__ acc, int accumulate, int32_t* __restrict__ nan_flag,
                                 float* __restrict__ loss_out) {
  if (threadIdx.x != 0) return;
  // every operand loaded before the first store (the counters are distinct: checked by the host), so
  // the launch is one memory round trip instead of a chain of read-modify-writes
  int64_t cv[kMaxCounters];
  float pv[kMaxParts];
  double av[kMaxParts];
#pragma unroll
  for (int i = 0; i < kMaxCounters; ++i) cv[i] = i < parts.nc ? parts.ctr[i][0] : 0;
#pragma unroll
  for (int i = 0; i < kMaxParts; ++i) {
    pv[i] = i < parts.n ? parts.p[i][0] : 0.f;
    av[i] = i < parts.n && accumulate ? acc[i] : 0.0;
  }
#pragma unroll
  for (int i = 0; i < kMaxCounters; ++i)
    if (i < parts.nc) parts.ctr[i][0] = cv[i] + 1;
  float s = 0.f;  // sum(losses) in fp32, left to right, as Python's sum over fp32 tensors
#pragma unroll
  for (int i = 0; i < kMaxParts; ++i) {
    if (i >= parts.n) break;
    const float v = pv[i];
    acc[i] = accumulate ? av[i] + (double)v : (double)v;
    s = i == 0 ? v : s + v;
  }
  if (s != s) nan_flag[0] |= 1;
  if (loss_out) loss_out[0] = s;  // the step's loss value (what the reference's train step returns)
}

}  // namespace

extern "C" int fr_step_book(const float* const* d_parts, int n, double* d_acc, int accumulate, int32_t* d_nan,
                            int64_t* const* d_counters, int n_counters, float* d_loss_out, void* stream) {
  FR_REQUIRE(n >= 1 && n <= kMaxParts, "1..8 loss parts");
  FR_REQUIRE(n_counters >= 0 && n_counters <= kMaxCounters, "0..8 counters");
  FR_REQUIRE(d_parts && d_acc && d_nan && (n_counters == 0 || d_counters), "null argument");
  Parts p{};
  for (int i = 0; i < n; ++i) {
    FR_REQUIRE(d_parts[i] != nullptr, "null loss part");
    p.p[i] = d_parts[i];
  }
  p.n = n;
  for (int i = 0; i < n_counters; ++i) {
    FR_REQUIRE(d_counters[i] != nullptr, "null counter");
    for (int j = 0; j < i; ++j) FR_REQUIRE(d_counters[j] != d_counters[i], "counters must be distinct");
    p.ctr[i] = d_counters[i];
  }
  p.nc = n_counters;
  hipLaunchKernelGGL(step_book_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), p, d_acc,
                     accumulate, d_nan, d_loss_out);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

// HealthRec's EmbLoss assembly (cikm_model.py:267-279 as the engine splits it): the fused BPR kernel
// returns the user / pos / neg norm sum `a`, the ingredient gather the two ingredient-block norms
// b[0..nb); reg = w * (a + (b_0 + ... ) / B) in the fp32 order of the torch expression it replaces
// (sum, divide, add, multiply).  Backward: da = g w, db_i = (g w) / B.  One launch each way instead
// of four and three.
namespace {

__global__ void reg_fwd_kernel(const float* __restrict__ a, const float* __restrict__ b, int nb, float B, float w,
                               float* __restrict__ out) {
  if (threadIdx.x != 0) return;
  float s = b[0];
  for (int i = 1; i < nb; ++i) s += b[i];
  out[0] = w * (a[0] + s / B);
}

__global__ void reg_bwd_kernel(const float* __restrict__ g, int nb, float B, float w, float* __restrict__ da,
                               float* __restrict__ db) {
  if (threadIdx.x != 0) return;
  const float gw = g[0] * w;
  da[0] = gw;
  const float gb = gw / B;
  for (int i = 0; i < nb; ++i) db[i] = gb;
}

}  // namespace

extern "C" int fr_reg_combine_fwd(const float* d_a, const float* d_b, int nb, float B, float w, float* d_out,
                                  void* stream) {
  FR_REQUIRE(d_a && d_b && d_out && nb >= 1 && B > 0.f, "bad argument");
  hipLaunchKernelGGL(reg_fwd_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), d_a, d_b, nb, B, w,
                     d_out);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_reg_combine_bwd(const float* d_g, int nb, float B, float w, float* d_da, float* d_db, void* stream) {
  FR_REQUIRE(d_g && d_da && d_db && nb >= 1 && B > 0.f, "bad argument");
  hipLaunchKernelGGL(reg_bwd_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), d_g, nb, B, w,
                     d_da, d_db);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

// ---- device wall-clock stamps (measurement): one single-lane kernel writes the constant-rate
// wall clock (s_memrealtime) with a vector store; stream order puts it after everything issued
// before it and before everything after, so two stamps bracket the kernels between them -- also
// inside a captured HIP graph, where timing events cannot be recorded (bench.py's roofline pass)
namespace {
__global__ void stamp_kernel(int64_t* out) {
  if (threadIdx.x == 0) out[threadIdx.x] = (int64_t)wall_clock64();
}
}  // namespace

extern "C" int fr_stamp(int64_t* d_slot, void* stream) {
  FR_REQUIRE(d_slot, "null stamp slot");
  hipLaunchKernelGGL(stamp_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), d_slot);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int64_t fr_stamp_hz() {
  int dev = 0, khz = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 0;
  if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0;
  return (int64_t)khz * 1000;
}
