// Per-item math of HealthRec's health / KD loss head (models/cikm_model.py:249-264, 304-308), shared
// by fr_health_kd.hip and the fused loss head (fr_modal_head.hip): one wave per item, lane = column.
// Elementwise formulas follow ATen's kernels (sigmoid 1/(1+exp(-x)); BCE with log/log1p clamped at
// -100; BCE backward (p-y)/max((1-p)p, 1e-12); cosine norms clamped at 1e-8).
#pragma once
#include "fr_common.h"

namespace {

constexpr int HEAD_D = 64;
constexpr int HMAX = 16;
constexpr int W1S = HEAD_D + 1;   // padded LDS row stride of W1 (conflict-free for lane = row and lane = column)
constexpr float kCosEps = 1e-8f;  // cosine_similarity eps
constexpr int NPART_BWD = HEAD_D * HEAD_D + HEAD_D + HMAX * HEAD_D + HMAX;  // dW1, db1, dW2 (HMAX rows), db2

__device__ __forceinline__ float wsum(float v) { return group_sum<64>(v); }

__device__ __forceinline__ float bcast(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// W1 (padded), b1, W2 (H rows, zero-padded to HMAX), b2 into LDS; T threads per block (compile-time
// trip counts: every thread's loads are in flight together).  Ends with a block barrier.
template <int T>
__device__ __forceinline__ void head_stage_weights(const float* __restrict__ w1, const float* __restrict__ b1,
                                                   const float* __restrict__ w2, const float* __restrict__ b2, int H,
                                                   float* sw1, float* sw2, float* sb) {
  constexpr int D = HEAD_D;
  float v1[D * D / T], v2[HMAX * D / T];
#pragma unroll
  for (int u = 0; u < D * D / T; ++u) v1[u] = w1[threadIdx.x + u * T];
#pragma unroll
  for (int u = 0; u < HMAX * D / T; ++u) {
    const int e = threadIdx.x + u * T;
    v2[u] = e < H * D ? w2[e] : 0.f;
  }
  const int e = threadIdx.x;
  const float vb = e < D ? b1[e] : (e < D + H ? b2[e - D] : 0.f);
#pragma unroll
  for (int u = 0; u < D * D / T; ++u) {
    const int f = threadIdx.x + u * T;
    sw1[(f >> 6) * W1S + (f & 63)] = v1[u];
  }
#pragma unroll
  for (int u = 0; u < HMAX * D / T; ++u) sw2[threadIdx.x + u * T] = v2[u];
  if (e < D + HMAX) sb[e] = vb;
  __syncthreads();
}

// z1 = W1 h + b1 for lane j (row j of W1), h broadcast by readlane; four interleaved partial sums
// (k mod 4) keep the dependent FMA chain 16 long instead of 64
__device__ __forceinline__ float head_layer1(const float* sw1, const float* sb, float h, int j) {
  float z[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < HEAD_D; ++k) z[k & 3] = fmaf(sw1[j * W1S + k], bcast(h, k), z[k & 3]);
  return ((z[0] + z[1]) + (z[2] + z[3])) + sb[j];
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + expf(-x)); }

__device__ __forceinline__ float bce(float p, float y) {
  const float lp = fmaxf(logf(p), -100.f), l1p = fmaxf(log1pf(-p), -100.f);
  return (y - 1.f) * l1p - y * lp;
}

}  // namespace
