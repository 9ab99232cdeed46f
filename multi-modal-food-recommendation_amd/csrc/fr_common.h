// Shared helpers for the FoodRec MI355X engine (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>
#include "fr_engine.h"
#include "fr_host.h"

namespace fr {

#define FR_HIP_CHECK(expr)                                                              \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess)                                                               \
      return ::fr::fail(FR_EHIP, std::string(__func__) + ": " #expr " -> " +          \
                                     hipGetErrorString(_e));                           \
  } while (0)

#define FR_LAUNCH_CHECK() FR_HIP_CHECK(hipGetLastError())

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

constexpr int kWave = 64;          // CDNA wavefront width
constexpr int kNumCU = 256;        // MI355X: 8 XCDs x 32 CUs

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }
inline int64_t align_up(int64_t a, int64_t b) { return ceil_div(a, b) * b; }

}  // namespace fr

// ---------------------------------------------------------------------------------------------
// device helpers
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float4 f4_fma(float s, float4 x, float4 acc) {
  acc.x = fmaf(s, x.x, acc.x);
  acc.y = fmaf(s, x.y, acc.y);
  acc.z = fmaf(s, x.z, acc.z);
  acc.w = fmaf(s, x.w, acc.w);
  return acc;
}

// Correctly rounded f32 sqrt: v_sqrt_f32 is accurate to 1 ulp only; pick among s-1ulp, s, s+1ulp
// by the sign of the fma residuals (the IEEE-exact expansion; matches x86 sqrtps bit for bit).
// Inputs below 2^-96 are scaled by 2^32 first (exact; v_sqrt_f32's 1-ulp bound holds for normal
// inputs) and the root by 2^-16 after (exact: the root is a normal number).  The bare instruction is
// used directly: the compiler's own correctly rounded sqrt expansion would repeat the selection.
__device__ __forceinline__ float sqrt_rn(float x) {
  const bool tiny = x < 0x1p-96f;
  const float xs = tiny ? x * 0x1p+32f : x;
  float s = __builtin_amdgcn_sqrtf(xs);
  const float s_dn = __int_as_float(__float_as_int(s) - 1);
  const float s_up = __int_as_float(__float_as_int(s) + 1);
  const float r_dn = fmaf(-s_dn, s, xs);
  const float r_up = fmaf(-s_up, s, xs);
  s = (r_dn <= 0.f) ? s_dn : s;
  s = (r_up > 0.f) ? s_up : s;
  return tiny ? s * 0x1p-16f : s;
}

__device__ __forceinline__ float4 f4_add(float4 a, float4 b) {
  return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

__device__ __forceinline__ float4 f4_scale(float s, float4 a) {
  return make_float4(s * a.x, s * a.y, s * a.z, s * a.w);
}

__device__ __forceinline__ float f4_dot(float4 a, float4 b) {
  return fmaf(a.w, b.w, fmaf(a.z, b.z, fmaf(a.y, b.y, a.x * b.x)));
}

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

__device__ __forceinline__ float lane_value(float v, int lane) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// sum over the `width` lanes of an aligned lane group (width power of two <= 64), the same value
// in every lane of the group.  Within a 16-lane DPP row the partners are swapped by VALU data-
// parallel moves (quad_perm xor 1, xor 2; row_half_mirror; row_mirror) instead of ds_bpermute
// round trips through the LDS crossbar; rows are then combined by gfx950's lane-swap moves:
// v_permlane16_swap on (v, v) gives every lane of rows 2k / 2k+1 the pair (row 2k, row 2k+1),
// v_permlane32_swap likewise the two 32-lane halves -- (row0 + row1) + (row2 + row3) in every lane,
// in a fixed order.  Every lane of the group must be active.
__device__ __forceinline__ float swap16_sum(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);  // (even row) + (odd row) in both rows
}
__device__ __forceinline__ float swap32_sum(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);  // (lanes 0-31) + (lanes 32-63) in both halves
}

template <int WIDTH>
__device__ __forceinline__ float group_sum(float v) {
  static_assert(WIDTH >= 1 && WIDTH <= 64 && (WIDTH & (WIDTH - 1)) == 0, "power-of-two group <= 64");
  if constexpr (WIDTH >= 2) v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  if constexpr (WIDTH >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (WIDTH >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror
  if constexpr (WIDTH >= 16) v += dpp_mov<0x140>(v); // row_mirror
  if constexpr (WIDTH >= 32) v = swap16_sum(v);
  if constexpr (WIDTH == 64) v = swap32_sum(v);
  return v;
}

template <int WIDTH>
__device__ __forceinline__ double group_sum_d(double v) {
#pragma unroll
  for (int off = WIDTH / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, WIDTH);
  return v;
}
