// bf16 storage helpers (BASELINE config 5: d=256 bf16 embedding tables, fp32 arithmetic).
//
// A bf16 value is the top half of an fp32; tables are row-major with 8 bf16 = 16 B per lane
// load (uint4).  Conversions round to nearest even, as torch's float -> bfloat16 cast does.
#pragma once
#include "fr_common.h"

__device__ __forceinline__ uint32_t fr_f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;  // NaN stays a (quiet) NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

__device__ __forceinline__ void fr_unpack8(uint4 x, float* o) {
  o[0] = __uint_as_float(x.x << 16);
  o[1] = __uint_as_float(x.x & 0xffff0000u);
  o[2] = __uint_as_float(x.y << 16);
  o[3] = __uint_as_float(x.y & 0xffff0000u);
  o[4] = __uint_as_float(x.z << 16);
  o[5] = __uint_as_float(x.z & 0xffff0000u);
  o[6] = __uint_as_float(x.w << 16);
  o[7] = __uint_as_float(x.w & 0xffff0000u);
}

__device__ __forceinline__ uint4 fr_pack8(const float* o) {
  uint4 r;
  r.x = fr_f2bf(o[0]) | (fr_f2bf(o[1]) << 16);
  r.y = fr_f2bf(o[2]) | (fr_f2bf(o[3]) << 16);
  r.z = fr_f2bf(o[4]) | (fr_f2bf(o[5]) << 16);
  r.w = fr_f2bf(o[6]) | (fr_f2bf(o[7]) << 16);
  return r;
}

__device__ __forceinline__ float fr_dot8(const float* a, const float* b) {
  float s = a[0] * b[0];
#pragma unroll
  for (int j = 1; j < 8; ++j) s = fmaf(a[j], b[j], s);
  return s;
}
