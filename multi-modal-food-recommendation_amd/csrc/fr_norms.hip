// Ingredient gather + the EmbLoss norms of its two halves (HealthRec), gfx950.
//
// HealthRec reads the ingredient table twice with the same ids (models/cikm_model.py:230 and
// :270-279): E = W[ids] for the encoder, and EmbLoss over nn.Embedding(ids) of the positive and the
// negative halves, i.e. the Frobenius norms ||E[:half]||, ||E[half:]|| (padding positions included in
// the forward, excluded from the gradient by padding_idx).
//   fr_gather_norms_fwd : E = W[ids] (16 lanes x float4 per 64-wide row) and per-block sums of squares
//                         of both halves; a one-wave finalize sums the block partials in a fixed
//                         order and takes the square roots (2 launches instead of gather + 2 norms).
//   fr_norms_bwd_coef   : G' = G + [ids != pad] * (gn[h] / nrm[h]) * E, h = the position's half (one
//                         launch instead of div / expand / ne / where / addcmul); G' then goes through
//                         the deterministic row scatter (fr_embedding_bwd).
#include "fr_common.h"

#include <algorithm>

namespace {

constexpr int D4 = 16;              // 64-wide rows as 16 float4
constexpr int ROWS_PER_BLOCK = 16;  // 256 threads
constexpr int MAX_BLOCKS = 1024;

__global__ __launch_bounds__(256) void gather_norms_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t half,
                                                           const float4* __restrict__ W4, int64_t ldw4,
                                                           float4* __restrict__ E4, float* __restrict__ part) {
  __shared__ float red[2][256];
  const int lane = threadIdx.x & 15, rg = threadIdx.x >> 4;
  float s0 = 0.f, s1 = 0.f;
  for (int64_t i = (int64_t)blockIdx.x * ROWS_PER_BLOCK + rg; i < n; i += (int64_t)gridDim.x * ROWS_PER_BLOCK) {
    const float4 v = W4[ids[i] * ldw4 + lane];
    E4[i * D4 + lane] = v;
    const float q = fmaf(v.x, v.x, fmaf(v.y, v.y, fmaf(v.z, v.z, v.w * v.w)));
    if (i < half) s0 += q; else s1 += q;
  }
  red[0][threadIdx.x] = s0;
  red[1][threadIdx.x] = s1;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {  // fixed-order tree
    if (threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = red[0][0];
    part[2 * blockIdx.x + 1] = red[1][0];
  }
}

// one block: the per-block partials in block order (strided per thread, then a fixed tree), sqrt
__global__ __launch_bounds__(256) void norms_final_kernel(const float* __restrict__ part, int nblk,
                                                          float* __restrict__ nrm) {
  __shared__ float red[2][256];
  float s0 = 0.f, s1 = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 256) {
    s0 += part[2 * b];
    s1 += part[2 * b + 1];
  }
  red[0][threadIdx.x] = s0;
  red[1][threadIdx.x] = s1;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (threadIdx.x < w) {
      red[0][threadIdx.x] += red[0][threadIdx.x + w];
      red[1][threadIdx.x] += red[1][threadIdx.x + w];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    nrm[0] = sqrtf(red[0][0]);
    nrm[1] = sqrtf(red[1][0]);
  }
}

__global__ __launch_bounds__(256) void norms_bwd_kernel(const int64_t* __restrict__ ids, int64_t n, int64_t half,
                                                        int64_t pad, const float4* __restrict__ G4,
                                                        const float4* __restrict__ E4, const float* __restrict__ gn,
                                                        int64_t gn_stride, const float* __restrict__ nrm,
                                                        float4* __restrict__ out4) {
  // vector_norm's backward: g * x / ||x||, zero where the norm is zero
  const float c0 = nrm[0] > 0.f ? gn[0] / nrm[0] : 0.f;
  const float c1 = nrm[1] > 0.f ? gn[gn_stride] / nrm[1] : 0.f;
  const int lane = threadIdx.x & 15;
  for (int64_t i = (int64_t)blockIdx.x * ROWS_PER_BLOCK + (threadIdx.x >> 4); i < n;
       i += (int64_t)gridDim.x * ROWS_PER_BLOCK) {
    const float c = ids[i] == pad ? 0.f : (i < half ? c0 : c1);
    const float4 g = G4[i * D4 + lane], e = E4[i * D4 + lane];
    out4[i * D4 + lane] = make_float4(fmaf(c, e.x, g.x), fmaf(c, e.y, g.y), fmaf(c, e.z, g.z), fmaf(c, e.w, g.w));
  }
}

int blocks_for(int64_t n) { return (int)std::min<int64_t>(fr::ceil_div(n, ROWS_PER_BLOCK), MAX_BLOCKS); }

}  // namespace

extern "C" int64_t fr_gather_norms_partials(int64_t n) { return n > 0 ? 2 * (int64_t)blocks_for(n) : 0; }

extern "C" int fr_gather_norms_fwd(const int64_t* d_ids, int64_t n, int64_t half, const float* d_w, int64_t ldw,
                                   float* d_e, float* d_partials, int64_t partial_floats, float* d_nrm,
                                   void* stream) {
  FR_REQUIRE(n > 0 && half >= 0 && half <= n, "n > 0 and 0 <= half <= n required");
  FR_REQUIRE(d_ids && d_w && d_e && d_partials, "null operand");
  FR_REQUIRE(ldw >= 64 && ldw % 4 == 0 && fr::aligned16(d_w) && fr::aligned16(d_e), "64-wide 16-B aligned rows");
  FR_REQUIRE(partial_floats >= fr_gather_norms_partials(n), "partial buffer too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = blocks_for(n);
  hipLaunchKernelGGL(gather_norms_kernel, dim3(nb), dim3(256), 0, s, d_ids, n, half,
                     reinterpret_cast<const float4*>(d_w), ldw / 4, reinterpret_cast<float4*>(d_e), d_partials);
  FR_LAUNCH_CHECK();
  if (d_nrm) {  // NULL: the finalize is left to fr_reg_combine_norms_fwd (the norms' only reader)
    hipLaunchKernelGGL(norms_final_kernel, dim3(1), dim3(256), 0, s, d_partials, nb, d_nrm);
    FR_LAUNCH_CHECK();
  }
  return FR_OK;
}

// the norms finalize (the same fixed-order sums as norms_final_kernel: bit-identical) with HealthRec's
// EmbLoss assembly in the same launch: reg = w * (a + (nrm0 + nrm1) / B) as fr_reg_combine_fwd
namespace {
__global__ __launch_bounds__(256) void reg_norms_kernel(const float* __restrict__ part, int nblk,
                                                        float* __restrict__ nrm, const float* __restrict__ a,
                                                        float B, float w, float* __restrict__ out) {
  __shared__ float red[2][256];
  float s0 = 0.f, s1 = 0.f;
  for (int b = threadIdx.x; b < nblk; b += 256) {
    s0 += part[2 * b];
    s1 += part[2 * b + 1];
  }
  red[0][threadIdx.x] = s0;
  red[1][threadIdx.x] = s1;
  __syncthreads();
  for (int q = 128; q > 0; q >>= 1) {
    if (threadIdx.x < q) {
      red[0][threadIdx.x] += red[0][threadIdx.x + q];
      red[1][threadIdx.x] += red[1][threadIdx.x + q];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const float n0 = sqrtf(red[0][0]), n1 = sqrtf(red[1][0]);
    nrm[0] = n0;
    nrm[1] = n1;
    if (out) out[0] = w * (a[0] + (n0 + n1) / B);
  }
}
}  // namespace

extern "C" int fr_reg_combine_norms_fwd(const float* d_a, const float* d_partials, int64_t n, float B, float w,
                                        float* d_nrm, float* d_out, void* stream) {
  FR_REQUIRE(n > 0 && d_partials && d_nrm && (!d_out || (d_a && B > 0.f)), "bad argument");
  hipLaunchKernelGGL(reg_norms_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), d_partials,
                     blocks_for(n), d_nrm, d_a, B, w, d_out);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_norms_bwd_coef(const int64_t* d_ids, int64_t n, int64_t half, int64_t pad, const float* d_g,
                                 const float* d_e, const float* d_gn, int64_t gn_stride, const float* d_nrm,
                                 float* d_out, void* stream) {
  FR_REQUIRE(n > 0 && half >= 0 && half <= n, "n > 0 and 0 <= half <= n required");
  FR_REQUIRE(d_ids && d_g && d_e && d_gn && d_nrm && d_out, "null operand");
  FR_REQUIRE(fr::aligned16(d_g) && fr::aligned16(d_e) && fr::aligned16(d_out), "16-B aligned rows");
  hipLaunchKernelGGL(norms_bwd_kernel, dim3(blocks_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     d_ids, n, half, pad, reinterpret_cast<const float4*>(d_g), reinterpret_cast<const float4*>(d_e),
                     d_gn, gn_stride, d_nrm, reinterpret_cast<float4*>(d_out));
  FR_LAUNCH_CHECK();
  return FR_OK;
}
