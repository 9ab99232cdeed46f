// LayerNorm over the last dimension (d <= 256, d % 4 == 0, d/4 a power of two), forward and
// backward, gfx950.
//
// Replaces nn.LayerNorm on the HealthRec step: the post-norm LayerNorms of the ingredient
// Transformer (cikm_model.py:33-35; [20480, 64] at B=512) and the shared Q/K LayerNorm of
// target_attention_layer (cikm_model.py:326-327, 349-350; eps 1e-12 over d/h = 32 features, up to
// 40960 rows).  One group of d/4 lanes per row (float4 per lane), mean and variance by two passes
// over the registers (shuffle reductions), rstd = 1/sqrt(var + eps).  Backward:
//   x_hat = (x - mean) rstd,  g = dy * gamma,
//   dx = rstd (g - mean(g) - x_hat mean(g x_hat)),  dgamma = sum dy x_hat,  dbeta = sum dy
// with dgamma/dbeta as per-block partials (rows in a fixed grid-stride order) summed in block order
// by a second kernel: deterministic.
#include "fr_common.h"

#include <algorithm>

namespace {

constexpr int kLnBlocks = 256;  // backward partial blocks (one per CU)

template <int LPR>
__device__ __forceinline__ float gsum(float v) {
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, LPR);
  return v;
}

template <int LPR>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const float* __restrict__ X, int64_t ldx, int64_t rows,
                                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                                     float eps, float* __restrict__ Y, int64_t ldy,
                                                     float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int GPB = 256 / LPR;
  constexpr float inv_d = 1.f / (4 * LPR);
  const int lane = threadIdx.x % LPR;
  const float4 gm = gamma ? reinterpret_cast<const float4*>(gamma)[lane] : make_float4(1.f, 1.f, 1.f, 1.f);
  const float4 bt = beta ? reinterpret_cast<const float4*>(beta)[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t r = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; r < rows; r += (int64_t)gridDim.x * GPB) {
    const float4 x = reinterpret_cast<const float4*>(X + r * ldx)[lane];
    const float mean = gsum<LPR>((x.x + x.y) + (x.z + x.w)) * inv_d;
    const float4 c = make_float4(x.x - mean, x.y - mean, x.z - mean, x.w - mean);
    const float var = gsum<LPR>((c.x * c.x + c.y * c.y) + (c.z * c.z + c.w * c.w)) * inv_d;
    const float rstd = 1.f / __builtin_sqrtf(var + eps);
    float4 y;
    y.x = fmaf(c.x * rstd, gm.x, bt.x);
    y.y = fmaf(c.y * rstd, gm.y, bt.y);
    y.z = fmaf(c.z * rstd, gm.z, bt.z);
    y.w = fmaf(c.w * rstd, gm.w, bt.w);
    reinterpret_cast<float4*>(Y + r * ldy)[lane] = y;
    if (lane == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
  }
}

// part: [gridDim.x][2][d] (dgamma, dbeta partials)
template <int LPR>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const float* __restrict__ dY, int64_t lddy,
                                                     const float* __restrict__ X, int64_t ldx, int64_t rows,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in,
                                                     const float* __restrict__ gamma, float* __restrict__ dX,
                                                     int64_t lddx, float* __restrict__ part) {
  constexpr int GPB = 256 / LPR;
  constexpr int D = 4 * LPR;
  constexpr float inv_d = 1.f / D;
  __shared__ float4 red[GPB][LPR][2];
  const int lane = threadIdx.x % LPR, grp = threadIdx.x / LPR;
  const float4 gm = gamma ? reinterpret_cast<const float4*>(gamma)[lane] : make_float4(1.f, 1.f, 1.f, 1.f);
  float4 dg = make_float4(0.f, 0.f, 0.f, 0.f), db = dg;
  for (int64_t r = (int64_t)blockIdx.x * GPB + grp; r < rows; r += (int64_t)gridDim.x * GPB) {
    const float4 x = reinterpret_cast<const float4*>(X + r * ldx)[lane];
    const float4 dy = reinterpret_cast<const float4*>(dY + r * lddy)[lane];
    const float mean = mean_in[r], rstd = rstd_in[r];
    const float4 xh = make_float4((x.x - mean) * rstd, (x.y - mean) * rstd, (x.z - mean) * rstd, (x.w - mean) * rstd);
    const float4 g = make_float4(dy.x * gm.x, dy.y * gm.y, dy.z * gm.z, dy.w * gm.w);
    const float mg = gsum<LPR>((g.x + g.y) + (g.z + g.w)) * inv_d;
    const float mgx = gsum<LPR>((g.x * xh.x + g.y * xh.y) + (g.z * xh.z + g.w * xh.w)) * inv_d;
    float4 dx;
    dx.x = rstd * (g.x - mg - xh.x * mgx);
    dx.y = rstd * (g.y - mg - xh.y * mgx);
    dx.z = rstd * (g.z - mg - xh.z * mgx);
    dx.w = rstd * (g.w - mg - xh.w * mgx);
    reinterpret_cast<float4*>(dX + r * lddx)[lane] = dx;
    dg = f4_fma(1.f, make_float4(dy.x * xh.x, dy.y * xh.y, dy.z * xh.z, dy.w * xh.w), dg);
    db = f4_add(db, dy);
  }
  if (!part) return;
  red[grp][lane][0] = dg;
  red[grp][lane][1] = db;
  __syncthreads();
  // groups combined in group order by the first LPR*2 threads
  if (threadIdx.x < 2 * LPR) {
    const int which = threadIdx.x / LPR, l = threadIdx.x % LPR;
    float4 acc = red[0][l][which];
#pragma unroll
    for (int k = 1; k < GPB; ++k) acc = f4_add(acc, red[k][l][which]);
    reinterpret_cast<float4*>(part + ((int64_t)blockIdx.x * 2 + which) * D)[l] = acc;
  }
}

// out[e] for e in [0, 2d): 16 outputs per block, 16 block-lanes each summing every 16th partial
// block (8 loads in flight), lanes combined in fixed order
__global__ __launch_bounds__(256) void ln_param_reduce_kernel(const float* __restrict__ part, int nblocks, int d,
                                                              float* __restrict__ dgamma,
                                                              float* __restrict__ dbeta) {
  __shared__ float red[16][17];
  const int el = threadIdx.x % 16, g = threadIdx.x / 16;
  const int e = blockIdx.x * 16 + el;
  float s = 0.f;
  if (e < 2 * d) {
    const int which = e / d, c = e % d;
    const float* src = part + (int64_t)which * d + c;
    const int64_t stride = 2 * (int64_t)d;
    int b = g;
    for (; b + 112 < nblocks; b += 128) {
      float v[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = src[(int64_t)(b + 16 * k) * stride];
#pragma unroll
      for (int k = 0; k < 8; ++k) s += v[k];
    }
    for (; b < nblocks; b += 16) s += src[(int64_t)b * stride];
  }
  red[g][el] = s;
  __syncthreads();
  if (g == 0 && e < 2 * d) {
    float r = red[0][el];
#pragma unroll
    for (int k = 1; k < 16; ++k) r += red[k][el];
    if (e < d) { if (dgamma) dgamma[e] = r; }
    else if (dbeta) dbeta[e - d] = r;
  }
}

template <int LPR>
hipError_t launch_fwd(const float* X, int64_t ldx, int64_t rows, const float* gamma, const float* beta, float eps,
                      float* Y, int64_t ldy, float* mean, float* rstd, hipStream_t s) {
  constexpr int GPB = 256 / LPR;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(rows, GPB), (int64_t)fr::kNumCU * 16));
  hipLaunchKernelGGL(ln_fwd_kernel<LPR>, dim3((unsigned)blocks), dim3(256), 0, s, X, ldx, rows, gamma, beta, eps, Y,
                     ldy, mean, rstd);
  return hipGetLastError();
}

template <int LPR>
hipError_t launch_bwd(const float* dY, int64_t lddy, const float* X, int64_t ldx, int64_t rows, const float* mean,
                      const float* rstd, const float* gamma, float* dX, int64_t lddx, float* part, int nblocks,
                      hipStream_t s) {
  hipLaunchKernelGGL(ln_bwd_kernel<LPR>, dim3((unsigned)nblocks), dim3(256), 0, s, dY, lddy, X, ldx, rows, mean,
                     rstd, gamma, dX, lddx, part);
  return hipGetLastError();
}

bool ln_shape_ok(int d) { return d >= 4 && d <= 256 && d % 4 == 0 && ((d / 4) & (d / 4 - 1)) == 0; }

}  // namespace

extern "C" int64_t fr_layernorm_bwd_workspace(int d) { return (int64_t)kLnBlocks * 2 * d * 4 + 256; }

extern "C" int fr_layernorm_fwd(const float* d_x, int64_t ldx, int64_t rows, int d, const float* d_gamma,
                                const float* d_beta, float eps, float* d_y, int64_t ldy, float* d_mean,
                                float* d_rstd, void* stream) {
  FR_REQUIRE(ln_shape_ok(d), "d must be 4 * 2^k <= 256");
  FR_REQUIRE(rows >= 0 && ldx >= d && ldy >= d && ldx % 4 == 0 && ldy % 4 == 0, "bad shape");
  FR_REQUIRE(rows == 0 || (d_x && d_y && d_mean && d_rstd && fr::aligned16(d_x) && fr::aligned16(d_y)),
             "bad pointers");
  FR_REQUIRE((!d_gamma || fr::aligned16(d_gamma)) && (!d_beta || fr::aligned16(d_beta)), "gamma/beta alignment");
  if (rows == 0) return FR_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e;
  switch (d / 4) {
    case 1: e = launch_fwd<1>(d_x, ldx, rows, d_gamma, d_beta, eps, d_y, ldy, d_mean, d_rstd, s); break;
    case 2: e = launch_fwd<2>(d_x, ldx, rows, d_gamma, d_beta, eps, d_y, ldy, d_mean, d_rstd, s); break;
    case 4: e = launch_fwd<4>(d_x, ldx, rows, d_gamma, d_beta, eps, d_y, ldy, d_mean, d_rstd, s); break;
    case 8: e = launch_fwd<8>(d_x, ldx, rows, d_gamma, d_beta, eps, d_y, ldy, d_mean, d_rstd, s); break;
    case 16: e = launch_fwd<16>(d_x, ldx, rows, d_gamma, d_beta, eps, d_y, ldy, d_mean, d_rstd, s); break;
    case 32: e = launch_fwd<32>(d_x, ldx, rows, d_gamma, d_beta, eps, d_y, ldy, d_mean, d_rstd, s); break;
    default: e = launch_fwd<64>(d_x, ldx, rows, d_gamma, d_beta, eps, d_y, ldy, d_mean, d_rstd, s); break;
  }
  FR_HIP_CHECK(e);
  return FR_OK;
}

extern "C" int fr_layernorm_bwd(const float* d_dy, int64_t lddy, const float* d_x, int64_t ldx, int64_t rows, int d,
                                const float* d_mean, const float* d_rstd, const float* d_gamma, float* d_dx,
                                int64_t lddx, float* d_dgamma, float* d_dbeta, void* d_workspace,
                                int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(ln_shape_ok(d), "d must be 4 * 2^k <= 256");
  FR_REQUIRE(rows >= 0 && lddy >= d && ldx >= d && lddx >= d && lddy % 4 == 0 && ldx % 4 == 0 && lddx % 4 == 0,
             "bad shape");
  FR_REQUIRE(rows == 0 || (d_dy && d_x && d_dx && d_mean && d_rstd && fr::aligned16(d_dy) && fr::aligned16(d_x) &&
                           fr::aligned16(d_dx)),
             "bad pointers");
  FR_REQUIRE(!d_gamma || fr::aligned16(d_gamma), "gamma alignment");
  const bool params = d_dgamma || d_dbeta;
  FR_REQUIRE(!params || (d_workspace && fr::aligned16(d_workspace) && workspace_bytes >= fr_layernorm_bwd_workspace(d)),
             "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float* part = params ? reinterpret_cast<float*>(d_workspace) : nullptr;
  const int nblocks = kLnBlocks;
  hipError_t e;
  switch (d / 4) {
    case 1: e = launch_bwd<1>(d_dy, lddy, d_x, ldx, rows, d_mean, d_rstd, d_gamma, d_dx, lddx, part, nblocks, s); break;
    case 2: e = launch_bwd<2>(d_dy, lddy, d_x, ldx, rows, d_mean, d_rstd, d_gamma, d_dx, lddx, part, nblocks, s); break;
    case 4: e = launch_bwd<4>(d_dy, lddy, d_x, ldx, rows, d_mean, d_rstd, d_gamma, d_dx, lddx, part, nblocks, s); break;
    case 8: e = launch_bwd<8>(d_dy, lddy, d_x, ldx, rows, d_mean, d_rstd, d_gamma, d_dx, lddx, part, nblocks, s); break;
    case 16: e = launch_bwd<16>(d_dy, lddy, d_x, ldx, rows, d_mean, d_rstd, d_gamma, d_dx, lddx, part, nblocks, s); break;
    case 32: e = launch_bwd<32>(d_dy, lddy, d_x, ldx, rows, d_mean, d_rstd, d_gamma, d_dx, lddx, part, nblocks, s); break;
    default: e = launch_bwd<64>(d_dy, lddy, d_x, ldx, rows, d_mean, d_rstd, d_gamma, d_dx, lddx, part, nblocks, s); break;
  }
  FR_HIP_CHECK(e);
  if (params) {
    hipLaunchKernelGGL(ln_param_reduce_kernel, dim3((unsigned)fr::ceil_div(2 * d, 16)), dim3(256), 0, s, part, nblocks,
                       d, d_dgamma, d_dbeta);
    FR_LAUNCH_CHECK();
  }
  return FR_OK;
}
