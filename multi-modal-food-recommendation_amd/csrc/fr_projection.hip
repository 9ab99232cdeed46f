// Modal projections of HealthRec over gathered feature rows (training forward + factored backward), gfx950.
//
// The reference projects the image / text features of the 2B batch items (models/cikm_model.py:240-241,
// image_trs / text_trs = Linear(2048 | 512 -> 64) over embImage / embText rows, both tables trainable):
//   forward   Y[i, :]   = X[ids[i], :] W^T + b                      (fr_gather_linear_fwd)
//   backward  dX[i, :]  = dY[i, :] W,  then rows of the table summed per id (index backward)
// Because W is shared, the table gradient of an id is (sum of its positions' dY rows) W: the
// backward segment-sums the 64-wide dY per id (fr_embedding_rowgrad on dY) and multiplies the compact
// rows once (fr_rows_matmul), so the [n x K] dX never exists and the data-parallel exchange moves
// 64-wide rows instead of K-wide ones.  dW = dY^T X[ids] is fr_linear_wgrad_gather (fr_linear.hip).
//
// Forward: 16 x 16 output tiles on v_mfma_f32_16x16x4_f32 (exact f32).  Each lane group h of a wave
// holds k = 4h..4h+3 of a 16-wide k chunk, so one float4 of the gathered row and one float4 of a W
// row feed four MFMAs.  KW = 16 waves split K: the problem is small (n = 2B = 1024 rows), so each
// wave's share of K is loaded in one or two rounds of four chunks (15.8 us against 16.4 us with 4
// waves over K at 1024 x (2048 + 512); one workgroup per 16 rows x all 64 columns, which reads each
// gathered row once, measured 27 us: half the CUs idle).
// (A K split over workgroups with an in-kernel ticket reduction measured slower: its device-scope
// fences cost more than the split saved.)
#include "fr_common.h"

#include <algorithm>

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int D = 64;            // output width (embedding size)
constexpr int WAVES = 4;
constexpr int KW = 16;           // waves over K per gathered-row tile (gather_linear_rows)

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// One workgroup per (16-row tile, 16-column tile): wave w takes chunks [C w / KW, C (w+1) / KW) of
// the C = K / 16 k chunks; the KW partial tiles are added in wave order through LDS and the bias
// added: no cross-workgroup traffic, deterministic.
__device__ __forceinline__ void gather_linear_rows(const int64_t* __restrict__ ids, int64_t n,
                                                   const float* __restrict__ X, int64_t ldx, int K,
                                                   const float* __restrict__ W, const float* __restrict__ b,
                                                   float* __restrict__ Y, int64_t ldy, int col0) {
  __shared__ float red[KW][256];
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = l & 15, h = l >> 4;
  const int64_t i = (int64_t)blockIdx.x * 16 + r;
  const float* __restrict__ xr = X + ids[i < n ? i : n - 1] * ldx;
  const float* __restrict__ wr = W + (int64_t)(col0 + r) * K;
  const int chunks = K / 16;
  const int q0 = chunks * w / KW, q1 = chunks * (w + 1) / KW;
  f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int c = q0; c < q1; c += 4) {
    float4 xa[4], wb[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = min(c + u, q1 - 1) * 16 + 4 * h;
      xa[u] = *reinterpret_cast<const float4*>(xr + k);
      wb[u] = *reinterpret_cast<const float4*>(wr + k);
    }
    __builtin_amdgcn_sched_barrier(0);  // the four chunks' loads in flight together
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (c + u < q1) {
        acc = mfma4(xa[u].x, wb[u].x, acc);
        acc = mfma4(xa[u].y, wb[u].y, acc);
        acc = mfma4(xa[u].z, wb[u].z, acc);
        acc = mfma4(xa[u].w, wb[u].w, acc);
      }
    }
  }
  // C layout: acc[q] = C[row 4h + q][col r]
#pragma unroll
  for (int q = 0; q < 4; ++q) red[w][(4 * h + q) * 16 + r] = acc[q];
  __syncthreads();
  if (threadIdx.x < 256) {
    const int e = threadIdx.x, rr = e / 16, cc = e % 16;
    float v = red[0][e];
#pragma unroll
    for (int k = 1; k < KW; ++k) v += red[k][e];
    const int64_t ii = (int64_t)blockIdx.x * 16 + rr;
    if (ii < n) Y[ii * ldy + col0 + cc] = v + (b ? b[col0 + cc] : 0.f);
  }
}

__global__ __launch_bounds__(64 * KW) void gather_linear_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                                const float* __restrict__ X, int64_t ldx, int K,
                                                                const float* __restrict__ W,
                                                                const float* __restrict__ b, float* __restrict__ Y,
                                                                int64_t ldy) {
  gather_linear_rows(ids, n, X, ldx, K, W, b, Y, ldy, blockIdx.y * 16);
}

// several tables at the same ids in one launch: blockIdx.z = table, its 64 output columns at 64 t
constexpr int kMaxProj = 4;
struct ProjTabs {
  const float* X[kMaxProj];
  int64_t ldx[kMaxProj];
  int K[kMaxProj];
  const float* W[kMaxProj];
  const float* b[kMaxProj];
};

__global__ __launch_bounds__(64 * KW) void gather_linear_multi_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                                      ProjTabs P, float* __restrict__ Y, int64_t ldy) {
  const int t = blockIdx.z;
  gather_linear_rows(ids, n, P.X[t], P.ldx[t], P.K[t], P.W[t], P.b[t], Y + (int64_t)t * D, ldy, blockIdx.y * 16);
}

// out[i, c] = sum_k S[i, k] W[k, c] for k < 64: 16 rows x 256 columns per workgroup, wave w the
// columns 64w..64w+63 as four 16x16 MFMA tiles over 16 k-steps.
__device__ __forceinline__ void rows_matmul_tile(const float* __restrict__ S, int64_t lds, int64_t n,
                                                 const float* __restrict__ W, int K, float* __restrict__ out,
                                                 int64_t ldo) {
  const int l = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int r = l & 15, h = l >> 4;
  const int64_t i0 = (int64_t)blockIdx.x * 16;
  const int64_t ia = min(i0 + r, n - 1);
  const int cbase = blockIdx.y * 256 + w * 64;
  // every operand load issued before the first MFMA (80 in flight per lane)
  float av[16], bv[16][4];
#pragma unroll
  for (int s = 0; s < 16; ++s) av[s] = S[ia * lds + 4 * s + h];  // A[r][k = 4s + h]
#pragma unroll
  for (int s = 0; s < 16; ++s) {
    const float* wr = W + (int64_t)(4 * s + h) * K;  // B[k = 4s + h][col]
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      const int c = min(cbase + 16 * t + r, K - 1);
      bv[s][t] = wr[c];
    }
  }
  __builtin_amdgcn_sched_barrier(0);  // all 80 loads issued before the first MFMA
  f32x4 acc[4];
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 16; ++s)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = mfma4(av[s], bv[s][t], acc[t]);
#pragma unroll
  for (int t = 0; t < 4; ++t) {
    const int c = cbase + 16 * t + r;
    if (c >= K) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t ii = i0 + 4 * h + q;
      if (ii < n) out[ii * ldo + c] = acc[t][q];
    }
  }
}

__global__ __launch_bounds__(64 * WAVES) void rows_matmul_kernel(const float* __restrict__ S, int64_t lds, int64_t n,
                                                                 const float* __restrict__ W, int K,
                                                                 float* __restrict__ out, int64_t ldo) {
  rows_matmul_tile(S, lds, n, W, K, out, ldo);
}

struct RowTabs {
  const float* W[kMaxProj];
  int K[kMaxProj];
  float* out[kMaxProj];
  int64_t ldo[kMaxProj];
};

// blockIdx.z = table t: S's 64-column block t times W_t; column blocks past K_t exit
__global__ __launch_bounds__(64 * WAVES) void rows_matmul_multi_kernel(const float* __restrict__ S, int64_t lds,
                                                                       int64_t n, RowTabs T) {
  const int t = blockIdx.z;
  if ((int)blockIdx.y * 256 >= T.K[t]) return;
  rows_matmul_tile(S + (int64_t)t * D, lds, n, T.W[t], T.K[t], T.out[t], T.ldo[t]);
}

}  // namespace

extern "C" int fr_gather_linear_fwd(const int64_t* d_ids, int64_t n, const float* d_x, int64_t ldx, int K,
                                    const float* d_w, const float* d_b, float* d_y, int64_t ldy, void* stream) {
  FR_REQUIRE(n > 0 && K > 0 && K % 16 == 0, "n > 0 and K a multiple of 16 required");
  FR_REQUIRE(d_ids && d_x && d_w && d_y, "null operand");
  FR_REQUIRE(ldx >= K && ldx % 4 == 0 && ldy >= D && fr::aligned16(d_x) && fr::aligned16(d_w),
             "X rows and W must be 16-byte aligned, ldx >= K, ldy >= 64");
  const int64_t tiles = fr::ceil_div(n, 16);
  FR_REQUIRE(tiles < (1ll << 31), "too many rows");
  hipLaunchKernelGGL(gather_linear_kernel, dim3((unsigned)tiles, D / 16), dim3(64 * KW), 0,
                     reinterpret_cast<hipStream_t>(stream), d_ids, n, d_x, ldx, K, d_w, d_b, d_y, ldy);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_rows_matmul(const float* d_s, int64_t lds, int64_t n, const float* d_w, int K, float* d_out,
                              int64_t ldo, void* stream) {
  FR_REQUIRE(n > 0 && K > 0, "empty problem");
  FR_REQUIRE(d_s && d_w && d_out && lds >= D && ldo >= K, "bad operands");
  hipLaunchKernelGGL(rows_matmul_kernel, dim3((unsigned)fr::ceil_div(n, 16), (unsigned)fr::ceil_div(K, 256)),
                     dim3(64 * WAVES), 0, reinterpret_cast<hipStream_t>(stream), d_s, lds, n, d_w, K, d_out, ldo);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_gather_linear_fwd_multi(const int64_t* d_ids, int64_t n, int n_tab, const float* const* d_x,
                                          const int64_t* ldx, const int* K, const float* const* d_w,
                                          const float* const* d_b, float* d_y, int64_t ldy, void* stream) {
  FR_REQUIRE(n > 0 && n_tab >= 1 && n_tab <= kMaxProj, "n > 0 and 1..4 tables required");
  FR_REQUIRE(d_ids && d_x && ldx && K && d_w && d_y && ldy >= D * n_tab, "null operand or ldy < 64 * tables");
  ProjTabs P{};
  for (int t = 0; t < n_tab; ++t) {
    FR_REQUIRE(K[t] > 0 && K[t] % 16 == 0 && ldx[t] >= K[t] && ldx[t] % 4 == 0 && d_x[t] && d_w[t] &&
                   fr::aligned16(d_x[t]) && fr::aligned16(d_w[t]),
               "table X rows / W must be 16-byte aligned, K a multiple of 16, ldx >= K");
    P.X[t] = d_x[t];
    P.ldx[t] = ldx[t];
    P.K[t] = K[t];
    P.W[t] = d_w[t];
    P.b[t] = d_b ? d_b[t] : nullptr;
  }
  const int64_t tiles = fr::ceil_div(n, 16);
  FR_REQUIRE(tiles < (1ll << 31), "too many rows");
  hipLaunchKernelGGL(gather_linear_multi_kernel, dim3((unsigned)tiles, D / 16, (unsigned)n_tab), dim3(64 * KW), 0,
                     reinterpret_cast<hipStream_t>(stream), d_ids, n, P, d_y, ldy);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_rows_matmul_multi(const float* d_s, int64_t lds, int64_t n, int n_tab, const float* const* d_w,
                                    const int* K, float* const* d_out, const int64_t* ldo, void* stream) {
  FR_REQUIRE(n > 0 && n_tab >= 1 && n_tab <= kMaxProj, "n > 0 and 1..4 tables required");
  FR_REQUIRE(d_s && d_w && K && d_out && ldo && lds >= D * n_tab, "null operand or lds < 64 * tables");
  RowTabs T{};
  int kmax = 0;
  for (int t = 0; t < n_tab; ++t) {
    FR_REQUIRE(K[t] > 0 && d_w[t] && d_out[t] && ldo[t] >= K[t], "bad table operands");
    T.W[t] = d_w[t];
    T.K[t] = K[t];
    T.out[t] = d_out[t];
    T.ldo[t] = ldo[t];
    kmax = std::max(kmax, K[t]);
  }
  hipLaunchKernelGGL(rows_matmul_multi_kernel,
                     dim3((unsigned)fr::ceil_div(n, 16), (unsigned)fr::ceil_div(kmax, 256), (unsigned)n_tab),
                     dim3(64 * WAVES), 0, reinterpret_cast<hipStream_t>(stream), d_s, lds, n, T);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
