// Weight/bias gradient of a Linear layer over many rows (split-K over the rows), gfx950.
//
//   dW[n, k] = sum_m dY[m, n] * X[m, k]        (dW = dY^T X, [N x K])
//   db[n]    = sum_m dY[m, n]
//
// The HealthRec ingredient Transformer (cikm_model.py:33-35: nn.TransformerEncoder, d=64, FF 4d)
// runs its four Linear layers over M = 2B x 20 = 20480 tokens: the weight gradients are
// [<=256 x 20480] x [20480 x <=256] -- tiny outputs, a huge reduction.  A library GEMM tiles the
// output and walks all 20480 rows in one workgroup per tile (~100 us each); here the rows are split
// into slabs, one workgroup per (slab, 64x64 output tile): the slab's 128 rows of both operands are
// loaded into LDS in one round (every load in flight at once: the kernel is latency-bound at these
// sizes), then each of the four waves runs a 16 x 64 strip of the tile on v_mfma_f32_16x16x4_f32
// (exact f32 products), db as one more MFMA chain against a ones operand.  Slab partials are summed in
// slab order by a second kernel: deterministic.
#include "fr_common.h"

#include <algorithm>

namespace {

constexpr int TN = 64, TK = 64;  // output tile
constexpr int kSlab = 128;       // rows per slab (split-K unit)
constexpr int LDT = TN + 16;     // LDS row stride (floats): the four row groups of an MFMA fragment read
                                 // land on disjoint banks

typedef float f32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 ld4_masked(const float* base, int64_t ld, int64_t m, int64_t M, int c, int C) {
  if (m < M && c < C) return *reinterpret_cast<const float4*>(base + m * ld + c);
  return make_float4(0.f, 0.f, 0.f, 0.f);
}

// grid: x = slab, y = n-tile * ktiles + k-tile.  part: [slabs][N][K], pdb: [slabs][N]
// X row m is X[ids[m]] when ids is given (gathered rows: the image / text projections)
__device__ __forceinline__ float4 ldx4(const float* X, int64_t ldx, const int64_t* ids, int64_t m, int64_t M, int c,
                                       int C) {
  if (m < M && c < C) return *reinterpret_cast<const float4*>(X + (ids ? ids[m] : m) * ldx + c);
  return make_float4(0.f, 0.f, 0.f, 0.f);
}

__device__ __forceinline__ void wgrad_slab(const float* __restrict__ dY, int64_t ldy, const float* __restrict__ X,
                                           int64_t ldx, const int64_t* __restrict__ ids, int64_t M, int N, int K,
                                           int ktiles, float* __restrict__ part, float* __restrict__ pdb,
                                           const int bx, const int by) {
  __shared__ __attribute__((aligned(16))) float As[kSlab][LDT];  // dY rows of the slab, columns n0..n0+63
  __shared__ __attribute__((aligned(16))) float Bs[kSlab][LDT];  // X rows of the slab, columns k0..k0+63
  const int t = threadIdx.x;
  const int n0 = (by / ktiles) * TN, k0 = (by % ktiles) * TK;
  const int64_t m0 = (int64_t)bx * kSlab;
  const int64_t m1 = min(M, m0 + kSlab);
  const bool want_db = pdb != nullptr && (by % ktiles) == 0;
  {  // 128 rows x 16 float4 per operand: 8 + 8 loads per thread, all issued before the LDS stores
    constexpr int J = kSlab * (TN / 4) / 256;
    const int r0 = t / 16, c4 = 4 * (t % 16);
    float4 ra[J], rb[J];
#pragma unroll
    for (int j = 0; j < J; ++j) {
      ra[j] = ld4_masked(dY, ldy, m0 + r0 + 16 * j, m1, n0 + c4, N);
      rb[j] = ldx4(X, ldx, ids, m0 + r0 + 16 * j, m1, k0 + c4, K);
    }
#pragma unroll
    for (int j = 0; j < J; ++j) {
      *reinterpret_cast<float4*>(&As[r0 + 16 * j][c4]) = ra[j];
      *reinterpret_cast<float4*>(&Bs[r0 + 16 * j][c4]) = rb[j];
    }
  }
  __syncthreads();
  // wave w: output rows n0 + 16w .. +15, all four 16-column k tiles.  MFMA operands: A[i][kk] =
  // dY[m][n0 + 16w + i], B[kk][j] = X[m][k0 + 16tt + j] at m = 4s + kk; lane (i16, h4) supplies row /
  // column i16 at kk = h4
  const int wave = t >> 6, lane = t & 63, i16 = lane & 15, h4 = lane >> 4;
  f32x4 acc[4], accb = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int tt = 0; tt < 4; ++tt) acc[tt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int st = 0; st < kSlab / 4; ++st) {
    const int m = 4 * st + h4;
    const float a = As[m][16 * wave + i16];
#pragma unroll
    for (int tt = 0; tt < 4; ++tt)
      acc[tt] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, Bs[m][16 * tt + i16], acc[tt], 0, 0, 0);
    if (want_db) accb = __builtin_amdgcn_mfma_f32_16x16x4f32(a, 1.f, accb, 0, 0, 0);
  }
  // C layout: acc[tt][q] = dW[n0 + 16 wave + 4 h4 + q][k0 + 16 tt + i16]
  const int64_t slab = bx;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n = n0 + 16 * wave + 4 * h4 + q;
    if (n >= N) continue;
#pragma unroll
    for (int tt = 0; tt < 4; ++tt) {
      const int k = k0 + 16 * tt + i16;
      if (k < K) part[(slab * N + n) * K + k] = acc[tt][q];
    }
    if (want_db && i16 == 0) pdb[slab * N + n] = accb[q];
  }
}

__global__ __launch_bounds__(256) void wgrad_slab_kernel(const float* __restrict__ dY, int64_t ldy,
                                                         const float* __restrict__ X, int64_t ldx,
                                                         const int64_t* __restrict__ ids, int64_t M,
                                                         int N, int K, int ktiles, float* __restrict__ part,
                                                         float* __restrict__ pdb) {
  wgrad_slab(dY, ldy, X, ldx, ids, M, N, K, ktiles, part, pdb, blockIdx.x, blockIdx.y);
}

// several gathered-input Linears over the same ids and rows (HealthRec's image / text projections):
// blockIdx.z = table, its own (N x K_t) tiles, partial slabs and reduction
constexpr int kMaxWg = 4;
struct WgTabs {
  const float* dy[kMaxWg];
  const float* X[kMaxWg];
  int64_t ldx[kMaxWg];
  int K[kMaxWg];
  int ktiles[kMaxWg];
  int tiles[kMaxWg];
  float* part[kMaxWg];
  float* pdb[kMaxWg];
  float* dW[kMaxWg];
  int64_t ldw[kMaxWg];
  float* db[kMaxWg];
  int64_t red_start[kMaxWg + 1];  // reduce: first block of table t
};

__global__ __launch_bounds__(256) void wgrad_slab_multi_kernel(int64_t ldy, const int64_t* __restrict__ ids,
                                                               int64_t M, int N, WgTabs T) {
  const int t = blockIdx.z;
  if ((int)blockIdx.y >= T.tiles[t]) return;
  wgrad_slab(T.dy[t], ldy, T.X[t], T.ldx[t], ids, M, N, T.K[t], T.ktiles[t], T.part[t], T.pdb[t], blockIdx.x,
             blockIdx.y);
}

// dW[n,k] = sum over slabs (in order, 4 interleaved slab lanes combined in fixed order).  A thread owns
// 4 consecutive outputs (one float4 per slab: 1 KiB per wave-load), a block 64 float4 columns; slab
// group g sums slabs g, g + 4, ... with 4 loads in flight, the 4 groups added in fixed order
__device__ __forceinline__ void wgrad_reduce(const float* __restrict__ part, int64_t slabs, int N, int K,
                                             float* __restrict__ dW, int64_t ldw, const float* __restrict__ pdb,
                                             float* __restrict__ db, int64_t bx) {
  __shared__ float4 red[4][64];
  const int e_local = threadIdx.x % 64, g = threadIdx.x / 64;
  const int64_t NK4 = (int64_t)N * K / 4;  // K % 4 == 0: a float4 never straddles two rows of dW
  const int64_t total4 = NK4 + (db ? N / 4 : 0);
  const int64_t e = bx * 64 + e_local;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (e < total4) {
    const float4* src = e < NK4 ? reinterpret_cast<const float4*>(part) + e
                                : reinterpret_cast<const float4*>(pdb) + (e - NK4);
    const int64_t stride = e < NK4 ? NK4 : N / 4;
    int64_t sl = g;
    for (; sl + 12 < slabs; sl += 16) {  // four loads in flight per lane
      const float4 v0 = src[sl * stride], v1 = src[(sl + 4) * stride];
      const float4 v2 = src[(sl + 8) * stride], v3 = src[(sl + 12) * stride];
      s = f4_add(s, v0); s = f4_add(s, v1); s = f4_add(s, v2); s = f4_add(s, v3);
    }
    for (; sl < slabs; sl += 4) s = f4_add(s, src[sl * stride]);
  }
  red[g][e_local] = s;
  __syncthreads();
  if (g == 0 && e < total4) {
    const float4 r = f4_add(f4_add(f4_add(red[0][e_local], red[1][e_local]), red[2][e_local]), red[3][e_local]);
    if (e < NK4) {
      const int64_t o = 4 * e;
      *reinterpret_cast<float4*>(dW + (o / K) * ldw + (o % K)) = r;
    } else {
      *reinterpret_cast<float4*>(db + 4 * (e - NK4)) = r;
    }
  }
}

__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int64_t slabs, int N,
                                                           int K, float* __restrict__ dW, int64_t ldw,
                                                           const float* __restrict__ pdb, float* __restrict__ db) {
  wgrad_reduce(part, slabs, N, K, dW, ldw, pdb, db, blockIdx.x);
}

__global__ __launch_bounds__(256) void wgrad_reduce_multi_kernel(int64_t slabs, int N, int n_tab, WgTabs T) {
  int t = 0;
  while (t + 1 < n_tab && (int64_t)blockIdx.x >= T.red_start[t + 1]) ++t;
  wgrad_reduce(T.part[t], slabs, N, T.K[t], T.dW[t], T.ldw[t], T.pdb[t], T.db[t], blockIdx.x - T.red_start[t]);
}

}  // namespace

extern "C" int64_t fr_linear_wgrad_workspace(int64_t M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0) return 0;
  const int64_t slabs = fr::ceil_div(M, kSlab);
  return fr::align_up(slabs * N * K * 4, 256) + fr::align_up(slabs * N * 4, 256);
}

static int wgrad_impl(const float* d_dy, int64_t ldy, const int64_t* d_ids, const float* d_x, int64_t ldx, int64_t M,
                      int N, int K, float* d_dw, int64_t ldw, float* d_db, void* d_workspace, int64_t workspace_bytes,
                      void* stream) {
  FR_REQUIRE(M > 0 && N > 0 && K > 0, "empty problem");
  FR_REQUIRE(N % 4 == 0 && K % 4 == 0, "N and K must be multiples of 4");
  FR_REQUIRE(d_dy && d_x && d_dw && ldy >= N && ldx >= K && ldw >= K && ldy % 4 == 0 && ldx % 4 == 0,
             "bad operands");
  FR_REQUIRE(fr::aligned16(d_dy) && fr::aligned16(d_x), "dY and X must be 16-byte aligned");
  FR_REQUIRE(fr::aligned16(d_dw) && ldw % 4 == 0 && (!d_db || fr::aligned16(d_db)),
             "dW (ld % 4 == 0) and db must be 16-byte aligned");
  FR_REQUIRE(d_workspace && fr::aligned16(d_workspace) && workspace_bytes >= fr_linear_wgrad_workspace(M, N, K),
             "workspace too small");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t slabs = fr::ceil_div(M, kSlab);
  FR_REQUIRE(slabs < (1u << 31), "too many rows");
  float* part = reinterpret_cast<float*>(d_workspace);
  float* pdb = reinterpret_cast<float*>(reinterpret_cast<char*>(d_workspace) + fr::align_up(slabs * N * K * 4, 256));
  const int ntiles = (int)fr::ceil_div(N, TN), ktiles = (int)fr::ceil_div(K, TK);
  hipLaunchKernelGGL(wgrad_slab_kernel, dim3((unsigned)slabs, (unsigned)(ntiles * ktiles)), dim3(256), 0, s, d_dy,
                     ldy, d_x, ldx, d_ids, M, N, K, ktiles, part, d_db ? pdb : nullptr);
  FR_LAUNCH_CHECK();
  const int64_t total4 = ((int64_t)N * K + (d_db ? N : 0)) / 4;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((unsigned)fr::ceil_div(total4, 64)), dim3(256), 0, s, part, slabs, N,
                     K, d_dw, ldw, pdb, d_db);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_linear_wgrad(const float* d_dy, int64_t ldy, const float* d_x, int64_t ldx, int64_t M, int N,
                               int K, float* d_dw, int64_t ldw, float* d_db, void* d_workspace,
                               int64_t workspace_bytes, void* stream) {
  return wgrad_impl(d_dy, ldy, nullptr, d_x, ldx, M, N, K, d_dw, ldw, d_db, d_workspace, workspace_bytes, stream);
}

extern "C" int fr_linear_wgrad_gather(const float* d_dy, int64_t ldy, const int64_t* d_ids, const float* d_x,
                                      int64_t ldx, int64_t M, int N, int K, float* d_dw, int64_t ldw, float* d_db,
                                      void* d_workspace, int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(d_ids, "null ids");
  return wgrad_impl(d_dy, ldy, d_ids, d_x, ldx, M, N, K, d_dw, ldw, d_db, d_workspace, workspace_bytes, stream);
}

extern "C" int64_t fr_linear_wgrad_gather_multi_workspace(int64_t M, int N, int n_tab, const int* K) {
  if (M <= 0 || N <= 0 || n_tab < 1 || n_tab > kMaxWg || !K) return 0;
  int64_t b = 0;
  for (int t = 0; t < n_tab; ++t) b += fr_linear_wgrad_workspace(M, N, K[t]);
  return b;
}

extern "C" int fr_linear_wgrad_gather_multi(const float* d_dy, int64_t ldy, const int64_t* d_ids, int64_t M, int N,
                                            int n_tab, const float* const* d_x, const int64_t* ldx, const int* K,
                                            float* const* d_dw, const int64_t* ldw, float* const* d_db,
                                            void* d_workspace, int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(M > 0 && N > 0 && N % 4 == 0 && n_tab >= 1 && n_tab <= kMaxWg, "bad sizes (1..4 tables)");
  FR_REQUIRE(d_dy && d_ids && d_x && ldx && K && d_dw && ldw && ldy >= N * n_tab && ldy % 4 == 0 &&
                 fr::aligned16(d_dy),
             "bad operands (dY holds the tables' N-wide blocks side by side)");
  FR_REQUIRE(d_workspace && fr::aligned16(d_workspace) &&
                 workspace_bytes >= fr_linear_wgrad_gather_multi_workspace(M, N, n_tab, K),
             "workspace too small");
  const int64_t slabs = fr::ceil_div(M, kSlab);
  FR_REQUIRE(slabs < (1u << 31), "too many rows");
  WgTabs T{};
  char* w = reinterpret_cast<char*>(d_workspace);
  int max_tiles = 0;
  int64_t blocks = 0;
  for (int t = 0; t < n_tab; ++t) {
    FR_REQUIRE(K[t] > 0 && K[t] % 4 == 0 && d_x[t] && d_dw[t] && ldx[t] >= K[t] && ldx[t] % 4 == 0 && ldw[t] >= K[t] &&
                   fr::aligned16(d_x[t]) && fr::aligned16(d_dw[t]) && ldw[t] % 4 == 0 &&
                   (!d_db || !d_db[t] || fr::aligned16(d_db[t])),
               "bad table operands (dW / db 16-byte aligned, ld % 4 == 0)");
    T.dy[t] = d_dy + (int64_t)t * N;
    T.X[t] = d_x[t];
    T.ldx[t] = ldx[t];
    T.K[t] = K[t];
    T.ktiles[t] = (int)fr::ceil_div(K[t], TK);
    T.tiles[t] = (int)fr::ceil_div(N, TN) * T.ktiles[t];
    T.part[t] = reinterpret_cast<float*>(w);
    T.pdb[t] = (d_db && d_db[t]) ? reinterpret_cast<float*>(w + fr::align_up(slabs * N * K[t] * 4, 256)) : nullptr;
    w += fr_linear_wgrad_workspace(M, N, K[t]);
    T.dW[t] = d_dw[t];
    T.ldw[t] = ldw[t];
    T.db[t] = d_db ? d_db[t] : nullptr;
    T.red_start[t] = blocks;
    blocks += fr::ceil_div(((int64_t)N * K[t] + (T.db[t] ? N : 0)) / 4, 64);
    max_tiles = std::max(max_tiles, T.tiles[t]);
  }
  T.red_start[n_tab] = blocks;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(wgrad_slab_multi_kernel, dim3((unsigned)slabs, (unsigned)max_tiles, (unsigned)n_tab), dim3(256),
                     0, s, ldy, d_ids, M, N, T);
  FR_LAUNCH_CHECK();
  hipLaunchKernelGGL(wgrad_reduce_multi_kernel, dim3((unsigned)blocks), dim3(256), 0, s, slabs, N, n_tab, T);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
