// Fused self-supervised losses of CLUSSL (PRICAI_ModelX):
//   * multi-view distance correlation  — correlation_distance, models/pricai_modelx.py:409-437,
//     called on three view pairs at :263.  All pairwise centred sums are computed from ONE set of
//     distance tiles per view (the reference builds each view's n x n distance matrix twice).
//   * InfoNCE / NT-Xent               — CL_loss, models/pricai_modelx.py:354-378.
//
// Both are n x n pair interactions over n = 2B = 1024 rows of d = 64: a few hundred MFLOP, so the
// kernels are LDS-tiled VALU (64x64 tiles, 4x4 outputs per thread) and never materialise the
// n x n matrices in HBM.  Reductions run in fp64 and in a fixed order (deterministic).
//
// dCor identity used (symmetric D, E; a_i = rowmean D, A = mean D):
//   sum_ij Dc_ij Ec_ij = sum D E - 2n sum_i a_i b_i + n^2 A B
// and its gradient: d(sum Dc Ec)/dD = Ec (the centring projector is idempotent and symmetric).
#include "fr_common.h"

#include <algorithm>

namespace {

constexpr int T = 64;     // tile rows
constexpr int PADT = 68;  // transposed tile row stride (floats): float4-aligned, spreads banks
constexpr int MAXV = 4;   // views
constexpr int MAXP = 10;  // unordered view pairs incl. (a,a): 4*5/2

struct Views {
  const float* x[MAXV];
  float* dx[MAXV];
};

struct PairTab {
  int n_pairs;           // requested dcor pairs
  int pa[16], pb[16];
};

__host__ __device__ inline int pair_index(int a, int b, int V) {
  if (a > b) { int t = a; a = b; b = t; }
  // index of (a,b), a<=b, in row-major upper triangle
  return a * V - a * (a - 1) / 2 + (b - a);
}

// rows [r0, r0+64) of X (ld = d) -> transposed LDS tile Xt[k*PADT + r] (0 beyond n)
__device__ __forceinline__ void load_tile_t(const float* __restrict__ X, int64_t n, int d, int64_t r0,
                                            float* Xt) {
  const int d4 = d >> 2;
  for (int idx = threadIdx.x; idx < T * d4; idx += blockDim.x) {
    const int r = idx / d4, k4 = idx - r * d4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < n) v = reinterpret_cast<const float4*>(X + (r0 + r) * d)[k4];
    Xt[(4 * k4 + 0) * PADT + r] = v.x;
    Xt[(4 * k4 + 1) * PADT + r] = v.y;
    Xt[(4 * k4 + 2) * PADT + r] = v.z;
    Xt[(4 * k4 + 3) * PADT + r] = v.w;
  }
}

// rows [r0, r0+64) of X -> row-major LDS tile Xr[r*(d+4) + k]
__device__ __forceinline__ void load_tile_r(const float* __restrict__ X, int64_t n, int d, int64_t r0,
                                            float* Xr) {
  const int d4 = d >> 2;
  const int ld = d + 4;
  for (int idx = threadIdx.x; idx < T * d4; idx += blockDim.x) {
    const int r = idx / d4, k4 = idx - r * d4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < n) v = reinterpret_cast<const float4*>(X + (r0 + r) * d)[k4];
    *reinterpret_cast<float4*>(Xr + r * ld + 4 * k4) = v;
  }
}

// load_tile_r for a compile-time d and block size: every thread's loads issued before its first LDS
// store (one global round trip per tile instead of one per strided step); NTILES tiles at once
template <int D, int NT, int NTILES = 1>
__device__ __forceinline__ void load_tiles_rc(const float* const (&X)[NTILES], int64_t n, const int64_t (&r0)[NTILES],
                                              float* const (&Xr)[NTILES]) {
  constexpr int D4 = D / 4, NST = T * D4 / NT, LD = D + 4;
  static_assert(T * D4 % NT == 0, "tile chunks must divide over the block");
  float4 v[NTILES][NST];
#pragma unroll
  for (int t = 0; t < NTILES; ++t)
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      const int idx = threadIdx.x + NT * u, r = idx / D4, k4 = idx - r * D4;
      v[t][u] = r0[t] + r < n ? reinterpret_cast<const float4*>(X[t] + (r0[t] + r) * D)[k4] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
  for (int t = 0; t < NTILES; ++t)
#pragma unroll
    for (int u = 0; u < NST; ++u) {
      const int idx = threadIdx.x + NT * u, r = idx / D4, k4 = idx - r * D4;
      *reinterpret_cast<float4*>(Xr[t] + r * LD + 4 * k4) = v[t][u];
    }
}

// 4x4 Gram block of thread (ti,tj): g[x][y] = <row 4ti+x of A, row 4tj+y of B>
__device__ __forceinline__ void gram4x4(const float* At, const float* Bt, int d, int ti, int tj,
                                        float g[4][4]) {
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) g[x][y] = 0.f;
  for (int k = 0; k < d; ++k) {
    const float4 a = *reinterpret_cast<const float4*>(At + k * PADT + 4 * ti);
    const float4 b = *reinterpret_cast<const float4*>(Bt + k * PADT + 4 * tj);
    const float av[4] = {a.x, a.y, a.z, a.w};
    const float bv[4] = {b.x, b.y, b.z, b.w};
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) g[x][y] = fmaf(av[x], bv[y], g[x][y]);
  }
}

// squared row norms of the 64 rows of a transposed tile (threads 0..63), fp32 like torch.sum(square)
__device__ __forceinline__ void row_sq(const float* Xt, int d, float* out) {
  if (threadIdx.x < T) {
    float s = 0.f;
    for (int k = 0; k < d; ++k) {
      const float v = Xt[k * PADT + threadIdx.x];
      s = fmaf(v, v, s);
    }
    out[threadIdx.x] = s;
  }
}

// block-wide fp64 sum (256 threads), result valid in thread 0
__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = group_sum_d<64>(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  if (threadIdx.x == 0)
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

// ============================ MFMA Gram tiles ==================================================
// The n x n Gram products of both losses on v_mfma_f32_16x16x4_f32 (exact fp32 products, fp32
// accumulation; the 16-wide k chunks permuted so a lane feeds four MFMAs from one float4 of each
// operand, as in fr_encoder.hip).  Tiles are row-major in LDS ([64][d + 4]); wave w owns rows
// [16w, 16w + 16) of the 64-row tile and all four 16-column tiles: acc[c][q] = C[16w + 4h + q][16c + i]
// for lane (i = lane & 15, h = lane >> 4).  fr_ssl_kernels selects them (default) or the VALU
// 4x4-per-thread tiles (A/B measurements).
typedef float f32x4 __attribute__((ext_vector_type(4)));
int g_ssl_mfma = 1;  // host-side kernel choice

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ float comp4(const float4& v, int m) {
  return m == 0 ? v.x : (m == 1 ? v.y : (m == 2 ? v.z : v.w));
}

// acc[c] = A[rows 16 rw..16 rw + 15] . B[rows 16 (c0 + c)..+15]^T over k < D, c < NC (A, B row-major,
// ld = D + 4)
template <int D, int NC = 4>
__device__ __forceinline__ void gram_mfma(const float* A, const float* B, f32x4 (&acc)[NC], int rw = -1, int c0 = 0) {
  constexpr int LD = D + 4;
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4;
  if (rw < 0) rw = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < NC; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < D / 16; ++kc) {
    const float4 a = *reinterpret_cast<const float4*>(A + (16 * rw + i) * LD + 16 * kc + 4 * h);
    float4 b[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) b[c] = *reinterpret_cast<const float4*>(B + (16 * (c0 + c) + i) * LD + 16 * kc + 4 * h);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < NC; ++c) acc[c] = mfma4(comp4(a, m), comp4(b[c], m), acc[c]);
  }
}

// acc[c] += W[rows 16 rw..16 rw + 15][0..64) . X[0..64)[cols 16 (c0 + c)..+15], c < NC (W row-major ld
// 65, X row-major ld D + 4): the backward's "sum_j w_ij x_j" over one 64-row tile of X
template <int D, int NC = D / 16>
__device__ __forceinline__ void wx_mfma(const float* W, const float* X, f32x4 (&acc)[NC], int rw = -1, int c0 = 0) {
  constexpr int LD = D + 4;
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4;
  if (rw < 0) rw = threadIdx.x >> 6;
#pragma unroll 4
  for (int jc = 0; jc < T / 16; ++jc) {
    float a[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) a[m] = W[(16 * rw + i) * 65 + 16 * jc + 4 * h + m];
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      float b[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) b[m] = X[(16 * jc + 4 * h + m) * LD + 16 * (c0 + c) + i];
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[c] = mfma4(a[m], b[m], acc[c]);
    }
  }
}

// squared row norms (fp32, k order) of the 64 rows of a row-major tile (threads 0..63)
template <int D>
__device__ __forceinline__ void row_sq_r(const float* X, float* out) {
  if (threadIdx.x < T) {
    float s = 0.f;
    for (int k = 0; k < D; ++k) {
      const float v = X[threadIdx.x * (D + 4) + k];
      s = fmaf(v, v, s);
    }
    out[threadIdx.x] = s;
  }
}

// ============================ distance correlation ============================================
// workspace layout (doubles unless noted):
//   S    [nblk][NP]          per-tile pair sums      (nblk = nt*nt)
//   row  [V][nt][n] floats   per-j-tile row sums of D_a
//   mean [V][n]              a_a[i] = rowmean(D_a)
//   Abar [V]                 mean(D_a)
//   coef [NP]                d(sum dcor)/d(centred pair sum), for unit upstream grad
//   out-scalars scratch
//   bwd partial P [JS][V][n][d] floats, rowm [JS][V][n] floats
constexpr int DCOR_JS = 16;  // j-splits of the backward tiles: 16 x 16 = 256 workgroups at n = 1024 (1 per CU)

constexpr int DCOR_BP = MAXV + 2 * MAXP;  // per means-block partials: sum mean, sum mean products, sum S

struct DcorWS {
  double* S; float* row; double* mean; double* Abar; double* coef;
  float* P; float* rowm; double* bpart;
  unsigned* ctr;  // means blocks done (zeroed by the tiles launch; the last block finalizes)
};

__host__ __device__ inline DcorWS dcor_ws(void* base, int64_t n, int V) {
  const int64_t nt = (n + T - 1) / T;
  const int NP = V * (V + 1) / 2;
  char* p = reinterpret_cast<char*>(base);
  DcorWS w;
  auto take = [&](int64_t bytes) { char* r = p; p += (bytes + 255) / 256 * 256; return r; };
  w.S = reinterpret_cast<double*>(take(nt * nt * NP * 8));
  w.row = reinterpret_cast<float*>(take((int64_t)V * nt * n * 4));
  w.mean = reinterpret_cast<double*>(take((int64_t)V * n * 8));
  w.Abar = reinterpret_cast<double*>(take(MAXV * 8));
  w.coef = reinterpret_cast<double*>(take(MAXP * 8));
  w.P = reinterpret_cast<float*>(take((int64_t)DCOR_JS * V * n * 128 * 4));
  w.rowm = reinterpret_cast<float*>(take((int64_t)DCOR_JS * V * n * 4));
  w.bpart = reinterpret_cast<double*>(take((n + 63) / 64 * DCOR_BP * 8));
  w.ctr = reinterpret_cast<unsigned*>(take(4));
  return w;
}

inline int64_t dcor_ws_bytes(int64_t n, int V) {
  const int64_t nt = (n + T - 1) / T;
  const int NP = V * (V + 1) / 2;
  auto r = [](int64_t b) { return (b + 255) / 256 * 256; };
  return r(nt * nt * NP * 8) + r((int64_t)V * nt * n * 4) + r((int64_t)V * n * 8) + r(MAXV * 8) +
         r(MAXP * 8) + r((int64_t)DCOR_JS * V * n * 128 * 4) + r((int64_t)DCOR_JS * V * n * 4) +
         r((n + 63) / 64 * DCOR_BP * 8) + r(4);
}

// distance tile of one view: D[x][y] for the thread's 4x4 block
__device__ __forceinline__ void dist4x4(const float* At, const float* Bt, const float* ra,
                                        const float* rb, int d, int ti, int tj, float D[4][4],
                                        float Q[4][4]) {
  float g[4][4];
  gram4x4(At, Bt, d, ti, tj, g);
#pragma unroll
  for (int x = 0; x < 4; ++x)
#pragma unroll
    for (int y = 0; y < 4; ++y) {
      // (r - 2 X X^T) + r^T, exactly the reference's evaluation order
      const float q = (ra[4 * ti + x] - 2.f * g[x][y]) + rb[4 * tj + y];
      Q[x][y] = q;
      D[x][y] = sqrtf(fmaxf(q, 0.f) + 1e-8f);
    }
}

// D is symmetric, so only the tiles it <= jt are computed: an off-diagonal tile gives the row sums
// of its it rows over column tile jt AND (as its column sums) the row sums of its jt rows over
// column tile it, and counts twice in the pair sums; blocks below the diagonal only zero their
// pair-sum slots.  (D_ij and D_ji differ in the last bits -- (r_i - 2g) + r_j vs (r_j - 2g) + r_i --
// so this is a rounding-level change from evaluating both.)
template <int V>
__global__ __launch_bounds__(256) void dcor_tiles_kernel(Views v, int64_t n, int d, DcorWS ws) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* At = smem;                 // [d][PADT]
  float* Bt = At + d * PADT;        // [d][PADT]
  float* ra = Bt + d * PADT;        // [64]
  float* rb = ra + T;               // [64]
  double* red = reinterpret_cast<double*>(rb + T);  // [4]
  __shared__ float colp[16][T];     // column partial sums (4 rows each) of an off-diagonal tile
  const int64_t nt = (n + T - 1) / T;
  const int it = blockIdx.x, jt = blockIdx.y;
  const int ti = threadIdx.x >> 4, tj = threadIdx.x & 15;
  const int NP = V * (V + 1) / 2;
  if (it == 0 && jt == 0 && threadIdx.x == 0) *ws.ctr = 0u;  // for the means launch's last block
  if (jt < it) {  // below the diagonal: the transposed tile carries it
    if (threadIdx.x < NP) ws.S[((int64_t)it * nt + jt) * NP + threadIdx.x] = 0.0;
    return;
  }
  const bool off = jt > it;
  float D[V][4][4];
#pragma unroll
  for (int a = 0; a < V; ++a) {
    __syncthreads();
    load_tile_t(v.x[a], n, d, (int64_t)it * T, At);
    load_tile_t(v.x[a], n, d, (int64_t)jt * T, Bt);
    __syncthreads();
    row_sq(At, d, ra);
    if (threadIdx.x >= T && threadIdx.x < 2 * T) {
      float s = 0.f;
      for (int k = 0; k < d; ++k) { const float t = Bt[k * PADT + threadIdx.x - T]; s = fmaf(t, t, s); }
      rb[threadIdx.x - T] = s;
    }
    __syncthreads();
    float Q[4][4];
    float Da[4][4];
    dist4x4(At, Bt, ra, rb, d, ti, tj, Da, Q);
#pragma unroll
    for (int x = 0; x < 4; ++x) {
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const bool ok = ((int64_t)it * T + 4 * ti + x < n) && ((int64_t)jt * T + 4 * tj + y < n);
        D[a][x][y] = ok ? Da[x][y] : 0.f;
      }
      // row sums over this j-tile
      float rs = D[a][x][0] + D[a][x][1] + D[a][x][2] + D[a][x][3];
      rs = group_sum<16>(rs);
      const int64_t gi = (int64_t)it * T + 4 * ti + x;
      if (tj == 0 && gi < n) ws.row[((int64_t)a * nt + jt) * n + gi] = rs;
    }
    if (off) {  // column sums = the jt rows' sums over column tile it (16 row groups, in order)
#pragma unroll
      for (int y = 0; y < 4; ++y) colp[ti][4 * tj + y] = ((D[a][0][y] + D[a][1][y]) + D[a][2][y]) + D[a][3][y];
      __syncthreads();
      if (threadIdx.x < T) {
        float cs = 0.f;
        for (int k = 0; k < 16; ++k) cs += colp[k][threadIdx.x];
        const int64_t gj = (int64_t)jt * T + threadIdx.x;
        if (gj < n) ws.row[((int64_t)a * nt + it) * n + gj] = cs;
      }
    }
  }
  // all unordered pair sums from the same tiles
  const int64_t blk = (int64_t)it * nt + jt;
#pragma unroll
  for (int a = 0; a < V; ++a)
#pragma unroll
    for (int b = a; b < V; ++b) {
      double s = 0.0;
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) s += (double)D[a][x][y] * (double)D[b][x][y];
      s = block_sum_d(s, red);
      if (threadIdx.x == 0) ws.S[blk * NP + pair_index(a, b, V)] = off ? 2.0 * s : s;
    }
}

// MFMA form of dcor_tiles_kernel: the distance tiles' Gram products on the matrix cores (wave w: rows
// [16w, 16w + 16), lane (i, h): columns 16c + i of rows 16w + 4h + q); row sums over the 16 lanes of a
// row, column sums of off-diagonal tiles through LDS in row-group order, pair sums as before
template <int V, int D>
__global__ __launch_bounds__(256) void dcor_tiles_mfma_kernel(Views v, int64_t n, DcorWS ws) {
  constexpr int LD = D + 4;
  // round 6: every view's i and j tiles staged by one load phase (was one load -> barrier -> compute
  // round trip per view), the column sums of all views behind one barrier, and all pair sums reduced
  // together (each in the same order as block_sum_d: wave sums, then waves 0..3)
  __shared__ __attribute__((aligned(16))) float At[V][T * LD];
  __shared__ __attribute__((aligned(16))) float Bt[V][T * LD];
  __shared__ float ra[V][T], rb[V][T];
  __shared__ float colp[V][16][T];
  constexpr int NP = V * (V + 1) / 2;
  __shared__ double red[4][NP];
  const int64_t nt = (n + T - 1) / T;
  const int it = blockIdx.x, jt = blockIdx.y;
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4, w = threadIdx.x >> 6;
  if (it == 0 && jt == 0 && threadIdx.x == 0) *ws.ctr = 0u;  // for the means launch's last block
  if (jt < it) {  // below the diagonal: the transposed tile carries it
    if (threadIdx.x < NP) ws.S[((int64_t)it * nt + jt) * NP + threadIdx.x] = 0.0;
    return;
  }
  const bool off = jt > it;
  {
    const float* src[2 * V];
    int64_t r0[2 * V];
    float* dst[2 * V];
#pragma unroll
    for (int a = 0; a < V; ++a) {
      src[2 * a] = v.x[a]; r0[2 * a] = (int64_t)it * T; dst[2 * a] = At[a];
      src[2 * a + 1] = v.x[a]; r0[2 * a + 1] = (int64_t)jt * T; dst[2 * a + 1] = Bt[a];
    }
    load_tiles_rc<D, 256, 2 * V>(src, n, r0, dst);
  }
  __syncthreads();
  // squared row norms (fp32, k order): threads 0..63 the i rows, 64..127 the j rows of every view
  if (threadIdx.x < 2 * T) {
    const int r = threadIdx.x & (T - 1);
#pragma unroll
    for (int a = 0; a < V; ++a) {
      const float* X = threadIdx.x < T ? At[a] : Bt[a];
      float sq = 0.f;
      for (int k = 0; k < D; ++k) { const float t = X[r * LD + k]; sq = fmaf(t, t, sq); }
      (threadIdx.x < T ? ra[a] : rb[a])[r] = sq;
    }
  }
  __syncthreads();
  float Dv[V][4][4];  // [view][column tile c][row q]
#pragma unroll
  for (int a = 0; a < V; ++a) {
    f32x4 g[4];
    gram_mfma<D>(At[a], Bt[a], g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 16 * w + 4 * h + q;
      const int64_t gi = (int64_t)it * T + r;
      float rs = 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int64_t gj = (int64_t)jt * T + 16 * c + i;
        // (r - 2 X X^T) + r^T, exactly the reference's evaluation order
        const float qv = (ra[a][r] - 2.f * g[c][q]) + rb[a][16 * c + i];
        Dv[a][c][q] = (gi < n && gj < n) ? sqrtf(fmaxf(qv, 0.f) + 1e-8f) : 0.f;
        rs += Dv[a][c][q];
      }
      rs = group_sum<16>(rs);
      if (i == 0 && gi < n) ws.row[((int64_t)a * nt + jt) * n + gi] = rs;
    }
    if (off) {  // column sums = the jt rows' sums over column tile it (16 row groups, in order)
#pragma unroll
      for (int c = 0; c < 4; ++c) colp[a][4 * w + h][16 * c + i] = ((Dv[a][c][0] + Dv[a][c][1]) + Dv[a][c][2]) + Dv[a][c][3];
    }
  }
  // all unordered pair sums from the same tiles: wave sums now, the waves in order below
  {
    int k = 0;
#pragma unroll
    for (int a = 0; a < V; ++a)
#pragma unroll
      for (int b = a; b < V; ++b, ++k) {
        double sum = 0.0;
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int q = 0; q < 4; ++q) sum += (double)Dv[a][c][q] * (double)Dv[b][c][q];
        sum = group_sum_d<64>(sum);
        if (lane == 0) red[w][pair_index(a, b, V)] = sum;
      }
  }
  __syncthreads();
  if (off && threadIdx.x < V * T) {
    const int a = threadIdx.x / T, col = threadIdx.x % T;
    float cs = 0.f;
    for (int k = 0; k < 16; ++k) cs += colp[a][k][col];
    const int64_t gj = (int64_t)jt * T + col;
    if (gj < n) ws.row[((int64_t)a * nt + it) * n + gj] = cs;
  }
  if (threadIdx.x < NP) {
    double sum = 0.0;
    for (int x = 0; x < 4; ++x) sum += red[x][threadIdx.x];
    ws.S[((int64_t)it * nt + jt) * NP + threadIdx.x] = off ? 2.0 * sum : sum;
  }
}

// the row means and the block partials of the centred sums: one wave per 64 rows (thread i: row i of
// every view, the j-tile row sums in fixed order), then per wave the sums of the means, of the pair
// products of the means and of a contiguous chunk of the per-tile pair sums -> ws.bpart[block]
template <int V>
__device__ __forceinline__ void dcor_means_block(int64_t n, DcorWS ws, int blk_id, int n_blk) {
  constexpr int NP = V * (V + 1) / 2;
  const int64_t nt = (n + T - 1) / T;
  const int lane = threadIdx.x & 63;
  const int64_t i = (int64_t)blk_id * 64 + lane;
  double mv[V];
  {  // every view's row sums: the loads of 8 j tiles of all views in flight together, added in j order
    double sv[V];
#pragma unroll
    for (int a = 0; a < V; ++a) sv[a] = 0.0;
    if (i < n) {
      int64_t jt = 0;
      for (; jt + 8 <= nt; jt += 8) {
        float x[V][8];
#pragma unroll
        for (int a = 0; a < V; ++a)
#pragma unroll
          for (int u = 0; u < 8; ++u) x[a][u] = ws.row[(int64_t)a * nt * n + i + (jt + u) * n];
#pragma unroll
        for (int a = 0; a < V; ++a)
#pragma unroll
          for (int u = 0; u < 8; ++u) sv[a] += (double)x[a][u];
      }
      for (; jt < nt; ++jt)
#pragma unroll
        for (int a = 0; a < V; ++a) sv[a] += (double)ws.row[(int64_t)a * nt * n + i + jt * n];
    }
#pragma unroll
    for (int a = 0; a < V; ++a) {
      mv[a] = i < n ? sv[a] / (double)n : 0.0;
      if (i < n) ws.mean[(int64_t)a * n + i] = mv[a];
    }
  }
  double* bp = ws.bpart + (int64_t)blk_id * DCOR_BP;
#pragma unroll
  for (int a = 0; a < V; ++a) {
    const double t = group_sum_d<64>(mv[a]);
    if (lane == 0) bp[a] = t;
  }
#pragma unroll
  for (int a = 0; a < V; ++a)
#pragma unroll
    for (int b = a; b < V; ++b) {
      const double t = group_sum_d<64>(mv[a] * mv[b]);
      if (lane == 0) bp[MAXV + pair_index(a, b, V)] = t;
    }
  const int64_t nblk = nt * nt, per = (nblk + n_blk - 1) / n_blk;
  const int64_t b0 = (int64_t)blk_id * per, b1 = b0 + per < nblk ? b0 + per : nblk;
  double lS[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) lS[k] = 0.0;
  for (int64_t blk = b0 + lane; blk < b1; blk += 64) {
    double x[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) x[k] = ws.S[blk * NP + k];
#pragma unroll
    for (int k = 0; k < NP; ++k) lS[k] += x[k];
  }
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const double t = group_sum_d<64>(lS[k]);
    if (lane == 0) bp[MAXV + MAXP + k] = t;
  }
}

// the block partials in block order -> Abar, centred sums, dcor values, backward coefficients
// (threads 0..DCOR_BP-1 of the workgroup; every thread reaches its barriers)
__device__ __forceinline__ void dcor_finalize_body(int V, int64_t n, int nb, const PairTab& pt, DcorWS ws,
                                                   float weight, float* out) {
  __shared__ double tot[DCOR_BP];
  __shared__ double Sc[MAXP];
  __shared__ double Ab[MAXV];
  const int NP = V * (V + 1) / 2;
  const int t = threadIdx.x;
  const bool used = t < DCOR_BP && (t < V || (t >= MAXV && t < MAXV + NP) || (t >= MAXV + MAXP && t < MAXV + MAXP + NP));
  if (used) {
    double s = 0.0;
    int b = 0;
    for (; b + 8 <= nb; b += 8) {  // 8 loads in flight, added in block order
      double x[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) x[u] = ws.bpart[(int64_t)(b + u) * DCOR_BP + t];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += x[u];
    }
    for (; b < nb; ++b) s += ws.bpart[(int64_t)b * DCOR_BP + t];
    tot[t] = s;
  }
  __syncthreads();
  if (t < V) {
    Ab[t] = tot[t] / (double)n;
    ws.Abar[t] = Ab[t];
  }
  __syncthreads();
  if (t < NP) {
    int a = 0, b = 0;
    for (int x = 0; x < V; ++x)
      for (int y = x; y < V; ++y)
        if (pair_index(x, y, V) == t) { a = x; b = y; }
    const double dn = (double)n;
    Sc[t] = tot[MAXV + MAXP + t] - 2.0 * dn * tot[MAXV + t] + dn * dn * Ab[a] * Ab[b];
  }
  __syncthreads();
  if (t == 0) {
    const double dn2 = (double)n * (double)n;
    double coef[MAXP];
    for (int k = 0; k < NP; ++k) coef[k] = 0.0;
    float total = 0.f;
    for (int k = 0; k < pt.n_pairs; ++k) {
      const int a = pt.pa[k], b = pt.pb[k];
      const int iab = pair_index(a, b, V), iaa = pair_index(a, a, V), ibb = pair_index(b, b, V);
      // fp32 scalar chain as the reference: dcov = sqrt(max(S/n^2, 0) + 1e-8)
      const float s12 = (float)(Sc[iab] / dn2), s11 = (float)(Sc[iaa] / dn2), s22 = (float)(Sc[ibb] / dn2);
      const float c12 = sqrtf(fmaxf(s12, 0.f) + 1e-8f);
      const float c11 = sqrtf(fmaxf(s11, 0.f) + 1e-8f);
      const float c22 = sqrtf(fmaxf(s22, 0.f) + 1e-8f);
      const float prod = c11 * c22;
      const float den = sqrtf(fmaxf(prod, 0.f) + 1e-10f);
      const float dc = c12 / den;
      out[k] = dc;
      total += dc;
      // gradients wrt the centred sums (torch.maximum passes half the grad at a tie)
      auto gate = [](float x) { return x > 0.f ? 1.0 : (x == 0.f ? 0.5 : 0.0); };
      const double d_c12 = 1.0 / den;
      const double d_den = -(double)c12 / ((double)den * den);
      const double d_prod = d_den * gate(prod) / (2.0 * den);
      const double d_c11 = d_prod * c22, d_c22 = d_prod * c11;
      coef[iab] += d_c12 * gate(s12) / (2.0 * c12) / dn2;
      coef[iaa] += d_c11 * gate(s11) / (2.0 * c11) / dn2;
      coef[ibb] += d_c22 * gate(s22) / (2.0 * c22) / dn2;
    }
    out[pt.n_pairs] = weight * total;  // (weight 1: the sum itself, exactly)
    for (int k = 0; k < NP; ++k) ws.coef[k] = coef[k];
  }
}

// The forward's second (and last) launch: one wave per 64 rows (the means stage); the last block
// to finish (a device-scope counter) runs the finalize over every block's partials in block order
// -- the same arithmetic as the round-5 means + finalize launches, so bit-identical.
template <int V>
__global__ __launch_bounds__(64) void dcor_means_finalize_kernel(int64_t n, int nb, PairTab pt, DcorWS ws,
                                                                 float weight, float* out) {
  __shared__ unsigned last;
  dcor_means_block<V>(n, ws, blockIdx.x, nb);
  __threadfence();  // this block's partials before its count
  if (threadIdx.x == 0) last = atomicAdd(ws.ctr, 1u) == (unsigned)nb - 1u;
  __syncthreads();
  if (!last) return;
  __threadfence();  // every block's partials after the count
  dcor_finalize_body(V, n, nb, pt, ws, weight, out);
}

// backward tiles: block (i-tile, j-split) accumulates P_a[i] = sum_j m_ij x_j and rowsum m
template <int V, int KPER>
__global__ __launch_bounds__(256) void dcor_bwd_tiles_kernel(Views v, int64_t n, DcorWS ws) {
  constexpr int d = 4 * KPER;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* Ait = smem;                    // [V][d][PADT] i-tiles (transposed)
  float* Bt = Ait + V * d * PADT;       // [d][PADT]
  float* Br = Bt + d * PADT;            // [64][d+4]
  float* Ms = Br + T * (d + 4);         // [64][65]
  float* ra = Ms + T * 65;              // [V][64]
  float* rb = ra + MAXV * T;            // [64]
  const int64_t nt = (n + T - 1) / T;
  const int it = blockIdx.x, js = blockIdx.y;
  const int ti = threadIdx.x >> 4, tj = threadIdx.x & 15;
  constexpr int NP = V * (V + 1) / 2;
  constexpr int kper = KPER;               // features per thread in the apply step
  const int ar = threadIdx.x & 63, aslot = threadIdx.x >> 6;
  double coef[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) coef[k] = ws.coef[k];
  for (int a = 0; a < V; ++a) load_tile_t(v.x[a], n, d, (int64_t)it * T, Ait + a * d * PADT);
  __syncthreads();
  for (int a = 0; a < V; ++a) row_sq(Ait + a * d * PADT, d, ra + a * T);
  __syncthreads();
  float acc[V][KPER];
  float rowm[V];
#pragma unroll
  for (int a = 0; a < V; ++a) {
    rowm[a] = 0.f;
#pragma unroll
    for (int k = 0; k < KPER; ++k) acc[a][k] = 0.f;
  }
  for (int64_t jt = js; jt < nt; jt += gridDim.y) {
    float D[V][4][4], Q[V][4][4];
#pragma unroll
    for (int a = 0; a < V; ++a) {
      __syncthreads();
      load_tile_t(v.x[a], n, d, jt * T, Bt);
      __syncthreads();
      if (threadIdx.x < T) {
        float s = 0.f;
        for (int k = 0; k < d; ++k) { const float t = Bt[k * PADT + threadIdx.x]; s = fmaf(t, t, s); }
        rb[threadIdx.x] = s;
      }
      __syncthreads();
      dist4x4(Ait + a * d * PADT, Bt, ra + a * T, rb, d, ti, tj, D[a], Q[a]);
    }
    // centred tiles (fp32 from fp64 means) for every view
    float Dc[V][4][4];
#pragma unroll
    for (int a = 0; a < V; ++a)
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          const int64_t gi = (int64_t)it * T + 4 * ti + x, gj = jt * T + 4 * tj + y;
          const bool ok = gi < n && gj < n;
          Dc[a][x][y] = ok ? (float)((double)D[a][x][y] - ws.mean[(int64_t)a * n + gi] -
                                     ws.mean[(int64_t)a * n + gj] + ws.Abar[a])
                           : 0.f;
        }
#pragma unroll
    for (int a = 0; a < V; ++a) {
      if (!v.dx[a]) continue;
      // m_ij = K_a(i,j) * gate(q) / (2 D), K_a = sum_b c_ab Dc_b (b != a) + 2 c_aa Dc_a
      __syncthreads();
#pragma unroll
      for (int x = 0; x < 4; ++x)
#pragma unroll
        for (int y = 0; y < 4; ++y) {
          double K = 2.0 * coef[pair_index(a, a, V)] * Dc[a][x][y];
#pragma unroll
          for (int b = 0; b < V; ++b)
            if (b != a) K += coef[pair_index(a, b, V)] * Dc[b][x][y];
          const float q = Q[a][x][y];
          const float gt = q > 0.f ? 1.f : (q == 0.f ? 0.5f : 0.f);
          const int64_t gi = (int64_t)it * T + 4 * ti + x, gj = jt * T + 4 * tj + y;
          const bool ok = gi < n && gj < n && gi != gj;
          Ms[(4 * ti + x) * 65 + 4 * tj + y] = ok ? (float)(K * gt / (2.0 * D[a][x][y])) : 0.f;
        }
      load_tile_r(v.x[a], n, d, jt * T, Br);
      __syncthreads();
      // apply: row ar, features [aslot*kper, +kper)
      float rm = 0.f;
      for (int j = 0; j < T; ++j) {
        const float w = Ms[ar * 65 + j];
        rm += w;
        const float* xr = Br + j * (d + 4) + aslot * kper;
#pragma unroll
        for (int k = 0; k < kper; ++k) acc[a][k] = fmaf(w, xr[k], acc[a][k]);
      }
      rowm[a] += rm;
    }
  }
  const int64_t gi = (int64_t)it * T + ar;
  if (gi < n) {
#pragma unroll
    for (int a = 0; a < V; ++a) {
      if (!v.dx[a]) continue;
      float* P = ws.P + (((int64_t)js * V + a) * n + gi) * d + aslot * kper;
#pragma unroll
      for (int k = 0; k < kper; ++k) P[k] = acc[a][k];
      if (aslot == 0) ws.rowm[((int64_t)js * V + a) * n + gi] = rowm[a];
    }
  }
}

// MFMA form of dcor_bwd_tiles_kernel: per j-tile the V distance tiles on the matrix cores, the
// centred tiles and m_ij = K_a(i,j) gate(q) / (2 D) on the VALU, m staged in LDS, then
// P_a += m X_a[j-tile] on the matrix cores (the view's j-tile reloaded row-major) and rowm_a from the
// fragments.  8 waves: wave w owns row block rw = w & 3 and the column half ch = w >> 2 (two 16-column
// tiles) of every 64 x 64 tile, so each lane holds 8 elements per view (two waves per SIMD).
// LDS: V i-tiles + one j-tile + m (D = 64, V <= 4).
constexpr int DB_NT = 512;
template <int V, int D>
__global__ __launch_bounds__(DB_NT) void dcor_bwd_mfma_kernel(Views v, int64_t n, DcorWS ws) {
  constexpr int LD = D + 4;
  constexpr int NC = D / 32;  // output column tiles per wave
  __shared__ __attribute__((aligned(16))) float Ai[V][T * LD];
  __shared__ __attribute__((aligned(16))) float Bt[T * LD];
  __shared__ float Ms[T * 65];
  __shared__ float ra[V][T], rb[T];
  __shared__ double mi[V][T], mj[V][T];
  __shared__ float rowp[2][V][T];
  const int64_t nt = (n + T - 1) / T;
  const int it = blockIdx.x, js = blockIdx.y;
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4, w = threadIdx.x >> 6;
  const int rw = w & 3, ch = w >> 2;
  constexpr int NP = V * (V + 1) / 2;
  double coef[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) coef[k] = ws.coef[k];
  for (int a = 0; a < V; ++a) load_tiles_rc<D, DB_NT>({v.x[a]}, n, {(int64_t)it * T}, {Ai[a]});
  if (threadIdx.x < T) {
    const int64_t gi = (int64_t)it * T + threadIdx.x;
    for (int a = 0; a < V; ++a) mi[a][threadIdx.x] = gi < n ? ws.mean[(int64_t)a * n + gi] : 0.0;
  }
  __syncthreads();
  for (int a = 0; a < V; ++a) row_sq_r<D>(Ai[a], ra[a]);
  f32x4 acc[V][NC];
  float rowm[V][4];
#pragma unroll
  for (int a = 0; a < V; ++a) {
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) rowm[a][q] = 0.f;
  }
  for (int64_t jt = js; jt < nt; jt += gridDim.y) {
    float Dd[V][2][4], Dc[V][2][4];  // [view][column tile 2 ch + c][row q]
    if (threadIdx.x < T) {
      const int64_t gj = jt * T + threadIdx.x;
      for (int a = 0; a < V; ++a) mj[a][threadIdx.x] = gj < n ? ws.mean[(int64_t)a * n + gj] : 0.0;
    }
#pragma unroll
    for (int a = 0; a < V; ++a) {
      __syncthreads();
      load_tiles_rc<D, DB_NT>({v.x[a]}, n, {jt * T}, {Bt});
      __syncthreads();
      if (threadIdx.x < T) {
        float sq = 0.f;
        for (int k = 0; k < D; ++k) { const float t = Bt[threadIdx.x * LD + k]; sq = fmaf(t, t, sq); }
        rb[threadIdx.x] = sq;
      }
      __syncthreads();
      f32x4 g[2];
      gram_mfma<D, 2>(Ai[a], Bt, g, rw, 2 * ch);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * rw + 4 * h + q;
        const int64_t gi = (int64_t)it * T + r;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int col = 16 * (2 * ch + c) + i;
          const int64_t gj = jt * T + col;
          const float qv = (ra[a][r] - 2.f * g[c][q]) + rb[col];
          const float dd = sqrtf(fmaxf(qv, 0.f) + 1e-8f);
          const float gt = qv > 0.f ? 1.f : (qv == 0.f ? 0.5f : 0.f);
          const bool ok = gi < n && gj < n;
          Dc[a][c][q] = ok ? (float)((double)dd - mi[a][r] - mj[a][col] + ws.Abar[a]) : 0.f;
          Dd[a][c][q] = (ok && gi != gj) ? gt / (2.f * dd) : 0.f;  // gate(q) / (2 D), 0 off the tile / diagonal
        }
      }
    }
#pragma unroll
    for (int a = 0; a < V; ++a) {
      if (!v.dx[a]) continue;
      __syncthreads();  // every wave is done with Ms and Bt
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * rw + 4 * h + q;
        float rs = 0.f;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          double K = 2.0 * coef[pair_index(a, a, V)] * Dc[a][c][q];
#pragma unroll
          for (int b = 0; b < V; ++b)
            if (b != a) K += coef[pair_index(a, b, V)] * Dc[b][c][q];
          const float mv = (float)(K * (double)Dd[a][c][q]);
          Ms[r * 65 + 16 * (2 * ch + c) + i] = mv;
          rs += mv;
        }
        rowm[a][q] += group_sum<16>(rs);
      }
      load_tiles_rc<D, DB_NT>({v.x[a]}, n, {jt * T}, {Bt});
      __syncthreads();
      wx_mfma<D, NC>(Ms, Bt, acc[a], rw, NC * ch);
    }
  }
  // row sums: the two column halves in order (ch 0, then 1)
#pragma unroll
  for (int a = 0; a < V; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (i == 0) rowp[ch][a][16 * rw + 4 * h + q] = rowm[a][q];
  __syncthreads();
#pragma unroll
  for (int a = 0; a < V; ++a) {
    if (!v.dx[a]) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 16 * rw + 4 * h + q;
      const int64_t gi = (int64_t)it * T + r;
      if (gi < n) {
        float* P = ws.P + (((int64_t)js * V + a) * n + gi) * D;
#pragma unroll
        for (int c = 0; c < NC; ++c) P[16 * (NC * ch + c) + i] = acc[a][c][q];
        if (i == 0 && ch == 0) ws.rowm[((int64_t)js * V + a) * n + gi] = rowp[0][a][r] + rowp[1][a][r];
      }
    }
  }
}

// Round-6 form of dcor_bwd_mfma_kernel for V <= 3 (the LDS holds every view's i AND j tiles): the
// i tiles, the first j tiles and the means issued in one load phase; per j tile ONE load phase for
// all views (the round-5 kernel loaded each view's j tile twice, each behind its own barrier pair).
// Same arithmetic in the same order.
template <int V, int D>
__global__ __launch_bounds__(DB_NT) void dcor_bwd_mfma_allb_kernel(Views v, int64_t n, DcorWS ws) {
  static_assert(V <= 3, "LDS holds 2V tiles for V <= 3");
  constexpr int LD = D + 4;
  constexpr int NC = D / 32;  // output column tiles per wave
  __shared__ __attribute__((aligned(16))) float Ai[V][T * LD];
  __shared__ __attribute__((aligned(16))) float Bt[V][T * LD];
  __shared__ float Ms[T * 65];
  __shared__ float ra[V][T], rb[V][T];
  __shared__ double mi[V][T], mj[V][T];
  __shared__ float rowp[2][V][T];
  const int64_t nt = (n + T - 1) / T;
  const int it = blockIdx.x, js = blockIdx.y;
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4, w = threadIdx.x >> 6;
  const int rw = w & 3, ch = w >> 2;
  constexpr int NP = V * (V + 1) / 2;
  double coef[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) coef[k] = ws.coef[k];
  f32x4 acc[V][NC];
  float rowm[V][4];
#pragma unroll
  for (int a = 0; a < V; ++a) {
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[a][c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int q = 0; q < 4; ++q) rowm[a][q] = 0.f;
  }
  bool first = true;
  for (int64_t jt = js; jt < nt; jt += gridDim.y, first = false) {
    if (!first) __syncthreads();  // every wave is done with the previous j tiles
    if (threadIdx.x < T) {
      const int64_t gi = (int64_t)it * T + threadIdx.x, gj = jt * T + threadIdx.x;
      for (int a = 0; a < V; ++a) {
        if (first) mi[a][threadIdx.x] = gi < n ? ws.mean[(int64_t)a * n + gi] : 0.0;
        mj[a][threadIdx.x] = gj < n ? ws.mean[(int64_t)a * n + gj] : 0.0;
      }
    }
    if (first) {
      const float* src[2 * V];
      int64_t r0[2 * V];
      float* dst[2 * V];
#pragma unroll
      for (int a = 0; a < V; ++a) {
        src[2 * a] = v.x[a]; r0[2 * a] = (int64_t)it * T; dst[2 * a] = Ai[a];
        src[2 * a + 1] = v.x[a]; r0[2 * a + 1] = jt * T; dst[2 * a + 1] = Bt[a];
      }
      load_tiles_rc<D, DB_NT, 2 * V>(src, n, r0, dst);
    } else {
      const float* src[V];
      int64_t r0[V];
      float* dst[V];
#pragma unroll
      for (int a = 0; a < V; ++a) { src[a] = v.x[a]; r0[a] = jt * T; dst[a] = Bt[a]; }
      load_tiles_rc<D, DB_NT, V>(src, n, r0, dst);
    }
    __syncthreads();
    // squared row norms (fp32, k order): wave pairs 2a / 2a + 1 the i / j rows of view a
    if (threadIdx.x < 2 * V * T) {
      const int a = threadIdx.x / (2 * T), r = threadIdx.x & (T - 1);
      const bool isj = (threadIdx.x / T) & 1;
      if (first || isj) {
        const float* X = isj ? Bt[a] : Ai[a];
        float sq = 0.f;
        for (int k = 0; k < D; ++k) { const float t = X[r * LD + k]; sq = fmaf(t, t, sq); }
        (isj ? rb[a] : ra[a])[r] = sq;
      }
    }
    __syncthreads();
    float Dd[V][2][4], Dc[V][2][4];  // [view][column tile 2 ch + c][row q]
#pragma unroll
    for (int a = 0; a < V; ++a) {
      f32x4 g[2];
      gram_mfma<D, 2>(Ai[a], Bt[a], g, rw, 2 * ch);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * rw + 4 * h + q;
        const int64_t gi = (int64_t)it * T + r;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const int col = 16 * (2 * ch + c) + i;
          const int64_t gj = jt * T + col;
          const float qv = (ra[a][r] - 2.f * g[c][q]) + rb[a][col];
          const float dd = sqrtf(fmaxf(qv, 0.f) + 1e-8f);
          const float gt = qv > 0.f ? 1.f : (qv == 0.f ? 0.5f : 0.f);
          const bool ok = gi < n && gj < n;
          Dc[a][c][q] = ok ? (float)((double)dd - mi[a][r] - mj[a][col] + ws.Abar[a]) : 0.f;
          Dd[a][c][q] = (ok && gi != gj) ? gt / (2.f * dd) : 0.f;  // gate(q) / (2 D), 0 off the tile / diagonal
        }
      }
    }
    bool ms_used = false;
#pragma unroll
    for (int a = 0; a < V; ++a) {
      if (!v.dx[a]) continue;
      if (ms_used) __syncthreads();  // every wave is done with Ms
      ms_used = true;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = 16 * rw + 4 * h + q;
        float rs = 0.f;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          double K = 2.0 * coef[pair_index(a, a, V)] * Dc[a][c][q];
#pragma unroll
          for (int b = 0; b < V; ++b)
            if (b != a) K += coef[pair_index(a, b, V)] * Dc[b][c][q];
          const float mv = (float)(K * (double)Dd[a][c][q]);
          Ms[r * 65 + 16 * (2 * ch + c) + i] = mv;
          rs += mv;
        }
        rowm[a][q] += group_sum<16>(rs);
      }
      __syncthreads();
      wx_mfma<D, NC>(Ms, Bt[a], acc[a], rw, NC * ch);
    }
  }
  // row sums: the two column halves in order (ch 0, then 1)
#pragma unroll
  for (int a = 0; a < V; ++a)
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (i == 0) rowp[ch][a][16 * rw + 4 * h + q] = rowm[a][q];
  __syncthreads();
#pragma unroll
  for (int a = 0; a < V; ++a) {
    if (!v.dx[a]) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 16 * rw + 4 * h + q;
      const int64_t gi = (int64_t)it * T + r;
      if (gi < n) {
        float* P = ws.P + (((int64_t)js * V + a) * n + gi) * D;
#pragma unroll
        for (int c = 0; c < NC; ++c) P[16 * (NC * ch + c) + i] = acc[a][c][q];
        if (i == 0 && ch == 0) ws.rowm[((int64_t)js * V + a) * n + gi] = rowp[0][a][r] + rowp[1][a][r];
      }
    }
  }
}

// dX_a[i][k] += 4 g (x_i[k] * rowm_i - P_i[k])   (sum over j-splits in order)
__global__ __launch_bounds__(256) void dcor_bwd_finalize_kernel(Views v, int V, int64_t n, int d,
                                                                int js_count, float g,
                                                                const float* gscale, int overwrite, DcorWS ws) {
  const float gg = 4.f * g * (gscale ? gscale[0] : 1.f);
  const int64_t total = (int64_t)V * n * d;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int a = (int)(t / (n * d));
    if (!v.dx[a]) continue;
    const int64_t rem = t - (int64_t)a * n * d;
    const int64_t i = rem / d;
    const int k = (int)(rem - i * d);
    // every split's partials loaded before the sums (added in split order)
    float rms[DCOR_JS], ps[DCOR_JS];
#pragma unroll
    for (int s = 0; s < DCOR_JS; ++s) {
      rms[s] = s < js_count ? ws.rowm[((int64_t)s * V + a) * n + i] : 0.f;
      ps[s] = s < js_count ? ws.P[(((int64_t)s * V + a) * n + i) * d + k] : 0.f;
    }
    const float xv = v.x[a][i * d + k];
    const float dv = overwrite ? 0.f : v.dx[a][i * d + k];
    float rm = 0.f, p = 0.f;
#pragma unroll
    for (int s = 0; s < DCOR_JS; ++s)
      if (s < js_count) {
        rm += rms[s];
        p += ps[s];
      }
    const float val = gg * (xv * rm - p);
    v.dx[a][i * d + k] = overwrite ? val : dv + val;
  }
}

// ============================ InfoNCE ==========================================================
// V views of b rows; pair p is H_p = [view pa[p] ; view pb[p]] (m = 2b rows).  All pairs of a step
// run in the same launches (blockIdx.z / y = pair), the views are normalised once, and the backward
// sums each view's upstream over the pairs it appears in before one normalize-backward per row
// (linear in the upstream), so CLUSSL's three InfoNCE pairs are 6 launches instead of 18 + glue.
// workspace: Hn [V][b][d] f32, nrm [V][b] f32, part (m,s) [P][JS][m] f32x2, lse [P][m] f32,
//            P [P][JS][m][d] f32 (bwd), rowsum [P][ceil(m/4)] f64
constexpr int NCE_JS = 8;
// the backward's product operand from a transposed copy of the j tile (true) or row-major dword reads
constexpr bool kNceBwdT = false;
// independent accumulator chains of the logits' MFMA products
constexpr int kNceChains = 1;
// the views normalised inside the log-sum-exp kernel's row staging (no normalize launch)
constexpr bool kNceFusedNorm = true;

struct NceWS { float* Hn; float* nrm; float2* part; float* lse; float* P; double* rowsum; };

__host__ __device__ inline int64_t nce_nparts(int64_t m) { return (m + 3) / 4; }

__host__ __device__ inline NceWS nce_ws(void* base, int V, int64_t b, int d, int P) {
  char* p = reinterpret_cast<char*>(base);
  auto take = [&](int64_t bytes) { char* r = p; p += (bytes + 255) / 256 * 256; return r; };
  const int64_t m = 2 * b;
  NceWS w;
  w.Hn = reinterpret_cast<float*>(take((int64_t)V * b * d * 4));
  w.nrm = reinterpret_cast<float*>(take((int64_t)V * b * 4));
  w.part = reinterpret_cast<float2*>(take((int64_t)P * NCE_JS * m * 8));
  w.lse = reinterpret_cast<float*>(take((int64_t)P * m * 4));
  w.P = reinterpret_cast<float*>(take((int64_t)P * NCE_JS * m * d * 4));
  w.rowsum = reinterpret_cast<double*>(take((int64_t)P * nce_nparts(m) * 8));
  return w;
}

inline int64_t nce_ws_bytes(int V, int64_t b, int d, int P) {
  auto r = [](int64_t x) { return (x + 255) / 256 * 256; };
  const int64_t m = 2 * b;
  return r((int64_t)V * b * d * 4) + r((int64_t)V * b * 4) + r((int64_t)P * NCE_JS * m * 8) + r((int64_t)P * m * 4) +
         r((int64_t)P * NCE_JS * m * d * 4) + r((int64_t)P * nce_nparts(m) * 8);
}

// normalised row r of pair p's H (rows [0, b) from view pa, [b, 2b) from view pb)
__device__ __forceinline__ const float* nce_row(const NceWS& ws, const PairTab& pt, int p, int64_t b, int d,
                                                int64_t r) {
  const int v = r < b ? pt.pa[p] : pt.pb[p];
  return ws.Hn + ((int64_t)v * b + (r < b ? r : r - b)) * d;
}

// rows [r0, r0+64) of pair p's H -> transposed LDS tile (0 beyond 2b)
__device__ __forceinline__ void nce_tile_t(const NceWS& ws, const PairTab& pt, int p, int64_t b, int d, int64_t r0,
                                           float* Xt) {
  const int d4 = d >> 2;
  for (int idx = threadIdx.x; idx < T * d4; idx += blockDim.x) {
    const int r = idx / d4, k4 = idx - r * d4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < 2 * b) v = reinterpret_cast<const float4*>(nce_row(ws, pt, p, b, d, r0 + r))[k4];
    Xt[(4 * k4 + 0) * PADT + r] = v.x;
    Xt[(4 * k4 + 1) * PADT + r] = v.y;
    Xt[(4 * k4 + 2) * PADT + r] = v.z;
    Xt[(4 * k4 + 3) * PADT + r] = v.w;
  }
}

// rows [r0, r0+64) of pair p's H -> row-major LDS tile Xr[r*(d+4) + k]
__device__ __forceinline__ void nce_tile_r(const NceWS& ws, const PairTab& pt, int p, int64_t b, int d, int64_t r0,
                                           float* Xr) {
  const int d4 = d >> 2;
  const int ld = d + 4;
  for (int idx = threadIdx.x; idx < T * d4; idx += blockDim.x) {
    const int r = idx / d4, k4 = idx - r * d4;
    float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
    if (r0 + r < 2 * b) v = reinterpret_cast<const float4*>(nce_row(ws, pt, p, b, d, r0 + r))[k4];
    *reinterpret_cast<float4*>(Xr + r * ld + 4 * k4) = v;
  }
}

// F.normalize(p=2, dim=-1) of every view row: x / max(||x||, 1e-12); one wave per row
// One row's squared norm the way the fused log-sum-exp staging computes it (nce_lse_mfma2_kernel<D,
// true>): a thread holds 4 adjacent float4 chunks of the row (lanes of a row: LPR = max(D / 16, 1)),
// each chunk folded w, z, y, x into one fmaf chain, then a DPP group sum over the row's lanes.  Both
// the normalize pass and the fused staging use it, so Hn / norms are bit-identical either way.
template <int D>
struct NceRowLayout {
  static constexpr int D4 = D / 4, LPR = D4 / 4 >= 1 ? D4 / 4 : 1;
};

template <int D>
__device__ __forceinline__ float nce_row_sumsq(const float4 (&fv)[4]) {
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    ss = fmaf(fv[q].x, fv[q].x, fmaf(fv[q].y, fv[q].y, fmaf(fv[q].z, fv[q].z, fmaf(fv[q].w, fv[q].w, ss))));
  return group_sum<NceRowLayout<D>::LPR>(ss);
}

// x / den rounded as fp32 division does, from one double reciprocal per row: RN32(x * RN64(1 / den)).
// A quotient of two fp32 numbers is never within 2^-49 (relative) of an fp32 rounding boundary when
// it is a normal number, and the double product is within 2^-52 of it, so the result is the correctly
// rounded quotient -- 3 operations per element instead of the ~10 of the division.  (Only a quotient
// below 2^-126, |x| < 2^-126 |den|, could land on a subnormal midpoint; normalised rows never come
// near that.)  Both the normalize pass and the fused staging use it: Hn stays bit-identical between them.
__device__ __forceinline__ float div_rden(float x, double rden) { return (float)((double)x * rden); }

// Hn = H / max(|H|, 1e-12) and the norms, rows of every view (the staging layout above: LPR lanes per
// row, every lane of a wave active for the DPP sum; rows past the end read zeros and store nothing)
template <int D>
__global__ __launch_bounds__(256) void nce_normalize_kernel(Views vw, int V, int64_t b, NceWS ws) {
  using Ly = NceRowLayout<D>;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = t / Ly::LPR, rows = (int64_t)V * b;
  const int c0 = (int)(t % Ly::LPR) * 4;
  const bool ok = r < rows;
  const float4* src = ok ? reinterpret_cast<const float4*>(vw.x[r / b] + (r % b) * D) + c0 : nullptr;
  float4 fv[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) fv[q] = ok && c0 + q < Ly::D4 ? src[q] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float nr = sqrtf(nce_row_sumsq<D>(fv));
  const float den = fmaxf(nr, 1e-12f);
  if (!ok) return;
  if (c0 == 0) ws.nrm[r] = nr;
  const double rd = 1.0 / (double)den;
#pragma unroll
  for (int q = 0; q < 4; ++q)
    if (c0 + q < Ly::D4)
      reinterpret_cast<float4*>(ws.Hn + r * D)[c0 + q] =
          make_float4(div_rden(fv[q].x, rd), div_rden(fv[q].y, rd), div_rden(fv[q].z, rd), div_rden(fv[q].w, rd));
}

__device__ __forceinline__ int64_t nce_partner(int64_t i, int64_t b) { return i < b ? i + b : i - b; }

// partial online log-sum-exp of row i of pair blockIdx.z over the column tiles of split js (self excluded)
__global__ __launch_bounds__(256) void nce_lse_tiles_kernel(int64_t b, int d, float inv_tau, PairTab pt, NceWS ws) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* At = smem;
  float* Bt = At + d * PADT;
  __shared__ float pm[T][17], ps[T][17];
  const int64_t m = 2 * b, nt = (m + T - 1) / T;
  const int it = blockIdx.x, js = blockIdx.y, p = blockIdx.z;
  const int ti = threadIdx.x >> 4, tj = threadIdx.x & 15;
  nce_tile_t(ws, pt, p, b, d, (int64_t)it * T, At);
  float mx[4], sm[4];
  for (int x = 0; x < 4; ++x) { mx[x] = -INFINITY; sm[x] = 0.f; }
  for (int64_t jt = js; jt < nt; jt += gridDim.y) {
    __syncthreads();
    nce_tile_t(ws, pt, p, b, d, jt * T, Bt);
    __syncthreads();
    float g[4][4];
    gram4x4(At, Bt, d, ti, tj, g);
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int64_t gi = (int64_t)it * T + 4 * ti + x, gj = jt * T + 4 * tj + y;
        if (gj >= m || gi == gj) continue;
        const float l = g[x][y] * inv_tau;
        if (l > mx[x]) { sm[x] = sm[x] * expf(mx[x] - l) + 1.f; mx[x] = l; }
        else sm[x] += expf(l - mx[x]);
      }
  }
  for (int x = 0; x < 4; ++x) { pm[4 * ti + x][tj] = mx[x]; ps[4 * ti + x][tj] = sm[x]; }
  __syncthreads();
  if (threadIdx.x < T) {
    const int r = threadIdx.x;
    float M = -INFINITY, S = 0.f;
    for (int k = 0; k < 16; ++k) {
      const float mk = pm[r][k], sk = ps[r][k];
      if (sk == 0.f) continue;
      if (mk > M) { S = S * expf(M - mk) + sk; M = mk; }
      else S += sk * expf(mk - M);
    }
    const int64_t gi = (int64_t)it * T + r;
    if (gi < m) ws.part[((int64_t)p * NCE_JS + js) * m + gi] = make_float2(M, S);
  }
}

// merge splits -> lse; row terms (lse_i - l_i,p(i)) of pair blockIdx.y.  One wave per row (lanes over
// the feature dim for the positive logit), 4 rows per block -> a per-block partial; nce_sum_kernel
// adds the partials in a fixed order (deterministic)
__global__ __launch_bounds__(256) void nce_finalize_kernel(int64_t b, int d, float inv_tau, int js_count, PairTab pt,
                                                           NceWS ws) {
  __shared__ double red[4];
  const int64_t m = 2 * b;
  const int p = blockIdx.y;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t i = (int64_t)blockIdx.x * 4 + wv;
  double v = 0.0;
  if (i < m) {
    // every load of the row issued up front (the split partials and both rows of the positive logit)
    const float* hi = nce_row(ws, pt, p, b, d, i);
    const float* hj = nce_row(ws, pt, p, b, d, nce_partner(i, b));
    const float h0 = lane < d ? hi[lane] : 0.f, j0 = lane < d ? hj[lane] : 0.f;
    const float h1 = lane + 64 < d ? hi[lane + 64] : 0.f, j1 = lane + 64 < d ? hj[lane + 64] : 0.f;
    float2 qs[NCE_JS];
#pragma unroll
    for (int s = 0; s < NCE_JS; ++s)
      qs[s] = s < js_count ? ws.part[((int64_t)p * NCE_JS + s) * m + i] : make_float2(0.f, 0.f);
    float M = -INFINITY, S = 0.f;
#pragma unroll
    for (int s = 0; s < NCE_JS; ++s) {
      const float2 q = qs[s];
      if (s >= js_count || q.y == 0.f) continue;
      if (q.x > M) { S = S * expf(M - q.x) + q.y; M = q.x; }
      else S += q.y * expf(q.x - M);
    }
    const float lse = M + logf(S);
    double dp = 0.0;
    if (lane < d) dp += (double)h0 * (double)j0;
    if (lane + 64 < d) dp += (double)h1 * (double)j1;
    const float dot = (float)group_sum_d<64>(dp);
    if (lane == 0) {
      ws.lse[(int64_t)p * m + i] = lse;
      v = (double)lse - (double)(dot * inv_tau);
    }
  }
  if (lane == 0) red[wv] = v;
  __syncthreads();
  if (threadIdx.x == 0) ws.rowsum[(int64_t)p * nce_nparts(m) + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// out_pairs[p] (optional) = pair p's loss (fp64 sum of its row terms in block order / b^2, rounded
// once); out[0] = their fp32 sum in pair order (Python's sum() over the pairs' fp32 losses)
__global__ __launch_bounds__(1024) void nce_sum_kernel(int64_t b, int n_pairs, NceWS ws, float weight, float* out,
                                                      float* out_pairs) {
  __shared__ double red[16 * 16];
  const int64_t nparts = nce_nparts(2 * b);
  // every pair's strided partial sums first (their loads in flight together), then the per-pair
  // reductions in the same order as before
  double locs[16];
  const bool first = (int64_t)threadIdx.x < nparts;
#pragma unroll
  for (int p = 0; p < 16; ++p)
    locs[p] = 0.0 + (p < n_pairs && first ? ws.rowsum[(int64_t)p * nparts + threadIdx.x] : 0.0);
  if (nparts > (int64_t)blockDim.x) {
#pragma unroll
    for (int p = 0; p < 16; ++p)
      if (p < n_pairs)
        for (int64_t k = threadIdx.x + blockDim.x; k < nparts; k += blockDim.x) locs[p] += ws.rowsum[(int64_t)p * nparts + k];
  }
#pragma unroll
  for (int p = 0; p < 16; ++p) {
    if (p < n_pairs) {  // (uniform)
      const double loc = group_sum_d<64>(locs[p]);
      if ((threadIdx.x & 63) == 0) red[16 * p + (threadIdx.x >> 6)] = loc;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float total = 0.f;
    for (int p = 0; p < n_pairs; ++p) {
      double s = 0.0;
      for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[16 * p + w];
      const float lp = (float)(s / ((double)b * (double)b));
      if (out_pairs) out_pairs[p] = lp;
      total = p == 0 ? lp : total + lp;
    }
    out[0] = weight * total;  // (weight 1: the sum itself, exactly)
  }
}

// dHn_i = (1/tau) sum_j W_ij Hn_j,  W_ij = dl_ij + dl_ji,  dl_ij = (P_ij - [j==p(i)]) * g / b^2  (pair blockIdx.z)
template <int KPER>
__global__ __launch_bounds__(256) void nce_bwd_tiles_kernel(int64_t b, float inv_tau, PairTab pt, NceWS ws) {
  constexpr int d = 4 * KPER;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* At = smem;
  float* Bt = At + d * PADT;
  float* Br = Bt + d * PADT;
  float* Ws = Br + T * (d + 4);
  __shared__ float lse_i[T], lse_j[T];
  const int64_t m = 2 * b, nt = (m + T - 1) / T;
  const int it = blockIdx.x, js = blockIdx.y, p = blockIdx.z;
  const float* lse = ws.lse + (int64_t)p * m;
  const int ti = threadIdx.x >> 4, tj = threadIdx.x & 15;
  const int ar = threadIdx.x & 63, aslot = threadIdx.x >> 6;
  constexpr int kper = KPER;
  nce_tile_t(ws, pt, p, b, d, (int64_t)it * T, At);
  if (threadIdx.x < T) {
    const int64_t gi = (int64_t)it * T + threadIdx.x;
    lse_i[threadIdx.x] = gi < m ? lse[gi] : 0.f;
  }
  float acc[KPER];
#pragma unroll
  for (int k = 0; k < KPER; ++k) acc[k] = 0.f;
  for (int64_t jt = js; jt < nt; jt += gridDim.y) {
    __syncthreads();
    nce_tile_t(ws, pt, p, b, d, jt * T, Bt);
    nce_tile_r(ws, pt, p, b, d, jt * T, Br);
    if (threadIdx.x < T) {
      const int64_t gj = jt * T + threadIdx.x;
      lse_j[threadIdx.x] = gj < m ? lse[gj] : 0.f;
    }
    __syncthreads();
    float g[4][4];
    gram4x4(At, Bt, d, ti, tj, g);
#pragma unroll
    for (int x = 0; x < 4; ++x)
#pragma unroll
      for (int y = 0; y < 4; ++y) {
        const int64_t gi = (int64_t)it * T + 4 * ti + x, gj = jt * T + 4 * tj + y;
        float w = 0.f;
        if (gi < m && gj < m && gi != gj) {
          const float l = g[x][y] * inv_tau;
          const float pij = expf(l - lse_i[4 * ti + x]) - (gj == nce_partner(gi, b) ? 1.f : 0.f);
          const float pji = expf(l - lse_j[4 * tj + y]) - (gi == nce_partner(gj, b) ? 1.f : 0.f);
          w = pij + pji;
        }
        Ws[(4 * ti + x) * 65 + 4 * tj + y] = w;
      }
    __syncthreads();
    for (int j = 0; j < T; ++j) {
      const float w = Ws[ar * 65 + j];
      const float* xr = Br + j * (d + 4) + aslot * kper;
#pragma unroll
      for (int k = 0; k < kper; ++k) acc[k] = fmaf(w, xr[k], acc[k]);
    }
  }
  const int64_t gi = (int64_t)it * T + ar;
  if (gi < m) {
    float* P = ws.P + (((int64_t)p * NCE_JS + js) * m + gi) * d + aslot * kper;
#pragma unroll
    for (int k = 0; k < kper; ++k) P[k] = acc[k];
  }
}

// MFMA form of nce_lse_tiles_kernel: the logits tile on the matrix cores, each lane keeping the online
// (max, sum) of its 4 rows over its columns; the 16 lanes of a row merged in a fixed order at the end.
// The MFMA forms take exp as v_exp_f32(x log2 e) (__expf: a few ulp, against expf's range reduction
// and fix-ups): the logits' exponentials are the kernels' VALU bulk -- InfoNCE fwd + bwd at b = 1,024,
// three pairs measured 123 -> 110 us (tools/profile_ssl.py); the loss and gradients stay inside the
// InfoNCE parity bars (tests/test_gpu_kernels.py, the CLUSSL InfoNCE fixture)
template <int D>
__global__ __launch_bounds__(256) void nce_lse_mfma_kernel(int64_t b, float inv_tau, PairTab pt, NceWS ws) {
  __shared__ __attribute__((aligned(16))) float At[T * (D + 4)];
  __shared__ __attribute__((aligned(16))) float Bt[T * (D + 4)];
  const int64_t m = 2 * b, nt = (m + T - 1) / T;
  const int it = blockIdx.x, js = blockIdx.y, p = blockIdx.z;
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4, w = threadIdx.x >> 6;
  nce_tile_r(ws, pt, p, b, D, (int64_t)it * T, At);
  float mx[4], sm[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) { mx[q] = -INFINITY; sm[q] = 0.f; }
  for (int64_t jt = js; jt < nt; jt += gridDim.y) {
    __syncthreads();
    nce_tile_r(ws, pt, p, b, D, jt * T, Bt);
    __syncthreads();
    f32x4 g[4];
    gram_mfma<D>(At, Bt, g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t gi = (int64_t)it * T + 16 * w + 4 * h + q;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int64_t gj = jt * T + 16 * c + i;
        if (gj >= m || gi == gj) continue;
        const float l = g[c][q] * inv_tau;
        if (l > mx[q]) { sm[q] = sm[q] * __expf(mx[q] - l) + 1.f; mx[q] = l; }
        else sm[q] += __expf(l - mx[q]);
      }
    }
  }
  // merge the 16 lanes of each row: lane i takes its neighbours' (M, S) at distance 1, 2, 4, 8
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    float M = mx[q], S = sm[q];
#pragma unroll
    for (int o = 1; o < 16; o <<= 1) {
      const float Mo = __shfl_xor(M, o, 16), So = __shfl_xor(S, o, 16);
      const float Mn = fmaxf(M, Mo);
      S = (S == 0.f ? 0.f : S * __expf(M - Mn)) + (So == 0.f ? 0.f : So * __expf(Mo - Mn));
      M = Mn;
    }
    const int64_t gi = (int64_t)it * T + 16 * w + 4 * h + q;
    if (i == 0 && gi < m) ws.part[((int64_t)p * NCE_JS + js) * m + gi] = make_float2(M, S);
  }
}

// the logits of a 16 x 16 sub-block: sum over k of the lane's A row (LDS, k-permuted float4 chunks)
// times its B fragments (registers), on kNceChains independent accumulators (k chunks dealt round
// robin) added at the end
template <int D>
__device__ __forceinline__ f32x4 nce_logits(const float* __restrict__ arow, const float4 (&bfr)[D / 16]) {
  f32x4 g[kNceChains];
#pragma unroll
  for (int c = 0; c < kNceChains; ++c) g[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < D / 16; ++kc) {
    const float4 a = *reinterpret_cast<const float4*>(arow + 16 * kc);
#pragma unroll
    for (int mm = 0; mm < 4; ++mm) g[(4 * kc + mm) % kNceChains] = mfma4(comp4(a, mm), comp4(bfr[kc], mm), g[(4 * kc + mm) % kNceChains]);
  }
#pragma unroll
  for (int c = 1; c < kNceChains; ++c) g[0] = g[0] + g[c];
  return g[0];
}

// Round 5 form of the InfoNCE log-sum-exp: the logits transposed per 16 x 16 sub-block (as
// nce_bwd_mfma2_kernel), S^T = Hn_j Hn_b^T, so each lane owns ONE b row (its B fragments in registers
// for the whole kernel: half the LDS reads of nce_lse_mfma_kernel) and keeps one online (max, sum)
// over the j values it holds; the 4 lane groups of a row are merged at the end in a fixed order.
template <int D, bool FUSED>
__global__ __launch_bounds__(256) void nce_lse_mfma2_kernel(int64_t b, float inv_tau, PairTab pt, NceWS ws, Views vw) {
  constexpr int LD = D + 4;
  __shared__ __attribute__((aligned(16))) float Bt[T * LD];
  const int64_t m = 2 * b, nt = (m + T - 1) / T;
  const int it = blockIdx.x, js = blockIdx.y, p = blockIdx.z;
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4, w = threadIdx.x >> 6;
  const int64_t gi = (int64_t)it * T + 16 * w + i;
  const bool ivalid = gi < m;
  constexpr int D4 = D / 4, NPF = T * D4 / 256;
  // FUSED: the rows are read raw (the views) and normalised where they are staged.  Staging layout:
  // a thread holds 4 adjacent float4 chunks of one row, a row spans LPR adjacent lanes; its sum of
  // squares is the thread's fmaf chain then a DPP group sum (the same order in every workgroup),
  // Hn = x / max(|x|, 1e-12) (nce_row_sumsq: the normalize pass's arithmetic).  The j == 0 split's workgroups also write their i rows' Hn and
  // norms for the finalize and the backward (no normalize launch)
  constexpr int LPR = NceRowLayout<D>::LPR, RPP = 256 / LPR, NPASS = (T + RPP - 1) / RPP;
  auto raw_row = [&](int64_t r) -> const float* {
    const int v = r < b ? pt.pa[p] : pt.pb[p];
    return vw.x[v] + (r < b ? r : r - b) * D;
  };
  auto fused_load = [&](int64_t r0, float4 (&fv)[NPASS][4]) {
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
      const int r = ps * RPP + (int)threadIdx.x / LPR, c0 = ((int)threadIdx.x % LPR) * 4;
      const bool ok = r < T && r0 + r < m;
      const float4* src = ok ? reinterpret_cast<const float4*>(raw_row(r0 + r)) + c0 : nullptr;
#pragma unroll
      for (int q = 0; q < 4; ++q) fv[ps][q] = ok && c0 + q < D4 ? src[q] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  };
  // normalise and store to Bt; owner: also write Hn / norms of rows r0 + r (global row index of pair p)
  auto fused_store = [&](int64_t r0, float4 (&fv)[NPASS][4], bool owner) {
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
      const int r = ps * RPP + (int)threadIdx.x / LPR, c0 = ((int)threadIdx.x % LPR) * 4;
      const float nr = sqrtf(nce_row_sumsq<D>(fv[ps]));
      const float den = fmaxf(nr, 1e-12f);
      const double rd = 1.0 / (double)den;
      if (r < T) {
        const int64_t gr = r0 + r;
        float* hn_g = nullptr;
        if (owner && gr < m) {
          const int v = gr < b ? pt.pa[p] : pt.pb[p];
          const int64_t vr = (int64_t)v * b + (gr < b ? gr : gr - b);
          hn_g = ws.Hn + vr * D;
          if (c0 == 0) ws.nrm[vr] = nr;
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          if (c0 + q >= D4) continue;
          const float4 x = fv[ps][q];
          const float4 hn = make_float4(div_rden(x.x, rd), div_rden(x.y, rd), div_rden(x.z, rd), div_rden(x.w, rd));
          *reinterpret_cast<float4*>(Bt + r * LD + 4 * (c0 + q)) = hn;
          if (hn_g) reinterpret_cast<float4*>(hn_g)[c0 + q] = hn;
        }
      }
    }
  };
  float4 bfr[D / 16];
  if constexpr (FUSED) {
    // the i tile staged normalised in Bt first, the B fragments read back from it
    float4 fi[NPASS][4];
    fused_load((int64_t)it * T, fi);
    fused_store((int64_t)it * T, fi, js == 0);
    __syncthreads();
#pragma unroll
    for (int kc = 0; kc < D / 16; ++kc)
      bfr[kc] = *reinterpret_cast<const float4*>(Bt + (16 * w + i) * LD + 16 * kc + 4 * h);
  } else {
    const float* row = ivalid ? nce_row(ws, pt, p, b, D, gi) : nullptr;
#pragma unroll
    for (int kc = 0; kc < D / 16; ++kc)
      bfr[kc] = ivalid ? *reinterpret_cast<const float4*>(row + 16 * kc + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  // base-2 online log-sum-exp, four logits at a time (no divergent rescale branch):
  // M' = max(M, max_q l2_q), S = S 2^(M - M') + sum_q 2^(l2_q - M')
  constexpr float kLog2e = 1.4426950408889634f;
  const float s2 = inv_tau * kLog2e;
  const int mi = (int)m, gi32 = (int)gi;
  float mx = -INFINITY, sm = 0.f;
  // the j tile's rows loaded into registers one tile ahead (in flight during the previous tile)
  float4 pf[FUSED ? 1 : NPF];
  float4 fj[FUSED ? NPASS : 1][4];
  auto load_tile = [&](int64_t jt) {
    if constexpr (FUSED) {
      fused_load(jt * T, fj);
    } else {
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        const int idx = threadIdx.x + 256 * u, r = idx / D4, k4 = idx - r * D4;
        pf[u] = jt * T + r < m ? reinterpret_cast<const float4*>(nce_row(ws, pt, p, b, D, jt * T + r))[k4]
                               : make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
  };
  if (js < nt) load_tile(js);
  for (int64_t jt = js; jt < nt; jt += gridDim.y) {
    __syncthreads();
    if constexpr (FUSED) {
      fused_store(jt * T, fj, false);
    } else {
#pragma unroll
      for (int u = 0; u < NPF; ++u) {
        const int idx = threadIdx.x + 256 * u, r = idx / D4, k4 = idx - r * D4;
        *reinterpret_cast<float4*>(Bt + r * LD + 4 * k4) = pf[u];
      }
    }
    __syncthreads();
    if (jt + gridDim.y < nt) load_tile(jt + gridDim.y);
#pragma unroll
    for (int jc = 0; jc < T / 16; ++jc) {
      const f32x4 g = nce_logits<D>(Bt + (16 * jc + i) * LD + 4 * h, bfr);
      float l2[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int gj = (int)jt * T + 16 * jc + 4 * h + q;
        l2[q] = (gj < mi && gj != gi32) ? g[q] * s2 : -INFINITY;
      }
      const float mn = fmaxf(mx, fmaxf(fmaxf(l2[0], l2[1]), fmaxf(l2[2], l2[3])));
      if (mn != -INFINITY) {  // (lane-uniform only by accident: a select, not a branch, in practice)
        float add = 0.f;
#pragma unroll
        for (int q = 0; q < 4; ++q) add += __builtin_amdgcn_exp2f(l2[q] - mn);
        sm = (sm == 0.f ? 0.f : sm * __builtin_amdgcn_exp2f(mx - mn)) + add;
        mx = mn;
      }
    }
  }
  // merge the 4 lane groups of the row (lanes i, i + 16, i + 32, i + 48): distance 16, then 32
#pragma unroll
  for (int o = 16; o < 64; o <<= 1) {
    const float Mo = __shfl_xor(mx, o, 64), So = __shfl_xor(sm, o, 64);
    const float Mn = fmaxf(mx, Mo);
    sm = (sm == 0.f ? 0.f : sm * __builtin_amdgcn_exp2f(mx - Mn)) + (So == 0.f ? 0.f : So * __builtin_amdgcn_exp2f(Mo - Mn));
    mx = Mn;
  }
  // (max, sum) in natural-log units for nce_finalize_kernel: M = M2 ln 2, S unchanged
  if (h == 0 && ivalid) ws.part[((int64_t)p * NCE_JS + js) * m + gi] = make_float2(mx * 0.69314718055994531f, sm);
}

// MFMA form of nce_bwd_tiles_kernel: the logits tile and W = dl + dl^T on the matrix cores / VALU,
// W staged in LDS, then sum_j W_ij Hn_j on the matrix cores into per-lane accumulators
template <int D>
__global__ __launch_bounds__(256) void nce_bwd_mfma_kernel(int64_t b, float inv_tau, PairTab pt, NceWS ws) {
  constexpr int LD = D + 4;
  __shared__ __attribute__((aligned(16))) float At[T * LD];
  __shared__ __attribute__((aligned(16))) float Bt[T * LD];
  __shared__ float Ws[T * 65];
  __shared__ float lse_i[T], lse_j[T];
  const int64_t m = 2 * b, nt = (m + T - 1) / T;
  const int it = blockIdx.x, js = blockIdx.y, p = blockIdx.z;
  const float* lse = ws.lse + (int64_t)p * m;
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4, w = threadIdx.x >> 6;
  nce_tile_r(ws, pt, p, b, D, (int64_t)it * T, At);
  if (threadIdx.x < T) {
    const int64_t gi = (int64_t)it * T + threadIdx.x;
    lse_i[threadIdx.x] = gi < m ? lse[gi] : 0.f;
  }
  f32x4 acc[D / 16];
#pragma unroll
  for (int c = 0; c < D / 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t jt = js; jt < nt; jt += gridDim.y) {
    __syncthreads();
    nce_tile_r(ws, pt, p, b, D, jt * T, Bt);
    if (threadIdx.x < T) {
      const int64_t gj = jt * T + threadIdx.x;
      lse_j[threadIdx.x] = gj < m ? lse[gj] : 0.f;
    }
    __syncthreads();
    f32x4 g[4];
    gram_mfma<D>(At, Bt, g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = 16 * w + 4 * h + q;
      const int64_t gi = (int64_t)it * T + r;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int64_t gj = jt * T + 16 * c + i;
        float wv = 0.f;
        if (gi < m && gj < m && gi != gj) {
          const float l = g[c][q] * inv_tau;
          const float pij = __expf(l - lse_i[r]) - (gj == nce_partner(gi, b) ? 1.f : 0.f);
          const float pji = __expf(l - lse_j[16 * c + i]) - (gi == nce_partner(gj, b) ? 1.f : 0.f);
          wv = pij + pji;
        }
        Ws[r * 65 + 16 * c + i] = wv;
      }
    }
    __syncthreads();
    wx_mfma<D>(Ws, Bt, acc);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t gi = (int64_t)it * T + 16 * w + 4 * h + q;
    if (gi < m) {
      float* P = ws.P + (((int64_t)p * NCE_JS + js) * m + gi) * D;
#pragma unroll
      for (int c = 0; c < D / 16; ++c) P[16 * c + i] = acc[c][q];
    }
  }
}

// Round 5 form of the InfoNCE backward: the logits are computed TRANSPOSED per 16 x 16 sub-block,
// S^T = Hn_j Hn_b^T (lane (i, h) holds S[j = 16 jc + 4h + q][b = 16 w + i]), and because W is symmetric
// those registers ARE the A operand of dHn_b = sum_j W_bj Hn_j (the k order of the 16-wide j chunk
// permuted so that lane group h feeds k = 4h + q to MFMA q).  No W staging in LDS, one barrier per
// column tile; the b-side rows' B fragments of the logits stay in registers for the whole kernel and
// the j tile is staged twice (row-major for the logits, transposed for the product: one ds_read_b128
// per B fragment).  Same partial layout as nce_bwd_mfma_kernel.
template <int D>
__global__ __launch_bounds__(256) void nce_bwd_mfma2_kernel(int64_t b, float inv_tau, PairTab pt, NceWS ws) {
  constexpr int LD = D + 4, LDT = T + 4;
  __shared__ __attribute__((aligned(16))) float Bt[T * LD];    // j rows, row-major (logits' A operand)
  __shared__ __attribute__((aligned(16))) float BtT[kNceBwdT ? D * LDT : 4];  // the same tile transposed (product's B operand)
  __shared__ float lse_j[T];
  const int64_t m = 2 * b, nt = (m + T - 1) / T;
  const int it = blockIdx.x, js = blockIdx.y, p = blockIdx.z;
  const float* lse = ws.lse + (int64_t)p * m;
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4, w = threadIdx.x >> 6;
  // 32-bit row indices (m < 2^31, checked by the caller); base-2 logits: exp(l - lse) = exp2(l2 - lse2)
  // with l2 = l log2(e).  The partner relation is an involution, so [i == partner(j)] = [j == partner(i)]:
  // W_ij = exp(l - lse_i) + exp(l - lse_j) - 2 [j == partner(i)]
  constexpr float kLog2e = 1.4426950408889634f;
  const float s2 = inv_tau * kLog2e;
  const int mi = (int)m;
  const int gi = it * T + 16 * w + i;  // this lane's b row (the product's A row)
  const bool ivalid = gi < mi;
  const float lse2_i = ivalid ? lse[gi] * kLog2e : 0.f;
  const int part_i = ivalid ? (int)nce_partner(gi, b) : -1;
  // B operand of the logits: row gi of Hn, k-permuted float4 chunks
  float4 bfr[D / 16];
  {
    const float* row = ivalid ? nce_row(ws, pt, p, b, D, gi) : nullptr;
#pragma unroll
    for (int kc = 0; kc < D / 16; ++kc)
      bfr[kc] = ivalid ? *reinterpret_cast<const float4*>(row + 16 * kc + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
  }
  f32x4 acc[D / 16];
#pragma unroll
  for (int c = 0; c < D / 16; ++c) acc[c] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t jt = js; jt < nt; jt += gridDim.y) {
    __syncthreads();
    {  // stage the j tile (every thread's loads issued before its first store), and its rows' lse
      constexpr int D4 = D / 4, NST = T * D4 / 256;
      float4 vs[NST];
#pragma unroll
      for (int u = 0; u < NST; ++u) {
        const int idx = threadIdx.x + 256 * u, r = idx / D4, k4 = idx - r * D4;
        vs[u] = jt * T + r < m ? reinterpret_cast<const float4*>(nce_row(ws, pt, p, b, D, jt * T + r))[k4]
                               : make_float4(0.f, 0.f, 0.f, 0.f);
      }
      const int64_t gj = jt * T + threadIdx.x;
      const float lj = threadIdx.x < T && gj < m ? lse[gj] * kLog2e : 0.f;
#pragma unroll
      for (int u = 0; u < NST; ++u) {
        const int idx = threadIdx.x + 256 * u, r = idx / D4, k4 = idx - r * D4;
        const float4 v = vs[u];
        *reinterpret_cast<float4*>(Bt + r * LD + 4 * k4) = v;
        if constexpr (kNceBwdT) {
          BtT[(4 * k4 + 0) * LDT + r] = v.x;
          BtT[(4 * k4 + 1) * LDT + r] = v.y;
          BtT[(4 * k4 + 2) * LDT + r] = v.z;
          BtT[(4 * k4 + 3) * LDT + r] = v.w;
        }
      }
      if (threadIdx.x < T) lse_j[threadIdx.x] = lj;
    }
    __syncthreads();
    const int j0 = (int)jt * T;
#pragma unroll
    for (int jc = 0; jc < T / 16; ++jc) {
      const f32x4 g = nce_logits<D>(Bt + (16 * jc + i) * LD + 4 * h, bfr);
      float wv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int jl = 16 * jc + 4 * h + q;
        const int gj = j0 + jl;
        const float l2 = g[q] * s2;
        const float e = (__builtin_amdgcn_exp2f(l2 - lse2_i) + __builtin_amdgcn_exp2f(l2 - lse_j[jl])) -
                        (gj == part_i ? 2.f : 0.f);
        wv[q] = (ivalid && gj < mi && gi != gj) ? e : 0.f;
      }
#pragma unroll
      for (int c = 0; c < D / 16; ++c) {
        float4 bx;
        if constexpr (kNceBwdT) {
          bx = *reinterpret_cast<const float4*>(BtT + (16 * c + i) * LDT + 16 * jc + 4 * h);
        } else {  // four conflict-free dword reads of the row-major tile (banks i + 16 h + 4 q)
          const float* bc = Bt + (16 * jc + 4 * h) * LD + 16 * c + i;
          bx = make_float4(bc[0], bc[LD], bc[2 * LD], bc[3 * LD]);
        }
#pragma unroll
        for (int q = 0; q < 4; ++q) acc[c] = mfma4(wv[q], comp4(bx, q), acc[c]);
      }
    }
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int64_t go = (int64_t)it * T + 16 * w + 4 * h + q;
    if (go < m) {
      float* P = ws.P + (((int64_t)p * NCE_JS + js) * m + go) * D;
#pragma unroll
      for (int c = 0; c < D / 16; ++c) P[16 * c + i] = acc[c][q];
    }
  }
}

// dview_v[r] = normalize_backward(gh) with gh = scale * (sum over the pairs holding view v, at the
// row's position in that pair, of the split partials); written (views that no pair holds: zeros)
__global__ __launch_bounds__(256) void nce_bwd_finalize_kernel(Views vw, int V, int64_t b, int d, float inv_tau,
                                                               int js_count, float g, const float* gscale, PairTab pt,
                                                               NceWS ws) {
  const float scale = g * (gscale ? gscale[0] : 1.f) / ((float)b * (float)b) * inv_tau;
  const int64_t m = 2 * b, rows = (int64_t)V * b;
  const int lane = threadIdx.x & 63;
  for (int64_t vr = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6; vr < rows;
       vr += ((int64_t)gridDim.x * blockDim.x) >> 6) {
    const int v = (int)(vr / b);
    const int64_t r = vr % b;
    float* dX = vw.dx[v];
    if (dX == nullptr) continue;
    const float nr = ws.nrm[vr];
    const float* hn = ws.Hn + vr * d;
    auto gsum = [&](int k) {
      float q = 0.f;
      for (int p = 0; p < pt.n_pairs; ++p) {
        for (int side = 0; side < 2; ++side) {
          if ((side ? pt.pb[p] : pt.pa[p]) != v) continue;
          // the pair's split partials of this row: loads issued together, added in split order
          const float* src = ws.P + ((int64_t)p * NCE_JS * m + (side ? b + r : r)) * d + k;
          float x[NCE_JS];
#pragma unroll
          for (int s = 0; s < NCE_JS; ++s) x[s] = s < js_count ? src[(int64_t)s * m * d] : 0.f;
#pragma unroll
          for (int s = 0; s < NCE_JS; ++s)
            if (s < js_count) q += x[s];
        }
      }
      return q * scale;
    };
    // this lane's columns k = lane, lane + 64 (d <= 128): the split partials are read once
    float gk[2];
    float dot = 0.f;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k = lane + 64 * t;
      gk[t] = k < d ? gsum(k) : 0.f;
      if (k < d) dot = fmaf(gk[t], hn[k], dot);
    }
    dot = group_sum<64>(dot);
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int k = lane + 64 * t;
      // d/dx [x / max(|x|, eps)]
      if (k < d) dX[r * d + k] = nr > 1e-12f ? (gk[t] - hn[k] * dot) / nr : gk[t] / 1e-12f;
    }
  }
}

}  // namespace

// ------------------------------------------------------------------------------------------ ABI
extern "C" int fr_ssl_kernels(int mfma) {
  const int prev = g_ssl_mfma;
  if (mfma >= 0) g_ssl_mfma = mfma > 2 ? 1 : mfma;
  return prev;
}

extern "C" int64_t fr_dcor_workspace(int64_t n, int n_views) {
  if (n <= 0 || n_views <= 0 || n_views > MAXV) return 0;
  return dcor_ws_bytes(n, n_views);
}

static int dcor_check(const float* const* views, int V, int64_t n, int d, const int32_t* pairs,
                      int P, void* ws, int64_t wsb) {
  FR_REQUIRE(views && V >= 1 && V <= MAXV, "1..4 views required");
  FR_REQUIRE(n >= 2, "need n >= 2 rows");
  FR_REQUIRE(d == 16 || d == 32 || d == 64 || d == 128, "d must be 16, 32, 64 or 128");
  FR_REQUIRE(pairs && P >= 1 && P <= 16, "1..16 pairs required");
  for (int k = 0; k < P; ++k)
    FR_REQUIRE(pairs[2 * k] >= 0 && pairs[2 * k] < V && pairs[2 * k + 1] >= 0 && pairs[2 * k + 1] < V,
               "pair view index out of range");
  for (int a = 0; a < V; ++a) FR_REQUIRE(views[a] && fr::aligned16(views[a]), "view null/unaligned");
  FR_REQUIRE(ws && wsb >= dcor_ws_bytes(n, V) && fr::aligned16(ws), "workspace too small");
  return FR_OK;
}

extern "C" int fr_dcor_fwd(const float* const* d_views, int n_views, int64_t n, int d,
                           const int32_t* pairs, int n_pairs, float* d_out, void* d_workspace,
                           int64_t workspace_bytes, void* stream) {
  return fr_dcor_fwd_ex(d_views, n_views, n, d, pairs, n_pairs, 1.f, d_out, d_workspace, workspace_bytes, stream);
}

extern "C" int fr_dcor_fwd_ex(const float* const* d_views, int n_views, int64_t n, int d,
                              const int32_t* pairs, int n_pairs, float weight, float* d_out, void* d_workspace,
                              int64_t workspace_bytes, void* stream) {
  int rc = dcor_check(d_views, n_views, n, d, pairs, n_pairs, d_workspace, workspace_bytes);
  if (rc) return rc;
  FR_REQUIRE(d_out, "out null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  Views v{};
  for (int a = 0; a < n_views; ++a) v.x[a] = d_views[a];
  PairTab pt{};
  pt.n_pairs = n_pairs;
  for (int k = 0; k < n_pairs; ++k) { pt.pa[k] = pairs[2 * k]; pt.pb[k] = pairs[2 * k + 1]; }
  DcorWS w = dcor_ws(d_workspace, n, n_views);
  const int64_t nt = fr::ceil_div(n, T);
  const size_t lds = (size_t)(2 * d * PADT + 2 * T) * 4 + 64;
  const dim3 grid((unsigned)nt, (unsigned)nt);
  if (g_ssl_mfma && d == 64) {
    switch (n_views) {
      case 1: hipLaunchKernelGGL((dcor_tiles_mfma_kernel<1, 64>), grid, dim3(256), 0, s, v, n, w); break;
      case 2: hipLaunchKernelGGL((dcor_tiles_mfma_kernel<2, 64>), grid, dim3(256), 0, s, v, n, w); break;
      case 3: hipLaunchKernelGGL((dcor_tiles_mfma_kernel<3, 64>), grid, dim3(256), 0, s, v, n, w); break;
      default: hipLaunchKernelGGL((dcor_tiles_mfma_kernel<4, 64>), grid, dim3(256), 0, s, v, n, w); break;
    }
  } else switch (n_views) {
    case 1: hipLaunchKernelGGL(dcor_tiles_kernel<1>, grid, dim3(256), lds, s, v, n, d, w); break;
    case 2: hipLaunchKernelGGL(dcor_tiles_kernel<2>, grid, dim3(256), lds, s, v, n, d, w); break;
    case 3: hipLaunchKernelGGL(dcor_tiles_kernel<3>, grid, dim3(256), lds, s, v, n, d, w); break;
    default: hipLaunchKernelGGL(dcor_tiles_kernel<4>, grid, dim3(256), lds, s, v, n, d, w); break;
  }
  FR_LAUNCH_CHECK();
  const int nb = (int)fr::ceil_div(n, 64);
  switch (n_views) {
#define FR_DCOR_MF(VV) \
  hipLaunchKernelGGL(dcor_means_finalize_kernel<VV>, dim3((unsigned)nb), dim3(64), 0, s, n, nb, pt, w, weight, d_out)
    case 1: FR_DCOR_MF(1); break;
    case 2: FR_DCOR_MF(2); break;
    case 3: FR_DCOR_MF(3); break;
    default: FR_DCOR_MF(4); break;
#undef FR_DCOR_MF
  }
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_dcor_bwd(const float* const* d_views, int n_views, int64_t n, int d,
                           const int32_t* pairs, int n_pairs, float g, const float* d_gscale,
                           float* const* d_dviews, void* d_workspace, int64_t workspace_bytes,
                           void* stream) {
  return fr_dcor_bwd_ex(d_views, n_views, n, d, pairs, n_pairs, g, d_gscale, d_dviews, 0, d_workspace,
                        workspace_bytes, stream);
}

extern "C" int fr_dcor_bwd_ex(const float* const* d_views, int n_views, int64_t n, int d,
                              const int32_t* pairs, int n_pairs, float g, const float* d_gscale,
                              float* const* d_dviews, int overwrite, void* d_workspace, int64_t workspace_bytes,
                              void* stream) {
  int rc = dcor_check(d_views, n_views, n, d, pairs, n_pairs, d_workspace, workspace_bytes);
  if (rc) return rc;
  FR_REQUIRE(d_dviews, "dviews null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  Views v{};
  for (int a = 0; a < n_views; ++a) {
    v.x[a] = d_views[a];
    v.dx[a] = d_dviews[a];
    FR_REQUIRE(!v.dx[a] || fr::aligned16(v.dx[a]), "dview unaligned");
  }
  DcorWS w = dcor_ws(d_workspace, n, n_views);
  const int64_t nt = fr::ceil_div(n, T);
  const int js = (int)std::min<int64_t>(DCOR_JS, nt);
  const size_t lds = (size_t)(n_views * d * PADT + d * PADT + T * (d + 4) + T * 65 + MAXV * T + T) * 4;
  FR_REQUIRE(lds <= 160 * 1024, "LDS budget exceeded (reduce views or d)");
  const dim3 grid((unsigned)nt, (unsigned)js);
  if (g_ssl_mfma && d == 64) {
    switch (n_views) {
      case 1: hipLaunchKernelGGL((dcor_bwd_mfma_allb_kernel<1, 64>), grid, dim3(DB_NT), 0, s, v, n, w); break;
      case 2: hipLaunchKernelGGL((dcor_bwd_mfma_allb_kernel<2, 64>), grid, dim3(DB_NT), 0, s, v, n, w); break;
      case 3: hipLaunchKernelGGL((dcor_bwd_mfma_allb_kernel<3, 64>), grid, dim3(DB_NT), 0, s, v, n, w); break;
      default: hipLaunchKernelGGL((dcor_bwd_mfma_kernel<4, 64>), grid, dim3(DB_NT), 0, s, v, n, w); break;
    }
    FR_LAUNCH_CHECK();
  } else {
#define FR_DCOR_BWD(VV, KK) \
  hipLaunchKernelGGL((dcor_bwd_tiles_kernel<VV, KK>), grid, dim3(256), lds, s, v, n, w)
#define FR_DCOR_BWD_V(KK)                          \
  switch (n_views) {                               \
    case 1: FR_DCOR_BWD(1, KK); break;             \
    case 2: FR_DCOR_BWD(2, KK); break;             \
    case 3: FR_DCOR_BWD(3, KK); break;             \
    default: FR_DCOR_BWD(4, KK); break;            \
  }
  switch (d) {
    case 16: FR_DCOR_BWD_V(4); break;
    case 32: FR_DCOR_BWD_V(8); break;
    case 64: FR_DCOR_BWD_V(16); break;
    default: FR_DCOR_BWD_V(32); break;
  }
#undef FR_DCOR_BWD_V
#undef FR_DCOR_BWD
  FR_LAUNCH_CHECK();
  }
  const int64_t total = (int64_t)n_views * n * d;
  const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(total, 256), 4096);
  hipLaunchKernelGGL(dcor_bwd_finalize_kernel, dim3(blocks), dim3(256), 0, s, v, n_views, n, d, js,
                     g, d_gscale, overwrite, w);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

static int nce_check(const float* const* views, int V, int64_t b, int d, const int32_t* pairs, int P, float tau,
                     void* ws, int64_t wsb) {
  FR_REQUIRE(views && V >= 1 && V <= MAXV, "1..4 views required");
  FR_REQUIRE(b >= 1, "b must be >= 1");
  FR_REQUIRE(d == 16 || d == 32 || d == 64 || d == 128, "d must be 16, 32, 64 or 128");
  FR_REQUIRE(tau > 0.f, "tau must be > 0");
  FR_REQUIRE(pairs && P >= 1 && P <= 16, "1..16 pairs required");
  for (int k = 0; k < P; ++k)
    FR_REQUIRE(pairs[2 * k] >= 0 && pairs[2 * k] < V && pairs[2 * k + 1] >= 0 && pairs[2 * k + 1] < V,
               "pair view index out of range");
  for (int a = 0; a < V; ++a) FR_REQUIRE(views[a] && fr::aligned16(views[a]), "view null/unaligned");
  FR_REQUIRE(ws && wsb >= nce_ws_bytes(V, b, d, P) && fr::aligned16(ws), "workspace too small");
  return FR_OK;
}

extern "C" int64_t fr_infonce_multi_workspace(int n_views, int64_t b, int d, int n_pairs) {
  if (b <= 0 || n_views <= 0 || n_views > MAXV || n_pairs <= 0 || n_pairs > 16 || d <= 0 || d > 128) return 0;
  return nce_ws_bytes(n_views, b, d, n_pairs);
}

// the log-sum-exp kernel of the MFMA forms: 1 = the round-5 transposed form, 2 = the round-4 one (A/B)
template <int D>
static void launch_lse(dim3 grid, hipStream_t s, int64_t b, float inv_tau, const PairTab& pt, const NceWS& w,
                       const Views& v, bool fused) {
  if (g_ssl_mfma == 2)
    hipLaunchKernelGGL(nce_lse_mfma_kernel<D>, grid, dim3(256), 0, s, b, inv_tau, pt, w);
  else if (fused)
    hipLaunchKernelGGL((nce_lse_mfma2_kernel<D, true>), grid, dim3(256), 0, s, b, inv_tau, pt, w, v);
  else
    hipLaunchKernelGGL((nce_lse_mfma2_kernel<D, false>), grid, dim3(256), 0, s, b, inv_tau, pt, w, v);
}

static int nce_fwd_impl(const float* const* d_views, int n_views, int64_t b, int d, const int32_t* pairs, int n_pairs,
                        float tau, float weight, float* d_out, float* d_out_pairs, void* d_workspace,
                        int64_t workspace_bytes, void* stream) {
  int rc = nce_check(d_views, n_views, b, d, pairs, n_pairs, tau, d_workspace, workspace_bytes);
  if (rc) return rc;
  FR_REQUIRE(d_out, "out null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t m = 2 * b;
  NceWS w = nce_ws(d_workspace, n_views, b, d, n_pairs);
  Views v{};
  for (int a = 0; a < n_views; ++a) v.x[a] = d_views[a];
  PairTab pt{};
  pt.n_pairs = n_pairs;
  for (int k = 0; k < n_pairs; ++k) { pt.pa[k] = pairs[2 * k]; pt.pb[k] = pairs[2 * k + 1]; }
  const float inv_tau = 1.f / tau;
  // the round-5 MFMA kernels normalise the views in their staging when every view is in a pair
  // (each view's rows are then some workgroup's i rows, whose Hn / norms it writes)
  bool every_view_paired = true;
  for (int a = 0; a < n_views; ++a) {
    bool in = false;
    for (int k = 0; k < n_pairs; ++k) in |= pt.pa[k] == a || pt.pb[k] == a;
    every_view_paired &= in;
  }
  const bool fused = kNceFusedNorm && g_ssl_mfma == 1 && every_view_paired;
  if (!fused) {
    const int lpr = d / 16;  // NceRowLayout<d>::LPR
    const unsigned nb = (unsigned)fr::ceil_div((int64_t)n_views * b * lpr, (int64_t)256);
    switch (d) {
      case 16: hipLaunchKernelGGL(nce_normalize_kernel<16>, dim3(nb), dim3(256), 0, s, v, n_views, b, w); break;
      case 32: hipLaunchKernelGGL(nce_normalize_kernel<32>, dim3(nb), dim3(256), 0, s, v, n_views, b, w); break;
      case 64: hipLaunchKernelGGL(nce_normalize_kernel<64>, dim3(nb), dim3(256), 0, s, v, n_views, b, w); break;
      default: hipLaunchKernelGGL(nce_normalize_kernel<128>, dim3(nb), dim3(256), 0, s, v, n_views, b, w); break;
    }
    FR_LAUNCH_CHECK();
  }
  const int64_t nt = fr::ceil_div(m, T);
  const int js = (int)std::min<int64_t>(NCE_JS, nt);
  const size_t lds = (size_t)(2 * d * PADT) * 4;
  const dim3 grid((unsigned)nt, (unsigned)js, (unsigned)n_pairs);
  if (g_ssl_mfma) {
    switch (d) {
      case 16: launch_lse<16>(grid, s, b, inv_tau, pt, w, v, fused); break;
      case 32: launch_lse<32>(grid, s, b, inv_tau, pt, w, v, fused); break;
      case 64: launch_lse<64>(grid, s, b, inv_tau, pt, w, v, fused); break;
      default: launch_lse<128>(grid, s, b, inv_tau, pt, w, v, fused); break;
    }
  } else {
    hipLaunchKernelGGL(nce_lse_tiles_kernel, grid, dim3(256), lds, s, b, d, inv_tau, pt, w);
  }
  FR_LAUNCH_CHECK();
  hipLaunchKernelGGL(nce_finalize_kernel, dim3((unsigned)nce_nparts(m), (unsigned)n_pairs), dim3(256), 0, s, b, d,
                     inv_tau, js, pt, w);
  FR_LAUNCH_CHECK();
  hipLaunchKernelGGL(nce_sum_kernel, dim3(1), dim3(1024), 0, s, b, n_pairs, w, weight, d_out, d_out_pairs);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_infonce_multi_fwd(const float* const* d_views, int n_views, int64_t b, int d, const int32_t* pairs,
                                    int n_pairs, float tau, float* d_out, void* d_workspace, int64_t workspace_bytes,
                                    void* stream) {
  return nce_fwd_impl(d_views, n_views, b, d, pairs, n_pairs, tau, 1.f, d_out, d_out ? d_out + 1 : nullptr, d_workspace,
                      workspace_bytes, stream);
}

extern "C" int fr_infonce_multi_fwd_ex(const float* const* d_views, int n_views, int64_t b, int d,
                                       const int32_t* pairs, int n_pairs, float tau, float weight, float* d_out,
                                       void* d_workspace, int64_t workspace_bytes, void* stream) {
  return nce_fwd_impl(d_views, n_views, b, d, pairs, n_pairs, tau, weight, d_out, d_out ? d_out + 1 : nullptr,
                      d_workspace, workspace_bytes, stream);
}

extern "C" int fr_infonce_multi_bwd(const float* const* d_views, int n_views, int64_t b, int d, const int32_t* pairs,
                                    int n_pairs, float tau, float g, const float* d_gscale, float* const* d_dviews,
                                    void* d_workspace, int64_t workspace_bytes, void* stream) {
  int rc = nce_check(d_views, n_views, b, d, pairs, n_pairs, tau, d_workspace, workspace_bytes);
  if (rc) return rc;
  FR_REQUIRE(d_dviews, "dviews null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t m = 2 * b;
  NceWS w = nce_ws(d_workspace, n_views, b, d, n_pairs);
  Views v{};
  for (int a = 0; a < n_views; ++a) {
    v.x[a] = d_views[a];
    v.dx[a] = d_dviews[a];
    FR_REQUIRE(!v.dx[a] || fr::aligned16(v.dx[a]), "dview unaligned");
  }
  PairTab pt{};
  pt.n_pairs = n_pairs;
  for (int k = 0; k < n_pairs; ++k) { pt.pa[k] = pairs[2 * k]; pt.pb[k] = pairs[2 * k + 1]; }
  const float inv_tau = 1.f / tau;
  const int64_t nt = fr::ceil_div(m, T);
  const int js = (int)std::min<int64_t>(NCE_JS, nt);
  const size_t lds = (size_t)(2 * d * PADT + T * (d + 4) + T * 65) * 4;
  const dim3 grid((unsigned)nt, (unsigned)js, (unsigned)n_pairs);
  if (g_ssl_mfma == 2) {  // the round-4 MFMA backward (W staged in LDS), for A/B
    switch (d) {
      case 16: hipLaunchKernelGGL(nce_bwd_mfma_kernel<16>, grid, dim3(256), 0, s, b, inv_tau, pt, w); break;
      case 32: hipLaunchKernelGGL(nce_bwd_mfma_kernel<32>, grid, dim3(256), 0, s, b, inv_tau, pt, w); break;
      case 64: hipLaunchKernelGGL(nce_bwd_mfma_kernel<64>, grid, dim3(256), 0, s, b, inv_tau, pt, w); break;
      default: hipLaunchKernelGGL(nce_bwd_mfma_kernel<128>, grid, dim3(256), 0, s, b, inv_tau, pt, w); break;
    }
  } else if (g_ssl_mfma) {
    switch (d) {
      case 16: hipLaunchKernelGGL(nce_bwd_mfma2_kernel<16>, grid, dim3(256), 0, s, b, inv_tau, pt, w); break;
      case 32: hipLaunchKernelGGL(nce_bwd_mfma2_kernel<32>, grid, dim3(256), 0, s, b, inv_tau, pt, w); break;
      case 64: hipLaunchKernelGGL(nce_bwd_mfma2_kernel<64>, grid, dim3(256), 0, s, b, inv_tau, pt, w); break;
      default: hipLaunchKernelGGL(nce_bwd_mfma2_kernel<128>, grid, dim3(256), 0, s, b, inv_tau, pt, w); break;
    }
  } else switch (d) {
    case 16: hipLaunchKernelGGL(nce_bwd_tiles_kernel<4>, grid, dim3(256), lds, s, b, inv_tau, pt, w); break;
    case 32: hipLaunchKernelGGL(nce_bwd_tiles_kernel<8>, grid, dim3(256), lds, s, b, inv_tau, pt, w); break;
    case 64: hipLaunchKernelGGL(nce_bwd_tiles_kernel<16>, grid, dim3(256), lds, s, b, inv_tau, pt, w); break;
    default: hipLaunchKernelGGL(nce_bwd_tiles_kernel<32>, grid, dim3(256), lds, s, b, inv_tau, pt, w); break;
  }
  FR_LAUNCH_CHECK();
  const unsigned nb = (unsigned)std::min<int64_t>(fr::ceil_div((int64_t)n_views * b, 4), 4096);
  hipLaunchKernelGGL(nce_bwd_finalize_kernel, dim3(nb), dim3(256), 0, s, v, n_views, b, d, inv_tau, js, g, d_gscale,
                     pt, w);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

// one pair over a contiguous H [2b, d]: the two halves as views 0 and 1
extern "C" int64_t fr_infonce_workspace(int64_t b) {
  if (b <= 0) return 0;
  return nce_ws_bytes(2, b, 128, 1);
}

extern "C" int fr_infonce_fwd(const float* d_H, int64_t b, int d, float tau, float* d_out,
                              void* d_workspace, int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(d_H && d_out && fr::aligned16(d_H) && b >= 1 && (b * d) % 4 == 0, "H/out null or unaligned");
  const float* views[2] = {d_H, d_H + b * d};
  const int32_t pair[2] = {0, 1};
  return nce_fwd_impl(views, 2, b, d, pair, 1, tau, 1.f, d_out, nullptr, d_workspace, workspace_bytes, stream);
}

extern "C" int fr_infonce_bwd(const float* d_H, int64_t b, int d, float tau, float g,
                              const float* d_gscale, float* d_dH, void* d_workspace,
                              int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(d_H && d_dH && fr::aligned16(d_H) && fr::aligned16(d_dH) && b >= 1 && (b * d) % 4 == 0,
             "H/dH null or unaligned");
  const float* views[2] = {d_H, d_H + b * d};
  float* dviews[2] = {d_dH, d_dH + b * d};
  const int32_t pair[2] = {0, 1};
  return fr_infonce_multi_bwd(views, 2, b, d, pair, 1, tau, g, d_gscale, dviews, d_workspace, workspace_bytes, stream);
}

// ------------------------------------------------------------------------------------------------
// CLUSSL's view sum and SSL gathers in one launch (pricai_modelx.py:227-263: item_emb = ingre +
// image + text, and the three views at the batch items): total = ((v0 + v1) + v2) in torch's add
// order (bit-identical), g_k[j] = v_k[ids[j]].  HBM stream: V reads + 1 write of the tables plus the
// gathered rows; one float4 per thread and iteration, grid-strided.  Ids outside [0, n) gather zeros.
// ------------------------------------------------------------------------------------------------
namespace {
struct ViewsSG {
  const float4* v[4];
  float4* g[4];
};

__global__ __launch_bounds__(256) void views_sum_gather_kernel(ViewsSG a, int V, int64_t n, int d4,
                                                               const int64_t* __restrict__ ids, int64_t m,
                                                               float4* __restrict__ total) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  const int64_t t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n4 = n * d4;
  for (int64_t i = t0; i < n4; i += stride) {
    float4 s = a.v[0][i];
    for (int k = 1; k < V; ++k) {
      const float4 x = a.v[k][i];
      s.x += x.x;
      s.y += x.y;
      s.z += x.z;
      s.w += x.w;
    }
    total[i] = s;
  }
  const int64_t m4 = m * d4;
  for (int64_t i = t0; i < m4 * V; i += stride) {
    const int k = (int)(i / m4);
    const int64_t j = i - (int64_t)k * m4, row = j / d4, c = j - row * d4;
    const int64_t r = ids[row];
    a.g[k][j] = (r >= 0 && r < n) ? a.v[k][r * d4 + c] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}
// backward, phase 1: dv_k = g_sum for every k (one read of g_sum, V writes)
__global__ __launch_bounds__(256) void views_bcast_kernel(ViewsSG a, int V, int64_t n4, const float4* __restrict__ gs) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n4; i += stride) {
    const float4 x = gs ? gs[i] : make_float4(0.f, 0.f, 0.f, 0.f);
    for (int k = 0; k < V; ++k) a.g[k][i] = x;
  }
}

// phase 2, default: one wave per id, lane = column, one float atomic wave-instruction per view over the
// 256 contiguous bytes of the row (the memory-side atomic units' full-rate shape); duplicate ids add
// in hardware order (as torch's index_add_)
__global__ __launch_bounds__(256) void views_scatter_atomic_kernel(ViewsSG a, int V, int64_t n, int d,
                                                                   const int64_t* __restrict__ ids, int64_t m) {
  const int lane = threadIdx.x & 63;
  const int64_t j = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (j >= m) return;
  const int64_t r = ids[j];
  if (r < 0 || r >= n) return;
  for (int c = lane; c < d; c += 64)
    for (int k = 0; k < V; ++k)
      atomicAdd(reinterpret_cast<float*>(a.g[k]) + r * d + c, reinterpret_cast<const float*>(a.v[k])[j * d + c]);
}

// deterministic mode, phase 0 (one workgroup, before phase 1 in stream order): the (id, j) keys of all ids sorted in LDS
// (bitonic network) -> keys[m].  key = (row + 1) << jbits | j; ids outside the table get row -1.
constexpr int VSG_MAX_IDS = 8192;

__global__ __launch_bounds__(1024) void views_sort_ids_kernel(const int64_t* __restrict__ ids, int64_t m, int64_t n,
                                                              int mp2, int jbits, uint64_t* __restrict__ keys) {
  __shared__ uint64_t key[VSG_MAX_IDS];
  for (int t = threadIdx.x; t < mp2; t += blockDim.x) {
    uint64_t k = ~0ull;  // padding keys sort last
    if (t < m) {
      const int64_t r = ids[t];
      k = (r >= 0 && r < n) ? ((uint64_t)(r + 1) << jbits) | (uint64_t)t : (uint64_t)t;
    }
    key[t] = k;
  }
  __syncthreads();
  for (int size = 2; size <= mp2; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int t = threadIdx.x; t < (mp2 >> 1); t += blockDim.x) {
        const int lo = 2 * t - (t & (stride - 1)), hi = lo + stride;
        const bool up = (lo & size) == 0;
        const uint64_t x = key[lo], y = key[hi];
        if ((x > y) == up) { key[lo] = y; key[hi] = x; }
      }
      __syncthreads();
    }
  for (int t = threadIdx.x; t < m; t += blockDim.x) keys[t] = key[t];
}

// phase 2: every distinct id adds, for every view k, the sum of g_k over its occurrences in increasing
// j -- each touched row written by one 16-lane group (the head of its run in the sorted keys), in a
// fixed order (deterministic, no atomics); one float4 column per lane
__global__ __launch_bounds__(256) void views_scatter_owner_kernel(ViewsSG a, int V, int d4,
                                                                  const uint64_t* __restrict__ keys, int64_t m,
                                                                  int jbits) {
  const uint64_t jmask = (1ull << jbits) - 1;
  const int q = threadIdx.x & 15;
  const int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  if (i >= m) return;
  const uint64_t rid = keys[i] >> jbits;
  if (rid == 0) return;                              // id outside the table
  if (i > 0 && (keys[i - 1] >> jbits) == rid) return;  // not the head of its run
  const int64_t r = (int64_t)rid - 1;
  int64_t e = i + 1;
  while (e < m && (keys[e] >> jbits) == rid) ++e;
  for (int c = q; c < d4; c += 16) {
    float4 acc[4];
    for (int k = 0; k < V; ++k) acc[k] = a.g[k][r * d4 + c];
    for (int64_t t = i; t < e; ++t) {
      const int64_t jj = (int64_t)(keys[t] & jmask);
      for (int k = 0; k < V; ++k) {
        const float4 x = a.v[k][jj * d4 + c];
        acc[k].x += x.x;
        acc[k].y += x.y;
        acc[k].z += x.z;
        acc[k].w += x.w;
      }
    }
    for (int k = 0; k < V; ++k) a.g[k][r * d4 + c] = acc[k];
  }
}
}  // namespace

extern "C" int64_t fr_views_sum_gather_bwd_workspace(int64_t m) { return m > 0 ? (m * 8 + 255) / 256 * 256 : 0; }

extern "C" int fr_views_sum_gather_bwd(const float* d_gsum, const float* const* d_grows, int n_views, int64_t n,
                                       int d, const int64_t* d_ids, int64_t m, float* const* d_dviews,
                                       int deterministic, void* d_workspace, int64_t workspace_bytes,
                                       void* stream) {
  FR_REQUIRE(d_dviews && n_views >= 1 && n_views <= 4 && n >= 1 && d >= 4 && d % 4 == 0 && m >= 0 &&
                 m <= VSG_MAX_IDS && (m == 0 || (d_ids && d_grows)) && (!d_gsum || fr::aligned16(d_gsum)),
             "views_sum_gather_bwd: bad arguments (m <= 8192)");
  FR_REQUIRE(!deterministic || m == 0 || (d_workspace && workspace_bytes >= m * 8 && fr::aligned16(d_workspace)),
             "views_sum_gather_bwd: workspace too small");
  ViewsSG a{};
  for (int k = 0; k < n_views; ++k) {
    FR_REQUIRE(d_dviews[k] && fr::aligned16(d_dviews[k]) && (m == 0 || (d_grows[k] && fr::aligned16(d_grows[k]))),
               "views_sum_gather_bwd: gradient table null or unaligned");
    a.g[k] = reinterpret_cast<float4*>(d_dviews[k]);
    a.v[k] = m ? reinterpret_cast<const float4*>(d_grows[k]) : nullptr;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int d4 = d / 4;
  int mp2 = 2, jbits = 1;
  while (mp2 < m) { mp2 <<= 1; ++jbits; }
  FR_REQUIRE(n < (int64_t(1) << (62 - jbits)), "views_sum_gather_bwd: table too large for the sort keys");
  uint64_t* keys = reinterpret_cast<uint64_t*>(d_workspace);
  if (m > 0 && deterministic) {
    hipLaunchKernelGGL(views_sort_ids_kernel, dim3(1), dim3(1024), 0, s, d_ids, m, n, mp2, jbits, keys);
    FR_LAUNCH_CHECK();
  }
  const int64_t work = n * d4;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(work, 256), (int64_t)fr::kNumCU * 16));
  hipLaunchKernelGGL(views_bcast_kernel, dim3((unsigned)blocks), dim3(256), 0, s, a, n_views, work,
                     reinterpret_cast<const float4*>(d_gsum));
  FR_LAUNCH_CHECK();
  if (m > 0 && deterministic) {
    hipLaunchKernelGGL(views_scatter_owner_kernel, dim3((unsigned)fr::ceil_div(m, 16)), dim3(256), 0, s, a, n_views,
                       d4, keys, m, jbits);
    FR_LAUNCH_CHECK();
  } else if (m > 0) {
    hipLaunchKernelGGL(views_scatter_atomic_kernel, dim3((unsigned)fr::ceil_div(m, 4)), dim3(256), 0, s, a, n_views, n,
                       d, d_ids, m);
    FR_LAUNCH_CHECK();
  }
  return FR_OK;
}

extern "C" int fr_views_sum_gather(const float* const* d_views, int n_views, int64_t n, int d,
                                   const int64_t* d_ids, int64_t m, float* d_total, float* const* d_gathered,
                                   void* stream) {
  FR_REQUIRE(d_views && d_gathered && d_total && n_views >= 1 && n_views <= 4 && n >= 1 && d >= 4 && d % 4 == 0 &&
                 m >= 0 && (m == 0 || d_ids) && fr::aligned16(d_total),
             "views_sum_gather: bad arguments");
  ViewsSG a{};
  for (int k = 0; k < n_views; ++k) {
    FR_REQUIRE(d_views[k] && fr::aligned16(d_views[k]) && (m == 0 || (d_gathered[k] && fr::aligned16(d_gathered[k]))),
               "views_sum_gather: view / gathered table null or unaligned");
    a.v[k] = reinterpret_cast<const float4*>(d_views[k]);
    a.g[k] = m ? reinterpret_cast<float4*>(d_gathered[k]) : nullptr;
  }
  const int d4 = d / 4;
  const int64_t work = n * d4;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(work, 256), (int64_t)fr::kNumCU * 16));
  hipLaunchKernelGGL(views_sum_gather_kernel, dim3((unsigned)blocks), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), a, n_views, n, d4, d_ids, m,
                     reinterpret_cast<float4*>(d_total));
  FR_LAUNCH_CHECK();
  return FR_OK;
}
