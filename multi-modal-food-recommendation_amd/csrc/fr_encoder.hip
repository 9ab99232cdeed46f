// Fused post-norm Transformer encoder layer (training forward + backward), gfx950.
//
// HealthRec's ingredient encoder (FoodRec/models/cikm_model.py:33-35, used at :232-238) is
// nn.TransformerEncoder over nn.TransformerEncoderLayer(d_model=64, nhead=2, dim_feedforward=256,
// dropout=p, activation=gelu), post-norm, run on 2B sequences of 20 ingredient tokens:
//
//   qkv = x W_in^T + b_in                      ctx = dropout(softmax(q k^T / sqrt(32) + mask)) v
//   x1  = LN1(x + dropout1(ctx W_o^T + b_o))   x2  = LN2(x1 + dropout2(dropout(act(x1 W1^T + b1)) W2^T + b2))
//
// torch runs this as ~20 forward and ~35 backward kernels per layer over [20480 x <=256] tensors,
// each a few microseconds of launch-bound work.  Here one workgroup owns G = 80/L whole sequences
// (80 token rows = five 16-row MFMA tiles) and keeps every intermediate in LDS: one forward and one
// backward launch per layer, plus one ordered reduction of the per-workgroup weight-gradient partials.
// 8 waves per workgroup (2 per SIMD): the VALU phases between the GEMMs (attention, LayerNorm, GELU,
// dropout hash) are latency-bound, and a second wave per SIMD is what hides that latency.
//
// * GEMMs on v_mfma_f32_16x16x4_f32 (exact f32 in / f32 accumulate, the f32 vector rate).  The k
//   order inside a 16-wide chunk is permuted so each lane feeds four MFMAs from one float4 of A and
//   one float4 of B (lane group h holds k = 4h..4h+3 of the chunk).
// * Attention (20 x 20 per head) on the VALU: two adjacent lanes per (sequence, head, query row), each
//   owning 16 of the head's 32 dimensions; partial dot products are combined by a DPP swap and the
//   score row stays in registers.
// * Dropout masks from a counter-based hash of (seed, step counter, site, element): the backward
//   regenerates them instead of storing them; the step counter is read on the device, so a captured
//   HIP graph draws fresh masks on every replay.
// * Weight/bias gradients: each workgroup writes its partial sums; fr_encoder_bwd sums them in
//   workgroup order (deterministic).
#include "fr_common.h"

namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int E = 64, HEADS = 2, HD = 32, FF = 256, QKV = 3 * E;
constexpr int ROWS = 80;                            // token rows per workgroup (5 MFMA row tiles)
constexpr int RT = ROWS / 16;
constexpr int LD_E = E + 4, LD_QKV = QKV + 4, LD_FF = FF + 4;
constexpr int NT = 512;                             // threads per workgroup: 8 waves, 2 per SIMD
// Wave w owns output column tiles by its SIMD slot sg = w & 3 (as a 4-wave layout would) and, within
// the SIMD, one of two row-tile ranges: hf = w >> 2 takes tiles [0, RT0) or [RT0, RT).  The two waves
// of a SIMD share its MFMA pipe and hide each other's LDS / global / transcendental latency.
constexpr int RT0 = (RT + 1) / 2;
constexpr int BUF_D = 6400;                         // attention p'/ds buffers (2*G*H*L*L) and scratch
// s_setprio 1 for the second-dispatched half (waves 4-7): the arbitration loser of every segment
// otherwise (MI355X_MICROARCH.md, two waves per SIMD, item 4)
constexpr int kEncPrio = 0;  // measured (round 6): bwd 70.6 vs 69.6 us alone -- off

// gradient partial sections (floats): the flat gradient buffer fr_encoder_bwd writes has the same
// offsets; inside the partials the four weight sections use the fragment layout (wgrad_tiles)
constexpr int OFF_WIN = 0, OFF_BIN = OFF_WIN + QKV * E, OFF_WO = OFF_BIN + QKV, OFF_BO = OFF_WO + E * E,
              OFF_G1 = OFF_BO + E, OFF_BE1 = OFF_G1 + E, OFF_W1 = OFF_BE1 + E, OFF_B1 = OFF_W1 + FF * E,
              OFF_W2 = OFF_B1 + FF, OFF_B2 = OFF_W2 + E * FF, OFF_G2 = OFF_B2 + E, OFF_BE2 = OFF_G2 + E,
              NPART = OFF_BE2 + E;
static_assert(NPART % 4 == 0, "partials are reduced as float4");

struct Weights {
  const float *w_in, *b_in, *w_o, *b_o, *g1, *be1, *w1, *b1, *w2, *b2, *g2, *be2;
  float eps1, eps2;
  uint32_t thr[4];     // dropout: element kept iff its 16-bit hash half >= thr  (sites: attn, out-proj, ff-act, ff-out)
  float scale[4];      // 1 / (1 - p)
  uint64_t seed;
  int gelu;
};

struct FwdArgs {
  Weights w;
  const float* x;      // [NS, L, 64]
  const float* mask;   // [NS, L] additive key mask (0 / -inf) or null
  int64_t ns;
  const int64_t* counter;
  int64_t* seed_out;   // counter value used (read back by the backward)
  float* out;          // [NS, L, 64]
  // saved for the backward: fact = dropout(act(pre)), dact = keep * scale * act'(pre)  [T, 256];
  // st: (mean, rstd) per token
  float *qkv, *ctx, *y1, *fact, *dact, *y2, *st1, *st2;
};

struct BwdArgs {
  Weights w;
  const float* dout;
  const float* x;
  const float* mask;
  int64_t ns;
  const int64_t* seed_in;
  const float *qkv, *ctx, *y1, *fact, *dact, *y2, *st1, *st2;
  float* dx;
  float* part;         // [n_wg, NPART]
  // optional: another backward call's partials ([n_wg, NPART], the same n_wg) summed into prev_grad
  // by this launch (every workgroup a slice of the columns, partials in workgroup order) -- the
  // previous layer's ordered reduction folded into this one's launch
  const float* prev_part;
  float* prev_grad;
};

// Phase timestamps (diagnostics, off unless fr_encoder_profile(1, ...)): workgroup 0's thread 0
// records s_memtime (shader clock) after each barrier of the forward (kind 0) / backward (kind 1).
__device__ int g_prof_on;
__device__ unsigned long long g_prof[2][32];
#define FR_MARK(kind, n)                                                       \
  do {                                                                         \
    if (prof && threadIdx.x == 0) g_prof[kind][n] = __builtin_amdgcn_s_memtime(); \
  } while (0)

// the same stamp from inside a device function (prof: the kernel's flag, workgroup 0; thread 0)
__device__ __forceinline__ void fr_mark(bool prof, int kind, int n) {
  if (prof && threadIdx.x == 0) g_prof[kind][n] = __builtin_amdgcn_s_memtime();
}

// keep the loads issued above this point above it (no instruction moves across): a prefetch the
// compiler would sink to its use otherwise
#define FR_SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)

// this thread's wave index as a scalar: the compiler cannot prove threadIdx.x >> 6 wave-uniform, and
// branches on it (job tables) must be scalar branches, not exec-masked ones
__device__ __forceinline__ int wave_id() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// per-(step, site) 32-bit hash keys: hi32(mix64(mix64(seed ^ mix64(counter + C)) + site + 1))
struct SiteKeys {
  uint32_t k[4];
};

__device__ __forceinline__ SiteKeys site_keys(uint64_t seed, int64_t counter) {
  const uint64_t key = mix64(seed ^ mix64((uint64_t)counter + 0x632BE59BD9B4E019ull));
  SiteKeys s;
#pragma unroll
  for (int i = 0; i < 4; ++i) s.k[i] = (uint32_t)(mix64(key + (uint64_t)(i + 1)) >> 32);
  return s;
}

// Dropout keep test.  Elements 2m and 2m+1 of a site share one 32-bit hash of m (Weyl step + the
// lowbias32 finalizer; its three 32-bit multiplies are quarter-rate): element e is kept iff the
// (e & 1) half of pair_hash(k, e >> 1) is >= thr = floor(p * 2^16).
__device__ __forceinline__ uint32_t pair_hash(uint32_t ks, uint32_t pair) {
  uint32_t x = pair * 0x9E3779B1u + ks;
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ bool half_keep(uint32_t h, uint32_t odd, uint32_t thr) {
  return (odd ? (h >> 16) : (h & 0xFFFFu)) >= thr;
}

__device__ __forceinline__ bool keep(uint32_t ks, uint32_t idx, uint32_t thr) {
  if (thr == 0u) return true;
  return half_keep(pair_hash(ks, idx >> 1), idx & 1u, thr);
}

__device__ __forceinline__ uint32_t pair_swap_u(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}

// Keep bits of the 4 elements (rows row0 + q, q = 0..3; column col) a lane holds in an MFMA output
// fragment of a [*, W] site (W even).  Adjacent columns are lanes 2k, 2k+1 and share each row's
// pair hash: the even lane hashes rows 0, 1, the odd lane rows 2, 3, and they swap (2 hashes per
// lane instead of 4).  Every lane of the wave must be active.
__device__ __forceinline__ uint32_t frag_keep4(uint32_t ks, int64_t tok_row0, int W, int col, uint32_t thr) {
  if (thr == 0u) return 0xFu;
  const uint32_t odd = col & 1;
  const uint32_t e0 = (uint32_t)((tok_row0 + 2 * odd) * W + col);
  const uint32_t ha = pair_hash(ks, e0 >> 1), hb = pair_hash(ks, (e0 + W) >> 1);
  const uint32_t oa = pair_swap_u(ha), ob = pair_swap_u(hb);
  const uint32_t h0 = odd ? oa : ha, h1 = odd ? ob : hb, h2 = odd ? ha : oa, h3 = odd ? hb : ob;
  return (uint32_t)half_keep(h0, odd, thr) | ((uint32_t)half_keep(h1, odd, thr) << 1) |
         ((uint32_t)half_keep(h2, odd, thr) << 2) | ((uint32_t)half_keep(h3, odd, thr) << 3);
}

// act(v) and act'(v) of two values at once: ReLU, or GELU(v) = v * Phi(v) (torch's exact-erf form).
// Phi and phi share one exp(-v^2/2); erf from Abramowitz & Stegun 7.1.26 (|err| <= 1.5e-7), with
// Phi(-|v|) = q computed directly (no cancellation for negative v).  The polynomial and products run
// on packed-fp32 VALU ops (v_pk_fma_f32 / v_pk_mul_f32), exp and rcp per element.
__device__ __forceinline__ void act_fwd_grad2(f32x2 v, int gelu, f32x2& act, f32x2& grad) {
  if (!gelu) {
    act = f32x2{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f)};
    grad = f32x2{v.x > 0.f ? 1.f : 0.f, v.y > 0.f ? 1.f : 0.f};
    return;
  }
  const f32x2 a = f32x2{fabsf(v.x), fabsf(v.y)} * 0.70710678118654752f;
  const f32x2 aa = a * a;
  const f32x2 e = f32x2{__expf(-aa.x), __expf(-aa.y)};
  const f32x2 den = __builtin_elementwise_fma(a, f32x2{0.3275911f, 0.3275911f}, f32x2{1.f, 1.f});
  const f32x2 t = f32x2{__builtin_amdgcn_rcpf(den.x), __builtin_amdgcn_rcpf(den.y)};
  f32x2 poly = __builtin_elementwise_fma(t, f32x2{1.061405429f, 1.061405429f}, f32x2{-1.453152027f, -1.453152027f});
  poly = __builtin_elementwise_fma(t, poly, f32x2{1.421413741f, 1.421413741f});
  poly = __builtin_elementwise_fma(t, poly, f32x2{-0.284496736f, -0.284496736f});
  poly = __builtin_elementwise_fma(t, poly, f32x2{0.254829592f, 0.254829592f});
  poly = t * poly;
  const f32x2 q = 0.5f * poly * e;
  const f32x2 cdf = f32x2{v.x >= 0.f ? 1.f - q.x : q.x, v.y >= 0.f ? 1.f - q.y : q.y};
  act = v * cdf;
  grad = __builtin_elementwise_fma(v, e * 0.39894228040143268f, cdf);
}

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float4 lds4(const float* p) { return *reinterpret_cast<const float4*>(p); }
__device__ __forceinline__ float comp(const float4& v, int m) {
  return m == 0 ? v.x : (m == 1 ? v.y : (m == 2 ? v.z : v.w));
}

constexpr float kScale = 0.17677669529663688f;  // 1 / sqrt(HD)


// offset of lane's float4 (4 rows of one column) of FF1 column tile (SIMD slot sg, c), row tile r, in
// the fragment-layout dact buffer [n_wg][ROWS * FF]
__device__ __forceinline__ int64_t dact_frag(int wg, int sg, int c, int r, int lane) {
  return (int64_t)wg * (ROWS * FF) + ((((sg * 4 + c) * RT + r) * 64 + lane) << 2);
}


// acc[r][c] (+)= A[rows of tiles R0..R0+NR-1] (LDS, lda) . W^T, W [N x K] row-major in global; column
// tiles c0..c0+NC-1; acc rows beyond NR are untouched.  The next chunk's W fragment is loaded before
// the current chunk's MFMAs (register double buffer).
template <int NC, int K, int R0, int NR, int NA>
__device__ __forceinline__ void gemm_xwt(const float* A, int lda, const float* __restrict__ W, int c0,
                                         f32x4 (&acc)[NA][NC]) {
  static_assert(NR <= NA, "accumulator rows");
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4;
  float4 bn[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) bn[c] = *reinterpret_cast<const float4*>(W + (int64_t)(16 * (c0 + c) + i) * K + 4 * h);
#pragma unroll 4
  for (int kc = 0; kc < K / 16; ++kc) {
    float4 a[NR], b[NC];
#pragma unroll
    for (int c = 0; c < NC; ++c) b[c] = bn[c];
    if (kc + 1 < K / 16) {
#pragma unroll
      for (int c = 0; c < NC; ++c)
        bn[c] = *reinterpret_cast<const float4*>(W + (int64_t)(16 * (c0 + c) + i) * K + (kc + 1) * 16 + 4 * h);
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) a[r] = lds4(A + (16 * (R0 + r) + i) * lda + kc * 16 + 4 * h);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[r][c] = mfma4(comp(a[r], m), comp(b[c], m), acc[r][c]);
  }
}

// acc[r][c] (+)= Y[rows of tiles R0..R0+NR-1] (LDS, ldy) . W, W [N x KO] row-major in global; output
// column tiles c0..
template <int NC, int N, int KO, int R0, int NR, int NA>
__device__ __forceinline__ void gemm_yw(const float* Y, int ldy, const float* __restrict__ W, int c0,
                                        f32x4 (&acc)[NA][NC]) {
  static_assert(NR <= NA, "accumulator rows");
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4;
  float bn[4][NC];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int c = 0; c < NC; ++c) bn[m][c] = W[(int64_t)(4 * h + m) * KO + 16 * (c0 + c) + i];
#pragma unroll 4
  for (int nc = 0; nc < N / 16; ++nc) {
    float4 a[NR];
    float b[4][NC];
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < NC; ++c) b[m][c] = bn[m][c];
    if (nc + 1 < N / 16) {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int c = 0; c < NC; ++c) bn[m][c] = W[(int64_t)((nc + 1) * 16 + 4 * h + m) * KO + 16 * (c0 + c) + i];
    }
#pragma unroll
    for (int r = 0; r < NR; ++r) a[r] = lds4(Y + (16 * (R0 + r) + i) * ldy + nc * 16 + 4 * h);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[r][c] = mfma4(comp(a[r], m), b[m][c], acc[r][c]);
  }
}

template <int NA, int NC>
__device__ __forceinline__ void zero_acc(f32x4 (&acc)[NA][NC]) {
#pragma unroll
  for (int r = 0; r < NA; ++r)
#pragma unroll
    for (int c = 0; c < NC; ++c) acc[r][c] = f32x4{0.f, 0.f, 0.f, 0.f};
}

// this wave's row tiles: [0, RT0) for hf == 0, [RT0, RT) for hf == 1 (wave-uniform)
#define FR_GEMM_XWT(NC, K, A, lda, W, c0, acc)                     \
  do {                                                             \
    if (hf == 0) gemm_xwt<NC, K, 0, RT0>(A, lda, W, c0, acc);      \
    else gemm_xwt<NC, K, RT0, RT - RT0>(A, lda, W, c0, acc);       \
  } while (0)
#define FR_GEMM_YW(NC, N, KO, Y, ldy, W, c0, acc)                  \
  do {                                                             \
    if (hf == 0) gemm_yw<NC, N, KO, 0, RT0>(Y, ldy, W, c0, acc);   \
    else gemm_yw<NC, N, KO, RT0, RT - RT0>(Y, ldy, W, c0, acc);    \
  } while (0)

// max / sum over the 4 lane rows (lanes l, l ^ 16, l ^ 32, l ^ 48), the same value in every lane
__device__ __forceinline__ float rows4_max(float v) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}
__device__ __forceinline__ float rows4_sum(float v) { return swap32_sum(swap16_sum(v)); }

// Weight-gradient partials are stored in the MFMA fragment layout of their [N x K] section (16 x 16
// tile (nt, kt) at float (nt * K / 16 + kt) * 256, lane l = 16 h + i's float4 at 4 l holding rows
// 16 nt + 4 h + q, column 16 kt + i): one coalesced 1 KiB float4 store per wave and tile instead of
// four 4-byte stores; the ordered reduction maps each float4 back to the gradient's row-major layout
// (grad_store4).  Bias / LayerNorm partials are plain.
struct FragSec {
  int base, K;
};
constexpr FragSec kFragSecs[4] = {{OFF_WIN, E}, {OFF_WO, E}, {OFF_W1, E}, {OFF_W2, FF}};
static_assert(OFF_WIN % 4 == 0 && OFF_WO % 4 == 0 && OFF_W1 % 4 == 0 && OFF_W2 % 4 == 0, "float4 sections");

// grad (row-major flat gradient) <- the reduced float4 c of the partial layout
__device__ __forceinline__ void grad_store4(float* __restrict__ grad, int c, float4 t) {
  const int f = 4 * c;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const FragSec sec = kFragSecs[k];
    const int n = k == 0 ? QKV : (k == 1 ? E : (k == 2 ? FF : E));
    if (f >= sec.base && f < sec.base + n * sec.K) {
      const int lf = f - sec.base, tile = lf >> 8, lane = (lf & 255) >> 2;
      const int nt = tile / (sec.K / 16), kt = tile % (sec.K / 16);
      const int row = 16 * nt + 4 * (lane >> 4), col = 16 * kt + (lane & 15);
      float* g = grad + sec.base + row * sec.K + col;
      g[0] = t.x;
      g[sec.K] = t.y;
      g[2 * sec.K] = t.z;
      g[3 * sec.K] = t.w;
      return;
    }
  }
  reinterpret_cast<float4*>(grad)[c] = t;
}

// weight-gradient partial  P[n][k] = sum_t Y[t][n] X[t][k] over the 80 rows; this wave owns
// n-tiles n0..n0+NN-1 x k-tiles k0..k0+NK-1; written to its section ``part`` ([N x K]) in the
// fragment layout above.  The wave reads every row of its Y columns as the MFMA A operand, so the
// bias gradient (the column sums of Y) comes with it: with ``bias`` set, the wave's columns' sums
// (lane (i, h): rows 4h..4h+3 of each 16-row tile in order, then the four lane rows added,
// rows4_sum) go to bias[16 (n0 + a) + i] -- VALU adds between the MFMAs instead of a separate pass.
template <int NN, int NK>
__device__ __forceinline__ void wgrad_tiles(const float* Y, int ldy, const float* X, int ldx, int n0, int k0,
                                            float* __restrict__ part, int K, float* __restrict__ bias = nullptr) {
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4;
  f32x4 acc[NN][NK];
  float cs[NN];
#pragma unroll
  for (int a = 0; a < NN; ++a) {
    cs[a] = 0.f;
#pragma unroll
    for (int b = 0; b < NK; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
#pragma unroll
  for (int tc = 0; tc < RT; ++tc) {
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int t = tc * 16 + 4 * h + m;
      float ya[NN], xb[NK];
#pragma unroll
      for (int a = 0; a < NN; ++a) ya[a] = Y[t * ldy + 16 * (n0 + a) + i];
#pragma unroll
      for (int b = 0; b < NK; ++b) xb[b] = X[t * ldx + 16 * (k0 + b) + i];
#pragma unroll
      for (int a = 0; a < NN; ++a) {
        cs[a] += ya[a];
#pragma unroll
        for (int b = 0; b < NK; ++b) acc[a][b] = mfma4(ya[a], xb[b], acc[a][b]);
      }
    }
  }
#pragma unroll
  for (int a = 0; a < NN; ++a)
#pragma unroll
    for (int b = 0; b < NK; ++b)
      *reinterpret_cast<float4*>(part + ((n0 + a) * (K / 16) + k0 + b) * 256 + 4 * lane) =
          make_float4(acc[a][b][0], acc[a][b][1], acc[a][b][2], acc[a][b][3]);
  if (bias) {
#pragma unroll
    for (int a = 0; a < NN; ++a) {
      const float t = rows4_sum(cs[a]);
      if (h == 0) bias[16 * (n0 + a) + i] = t;
    }
  }
}

// zero a [rows x cols] LDS region (cols % 4 == 0)
__device__ __forceinline__ void lds_zero(float* p, int ld, int rows, int cols) {
  const int per = cols / 4;
  for (int e = threadIdx.x; e < rows * per; e += NT)
    *reinterpret_cast<float4*>(p + (e / per) * ld + 4 * (e % per)) = make_float4(0.f, 0.f, 0.f, 0.f);
}

// load rows [0, tv) of a [*, COLS] global tensor into LDS (ld), zero rows [tv, 80).  All loads of a
// thread are issued before the first LDS store (unconditional addresses, rows clamped), so the
// copy costs one memory latency, not one per row.
template <int COLS>
__device__ __forceinline__ void lds_load(float* p, int ld, const float* __restrict__ g, int tv) {
  constexpr int PER = COLS / 4, TOT = ROWS * PER, ITER = (TOT + NT - 1) / NT;
  float4 v[ITER];
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int e = min((int)threadIdx.x + k * NT, TOT - 1), r = e / PER, c4 = e % PER;
    v[k] = *reinterpret_cast<const float4*>(g + (int64_t)min(r, tv - 1) * COLS + 4 * c4);
  }
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int e = threadIdx.x + k * NT, r = e / PER, c4 = e % PER;
    if (TOT % NT == 0 || e < TOT)
      *reinterpret_cast<float4*>(p + r * ld + 4 * c4) = r < tv ? v[k] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// store rows [0, tv) of an LDS tile (ld) to a [*, COLS] global tensor, float4 per thread
template <int COLS>
__device__ __forceinline__ void lds_store(const float* p, int ld, float* __restrict__ g, int tv) {
  constexpr int PER = COLS / 4, TOT = ROWS * PER, ITER = (TOT + NT - 1) / NT;
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int e = threadIdx.x + k * NT, r = e / PER, c4 = e % PER;
    if ((TOT % NT == 0 || e < TOT) && r < tv)
      *reinterpret_cast<float4*>(g + (int64_t)r * COLS + 4 * c4) = lds4(p + r * ld + 4 * c4);
  }
}

// A global -> LDS tile copy split in two: pf_issue puts this thread's loads in flight (rows [0, tv) of a
// [*, COLS] tensor, rows clamped), pf_commit writes them to LDS (zero rows [tv, 80)).  Loads retire in
// issue order (vmcnt), so a prefetch overlaps the work between the two calls only when no load issued
// after it is waited for in between: the backward issues each phase's global operands (weight
// fragments included) BEFORE the prefetch that must survive that phase.
template <int COLS>
struct TilePf {
  static constexpr int PER = COLS / 4, TOT = ROWS * PER, ITER = (TOT + NT - 1) / NT;
  float4 v[ITER];
};

template <int COLS>
__device__ __forceinline__ void pf_issue(TilePf<COLS>& pf, const float* __restrict__ g, int tv) {
  using P = TilePf<COLS>;
#pragma unroll
  for (int k = 0; k < P::ITER; ++k) {
    const int e = min((int)threadIdx.x + k * NT, P::TOT - 1), r = e / P::PER, c4 = e % P::PER;
    pf.v[k] = *reinterpret_cast<const float4*>(g + (int64_t)min(r, tv - 1) * COLS + 4 * c4);
  }
}

template <int COLS>
__device__ __forceinline__ void pf_commit(const TilePf<COLS>& pf, float* p, int ld, int tv) {
  using P = TilePf<COLS>;
#pragma unroll
  for (int k = 0; k < P::ITER; ++k) {
    const int e = threadIdx.x + k * NT, r = e / P::PER, c4 = e % P::PER;
    if (P::TOT % NT == 0 || e < P::TOT)
      *reinterpret_cast<float4*>(p + r * ld + 4 * c4) = r < tv ? pf.v[k] : make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// the per-row operands of a LayerNorm backward (or of the LN1 recompute) for this thread's rows
// (16 lanes x float4 per row, rows grp, grp + 32, grp + 64): saved input rows, (mean, rstd), gamma
// (and beta), issued ahead of their use
struct LnPf {
  static constexpr int NG = NT / 16, NR = (ROWS + NG - 1) / NG;
  float4 yv[NR];
  float2 sv[NR];
  float4 gg, bb;
};

__device__ __forceinline__ void ln_issue(LnPf& pf, const float* __restrict__ y, const float* __restrict__ st,
                                         const float* __restrict__ g, const float* __restrict__ b, int tv) {
  const int grp = threadIdx.x >> 4, l = threadIdx.x & 15;
  pf.gg = *reinterpret_cast<const float4*>(g + 4 * l);
  if (b) pf.bb = *reinterpret_cast<const float4*>(b + 4 * l);
#pragma unroll
  for (int k = 0; k < LnPf::NR; ++k) {
    const int r = min(grp + k * LnPf::NG, tv - 1);
    pf.yv[k] = *reinterpret_cast<const float4*>(y + (int64_t)r * E + 4 * l);
    pf.sv[k] = *reinterpret_cast<const float2*>(st + 2 * r);
  }
}

// the gemm_yw B operand (W [N x KO] row-major, output column tiles c0..c0+NC-1) for every N chunk,
// loaded ahead of the GEMM (gemm_yw_pre)
template <int NC, int N, int KO>
struct YwFrags {
  float b[N / 16][4][NC];
};

template <int NC, int N, int KO>
__device__ __forceinline__ void yw_issue(YwFrags<NC, N, KO>& f, const float* __restrict__ W, int c0) {
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4;
#pragma unroll
  for (int nc = 0; nc < N / 16; ++nc)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < NC; ++c) f.b[nc][m][c] = W[(int64_t)(nc * 16 + 4 * h + m) * KO + 16 * (c0 + c) + i];
}

// gemm_yw with the B fragments already in registers (no global loads inside)
template <int NC, int N, int KO, int R0, int NR, int NA>
__device__ __forceinline__ void gemm_yw_pre(const float* Y, int ldy, const YwFrags<NC, N, KO>& f,
                                            f32x4 (&acc)[NA][NC]) {
  static_assert(NR <= NA, "accumulator rows");
  const int lane = threadIdx.x & 63, i = lane & 15, h = lane >> 4;
#pragma unroll
  for (int nc = 0; nc < N / 16; ++nc) {
    float4 a[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) a[r] = lds4(Y + (16 * (R0 + r) + i) * ldy + nc * 16 + 4 * h);
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int r = 0; r < NR; ++r)
#pragma unroll
        for (int c = 0; c < NC; ++c) acc[r][c] = mfma4(comp(a[r], m), f.b[nc][m][c], acc[r][c]);
    // (fully unrolled: without a fence every 4 chunks the scheduler hoists all the chunks' LDS
    // reads to the top -- N / 16 x NR float4 live at once -- and spills)
    if ((nc & 3) == 3) FR_SCHED_FENCE();
  }
}

// LayerNorm forward over the 80 rows of an LDS [80 x 64] tile, in place; 16 lanes x float4 per row.
// Saves y (the LN input) and (mean, rstd) for rows < tv.
__device__ __forceinline__ void ln_rows_fwd(float* X, const float* __restrict__ g, const float* __restrict__ b,
                                            float eps, int tv, float* __restrict__ ysave, float* __restrict__ st,
                                            float* __restrict__ gout) {
  const int grp = threadIdx.x >> 4, l = threadIdx.x & 15;
  const float4 gg = *reinterpret_cast<const float4*>(g + 4 * l);
  const float4 bb = *reinterpret_cast<const float4*>(b + 4 * l);
  for (int r = grp; r < ROWS; r += NT / 16) {
    float4 v = lds4(X + r * LD_E + 4 * l);
    const float mean = group_sum<16>(v.x + v.y + v.z + v.w) * (1.f / E);
    const float4 d = make_float4(v.x - mean, v.y - mean, v.z - mean, v.w - mean);
    const float var = group_sum<16>(d.x * d.x + d.y * d.y + d.z * d.z + d.w * d.w) * (1.f / E);
    const float rstd = rsqrtf(var + eps);
    const float4 o = make_float4(fmaf(d.x * rstd, gg.x, bb.x), fmaf(d.y * rstd, gg.y, bb.y),
                                 fmaf(d.z * rstd, gg.z, bb.z), fmaf(d.w * rstd, gg.w, bb.w));
    *reinterpret_cast<float4*>(X + r * LD_E + 4 * l) = o;
    if (r < tv) {
      if (ysave) *reinterpret_cast<float4*>(ysave + (int64_t)r * E + 4 * l) = v;
      if (gout) *reinterpret_cast<float4*>(gout + (int64_t)r * E + 4 * l) = o;
      if (l == 0) {
        st[2 * r] = mean;
        st[2 * r + 1] = rstd;
      }
    }
  }
}

// LayerNorm backward over the rows of an LDS [80 x 64] tile of upstream gradients, in place
// (dY -> dX).  y: saved LN input rows (global), st: (mean, rstd).  dgamma / dbeta partials via the
// scratch (NT / 16 row groups x 64, summed in group order) -> pg / pb.  The residual branch's dropout
// backward is fused in: G = dropout(dX) (site key ks, one pair hash per two adjacent columns, the
// masks drop_pairs draws) written to ``G`` (rows >= tv zero) and its column sums (the branch bias's
// gradient) reduced with dgamma / dbeta -> pbias.
__device__ __forceinline__ void ln_rows_bwd(float* D, const LnPf& pf, int tv, float* scratch,
                                            float* __restrict__ pg, float* __restrict__ pb, float* G, uint32_t ks,
                                            int64_t tok0, uint32_t thr, float scale, float* __restrict__ pbias) {
  const int grp = threadIdx.x >> 4, l = threadIdx.x & 15;
  constexpr int NG = LnPf::NG, NR = LnPf::NR;
  const float4 gg = pf.gg;
  float4 sg = make_float4(0.f, 0.f, 0.f, 0.f), sb = sg, sd = sg;
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    const int r = grp + k * NG;
    if (r >= ROWS) break;
    if (r >= tv) {
      *reinterpret_cast<float4*>(G + r * LD_E + 4 * l) = make_float4(0.f, 0.f, 0.f, 0.f);
      continue;
    }
    const float4 dy = lds4(D + r * LD_E + 4 * l);
    const float4 v = pf.yv[k];
    const float mean = pf.sv[k].x, rstd = pf.sv[k].y;
    const float4 xh = make_float4((v.x - mean) * rstd, (v.y - mean) * rstd, (v.z - mean) * rstd, (v.w - mean) * rstd);
    const float4 gd = make_float4(dy.x * gg.x, dy.y * gg.y, dy.z * gg.z, dy.w * gg.w);
    const float m1 = group_sum<16>(gd.x + gd.y + gd.z + gd.w) * (1.f / E);
    const float m2 = group_sum<16>(gd.x * xh.x + gd.y * xh.y + gd.z * xh.z + gd.w * xh.w) * (1.f / E);
    const float4 dx = make_float4(rstd * (gd.x - m1 - xh.x * m2), rstd * (gd.y - m1 - xh.y * m2),
                                  rstd * (gd.z - m1 - xh.z * m2), rstd * (gd.w - m1 - xh.w * m2));
    *reinterpret_cast<float4*>(D + r * LD_E + 4 * l) = dx;
    float4 o = make_float4(dx.x * scale, dx.y * scale, dx.z * scale, dx.w * scale);
    if (thr != 0u) {
      const uint32_t p0 = (uint32_t)(((tok0 + r) * E + 4 * l) >> 1);
      const uint32_t h0 = pair_hash(ks, p0), h1 = pair_hash(ks, p0 + 1);
      o.x = half_keep(h0, 0, thr) ? o.x : 0.f;
      o.y = half_keep(h0, 1, thr) ? o.y : 0.f;
      o.z = half_keep(h1, 0, thr) ? o.z : 0.f;
      o.w = half_keep(h1, 1, thr) ? o.w : 0.f;
    }
    *reinterpret_cast<float4*>(G + r * LD_E + 4 * l) = o;
    sg = make_float4(fmaf(dy.x, xh.x, sg.x), fmaf(dy.y, xh.y, sg.y), fmaf(dy.z, xh.z, sg.z), fmaf(dy.w, xh.w, sg.w));
    sb = f4_add(sb, dy);
    sd = f4_add(sd, o);
  }
  *reinterpret_cast<float4*>(scratch + grp * E + 4 * l) = sg;
  *reinterpret_cast<float4*>(scratch + NG * E + grp * E + 4 * l) = sb;
  *reinterpret_cast<float4*>(scratch + 2 * NG * E + grp * E + 4 * l) = sd;
  __syncthreads();
  if (threadIdx.x < 3 * E) {
    const int which = threadIdx.x / E, c = threadIdx.x % E;
    float s = 0.f;
#pragma unroll 8
    for (int q = 0; q < NG; ++q) s += scratch[which * NG * E + q * E + c];
    (which == 0 ? pg : (which == 1 ? pb : pbias))[c] = s;
  }
  __syncthreads();
}

// ---------------------------------------------------------------------------------------------
// attention on MFMA (v_mfma_f32_16x16x4_f32)
// ---------------------------------------------------------------------------------------------
// A query tile R (token rows 16R .. 16R+15 of the workgroup) attends only to the keys of the
// sequences its rows belong to: key tiles band_lo(R) .. band_hi(R) (at most 3; 13 of the 25
// 16 x 16 tiles of the 80 x 80 score matrix for L = 20).  Scores are computed transposed,
// S^T = K Q^T: lane (i = l & 15, g4 = l >> 4) holds S^T[key 16c + 4 g4 + q][query 16R + i], so each
// lane owns one query column, the softmax over keys is lane-local over (c, q) plus the 4 lane rows
// (permlane swaps), and the probabilities in registers are directly the A operand of the next
// product over keys (ctx = P'V, dQ = dS K: k = key 4 g4 + q of each 16-key chunk).
template <int L> constexpr int band_lo(int r) { return ((16 * r) / L) * L / 16; }
template <int L> constexpr int band_hi(int r) {
  const int e = ((16 * r + 15) / L + 1) * L - 1;
  return (e > ROWS - 1 ? ROWS - 1 : e) / 16;
}
template <int L> constexpr int band_n(int r) { return band_hi<L>(r) - band_lo<L>(r) + 1; }
template <int L> constexpr int band_slot(int r) {
  int s = 0;
  for (int k = 0; k < r; ++k) s += band_n<L>(k);
  return s;
}
constexpr int TILE_LD = 20;               // scratch score tiles [16 keys][16 queries], rows padded to 20
constexpr int TILE_SZ = 16 * TILE_LD;
constexpr int MAX_SLOTS = 13;             // band tiles of the 5 query tiles, max over supported L
constexpr int DQ_LD = HD + 4;


// S^T tiles of query tile R, head hh: s[c] = K[key tile C0 + c] Q[tile R]^T (unscaled).  ``OFF``:
// column offset of the left operand (E: K for scores; 2E: V for dP'^T = V dctx^T with Bsrc = dctx).
// All operands are read first, then the NC independent accumulation chains are interleaved.
template <int R, int C0, int NC>
__device__ __forceinline__ void tiles_t(const float* RA, int off, const float* Bsrc, int ldb, int hh, f32x4 (&s)[NC]) {
  const int lane = threadIdx.x & 63, i = lane & 15, g4 = lane >> 4;
  float4 a[NC][HD / 16], b[HD / 16];
#pragma unroll
  for (int kc = 0; kc < HD / 16; ++kc) {
    b[kc] = lds4(Bsrc + (16 * R + i) * ldb + hh * HD + 16 * kc + 4 * g4);
#pragma unroll
    for (int c = 0; c < NC; ++c) a[c][kc] = lds4(RA + (16 * (C0 + c) + i) * LD_QKV + off + hh * HD + 16 * kc + 4 * g4);
  }
#pragma unroll
  for (int c = 0; c < NC; ++c) s[c] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int kc = 0; kc < HD / 16; ++kc)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int c = 0; c < NC; ++c) s[c] = mfma4(comp(a[c][kc], m), comp(b[kc], m), s[c]);
}

// out[dt] = X^T-tiles (registers, A operand: k = key 4 g4 + m of each 16-key chunk) times the rows
// of RA at column offset ``off`` (keys of the band, B operand as scalars), both column tiles of the head
template <int C0, int NC>
__device__ __forceinline__ void keys_product(const f32x4 (&x)[NC], const float* RA, int off, int hh,
                                             f32x4 (&out)[HD / 16]) {
  const int lane = threadIdx.x & 63, i = lane & 15, g4 = lane >> 4;
  float b[HD / 16][NC][4];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
    for (int c = 0; c < NC; ++c)
#pragma unroll
      for (int m = 0; m < 4; ++m) b[dt][c][m] = RA[(16 * (C0 + c) + 4 * g4 + m) * LD_QKV + off + hh * HD + 16 * dt + i];
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt) out[dt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int m = 0; m < 4; ++m)
#pragma unroll
      for (int dt = 0; dt < HD / 16; ++dt) out[dt] = mfma4(x[c][m], b[dt][c][m], out[dt]);
}

// e^x as 2^(x log2 e) on v_exp_f32 (exact at -inf -> 0; relative error a few 1e-7 over the
// softmax's range x in [-30, 0], far inside the layer's 2e-5 tolerance)
__device__ __forceinline__ float exp_fast(float x) { return __builtin_amdgcn_exp2f(x * 1.4426950408889634f); }

// scale + key masks (other sequences, key padding) and the softmax over keys, in place: s -> p
template <int L, int C0, int NC>
__device__ __forceinline__ void softmax_t(const float* MS, int qrow, f32x4 (&s)[NC]) {
  const int g4 = (threadIdx.x & 63) >> 4, lo = (qrow / L) * L;
  float mx = -INFINITY;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int key = 16 * (C0 + c) + 4 * g4 + q;
      const float ms = MS[key];  // key < 80 always: an unconditional load, no branch
      const float v = (unsigned)(key - lo) < (unsigned)L ? s[c][q] * kScale + ms : -INFINITY;
      s[c][q] = v;
      mx = fmaxf(mx, v);
    }
  mx = rows4_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float e = exp_fast(s[c][q] - mx);
      s[c][q] = e;
      sum += e;
    }
  const float inv = 1.f / rows4_sum(sum);
#pragma unroll
  for (int c = 0; c < NC; ++c) s[c] = s[c] * inv;
}

// keep bits of the attention dropout at this lane's (key, query) elements: bit 4c + q.  A lane's
// four keys of a tile are consecutive elements of one score row; for even L a row starts on a pair
// boundary, so q = 0, 1 and q = 2, 3 share one pair hash (keep()'s halves)
template <int L, int C0, int NC>
__device__ __forceinline__ uint32_t att_keep_bits(uint32_t ks, uint32_t thr, int64_t seq0, int hh, int qrow) {
  if (thr == 0u) return 0xFFFFFFFFu;
  const int g4 = (threadIdx.x & 63) >> 4, g = qrow / L;
  const uint32_t base = (uint32_t)((((seq0 + g) * HEADS + hh) * L + (qrow - g * L)) * L);
  uint32_t bits = 0;
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    // keys of other sequences have p = 0: whatever their bit, they contribute nothing
    const uint32_t e0 = base + (uint32_t)(16 * (C0 + c) + 4 * g4 - g * L);
    if constexpr (L % 2 == 0) {
      const uint32_t h0 = pair_hash(ks, e0 >> 1), h1 = pair_hash(ks, (e0 >> 1) + 1);
      bits |= ((uint32_t)half_keep(h0, 0, thr) | ((uint32_t)half_keep(h0, 1, thr) << 1) |
               ((uint32_t)half_keep(h1, 0, thr) << 2) | ((uint32_t)half_keep(h1, 1, thr) << 3)) << (4 * c);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) bits |= (uint32_t)keep(ks, e0 + q, thr) << (4 * c + q);
    }
  }
  return bits;
}

// forward: ctx rows of query tile R, head hh, written over the tile's q slots in RA
template <int L, int R>
__device__ __forceinline__ void attn_fwd_tile(float* RA, const float* MS, int hh, int64_t seq0, uint32_t ks,
                                              const Weights& w, bool prof) {
  constexpr int C0 = band_lo<L>(R), NC = band_n<L>(R);
  const int lane = threadIdx.x & 63, i = lane & 15, g4 = lane >> 4;
  const int qrow = 16 * R + i;
  f32x4 s[NC];
  tiles_t<R, C0, NC>(RA, E, RA, LD_QKV, hh, s);
  fr_mark(prof, 0, 21);
  softmax_t<L, C0, NC>(MS, qrow, s);
  fr_mark(prof, 0, 22);
  const uint32_t kb = att_keep_bits<L, C0, NC>(ks, w.thr[0], seq0, hh, qrow);
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) s[c][q] = ((kb >> (4 * c + q)) & 1u) ? s[c][q] * w.scale[0] : 0.f;
  fr_mark(prof, 0, 23);
  f32x4 ctx[HD / 16];
  keys_product<C0, NC>(s, RA, 2 * E, hh, ctx);
  // only this job reads the q slots of (tile R, head hh), and it is done with them
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
    for (int q = 0; q < 4; ++q) RA[(16 * R + 4 * g4 + q) * LD_QKV + hh * HD + 16 * dt + i] = ctx[dt][q];
  fr_mark(prof, 0, 24);
}

// the 10 (query tile, head) jobs over 8 waves: tiles 1-3 (3 band tiles for L = 20, 10, 5) one per
// wave, tiles 0 and 4 (2 band tiles) two per wave on waves 6 and 7
template <int L>
__device__ __forceinline__ void attn_fwd(float* RA, const float* MS, int64_t seq0, uint32_t ks, const Weights& w,
                                         bool prof) {
  static_assert(RT == 5 && HEADS == 2 && NT / 64 == 8, "job table");
  const int wave = wave_id();
  for (int j = wave; j < RT * HEADS; j += (wave >= 6 ? 2 : RT * HEADS)) {
    const int R = j < 6 ? 1 + j % 3 : ((j - 6) % 2 ? 4 : 0), hh = j < 6 ? j / 3 : (j - 6) / 2;
    switch (R) {
      case 0: attn_fwd_tile<L, 0>(RA, MS, hh, seq0, ks, w, prof); break;
      case 1: attn_fwd_tile<L, 1>(RA, MS, hh, seq0, ks, w, prof); break;
      case 2: attn_fwd_tile<L, 2>(RA, MS, hh, seq0, ks, w, prof); break;
      case 3: attn_fwd_tile<L, 3>(RA, MS, hh, seq0, ks, w, prof); break;
      default: attn_fwd_tile<L, 4>(RA, MS, hh, seq0, ks, w, prof); break;
    }
  }
}

// backward, phase 1 (query tile R, head hh): recompute P, dP'^T = V dctx^T, dropout backward,
// dS = P (dP - D) / sqrt(HD); P' and dS tiles to the scratch ([key][query], TILE_LD), dQ = dS K to DQ
template <int L, int R>
__device__ __forceinline__ void attn_bwd_rows(const float* RA, const float* RC, const float* MS, int hh, int64_t seq0,
                                              uint32_t ks, const Weights& w, float* SP, float* SS, float* DQ,
                                              bool prof) {
  constexpr int C0 = band_lo<L>(R), NC = band_n<L>(R), S0 = band_slot<L>(R);
  const int lane = threadIdx.x & 63, i = lane & 15, g4 = lane >> 4;
  const int qrow = 16 * R + i;
  f32x4 p[NC], d[NC];
  tiles_t<R, C0, NC>(RA, E, RA, LD_QKV, hh, p);      // S^T = K Q^T
  tiles_t<R, C0, NC>(RA, 2 * E, RC, LD_E, hh, d);    // dP'^T = V dctx^T
  if (hh == 0) fr_mark(prof, 1, 13);
  softmax_t<L, C0, NC>(MS, qrow, p);
  const uint32_t kb = att_keep_bits<L, C0, NC>(ks, w.thr[0], seq0, hh, qrow);
  if (hh == 0) fr_mark(prof, 1, 14);
  float D = 0.f;
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float dpj = ((kb >> (4 * c + q)) & 1u) ? d[c][q] * w.scale[0] : 0.f;  // dL/dp
      d[c][q] = dpj;
      D = fmaf(p[c][q], dpj, D);
    }
  D = rows4_sum(D);
#pragma unroll
  for (int c = 0; c < NC; ++c)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float pv = p[c][q];
      const float ds = pv * (d[c][q] - D) * kScale;
      d[c][q] = ds;
      const int o = (S0 + c) * TILE_SZ + (4 * g4 + q) * TILE_LD + i;
      SS[o] = ds;
      SP[o] = ((kb >> (4 * c + q)) & 1u) ? pv * w.scale[0] : 0.f;  // p'
    }
  if (hh == 0) fr_mark(prof, 1, 15);
  f32x4 dq[HD / 16];
  keys_product<C0, NC>(d, RA, E, hh, dq);  // dQ = dS K
#pragma unroll
  for (int dt = 0; dt < HD / 16; ++dt)
#pragma unroll
    for (int q = 0; q < 4; ++q) DQ[(16 * R + 4 * g4 + q) * DQ_LD + 16 * dt + i] = dq[dt][q];
  if (hh == 0) fr_mark(prof, 1, 16);
}

// backward, phase 2 (key tile c, head hh, column tile dt): dK = dS^T Q (kind 0) or dV = P'^T dctx
// (kind 1) over the query tiles whose band holds c, written over the key rows' k / v slots
template <int L>
__device__ __forceinline__ void attn_bwd_keys(float* RA, const float* RC, const float* SP, const float* SS, int hh,
                                              int c, int kind, int dt) {
  const int lane = threadIdx.x & 63, i = lane & 15, g4 = lane >> 4;
  const float* T = kind ? SP : SS;
  const float* Bm = kind ? RC : RA;
  const int ldb = kind ? LD_E : LD_QKV;
  float4 a[RT];
  float b[RT][4];
#pragma unroll
  for (int r = 0; r < RT; ++r) {  // operands of every query tile first (tiles outside the band: zeros)
    const bool in = c >= band_lo<L>(r) && c <= band_hi<L>(r);
    const int slot = in ? band_slot<L>(r) + c - band_lo<L>(r) : 0;
    a[r] = lds4(T + slot * TILE_SZ + i * TILE_LD + 4 * g4);
    if (!in) a[r] = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int m = 0; m < 4; ++m) b[r][m] = Bm[(16 * r + 4 * g4 + m) * ldb + hh * HD + 16 * dt + i];
  }
  f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;  // two chains (even / odd query tiles), summed at the end
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      if (r % 2 == 0) acc0 = mfma4(comp(a[r], m), b[r][m], acc0);
      else acc1 = mfma4(comp(a[r], m), b[r][m], acc1);
    }
#pragma unroll
  for (int q = 0; q < 4; ++q)
    RA[(16 * c + 4 * g4 + q) * LD_QKV + (kind ? 2 * E : E) + hh * HD + 16 * dt + i] = acc0[q] + acc1[q];
}

template <int L>
__device__ __forceinline__ void attn_bwd_rows_any(int R, const float* RA, const float* RC, const float* MS, int hh,
                                                  int64_t seq0, uint32_t ks, const Weights& w, float* SP, float* SS,
                                                  float* DQ, bool prof) {
  switch (R) {
    case 0: attn_bwd_rows<L, 0>(RA, RC, MS, hh, seq0, ks, w, SP, SS, DQ, prof); break;
    case 1: attn_bwd_rows<L, 1>(RA, RC, MS, hh, seq0, ks, w, SP, SS, DQ, prof); break;
    case 2: attn_bwd_rows<L, 2>(RA, RC, MS, hh, seq0, ks, w, SP, SS, DQ, prof); break;
    case 3: attn_bwd_rows<L, 3>(RA, RC, MS, hh, seq0, ks, w, SP, SS, DQ, prof); break;
    default: attn_bwd_rows<L, 4>(RA, RC, MS, hh, seq0, ks, w, SP, SS, DQ, prof); break;
  }
}

// ---------------------------------------------------------------------------------------------
// attention per (sequence, head) on one wave, v_mfma_f32_32x32x2_f32 (L = 20: a sequence padded to
// one 32 x 32 tile).  The workgroup's 4 sequences x 2 heads are exactly its 8 waves: no job table,
// no barrier between the products, no scratch shared between waves.  Layout of a 32 x 32 output:
// lane l holds column j = l & 31, register v row tile_row(v, hf = l >> 5).  Scores are computed
// transposed, S^T = K Q^T (rows keys, lane = query): the softmax over keys is lane-local plus the
// partner half (permlane32 swap), and register s is directly the A operand of a product over keys
// (contraction index key(s, hf) = tile_row(s, hf): 12 steps cover keys 0..23).  Products over
// queries (dK, dV) read dS / P' back transposed from a 20 x 24 slice of LDS private to the wave
// (contraction index query 2s + hf: 10 steps).  Operand rows past the sequence (keys / queries
// >= L) are read as zeros, so padded rows contribute nothing (0 x garbage never enters an MFMA).
typedef float f32x16 __attribute__((ext_vector_type(16)));

// v & msk bitwise (msk all ones or zero): a branch-free zero of operands past the sequence
__device__ __forceinline__ float mask1(float v, uint32_t msk) { return __uint_as_float(__float_as_uint(v) & msk); }
__device__ __forceinline__ float4 mask4(float4 v, uint32_t msk) {
  return make_float4(mask1(v.x, msk), mask1(v.y, msk), mask1(v.z, msk), mask1(v.w, msk));
}

__device__ __forceinline__ f32x16 mfma32(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int tile_row(int v, int hf) { return 8 * (v >> 2) + 4 * hf + (v & 3); }
__device__ __forceinline__ float swap32_max(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}

constexpr int SEQ_TLD = 24;                       // private transposed dS / P' slices: [key][query]
constexpr int SEQ_TSZ = 20 * SEQ_TLD;             // floats per slice (L = 20)

// this wave's (sequence g, head hh) for L = 20
struct SeqJob {
  int g, hh, base, j, hf;
  bool jv;
};
template <int L>
__device__ __forceinline__ SeqJob seq_job() {
  const int w = wave_id(), lane = threadIdx.x & 63;
  SeqJob q;
  q.g = w & 3;
  q.hh = w >> 2;
  q.base = q.g * L;
  q.j = lane & 31;
  q.hf = lane >> 5;
  q.jv = q.j < L;
  return q;
}

// S^T = K Q^T of the job (unscaled, rows keys, lane = query); optionally the same product with
// V (A) and dctx (B) -> dP'^T
template <int L>
__device__ __forceinline__ f32x16 seq_scores(const float* RA, int offA, const float* Bsrc, int ldb, int offB,
                                             const SeqJob& q) {
  const int row = q.base + (q.jv ? q.j : 0);
  const float* ar = RA + row * LD_QKV + offA + q.hh * HD + 16 * q.hf;
  const float* br = Bsrc + row * ldb + offB + q.hh * HD + 16 * q.hf;
  // rows past L read the sequence's first row (finite) and are zeroed by a lane mask: no branch between
  // the loads, all eight in flight at once
  const uint32_t msk = q.jv ? 0xFFFFFFFFu : 0u;
  float4 av[4], bv[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    av[k] = lds4(ar + 4 * k);
    bv[k] = lds4(br + 4 * k);
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    av[k] = mask4(av[k], msk);
    bv[k] = mask4(bv[k], msk);
  }
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
#pragma unroll
  for (int st = 0; st < 16; ++st) acc = mfma32(comp(av[st >> 2], st & 3), comp(bv[st >> 2], st & 3), acc);
  return acc;
}

// scale + key masks + softmax over keys, in place (S^T -> P^T); keys >= L get p = 0
template <int L>
__device__ __forceinline__ void seq_softmax(f32x16& s, const float* MS, const SeqJob& q) {
  float mx = -INFINITY;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int key = tile_row(v, q.hf);
    const float ms = MS[q.base + (key < L ? key : 0)];
    const float x = key < L ? s[v] * kScale + ms : -INFINITY;
    s[v] = x;
    mx = fmaxf(mx, x);
  }
  mx = swap32_max(mx);
  float sum = 0.f;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const float e = exp_fast(s[v] - mx);
    s[v] = e;
    sum += e;
  }
  const float inv = 1.f / swap32_sum(sum);
#pragma unroll
  for (int v = 0; v < 16; ++v) s[v] *= inv;
}

// attention-dropout keep bits of the lane's 16 (query j, key tile_row(v, hf)) elements, bit v; keys
// come in aligned groups of 4, so pairs (k, k + 1) share one hash (keep()'s halves)
template <int L>
__device__ __forceinline__ uint32_t seq_keep_bits(uint32_t ks, uint32_t thr, int64_t seq0, const SeqJob& q) {
  static_assert(L % 2 == 0, "pair hashes need even rows");
  if (thr == 0u) return 0xFFFFu;
  const uint32_t rowb = (uint32_t)((((seq0 + q.g) * HEADS + q.hh) * L + q.j) * L);
  uint32_t bits = 0;
#pragma unroll
  for (int grp = 0; grp < 4; ++grp) {
    const int k0 = 8 * grp + 4 * q.hf;
    const uint32_t p0 = (rowb + (uint32_t)k0) >> 1;
    const uint32_t h0 = pair_hash(ks, p0), h1 = pair_hash(ks, p0 + 1);
    bits |= ((uint32_t)half_keep(h0, 0, thr) | ((uint32_t)half_keep(h0, 1, thr) << 1) |
             ((uint32_t)half_keep(h1, 0, thr) << 2) | ((uint32_t)half_keep(h1, 1, thr) << 3)) << (4 * grp);
  }
  return bits;
}

// out[query][d] (+)= sum over keys X^T[key][query] Bm[key][d]: X^T in registers (A operand, key(s, hf) =
// tile_row(s, hf)), Bm rows of the sequence's keys at column offset off (head hh), zero past L
template <int L>
__device__ __forceinline__ f32x16 seq_keys_product(const f32x16& x, const float* Bm, int ldb, int off,
                                                   const SeqJob& q) {
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  float b[12];
#pragma unroll
  for (int st = 0; st < 12; ++st) {
    const int key = tile_row(st, q.hf);
    b[st] = Bm[(q.base + (key < L ? key : 0)) * ldb + off + q.hh * HD + q.j];
  }
#pragma unroll
  for (int st = 0; st < 12; ++st) b[st] = mask1(b[st], tile_row(st, q.hf) < L ? 0xFFFFFFFFu : 0u);
#pragma unroll
  for (int st = 0; st < 12; ++st) acc = mfma32(x[st], b[st], acc);
  return acc;
}

// out[key][d] = sum over queries T[key][query] Bm[query][d]: T the wave's transposed slice (A
// operand: lane = key, query 2s + hf), Bm the sequence's query rows (column offset off, head hh)
template <int L>
__device__ __forceinline__ f32x16 seq_queries_product(const float* T, const float* Bm, int ldb, int off,
                                                      const SeqJob& q) {
  static_assert(L == 20, "10 steps of 2 queries");
  f32x16 acc;
#pragma unroll
  for (int v = 0; v < 16; ++v) acc[v] = 0.f;
  float a[10], b[10];
  const int jr = q.jv ? q.j : 0;
  const uint32_t msk = q.jv ? 0xFFFFFFFFu : 0u;
#pragma unroll
  for (int st = 0; st < 10; ++st) {
    const int qr = 2 * st + q.hf;
    a[st] = T[jr * SEQ_TLD + qr];
    b[st] = Bm[(q.base + qr) * ldb + off + q.hh * HD + q.j];
  }
#pragma unroll
  for (int st = 0; st < 10; ++st) a[st] = mask1(a[st], msk);
#pragma unroll
  for (int st = 0; st < 10; ++st) acc = mfma32(a[st], b[st], acc);
  return acc;
}

// store the rows < L of a 32 x 32 output (rows tile_row(v, hf), column j = d) to LDS rows of the
// sequence at column offset off (head hh)
template <int L>
__device__ __forceinline__ void seq_store(float* dst, int ld, int off, const f32x16& o, const SeqJob& q) {
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const int r = tile_row(v, q.hf);
    if (r < L) dst[(q.base + r) * ld + off + q.hh * HD + q.j] = o[v];
  }
}

// forward: ctx = dropout(softmax(q k^T / sqrt(32) + mask)) v of the wave's (sequence, head), over the
// q slots of RA
template <int L>
__device__ __forceinline__ void attn_fwd_seq(float* RA, const float* MS, int64_t seq0, uint32_t ks, const Weights& w) {
  const SeqJob q = seq_job<L>();
  f32x16 p = seq_scores<L>(RA, E, RA, LD_QKV, 0, q);  // S^T = K Q^T
  seq_softmax<L>(p, MS, q);
  const uint32_t kb = seq_keep_bits<L>(ks, w.thr[0], seq0, q);
#pragma unroll
  for (int v = 0; v < 16; ++v) p[v] = ((kb >> v) & 1u) ? p[v] * w.scale[0] : 0.f;
  const f32x16 ctx = seq_keys_product<L>(p, RA, LD_QKV, 2 * E, q);  // P' V
  seq_store<L>(RA, LD_QKV, 0, ctx, q);  // only this wave reads the (sequence, head) q slots
}

// backward of the wave's (sequence, head): dQ, dK, dV over the q / k / v slots of RA (each wave owns
// its slots: no other wave reads them).  RC: dctx.  TB: 2 x SEQ_TSZ floats private to the wave.
template <int L>
__device__ __forceinline__ void attn_bwd_seq(float* RA, const float* RC, const float* MS, int64_t seq0, uint32_t ks,
                                             const Weights& w, float* TB) {
  const SeqJob q = seq_job<L>();
  f32x16 p = seq_scores<L>(RA, E, RA, LD_QKV, 0, q);        // S^T = K Q^T
  f32x16 d = seq_scores<L>(RA, 2 * E, RC, LD_E, 0, q);      // dP'^T = V dctx^T
  seq_softmax<L>(p, MS, q);
  const uint32_t kb = seq_keep_bits<L>(ks, w.thr[0], seq0, q);
  float D = 0.f;
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const float dpj = ((kb >> v) & 1u) ? d[v] * w.scale[0] : 0.f;  // dL/dp
    d[v] = dpj;
    D = fmaf(p[v], dpj, D);
  }
  D = swap32_sum(D);
  float* TS = TB;            // dS^T as [key][query]
  float* TP = TB + SEQ_TSZ;  // P'^T
#pragma unroll
  for (int v = 0; v < 16; ++v) {
    const float pv = p[v];
    const float ds = pv * (d[v] - D) * kScale;
    d[v] = ds;
    const int key = tile_row(v, q.hf);
    if (key < L && q.jv) {
      TS[key * SEQ_TLD + q.j] = ds;
      TP[key * SEQ_TLD + q.j] = ((kb >> v) & 1u) ? pv * w.scale[0] : 0.f;
    }
  }
  const f32x16 dq = seq_keys_product<L>(d, RA, LD_QKV, E, q);          // dQ = dS K
  const f32x16 dk = seq_queries_product<L>(TS, RA, LD_QKV, 0, q);       // dK = dS^T Q
  const f32x16 dv = seq_queries_product<L>(TP, RC, LD_E, 0, q);         // dV = P'^T dctx
  seq_store<L>(RA, LD_QKV, 0, dq, q);
  seq_store<L>(RA, LD_QKV, E, dk, q);
  seq_store<L>(RA, LD_QKV, 2 * E, dv, q);
}

// The ordered reduction of another backward call's partials, folded into this launch: workgroup b
// owns float4 columns [b C, (b + 1) C) of the NPART / 4 (C = ceil(NPART / 4 / n_wg)), taken in chunks
// of PR_CH columns (what the scratch holds); PR_SL slices of its threads sum workgroups s, s + PR_SL,
// ... in order (PR_UNR loads in flight per thread), then the slices are added in slice order through
// LDS (scratch: PR_SL x PR_CH float4).  The same column always gets the same order of additions:
// deterministic, independent of placement and timing.
constexpr int PR_SL = 10, PR_UNR = 26, PR_CH = (BUF_D / 4) / PR_SL;  // (256 workgroups: one batch of loads)
__device__ __forceinline__ void prev_reduce(const float* __restrict__ prev, int nwg, float* __restrict__ out,
                                            float* scratch) {
  constexpr int N4 = NPART / 4;
  const int C = (N4 + nwg - 1) / nwg;
  const int c0 = blockIdx.x * C;
  const float4* p4 = reinterpret_cast<const float4*>(prev);
  float4* s4 = reinterpret_cast<float4*>(scratch);
  for (int cb = 0; cb < C; cb += PR_CH) {
    const int cn = min(PR_CH, C - cb);
    for (int e = threadIdx.x; e < PR_SL * cn; e += NT) {
      const int cl = e % cn, sl = e / cn, c = min(c0 + cb + cl, N4 - 1);
      float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int g0 = sl; g0 < nwg; g0 += PR_SL * PR_UNR) {
        float4 v[PR_UNR];
#pragma unroll
        for (int k = 0; k < PR_UNR; ++k) v[k] = p4[(int64_t)min(g0 + k * PR_SL, nwg - 1) * N4 + c];
#pragma unroll
        for (int k = 0; k < PR_UNR; ++k)
          if (g0 + k * PR_SL < nwg) s = f4_add(s, v[k]);
      }
      s4[sl * cn + cl] = s;
    }
    __syncthreads();
    for (int cl = threadIdx.x; cl < cn; cl += NT) {
      if (c0 + cb + cl >= N4) break;
      float4 t = s4[cl];
#pragma unroll
      for (int k = 1; k < PR_SL; ++k) t = f4_add(t, s4[k * cn + cl]);
      grad_store4(out, c0 + cb + cl, t);
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------------------
template <int L>
__global__ __launch_bounds__(NT) void enc_fwd_kernel(FwdArgs a) {
  constexpr int G = ROWS / L;
  __shared__ __attribute__((aligned(16))) float RA[ROWS * LD_FF];  // qkv (ctx in the q slots), then act
  __shared__ __attribute__((aligned(16))) float RB[ROWS * LD_E];   // x -> y1 -> x1 -> y2
  __shared__ float MS[ROWS];                                        // key mask of the tile's tokens
  const Weights& w = a.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i16 = lane & 15, h4 = lane >> 4;
  const int sg = wave & 3, hf = wave >> 2, r0 = hf ? RT0 : 0, nr = hf ? RT - RT0 : RT0;
  const int64_t seq0 = (int64_t)blockIdx.x * G;
  const int nseq = (int)min<int64_t>(G, a.ns - seq0);
  const int tv = nseq * L;
  const int64_t tok0 = seq0 * L;
  const bool prof = g_prof_on && blockIdx.x == 0;
  if (kEncPrio && wave_id() >= 4) __builtin_amdgcn_s_setprio(1);
  FR_MARK(0, 0);
  const int64_t counter = *a.counter;
  const SiteKeys ks = site_keys(w.seed, counter);
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.seed_out = counter;

  if (threadIdx.x < ROWS) MS[threadIdx.x] = (a.mask && threadIdx.x < tv) ? a.mask[tok0 + threadIdx.x] : 0.f;
  lds_load<E>(RB, LD_E, a.x + tok0 * E, tv);
  __syncthreads();
  FR_MARK(0, 1);

  {  // qkv = x W_in^T + b_in  (SIMD slot sg: column tiles 3sg..3sg+2)
    f32x4 acc[RT0][3];
    zero_acc(acc);
    FR_GEMM_XWT(3, E, RB, LD_E, w.w_in, 3 * sg, acc);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const int col = 16 * (3 * sg + c) + i16;
      const float bias = w.b_in[col];
#pragma unroll
      for (int r = 0; r < RT0; ++r) {
        if (r >= nr) break;
#pragma unroll
        for (int q = 0; q < 4; ++q) RA[(16 * (r0 + r) + 4 * h4 + q) * LD_QKV + col] = acc[r][c][q] + bias;
      }
    }
  }
  __syncthreads();
  FR_MARK(0, 2);
  lds_store<QKV>(RA, LD_QKV, a.qkv + tok0 * QKV, tv);
  __syncthreads();  // the copy has read every q slot before attention overwrites them with ctx
  FR_MARK(0, 20);

  // attention on MFMA: 10 (query tile, head) jobs over the 8 waves; ctx over the q slots
  if constexpr (L == 20) attn_fwd_seq<L>(RA, MS, seq0, ks.k[0], w);
  else attn_fwd<L>(RA, MS, seq0, ks.k[0], w, prof);
  __syncthreads();
  FR_MARK(0, 3);
  lds_store<E>(RA, LD_QKV, a.ctx + tok0 * E, tv);  // ctx (saved for the backward): cols 0..63 of RA

  {  // y1 = x + dropout1(ctx W_o^T + b_o)   (column tile sg); ctx rows of padded sequences are stale
    f32x4 acc[RT0][1];
    zero_acc(acc);
    FR_GEMM_XWT(1, E, RA, LD_QKV, w.w_o, sg, acc);
    const int col = 16 * sg + i16;
    const float bias = w.b_o[col];
#pragma unroll
    for (int r = 0; r < RT0; ++r) {
      if (r >= nr) break;
      const int row0 = 16 * (r0 + r) + 4 * h4;
      const uint32_t kb = frag_keep4(ks.k[1], tok0 + row0, E, col, w.thr[1]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float o = acc[r][0][q] + bias;
        RB[(row0 + q) * LD_E + col] += ((kb >> q) & 1u) ? o * w.scale[1] : 0.f;
      }
    }
  }
  __syncthreads();
  FR_MARK(0, 4);
  ln_rows_fwd(RB, w.g1, w.be1, w.eps1, tv, a.y1 + tok0 * E, a.st1 + 2 * tok0, nullptr);
  __syncthreads();
  FR_MARK(0, 5);

  {  // pre = x1 W1^T + b1; act' = dropout(act(pre)) -> RA.  Column split (wave: tiles 4sg + 2hf, +1;
     // every row tile), so both waves of a SIMD get the same share of the GELU / dropout epilogue.
     // One column tile at a time (GEMM, then its epilogue): 20 accumulator registers live instead of
     // 40 keeps the kernel at <= 128 VGPRs, so a SIMD can hold two of its waves beside two waves of a
     // 128-register kernel (the background Adam slice) in the training step's graph
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      f32x4 acc[RT][1];
      zero_acc(acc);
      const int c = 2 * hf + cc;  // column tile within the SIMD slot's four (dact fragment index)
      gemm_xwt<1, E, 0, RT>(RB, LD_E, w.w1, 4 * sg + c, acc);
      const int col = 16 * (4 * sg + c) + i16;
      const float bias = w.b1[col];
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        const int row0 = 16 * r + 4 * h4;
        const uint32_t kb = frag_keep4(ks.k[2], tok0 + row0, FF, col, w.thr[2]);
        float d[4];
#pragma unroll
        for (int q2 = 0; q2 < 2; ++q2) {
          f32x2 av, gv;
          act_fwd_grad2(f32x2{acc[r][0][2 * q2], acc[r][0][2 * q2 + 1]} + bias, w.gelu, av, gv);
          av = av * w.scale[2];
          gv = gv * w.scale[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int q = 2 * q2 + u;
            const bool kp = (kb >> q) & 1u;
            RA[(row0 + q) * LD_FF + col] = kp ? av[u] : 0.f;
            d[q] = kp ? gv[u] : 0.f;
          }
        }
        // dact in the MFMA fragment layout: one coalesced float4 per lane, read back the same way
        *reinterpret_cast<float4*>(a.dact + dact_frag(blockIdx.x, sg, c, r, lane)) = make_float4(d[0], d[1], d[2], d[3]);
      }
      FR_SCHED_FENCE();
    }
  }
  __syncthreads();
  FR_MARK(0, 6);

  {  // y2 = x1 + dropout2(act' W2^T + b2)  (column tile sg, K = 256)
    f32x4 acc[RT0][1];
    zero_acc(acc);
    FR_GEMM_XWT(1, FF, RA, LD_FF, w.w2, sg, acc);
    const int col = 16 * sg + i16;
    const float bias = w.b2[col];
#pragma unroll
    for (int r = 0; r < RT0; ++r) {
      if (r >= nr) break;
      const int row0 = 16 * (r0 + r) + 4 * h4;
      const uint32_t kb = frag_keep4(ks.k[3], tok0 + row0, E, col, w.thr[3]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float o = acc[r][0][q] + bias;
        RB[(row0 + q) * LD_E + col] += ((kb >> q) & 1u) ? o * w.scale[3] : 0.f;
      }
    }
  }
  __syncthreads();
  FR_MARK(0, 7);
  lds_store<FF>(RA, LD_FF, a.fact + tok0 * FF, tv);  // act' (RA is final after the FF2 barrier)
  ln_rows_fwd(RB, w.g2, w.be2, w.eps2, tv, a.y2 + tok0 * E, a.st2 + 2 * tok0, a.out + tok0 * E);
  FR_MARK(0, 31);
}

// ---------------------------------------------------------------------------------------------
// backward
// ---------------------------------------------------------------------------------------------
template <int L>
__global__ __launch_bounds__(NT) void enc_bwd_kernel(BwdArgs a) {
  constexpr int G = ROWS / L;
  // one LDS image: RA [80 x 260] | RC [80 x 68] | RB [80 x 68] | RD [BUF_D]; the attention backward's
  // scratch (P' and dS tiles, dQ) overlays RB + RD (dY1 is held in registers across it)
  constexpr int OFF_RC = ROWS * LD_FF, OFF_RB = OFF_RC + ROWS * LD_E, OFF_RD = OFF_RB + ROWS * LD_E;
  constexpr int SCR_FLOATS = 2 * MAX_SLOTS * TILE_SZ + ROWS * DQ_LD;
  static_assert(SCR_FLOATS <= ROWS * LD_E + BUF_D, "attention scratch fits RB + RD");
  static_assert((NT / 64) * 2 * SEQ_TSZ <= ROWS * LD_E + BUF_D, "per-wave transposed slices fit RB + RD");
  static_assert(ROWS * LD_E <= BUF_D && 3 * (NT / 16) * E <= BUF_D, "LayerNorm scratch / ctx in RD");
  static_assert(band_slot<L>(RT) <= MAX_SLOTS, "band tiles");
  __shared__ __attribute__((aligned(16))) float LDSB[OFF_RD + BUF_D];
  float* const RA = LDSB;
  float* const RC = LDSB + OFF_RC;
  float* const RB = LDSB + OFF_RB;
  float* const RD = LDSB + OFF_RD;
  float* const SP = RB;                            // P' tiles   [MAX_SLOTS][16][TILE_LD]
  float* const SS = RB + MAX_SLOTS * TILE_SZ;      // dS tiles
  float* const DQ = RB + 2 * MAX_SLOTS * TILE_SZ;  // dQ of one head [80][DQ_LD]
  const Weights& w = a.w;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, i16 = lane & 15, h4 = lane >> 4;
  const int sg = wave & 3, hf = wave >> 2, r0 = hf ? RT0 : 0, nr = hf ? RT - RT0 : RT0;
  const int64_t seq0 = (int64_t)blockIdx.x * G;
  const int nseq = (int)min<int64_t>(G, a.ns - seq0);
  const int tv = nseq * L;
  const int64_t tok0 = seq0 * L;
  const bool prof = g_prof_on && blockIdx.x == 0;
  if (kEncPrio && wave_id() >= 4) __builtin_amdgcn_s_setprio(1);
  FR_MARK(1, 0);
  const SiteKeys ks = site_keys(w.seed, *a.seed_in);
  float* part = a.part + (int64_t)blockIdx.x * NPART;
  __shared__ float MS[ROWS];
  if (threadIdx.x < ROWS) MS[threadIdx.x] = (a.mask && threadIdx.x < tv) ? a.mask[tok0 + threadIdx.x] : 0.f;

  // 0. (optional) the previous backward call's weight-gradient partials: this workgroup's slice of
  //    the columns, summed over that call's workgroups in order (deterministic)
  if (a.prev_part) prev_reduce(a.prev_part, (int)gridDim.x, a.prev_grad, RD);

  // Global operands are issued one phase ahead of their use, in the order they are waited for (loads
  // retire in order): dY2, then LN2's rows, then act' (its ~80 KB per workgroup lands during LN2).
  // (act' is issued only once dY2 has landed: a burst issued ahead of it stalls the issuing waves for
  // its whole transfer -- the loads are bandwidth-, not latency-bound -- and dY2 waits behind it)
  TilePf<E> pf_dout;
  pf_issue(pf_dout, a.dout + tok0 * E, tv);
  LnPf ln2;
  ln_issue(ln2, a.y2 + tok0 * E, a.st2 + 2 * tok0, w.g2, nullptr, tv);

  // 1. LN2 backward: RB = dY2 (pad rows 0), and dG = dropout2'(dY2) -> RC, db2
  pf_commit(pf_dout, RB, LD_E, tv);
  TilePf<FF> pf_fact;
  pf_issue(pf_fact, a.fact + tok0 * FF, tv);
  __syncthreads();
  FR_MARK(1, 1);
  ln_rows_bwd(RB, ln2, tv, RD, part + OFF_G2, part + OFF_BE2, RC, ks.k[3], tok0, w.thr[3], w.scale[3],
              part + OFF_B2);

  // 2. act' (saved by the forward) -> RA
  pf_commit(pf_fact, RA, LD_FF, tv);
  __syncthreads();
  FR_MARK(1, 2);

  // the step-4 GEMM's W2 fragments, then dact at this lane's step-4 output elements (fragment
  // layout): both in flight across the dW2 slab below
  YwFrags<2, E, FF> w2f;
  yw_issue(w2f, w.w2, 4 * sg + 2 * hf);
  float4 pv[2][RT];
#pragma unroll
  for (int cc = 0; cc < 2; ++cc)
#pragma unroll
    for (int r = 0; r < RT; ++r)
      pv[cc][r] = *reinterpret_cast<const float4*>(a.dact + dact_frag(blockIdx.x, sg, 2 * hf + cc, r, lane));
  // the scheduler would otherwise sink these loads to their use (the register pressure heuristic):
  // the W2 fragments into the step-4 GEMM loop (vmcnt waits between its MFMAs), dact behind it
  FR_SCHED_FENCE();

  // 3. dW2 = dG^T act'  [64 x 256] (wave: k-tiles 2w, 2w+1);  db2
  wgrad_tiles<4, 2>(RC, LD_E, RA, LD_FF, 0, 2 * wave, part + OFF_W2, FF);  // (db2: with the LN2 backward)

  LnPf ln1;  // y1 rows / stats, gamma1 / beta1: the LN1 recompute (step 5) and the LN1 backward (step 8)
  {  // 4. dact' = dG W2 [80 x 256]; dpre = dact' * (keep * scale * act'(pre)) -> RA  (wave: column tiles
     // 4sg + 2hf, +1; every row tile)
    f32x4 acc[RT][2];
    zero_acc(acc);
    gemm_yw_pre<2, E, FF, 0, RT>(RC, LD_E, w2f, acc);
    ln_issue(ln1, a.y1 + tok0 * E, a.st1 + 2 * tok0, w.g1, w.be1, tv);
    __syncthreads();  // every wave is done reading act' from RA
    FR_MARK(1, 3);
#pragma unroll
    for (int cc = 0; cc < 2; ++cc) {
      const int col = 16 * (4 * sg + 2 * hf + cc) + i16;
#pragma unroll
      for (int r = 0; r < RT; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int row = 16 * r + 4 * h4 + q;
          RA[row * LD_FF + col] = row < tv ? acc[r][cc][q] * comp(pv[cc][r], q) : 0.f;
        }
    }
  }
  __syncthreads();
  FR_MARK(1, 4);

  // the step-7 GEMM's W1 fragments (the whole K = 256 column slice of this SIMD slot: 64 registers),
  // in flight across the LN1 recompute and the dW1 slab instead of one chunk ahead inside the loop
  YwFrags<1, FF, E> w1f;
  yw_issue(w1f, w.w1, sg);
  FR_SCHED_FENCE();

  // 5. x1 = LN1(y1) recomputed -> RC  (db1: with dW1 below)
  {
    const int grp = threadIdx.x >> 4, l = threadIdx.x & 15;
    const float4 gg = ln1.gg, bb = ln1.bb;
#pragma unroll
    for (int k = 0; k < LnPf::NR; ++k) {
      const int r = grp + k * LnPf::NG;
      if (r >= ROWS) break;
      const float4 v = ln1.yv[k];
      const float mean = ln1.sv[k].x, rstd = ln1.sv[k].y;
      const float4 o = make_float4(fmaf((v.x - mean) * rstd, gg.x, bb.x), fmaf((v.y - mean) * rstd, gg.y, bb.y),
                                   fmaf((v.z - mean) * rstd, gg.z, bb.z), fmaf((v.w - mean) * rstd, gg.w, bb.w));
      *reinterpret_cast<float4*>(RC + r * LD_E + 4 * l) = r < tv ? o : make_float4(0.f, 0.f, 0.f, 0.f);
    }
  }
  __syncthreads();
  FR_MARK(1, 5);

  // 6. dW1 = dpre^T x1  [256 x 64] (wave: n-tiles 2w, 2w+1);  db1
  wgrad_tiles<2, 4>(RA, LD_FF, RC, LD_E, 2 * wave, 0, part + OFF_W1, E, part + OFF_B1);

  {  // 7. dX1 = dY2 + dpre W1  -> RB
    f32x4 acc[RT0][1];
    zero_acc(acc);
    if (hf == 0) gemm_yw_pre<1, FF, E, 0, RT0>(RA, LD_FF, w1f, acc);
    else gemm_yw_pre<1, FF, E, RT0, RT - RT0>(RA, LD_FF, w1f, acc);
    const int col = 16 * sg + i16;
#pragma unroll
    for (int r = 0; r < RT0; ++r) {
      if (r >= nr) break;
#pragma unroll
      for (int q = 0; q < 4; ++q) RB[(16 * (r0 + r) + 4 * h4 + q) * LD_E + col] += acc[r][0][q];
    }
  }
  // ctx (step 9) and the step-11 W_o fragments: in flight across the LN1 backward
  TilePf<E> pf_ctx;
  pf_issue(pf_ctx, a.ctx + tok0 * E, tv);
  YwFrags<1, E, E> wof;
  yw_issue(wof, w.w_o, sg);
  __syncthreads();
  FR_MARK(1, 6);

  // 8. LN1 backward: RB = dY1, and dO = dropout1'(dY1) -> RC, db_o
  ln_rows_bwd(RB, ln1, tv, RD, part + OFF_G1, part + OFF_BE1, RC, ks.k[1], tok0, w.thr[1], w.scale[1],
              part + OFF_BO);

  // 9. ctx -> RD
  pf_commit(pf_ctx, RD, LD_E, tv);
  TilePf<QKV> pf_qkv;  // qkv (step 11): in flight across the dW_o slab and the dctx GEMM
  pf_issue(pf_qkv, a.qkv + tok0 * QKV, tv);
  __syncthreads();
  FR_MARK(1, 7);

  // 10. dW_o = dO^T ctx [64 x 64] (wave: n-tile sg, k-tiles 2hf, 2hf+1)
  wgrad_tiles<1, 2>(RC, LD_E, RD, LD_E, sg, 2 * hf, part + OFF_WO, E);  // (db_o: with the LN1 backward)

  // dY1 rows of this lane's final dX elements, held in registers: the attention scratch overlays RB
  float dy1[RT0][4];
#pragma unroll
  for (int r = 0; r < RT0; ++r)
#pragma unroll
    for (int q = 0; q < 4; ++q) dy1[r][q] = r < nr ? RB[(16 * (r0 + r) + 4 * h4 + q) * LD_E + 16 * sg + i16] : 0.f;

  {  // 11. dctx = dO W_o -> RC;  qkv -> RA
    f32x4 acc[RT0][1];
    zero_acc(acc);
    if (hf == 0) gemm_yw_pre<1, E, E, 0, RT0>(RC, LD_E, wof, acc);
    else gemm_yw_pre<1, E, E, RT0, RT - RT0>(RC, LD_E, wof, acc);
    pf_commit(pf_qkv, RA, LD_QKV, tv);
    __syncthreads();
    FR_MARK(1, 8);
    const int col = 16 * sg + i16;
#pragma unroll
    for (int r = 0; r < RT0; ++r) {
      if (r >= nr) break;
#pragma unroll
      for (int q = 0; q < 4; ++q) RC[(16 * (r0 + r) + 4 * h4 + q) * LD_E + col] = acc[r][0][q];
    }
  }
  __syncthreads();
  FR_MARK(1, 9);

  // 12. attention backward on MFMA, one head at a time (the scratch holds one head's tiles):
  //   phase 1: query tiles (5 waves): P, dP'^T, dS, the P' / dS tiles, dQ -> DQ
  //   phase 2: (key tile, dK | dV, column tile) jobs: dK = dS^T Q, dV = P'^T dctx over the k / v slots
  //   then dQ over the head's q slots (phase 2 has read them)
  const int wv = wave_id();
  if constexpr (L == 20) {
    attn_bwd_seq<L>(RA, RC, MS, seq0, ks.k[0], w, RB + wv * 2 * SEQ_TSZ);
    __syncthreads();
  } else
  for (int hh = 0; hh < HEADS; ++hh) {
    if (wv < RT) attn_bwd_rows_any<L>(wv, RA, RC, MS, hh, seq0, ks.k[0], w, SP, SS, DQ, prof);
    __syncthreads();
    if (hh == 0) FR_MARK(1, 18);
    for (int j = wv; j < RT * 2 * (HD / 16); j += NT / 64)
      attn_bwd_keys<L>(RA, RC, SP, SS, hh, j % RT, (j / RT) % 2, j / (2 * RT));
    __syncthreads();
    if (hh == 0) FR_MARK(1, 19);
    for (int e = threadIdx.x; e < ROWS * (HD / 4); e += NT) {
      const int r = e / (HD / 4), c4 = e % (HD / 4);
      *reinterpret_cast<float4*>(RA + r * LD_QKV + hh * HD + 4 * c4) = lds4(DQ + r * DQ_LD + 4 * c4);
    }
    __syncthreads();
  }
  FR_MARK(1, 10);
  // x (step 13), then the step-14 GEMM's W_in fragments (K = 192: 48 registers, in flight across the
  // dW_in slab); x's commit waits only for its own loads (issued first: loads retire in order)
  TilePf<E> pf_x;
  pf_issue(pf_x, a.x + tok0 * E, tv);
  YwFrags<1, QKV, E> winf;
  yw_issue(winf, w.w_in, sg);
  FR_SCHED_FENCE();
  if (tv < ROWS) lds_zero(RA + tv * LD_QKV, LD_QKV, ROWS - tv, QKV);
  pf_commit(pf_x, RC, LD_E, tv);
  __syncthreads();
  FR_MARK(1, 12);

  // 13. db_in; dW_in = dqkv^T x [192 x 64] (wave: n-tiles 3sg..3sg+2, k-tiles 2hf, 2hf+1)
  wgrad_tiles<3, 2>(RA, LD_QKV, RC, LD_E, 3 * sg, 2 * hf, part + OFF_WIN, E, hf == 0 ? part + OFF_BIN : nullptr);

  {  // 14. dX = dY1 + dqkv W_in
    f32x4 acc[RT0][1];
    zero_acc(acc);
    if (hf == 0) gemm_yw_pre<1, QKV, E, 0, RT0>(RA, LD_QKV, winf, acc);
    else gemm_yw_pre<1, QKV, E, RT0, RT - RT0>(RA, LD_QKV, winf, acc);
    const int col = 16 * sg + i16;
#pragma unroll
    for (int r = 0; r < RT0; ++r) {
      if (r >= nr) break;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int row = 16 * (r0 + r) + 4 * h4 + q;
        if (row < tv) a.dx[(tok0 + row) * E + col] = dy1[r][q] + acc[r][0][q];
      }
    }
  }
  FR_MARK(1, 31);
}

// grad[j] = sum over workgroups of part[wg][j], in a fixed order (deterministic).  A block owns 16
// float4 columns and 16 slices; slice s sums workgroups s, s + 16, s + 32, ... in order (all of its
// loads in flight at once: 16 per thread at 256 workgroups), then the slices are added in slice
// order.  781 blocks for the 12,496 float4 columns: three per CU, every CU streaming.
constexpr int RED_COLS = 16, RED_SL = 16, RED_UNR = 16;
__global__ __launch_bounds__(256) void enc_reduce_kernel(const float4* __restrict__ part, int nwg,
                                                         float4* __restrict__ grad) {
  constexpr int N4 = NPART / 4;
  __shared__ float4 sl[RED_SL][RED_COLS];
  const int c = blockIdx.x * RED_COLS + (threadIdx.x % RED_COLS), slice = threadIdx.x / RED_COLS;
  const int cc = min(c, N4 - 1);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int g0 = slice; g0 < nwg; g0 += RED_SL * RED_UNR) {
    float4 v[RED_UNR];
#pragma unroll
    for (int k = 0; k < RED_UNR; ++k) {
      const int g = min(g0 + k * RED_SL, nwg - 1);
      v[k] = part[(int64_t)g * N4 + cc];
    }
#pragma unroll
    for (int k = 0; k < RED_UNR; ++k)
      if (g0 + k * RED_SL < nwg) s = f4_add(s, v[k]);
  }
  sl[slice][threadIdx.x % RED_COLS] = s;
  __syncthreads();
  if (slice == 0 && c < N4) {
    float4 t = sl[0][threadIdx.x];
#pragma unroll
    for (int k = 1; k < RED_SL; ++k) t = f4_add(t, sl[k][threadIdx.x]);
    grad_store4(reinterpret_cast<float*>(grad), c, t);
  }
}

// The same sum with every load a contiguous 1 KiB piece of one workgroup's partial row (round 5): a
// block owns 64 float4 columns (lane = column) and RW_W waves; wave w sums workgroups w, w + RW_W,
// w + 2 RW_W, ... in order (RW_UNR loads in flight), then the waves' sums are added in wave order
// through LDS.  Deterministic like the kernel above (a different fixed order).  196 blocks of 16 waves
// at NPART: every load streams whole 128-B lines of one partial row.
constexpr int RW_W = 16, RW_UNR = 16;
__global__ __launch_bounds__(64 * RW_W) void enc_reduce_rows_kernel(const float4* __restrict__ part, int nwg,
                                                                   float4* __restrict__ grad) {
  constexpr int N4 = NPART / 4;
  __shared__ float4 sl[RW_W][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, cc = min(c, N4 - 1);
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int g0 = w; g0 < nwg; g0 += RW_W * RW_UNR) {
    float4 v[RW_UNR];
#pragma unroll
    for (int k = 0; k < RW_UNR; ++k) v[k] = part[(int64_t)min(g0 + k * RW_W, nwg - 1) * N4 + cc];
#pragma unroll
    for (int k = 0; k < RW_UNR; ++k)
      if (g0 + k * RW_W < nwg) s = f4_add(s, v[k]);
  }
  sl[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < N4) {
    float4 t = sl[0][lane];
#pragma unroll
    for (int k = 1; k < RW_W; ++k) t = f4_add(t, sl[k][lane]);
    grad_store4(reinterpret_cast<float*>(grad), c, t);
  }
}

// 0: enc_reduce_kernel (default), 1: enc_reduce_rows_kernel (A/B: fr_encoder_options; measured
// 9.9 vs 9.7 us alone at HealthRec's shape, not kept as the default)
int g_reduce_mode = 0;

void launch_reduce(const float* part, int64_t nwg, float* grad, hipStream_t s) {
  if (g_reduce_mode == 1)
    hipLaunchKernelGGL(enc_reduce_rows_kernel, dim3((unsigned)fr::ceil_div(NPART / 4, 64)), dim3(64 * RW_W), 0, s,
                       reinterpret_cast<const float4*>(part), (int)nwg, reinterpret_cast<float4*>(grad));
  else
    hipLaunchKernelGGL(enc_reduce_kernel, dim3((unsigned)fr::ceil_div(NPART / 4, RED_COLS)), dim3(256), 0, s,
                       reinterpret_cast<const float4*>(part), (int)nwg, reinterpret_cast<float4*>(grad));
}

template <int L>
int launch_fwd(const FwdArgs& a, hipStream_t s) {
  const int64_t nwg = fr::ceil_div(a.ns, ROWS / L);
  hipLaunchKernelGGL(enc_fwd_kernel<L>, dim3((unsigned)nwg), dim3(NT), 0, s, a);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

template <int L>
int launch_bwd(const BwdArgs& a, float* grad, hipStream_t s) {
  const int64_t nwg = fr::ceil_div(a.ns, ROWS / L);
  hipLaunchKernelGGL(enc_bwd_kernel<L>, dim3((unsigned)nwg), dim3(NT), 0, s, a);
  FR_LAUNCH_CHECK();
  if (grad) {
    launch_reduce(a.part, nwg, grad, s);
    FR_LAUNCH_CHECK();
  }
  return FR_OK;
}

bool supported_len(int L) { return L == 20 || L == 16 || L == 10 || L == 8 || L == 5 || L == 4; }

int fill_weights(Weights& w, const float* const* p, const float* eps, const float* drop, uint64_t seed, int gelu) {
  w.w_in = p[0]; w.b_in = p[1]; w.w_o = p[2]; w.b_o = p[3]; w.g1 = p[4]; w.be1 = p[5];
  w.w1 = p[6]; w.b1 = p[7]; w.w2 = p[8]; w.b2 = p[9]; w.g2 = p[10]; w.be2 = p[11];
  for (int k = 0; k < 12; ++k) FR_REQUIRE(p[k] && fr::aligned16(p[k]), "parameter pointers must be 16-byte aligned");
  w.eps1 = eps[0];
  w.eps2 = eps[1];
  for (int k = 0; k < 4; ++k) {
    FR_REQUIRE(drop[k] >= 0.f && drop[k] < 1.f, "dropout probability must be in [0, 1)");
    const double t = (double)drop[k] * 65536.0;
    w.thr[k] = drop[k] == 0.f ? 0u : (uint32_t)(t >= 65535.0 ? 65535.0 : t);
    w.scale[k] = 1.f / (1.f - drop[k]);
  }
  w.seed = seed;
  w.gelu = gelu;
  return FR_OK;
}

}  // namespace

extern "C" int64_t fr_encoder_partials(int64_t n_seq, int L) {
  if (n_seq <= 0 || !supported_len(L)) return 0;
  return fr::ceil_div(n_seq, ROWS / L) * (int64_t)NPART;
}

extern "C" int64_t fr_encoder_grad_numel(void) { return NPART; }

// floats of the forward's dact buffer (per-workgroup MFMA fragment layout, ROWS x FF per workgroup)
extern "C" int64_t fr_encoder_dact_numel(int64_t n_seq, int L) {
  if (n_seq <= 0 || !supported_len(L)) return 0;
  return fr::ceil_div(n_seq, ROWS / L) * (int64_t)(ROWS * FF);
}

extern "C" int fr_encoder_profile(int enable, uint64_t* host_marks) {
  if (enable >= 0) {
    const int on = enable ? 1 : 0;
    FR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_prof_on), &on, sizeof(on)));
  }
  if (host_marks) FR_HIP_CHECK(hipMemcpyFromSymbol(host_marks, HIP_SYMBOL(g_prof), sizeof(g_prof)));
  return FR_OK;
}

extern "C" int fr_encoder_fwd(const float* d_x, const float* d_mask, int64_t n_seq, int L,
                              const float* const* d_params, const float* eps, const float* drop, uint64_t seed,
                              int gelu, const int64_t* d_counter, int64_t* d_seed_out, float* d_out,
                              float* d_qkv, float* d_ctx, float* d_y1, float* d_fact, float* d_dact, float* d_y2,
                              float* d_st1, float* d_st2, void* stream) {
  FR_REQUIRE(n_seq > 0 && supported_len(L), "L must be one of 4, 5, 8, 10, 16, 20 and n_seq > 0");
  FR_REQUIRE(n_seq * L * FF < (int64_t)1 << 32 && n_seq * HEADS * L * L < (int64_t)1 << 32,
             "too many tokens for the 32-bit dropout element index");
  FR_REQUIRE(d_x && d_out && d_counter && d_seed_out && d_qkv && d_ctx && d_y1 && d_fact && d_dact && d_y2 &&
                 d_st1 && d_st2,
             "null operand");
  FR_REQUIRE(fr::aligned16(d_x) && fr::aligned16(d_out) && fr::aligned16(d_qkv) && fr::aligned16(d_ctx) &&
                 fr::aligned16(d_y1) && fr::aligned16(d_fact) && fr::aligned16(d_dact) && fr::aligned16(d_y2),
             "tensors must be 16-byte aligned");
  FwdArgs a{};
  int rc = fill_weights(a.w, d_params, eps, drop, seed, gelu);
  if (rc) return rc;
  a.x = d_x; a.mask = d_mask; a.ns = n_seq; a.counter = d_counter; a.seed_out = d_seed_out; a.out = d_out;
  a.qkv = d_qkv; a.ctx = d_ctx; a.y1 = d_y1; a.fact = d_fact; a.dact = d_dact; a.y2 = d_y2; a.st1 = d_st1; a.st2 = d_st2;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (L) {
    case 20: return launch_fwd<20>(a, s);
    case 16: return launch_fwd<16>(a, s);
    case 10: return launch_fwd<10>(a, s);
    case 8: return launch_fwd<8>(a, s);
    case 5: return launch_fwd<5>(a, s);
    default: return launch_fwd<4>(a, s);
  }
}

extern "C" int fr_encoder_bwd(const float* d_dout, const float* d_x, const float* d_mask, int64_t n_seq, int L,
                              const float* const* d_params, const float* eps, const float* drop, uint64_t seed,
                              int gelu, const int64_t* d_seed_in, const float* d_qkv, const float* d_ctx,
                              const float* d_y1, const float* d_fact, const float* d_dact, const float* d_y2,
                              const float* d_st1, const float* d_st2, float* d_dx, float* d_grad, float* d_partials,
                              int64_t partial_floats, const float* d_prev_partials, float* d_prev_grad,
                              void* stream) {
  FR_REQUIRE(n_seq > 0 && supported_len(L), "L must be one of 4, 5, 8, 10, 16, 20 and n_seq > 0");
  FR_REQUIRE(d_dout && d_x && d_seed_in && d_qkv && d_ctx && d_y1 && d_fact && d_dact && d_y2 && d_st1 && d_st2 &&
                 d_dx && d_partials,
             "null operand");
  FR_REQUIRE(!d_prev_partials == !d_prev_grad, "d_prev_partials and d_prev_grad go together");
  FR_REQUIRE(fr::aligned16(d_dout) && fr::aligned16(d_x) && fr::aligned16(d_dx) && fr::aligned16(d_grad) &&
                 fr::aligned16(d_partials) && fr::aligned16(d_qkv) && fr::aligned16(d_ctx) && fr::aligned16(d_y1) &&
                 fr::aligned16(d_y2) && fr::aligned16(d_prev_partials) && fr::aligned16(d_prev_grad),
             "tensors must be 16-byte aligned");
  FR_REQUIRE(partial_floats >= fr_encoder_partials(n_seq, L), "partial buffer too small");
  BwdArgs a{};
  int rc = fill_weights(a.w, d_params, eps, drop, seed, gelu);
  if (rc) return rc;
  a.dout = d_dout; a.x = d_x; a.mask = d_mask; a.ns = n_seq; a.seed_in = d_seed_in;
  a.qkv = d_qkv; a.ctx = d_ctx; a.y1 = d_y1; a.fact = d_fact; a.dact = d_dact; a.y2 = d_y2; a.st1 = d_st1; a.st2 = d_st2;
  a.dx = d_dx; a.part = d_partials; a.prev_part = d_prev_partials; a.prev_grad = d_prev_grad;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  switch (L) {
    case 20: return launch_bwd<20>(a, d_grad, s);
    case 16: return launch_bwd<16>(a, d_grad, s);
    case 10: return launch_bwd<10>(a, d_grad, s);
    case 8: return launch_bwd<8>(a, d_grad, s);
    case 5: return launch_bwd<5>(a, d_grad, s);
    default: return launch_bwd<4>(a, d_grad, s);
  }
}

extern "C" int fr_encoder_reduce(const float* d_partials, int64_t n_seq, int L, float* d_grad, void* stream) {
  FR_REQUIRE(n_seq > 0 && supported_len(L), "L must be one of 4, 5, 8, 10, 16, 20 and n_seq > 0");
  FR_REQUIRE(d_partials && d_grad && fr::aligned16(d_partials) && fr::aligned16(d_grad), "null or unaligned operand");
  const int64_t nwg = fr::ceil_div(n_seq, ROWS / L);
  launch_reduce(d_partials, nwg, d_grad, reinterpret_cast<hipStream_t>(stream));
  FR_LAUNCH_CHECK();
  return FR_OK;
}

// A/B switches of the encoder's launches (host-side state of this library): reduce_mode 0 = the
// column-slice ordered reduction (default), 1 = the row-streaming one; -1 leaves it.
extern "C" int fr_encoder_options(int reduce_mode) {
  FR_REQUIRE(reduce_mode >= -1 && reduce_mode <= 1, "reduce_mode must be -1, 0 or 1");
  if (reduce_mode >= 0) g_reduce_mode = reduce_mode;
  return FR_OK;
}
