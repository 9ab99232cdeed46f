// Fused health / knowledge-distillation loss head of HealthRec (training forward + backward), gfx950.
//
// Replaces, over the 2B batch items (models/cikm_model.py:249-264, 304-308; common/trainer.py sums
// the returned terms):
//   health_pred = sigmoid(Linear(H<-64)(relu(Linear(64<-64)(hin))))           (self.health_mlp)
//   out[0]      = w_h * sum(BCELoss(reduction='none')(health_pred, labels))     (loss_health * ...)
//   kd          = 1 - cosine_similarity(know, rows, dim=-1).mean()              (rows = item_all[ids])
//   out[1]      = w_k * max(0, kd - kd_threshold)                               (loss_kd * norm_loss)
// torch runs this as ~20 kernels forward and ~25 backward (addmm, relu, sigmoid, BCE, norms, clamps,
// divisions, reductions), each a few microseconds at n = 1024.  Here one wave owns one item with
// lane = embedding column: the 64x64 Linear is lane-local FMAs against a padded LDS copy of W1 (row
// stride 65: conflict-free both for lane = row in the forward and lane = column in the backward)
// with the input broadcast by readlane; the H outputs, the norms and the cosine are wave sums.
// Elementwise formulas follow ATen's kernels (sigmoid 1/(1+exp(-x)); BCE with log/log1p clamped at
// -100; BCE backward (p-y)/max((1-p)p, 1e-12); sigmoid backward g(1-p)p; cosine norms clamped at
// 1e-8; maximum's backward halves the gradient on a tie).
// Loss sums are per-block partials summed by a one-wave finalize launch (fixed-order wave sum);
// parameter gradients are per-block partials summed in a fixed order by a reduce kernel.
// Forward item inputs are loaded one item ahead; every load loop has a compile-time trip count.
#include "fr_head_math.h"

namespace {

constexpr int D = 64;
constexpr int WAVES = 8;          // forward: waves per block (2 per SIMD), up to 128 blocks
constexpr int BWAVES = 4;         // backward: 4 waves per block (its 64 dW1 accumulators per lane need the
                                  // full register file), up to 256 blocks
constexpr int MAX_BLOCKS = 128;   // forward grid cap (1024 items: one per wave)
constexpr int MAX_BLOCKS_BWD = 256;  // backward grid cap: bounds the parameter-gradient partials

struct HeadArgs {
  const float* hin;     // [n, 64]
  const float* know;    // [n, 64]
  const float* rows;    // [n, 64] item_all[ids]
  const float* labels;  // [n, H]
  int64_t n;
  int H;
  const float *w1, *b1, *w2, *b2;  // [64,64], [64], [H,64], [H]
  float thr, wh, wk;
  float* out;           // [3]: w_h * health, w_k * kd_term, kd - thr (the gate, for the backward)
  float* part;          // forward: [nblk, 2]; backward: [nblk, NPART_BWD]
  // backward
  const float* gh;      // d loss / d out[0]  (device scalar)
  const float* gk;      // d loss / d out[1]
  float *dhin, *dknow, *drows;
  float *dw1, *db1, *dw2, *db2;
};

template <int NW>
__device__ __forceinline__ void stage_weights(const HeadArgs& a, float* sw1, float* sw2, float* sb) {
  head_stage_weights<64 * NW>(a.w1, a.b1, a.w2, a.b2, a.H, sw1, sw2, sb);
}

// one item's inputs for lane j (loaded one item ahead of use)
struct ItemIn {
  float h, k, r, y[HMAX];
};

__device__ __forceinline__ ItemIn load_item(const HeadArgs& a, int64_t i, int j) {
  ItemIn x;
  const int64_t c = i < a.n ? i : a.n - 1;  // clamped: the prefetch past the end is never used
  x.h = a.hin[c * D + j];
  x.k = a.know[c * D + j];
  x.r = a.rows[c * D + j];
#pragma unroll
  for (int t = 0; t < HMAX; ++t) x.y[t] = t < a.H ? a.labels[c * a.H + t] : 0.f;
  return x;
}

__device__ __forceinline__ float layer1(const float* sw1, const float* sb, float h, int j) {
  return head_layer1(sw1, sb, h, j);
}

__global__ __launch_bounds__(64 * WAVES) void head_fwd_kernel(HeadArgs a) {
  __shared__ float sw1[D * W1S];
  __shared__ float sw2[HMAX * D];
  __shared__ float sb[D + HMAX];
  __shared__ float red[WAVES][2];
  stage_weights<WAVES>(a, sw1, sw2, sb);
  const int j = threadIdx.x & 63, w = threadIdx.x >> 6;
  float sum_bce = 0.f, sum_cos = 0.f;
  const int64_t stride = (int64_t)gridDim.x * WAVES;
  int64_t i = (int64_t)blockIdx.x * WAVES + w;
  ItemIn cur = load_item(a, i, j);
  for (; i < a.n; i += stride) {
    const ItemIn nxt = load_item(a, i + stride, j);
    const float a1 = fmaxf(layer1(sw1, sb, cur.h, j), 0.f);
    float z2[HMAX];
#pragma unroll
    for (int t = 0; t < HMAX; ++t) z2[t] = t < a.H ? sw2[t * D + j] * a1 : 0.f;
#pragma unroll
    for (int t = 0; t < HMAX; ++t)
      if (t < a.H) z2[t] = wsum(z2[t]);
    float item_bce = 0.f;
#pragma unroll
    for (int t = 0; t < HMAX; ++t)
      if (t < a.H) item_bce += bce(sigmoidf_(z2[t] + sb[D + t]), cur.y[t]);
    sum_bce += item_bce;
    const float n1 = fmaxf(sqrtf(wsum(cur.k * cur.k)), kCosEps), n2 = fmaxf(sqrtf(wsum(cur.r * cur.r)), kCosEps);
    sum_cos += wsum((cur.k / n1) * (cur.r / n2));
    cur = nxt;
  }
  if (j == 0) { red[w][0] = sum_bce; red[w][1] = sum_cos; }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sb_ = 0.f, sc = 0.f;
    for (int q = 0; q < WAVES; ++q) { sb_ += red[q][0]; sc += red[q][1]; }
    a.part[2 * blockIdx.x] = sb_;
    a.part[2 * blockIdx.x + 1] = sc;
  }
}

// the loss terms from the <= 128 block partials (lane j: blocks j, j + 64 in that order), one
// fixed-order wave sum each
__global__ __launch_bounds__(64) void head_final_kernel(HeadArgs a, int nblk) {
  const int j = threadIdx.x;
  float sb_ = 0.f, sc = 0.f;
  for (int b = j; b < nblk; b += 64) {
    sb_ += a.part[2 * b];
    sc += a.part[2 * b + 1];
  }
  const float tb = wsum(sb_);
  const float tc = wsum(sc);
  if (j != 0) return;
  const float kd = 1.f - tc / (float)a.n;
  const float x = kd - a.thr;
  a.out[0] = a.wh * tb;
  a.out[1] = a.wk * fmaxf(0.f, x);
  a.out[2] = x;
}

__global__ __launch_bounds__(64 * BWAVES) void head_bwd_kernel(HeadArgs a) {
  __shared__ float sw1[D * W1S];
  __shared__ float sw2[HMAX * D];
  __shared__ float sb[D + HMAX];
  __shared__ float comb[D * D + D + HMAX * D + HMAX];
  stage_weights<BWAVES>(a, sw1, sw2, sb);
  const int j = threadIdx.x & 63, w = threadIdx.x >> 6;
  const float gh = *a.gh * a.wh;
  // maximum(0, x) backward for x: g where x > 0, g / 2 on a tie, 0 below
  const float x = a.out[2];
  const float gk = *a.gk * a.wk;
  const float dkd = x > 0.f ? gk : (x == 0.f ? gk * 0.5f : 0.f);
  const float dc = -dkd / (float)a.n;  // mean backward, then (1 - mean)
  float gw1[D];
#pragma unroll
  for (int k = 0; k < D; ++k) gw1[k] = 0.f;
  float gb1 = 0.f, gw2[HMAX], gb2[HMAX];
#pragma unroll
  for (int t = 0; t < HMAX; ++t) { gw2[t] = 0.f; gb2[t] = 0.f; }
  const int64_t stride = (int64_t)gridDim.x * BWAVES;
  for (int64_t i = (int64_t)blockIdx.x * BWAVES + w; i < a.n; i += stride) {
    const ItemIn cur = load_item(a, i, j);  // one item per wave at n <= 1024: no prefetch registers
    // health branch
    const float h = cur.h;
    const float z1 = layer1(sw1, sb, h, j);
    const float a1 = fmaxf(z1, 0.f);
    float z2s[HMAX];
#pragma unroll
    for (int t = 0; t < HMAX; ++t) z2s[t] = t < a.H ? sw2[t * D + j] * a1 : 0.f;
#pragma unroll
    for (int t = 0; t < HMAX; ++t)
      if (t < a.H) z2s[t] = wsum(z2s[t]);
    float da1 = 0.f;
#pragma unroll
    for (int t = 0; t < HMAX; ++t) {
      if (t < a.H) {
        const float z2 = z2s[t] + sb[D + t];
        const float p = sigmoidf_(z2), y = cur.y[t];
        const float g = gh * (p - y) / fmaxf((1.f - p) * p, 1e-12f);
        const float dz2 = g * (1.f - p) * p;
        gw2[t] = fmaf(dz2, a1, gw2[t]);
        gb2[t] += dz2;
        da1 = fmaf(sw2[t * D + j], dz2, da1);
      }
    }
    const float dz1 = a1 > 0.f ? da1 : 0.f;
    gb1 += dz1;
    float dh = 0.f;
#pragma unroll
    for (int k = 0; k < D; ++k) {
      const float dzk = bcast(dz1, k);
      dh = fmaf(sw1[k * W1S + j], dzk, dh);  // lane j: column j of W1
      gw1[k] = fmaf(dzk, h, gw1[k]);         // lane j holds column j: dW1[k][j] += dz1_k h_j
    }
    a.dhin[i * D + j] = dh;
    // KD branch
    const float kv = cur.k, rv = cur.r;
    const float n1 = fmaxf(sqrtf(wsum(kv * kv)), kCosEps), n2 = fmaxf(sqrtf(wsum(rv * rv)), kCosEps);
    const float kh = kv / n1, rh = rv / n2;
    const float c = wsum(kh * rh);
    a.dknow[i * D + j] = dc * (rh - c * kh) / n1;
    a.drows[i * D + j] = dc * (kh - c * rh) / n2;
  }
  // combine the waves' accumulators in wave order, then one partial per block
  for (int q = 0; q < BWAVES; ++q) {
    if (w == q) {
#pragma unroll
      for (int k = 0; k < D; ++k) comb[k * D + j] = (q ? comb[k * D + j] : 0.f) + gw1[k];
      comb[D * D + j] = (q ? comb[D * D + j] : 0.f) + gb1;
#pragma unroll
      for (int t = 0; t < HMAX; ++t) comb[D * D + D + t * D + j] = (q ? comb[D * D + D + t * D + j] : 0.f) + gw2[t];
      if (j < HMAX) {
        float v = 0.f;
#pragma unroll
        for (int t = 0; t < HMAX; ++t) v = t == j ? gb2[t] : v;
        // dz2 is a wave sum, so every lane holds the same gb2[]; lane t writes entry t
        comb[D * D + D + HMAX * D + j] = (q ? comb[D * D + D + HMAX * D + j] : 0.f) + v;
      }
    }
    __syncthreads();
  }
  float* dst = a.part + (int64_t)blockIdx.x * NPART_BWD;
  for (int e = threadIdx.x; e < NPART_BWD; e += blockDim.x) dst[e] = comb[e];
}

// sums the per-block partials into dW1, db1, dW2, db2: 32 outputs x 8 block slices per workgroup,
// each thread's <= 32 loads in flight (nblk <= 256), slices added in slice order (deterministic)
__global__ __launch_bounds__(256) void head_reduce_kernel(const float* __restrict__ part, int nblk, int H,
                                                          float* __restrict__ dw1, float* __restrict__ db1,
                                                          float* __restrict__ dw2, float* __restrict__ db2) {
  __shared__ float red[8][32];
  const int o = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int e = blockIdx.x * 32 + o;
  float v[MAX_BLOCKS_BWD / 8];
#pragma unroll
  for (int u = 0; u < MAX_BLOCKS_BWD / 8; ++u) {
    const int b = sl + 8 * u;
    v[u] = (b < nblk && e < NPART_BWD) ? part[(int64_t)b * NPART_BWD + e] : 0.f;
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < MAX_BLOCKS_BWD / 8; ++u) s += v[u];
  red[sl][o] = s;
  __syncthreads();
  if (sl != 0 || e >= NPART_BWD) return;
  float t = red[0][o];
#pragma unroll
  for (int q = 1; q < 8; ++q) t += red[q][o];
  if (e < D * D) {
    dw1[e] = t;
  } else if (e < D * D + D) {
    db1[e - D * D] = t;
  } else if (e < D * D + D + HMAX * D) {
    if ((e - D * D - D) / D < H) dw2[e - D * D - D] = t;
  } else if (e - D * D - D - HMAX * D < H) {
    db2[e - D * D - D - HMAX * D] = t;
  }
}

int blocks_for(int64_t n) { return (int)std::min<int64_t>(fr::ceil_div(n, WAVES), MAX_BLOCKS); }
int bwd_blocks_for(int64_t n) { return (int)std::min<int64_t>(fr::ceil_div(n, BWAVES), MAX_BLOCKS_BWD); }

int common_args(HeadArgs& a, const float* hin, const float* know, const float* rows, const float* labels, int64_t n,
                int H, const float* const* mlp, float thr, float wh, float wk, float* out) {
  FR_REQUIRE(n > 0 && H >= 1 && H <= HMAX, "n > 0 and 1 <= H <= 16 required");
  FR_REQUIRE(hin && know && rows && labels && mlp && mlp[0] && mlp[1] && mlp[2] && mlp[3] && out, "null operand");
  a.hin = hin; a.know = know; a.rows = rows; a.labels = labels; a.n = n; a.H = H;
  a.w1 = mlp[0]; a.b1 = mlp[1]; a.w2 = mlp[2]; a.b2 = mlp[3];
  a.thr = thr; a.wh = wh; a.wk = wk; a.out = out;
  return FR_OK;
}

}  // namespace

extern "C" int64_t fr_health_kd_partials(int64_t n_items, int backward) {
  if (n_items <= 0) return 0;
  return backward ? bwd_blocks_for(n_items) * NPART_BWD : 1 + 2 * blocks_for(n_items);  // forward: the ticket word, then 2 floats per block
}

extern "C" int fr_health_kd_fwd(const float* d_hin, const float* d_know, const float* d_rows, const float* d_labels,
                                int64_t n_items, int H, const float* const* d_mlp, float kd_threshold, float w_health,
                                float w_kd, float* d_out, float* d_partials, int64_t partial_floats, void* stream) {
  HeadArgs a{};
  int rc = common_args(a, d_hin, d_know, d_rows, d_labels, n_items, H, d_mlp, kd_threshold, w_health, w_kd, d_out);
  if (rc) return rc;
  FR_REQUIRE(d_partials && partial_floats >= fr_health_kd_partials(n_items, 0), "partial buffer too small");
  const int nb = blocks_for(n_items);
  a.part = d_partials + 1;  // word 0 is unused (kept for the partial-buffer layout)
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(head_fwd_kernel, dim3(nb), dim3(64 * WAVES), 0, s, a);
  FR_LAUNCH_CHECK();
  // a second launch instead of an in-kernel last-block reduction: a device-scope fence per block
  // costs more than the kernel boundary
  hipLaunchKernelGGL(head_final_kernel, dim3(1), dim3(64), 0, s, a, nb);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_health_kd_bwd(const float* d_hin, const float* d_know, const float* d_rows, const float* d_labels,
                                int64_t n_items, int H, const float* const* d_mlp, float kd_threshold, float w_health,
                                float w_kd, const float* d_out, const float* d_gh, const float* d_gk, float* d_dhin,
                                float* d_dknow, float* d_drows, float* const* d_dmlp, float* d_partials,
                                int64_t partial_floats, void* stream) {
  HeadArgs a{};
  int rc = common_args(a, d_hin, d_know, d_rows, d_labels, n_items, H, d_mlp, kd_threshold, w_health, w_kd,
                       const_cast<float*>(d_out));
  if (rc) return rc;
  FR_REQUIRE(d_gh && d_gk && d_dhin && d_dknow && d_drows && d_dmlp && d_dmlp[0] && d_dmlp[1] && d_dmlp[2] &&
                 d_dmlp[3] && d_partials, "null operand");
  FR_REQUIRE(partial_floats >= fr_health_kd_partials(n_items, 1), "partial buffer too small");
  a.gh = d_gh; a.gk = d_gk; a.dhin = d_dhin; a.dknow = d_dknow; a.drows = d_drows; a.part = d_partials;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int nb = bwd_blocks_for(n_items);
  hipLaunchKernelGGL(head_bwd_kernel, dim3(nb), dim3(64 * BWAVES), 0, s, a);
  FR_LAUNCH_CHECK();
  hipLaunchKernelGGL(head_reduce_kernel, dim3(fr::ceil_div(NPART_BWD, 32)), dim3(256), 0, s, d_partials, nb, H,
                     d_dmlp[0], d_dmlp[1], d_dmlp[2], d_dmlp[3]);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
