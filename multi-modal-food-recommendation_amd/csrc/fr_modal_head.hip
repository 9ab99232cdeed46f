// HealthRec's loss head after the ingredient encoder, fused (training forward + backward), gfx950.
//
// One autograd node for models/cikm_model.py:245-264 (+ 304-308, 311-369) over the 2B batch items:
//   know, hin  = the two target attentions + F.normalize heads          (fr_fusion.hip's per-item math)
//   out[0]     = w_h * sum(BCELoss(sigmoid(health_mlp(hin)), labels))  (fr_health_kd.hip's per-item math)
//   out[1]     = w_k * max(0, 1 - cosine_similarity(know, rows).mean() - kd_threshold)
// The separate path runs fusion_fwd -> head_fwd -> head_final forward and head_bwd -> head_reduce ->
// fusion_bwd -> fusion_reduce backward: seven launches in a serial chain of latency-bound kernels,
// know / hin / their gradients round-tripping through memory.  Here:
//   forward   modal_head_fwd: per item (one wave, lane = column) the fusion forward and the head's
//             forward in registers; per-block (BCE, cosine) partials; head_final-style one-wave
//             finalize (fixed-order sums) writes out[0..2];
//   backward  modal_head_bwd: per item the fusion forward recomputed, the head's backward (dhin,
//             dknow in registers, drows written for the BPR kernel's item rows), then the fusion
//             backward from them (d enc, d query); every parameter gradient of the block (health
//             MLP, both LayerNorms) as one partial row; one ordered column reduction afterwards (it
//             feeds only the optimiser: the caller may run it beside the encoder backward).
// Deterministic: fixed per-block wave order, partials summed in block order.
#include "fr_fusion_item.h"
#include "fr_head_math.h"

namespace {

constexpr int WAVES = 4;  // items per block (one per wave); 256 threads
constexpr int NT = 64 * WAVES;
constexpr int NPF = 4 * HD;                 // fusion LayerNorm-parameter gradients: dga, dba, dgb, dbb [32]
constexpr int NPH = NPART_BWD;              // health MLP: dW1 [64x64], db1, dW2 [HMAX x 64], db2 [HMAX]
constexpr int NPART_ROW = NPH + NPF;        // one block's partial row

struct HeadArgs {
  FusionArgs f;               // enc, query, ids, num, pad_id, n_items, LayerNorm params, eps; denc, dquery
  const float* rows;          // [n, 64] item_all[ids] (the BPR kernel's item rows)
  const float* labels;        // [n, H]
  int H;
  const float *w1, *b1, *w2, *b2;
  float thr, wh, wk;
  float* out;                 // [3]: w_h * health, w_k * kd term, kd - thr (the gate)
  float* part;                // forward: [nblk, 2]; backward: [nblk, NPART_ROW]
  int32_t* ticket;            // forward: zero-initialised arrival counter (the last block finalises; reset to 0)
  const float *gh, *gk;       // upstream gradients of out[0], out[1] (device scalars)
  float* drows;               // [n, 64]
};

// head forward of one item: (BCE sum over the H labels, cosine(know, rows)) -- wave-uniform
__device__ __forceinline__ float2 head_item_fwd(const HeadArgs& a, const float* sw1, const float* sw2, const float* sb,
                                                int64_t item, int j, float know, float hin) {
  const float a1 = fmaxf(head_layer1(sw1, sb, hin, j), 0.f);
  float z2[HMAX];
#pragma unroll
  for (int t = 0; t < HMAX; ++t) z2[t] = t < a.H ? wsum(sw2[t * HEAD_D + j] * a1) : 0.f;
  float item_bce = 0.f;
#pragma unroll
  for (int t = 0; t < HMAX; ++t)
    if (t < a.H) item_bce += bce(sigmoidf_(z2[t] + sb[HEAD_D + t]), a.labels[item * a.H + t]);
  const float r = a.rows[item * HEAD_D + j];
  const float n1 = fmaxf(sqrtf(wsum(know * know)), kCosEps), n2 = fmaxf(sqrtf(wsum(r * r)), kCosEps);
  return make_float2(item_bce, wsum((know / n1) * (r / n2)));
}

__device__ __forceinline__ void head_final(const HeadArgs& a, int nblk, int j);

template <int L>
__global__ __launch_bounds__(NT) void modal_head_fwd_kernel(HeadArgs a) {
  __shared__ float sw1[HEAD_D * W1S];
  __shared__ float sw2[HMAX * HEAD_D];
  __shared__ float sb[HEAD_D + HMAX];
  __shared__ float red[WAVES][2];
  head_stage_weights<NT>(a.w1, a.b1, a.w2, a.b2, a.H, sw1, sw2, sb);
  const int w = threadIdx.x >> 6, c = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * WAVES + w;
  float2 v = make_float2(0.f, 0.f);
  if (item < a.f.n_items) {  // wave-uniform
    ItemFwd<L> f;
    f.run(a.f, item, c);
    float know, hin;
    fusion_item_out(f, (float)a.f.num[item], know, hin);
    v = head_item_fwd(a, sw1, sw2, sb, item, c, know, hin);
  }
  if (c == 0) {
    red[w][0] = v.x;
    red[w][1] = v.y;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sbce = 0.f, scos = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) {
      sbce += red[q][0];
      scos += red[q][1];
    }
    a.part[2 * blockIdx.x] = sbce;
    a.part[2 * blockIdx.x + 1] = scos;
  }
  if (a.ticket) {  // the last block to arrive sums every block's partials (the final kernel's work)
    __shared__ int last;
    if (threadIdx.x == 0) {
      __threadfence();  // this block's partials before its arrival
      last = atomicAdd(a.ticket, 1) == (int)gridDim.x - 1;
    }
    __syncthreads();
    if (last) {
      __threadfence();  // every block's partials visible to this one
      if (threadIdx.x < 64) head_final(a, (int)gridDim.x, threadIdx.x);
      if (threadIdx.x == 0) a.ticket[0] = 0;  // ready for the next launch (graph replays)
    }
  }
}

// the loss terms from the block partials (lane j: blocks j, j + 64, ... in that order), one
// fixed-order wave sum each (one wave)
__device__ __forceinline__ void head_final(const HeadArgs& a, int nblk, int j) {
  float sbce = 0.f, scos = 0.f;
  for (int b0 = j; b0 < nblk; b0 += 256) {  // four blocks' partials in flight, added in block order
    float2 x[4];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      x[u] = b0 + 64 * u < nblk ? make_float2(a.part[2 * (b0 + 64 * u)], a.part[2 * (b0 + 64 * u) + 1])
                                : make_float2(0.f, 0.f);
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b0 + 64 * u < nblk) {
        sbce += x[u].x;
        scos += x[u].y;
      }
  }
  const float tb = wsum(sbce), tc = wsum(scos);
  if (j != 0) return;
  const float x = (1.f - tc / (float)a.f.n_items) - a.thr;
  a.out[0] = a.wh * tb;
  a.out[1] = a.wk * fmaxf(0.f, x);
  a.out[2] = x;
}

__global__ __launch_bounds__(64) void modal_head_final_kernel(HeadArgs a, int nblk) { head_final(a, nblk, threadIdx.x); }

template <int L>
__global__ __launch_bounds__(NT) void modal_head_bwd_kernel(HeadArgs a) {
  __shared__ float sw1[HEAD_D * W1S];
  __shared__ float sw2[HMAX * HEAD_D];
  __shared__ float sb[HEAD_D + HMAX];
  __shared__ float s_dz1[WAVES][HEAD_D], s_h[WAVES][HEAD_D], s_a1[WAVES][HEAD_D], s_dz2[WAVES][HMAX];
  __shared__ float s_ln[WAVES][NPARAM];
  head_stage_weights<NT>(a.w1, a.b1, a.w2, a.b2, a.H, sw1, sw2, sb);
  const int w = threadIdx.x >> 6, j = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * WAVES + w;
  const int64_t n = a.f.n_items;
  // maximum(0, x) backward: g where x > 0, g / 2 on a tie, 0 below; then the mean and (1 - mean)
  const float x = a.out[2];
  const float gk = *a.gk * a.wk, gh = *a.gh * a.wh;
  const float dkd = x > 0.f ? gk : (x == 0.f ? gk * 0.5f : 0.f);
  const float dc = -dkd / (float)n;
  float pg_a = 0.f, pb_a = 0.f, pg_b = 0.f, pb_b = 0.f;
  float dz1 = 0.f, h = 0.f, a1 = 0.f, dz2v = 0.f;
  if (item < n) {  // wave-uniform
    ItemFwd<L> f;
    f.run(a.f, item, j);
    const float num = (float)a.f.num[item];
    float know;
    fusion_item_out(f, num, know, h);
    // health branch
    const float z1 = head_layer1(sw1, sb, h, j);
    a1 = fmaxf(z1, 0.f);
    float z2s[HMAX];
#pragma unroll
    for (int t = 0; t < HMAX; ++t) z2s[t] = t < a.H ? wsum(sw2[t * HEAD_D + j] * a1) : 0.f;
    float da1 = 0.f;
#pragma unroll
    for (int t = 0; t < HMAX; ++t) {
      if (t < a.H) {
        const float p = sigmoidf_(z2s[t] + sb[HEAD_D + t]), y = a.labels[item * a.H + t];
        const float g = gh * (p - y) / fmaxf((1.f - p) * p, 1e-12f);
        const float dz2 = g * (1.f - p) * p;  // wave-uniform
        dz2v = t == j ? dz2 : dz2v;           // lane t keeps entry t for the partial
        da1 = fmaf(sw2[t * HEAD_D + j], dz2, da1);
      }
    }
    dz1 = a1 > 0.f ? da1 : 0.f;
    float dh = 0.f;
#pragma unroll
    for (int k = 0; k < HEAD_D; ++k) dh = fmaf(sw1[k * W1S + j], bcast(dz1, k), dh);  // lane j: column j of W1
    // KD branch
    const float rv = a.rows[item * HEAD_D + j];
    const float n1 = fmaxf(sqrtf(wsum(know * know)), kCosEps), n2 = fmaxf(sqrtf(wsum(rv * rv)), kCosEps);
    const float kh = know / n1, rh = rv / n2;
    const float cs = wsum(kh * rh);
    const float dknow = dc * (rh - cs * kh) / n1;
    a.drows[item * HEAD_D + j] = dc * (kh - cs * rh) / n2;
    // the fusion backward from d know / d hin
    fusion_item_bwd(f, a.f, item, j, dknow / num, dh * 0.5f, pg_a, pb_a, pg_b, pb_b);
  }
  s_dz1[w][j] = dz1;
  s_h[w][j] = h;
  s_a1[w][j] = a1;
  if (j < HMAX) s_dz2[w][j] = dz2v;
  s_ln[w][j] = pg_a;
  s_ln[w][HEAD_D + j] = pb_a;
  s_ln[w][2 * HEAD_D + j] = pg_b;
  s_ln[w][3 * HEAD_D + j] = pb_b;
  __syncthreads();
  // the block's partial row, waves summed in order: dW1[k][i] = sum_w dz1_w[k] h_w[i], db1, dW2[t][i] =
  // sum_w dz2_w[t] a1_w[i], db2, then the LayerNorm partials folded over the head halves (j, j + 32)
  float* dst = a.part + (int64_t)blockIdx.x * NPART_ROW;
#pragma unroll
  for (int u = 0; u < HEAD_D * HEAD_D / NT; ++u) {
    const int e = threadIdx.x + u * NT, k = e >> 6, i = e & 63;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) s = fmaf(s_dz1[q][k], s_h[q][i], s);
    dst[e] = s;
  }
#pragma unroll
  for (int u = 0; u < HMAX * HEAD_D / NT; ++u) {
    const int e = threadIdx.x + u * NT, t = e >> 6, i = e & 63;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) s = fmaf(s_dz2[q][t], s_a1[q][i], s);
    dst[HEAD_D * HEAD_D + HEAD_D + e] = s;
  }
  if (threadIdx.x < HEAD_D) {
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) s += s_dz1[q][threadIdx.x];
    dst[HEAD_D * HEAD_D + threadIdx.x] = s;
  } else if (threadIdx.x < HEAD_D + HMAX) {
    const int t = threadIdx.x - HEAD_D;
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) s += s_dz2[q][t];
    dst[HEAD_D * HEAD_D + HEAD_D + HMAX * HEAD_D + t] = s;
  } else if (threadIdx.x >= 128) {
    const int e = threadIdx.x - 128, kind = e / HD, i = e % HD;  // 128 LayerNorm outputs
    float s = 0.f;
#pragma unroll
    for (int q = 0; q < WAVES; ++q) s += s_ln[q][kind * HEAD_D + i] + s_ln[q][kind * HEAD_D + i + HD];
    dst[NPH + e] = s;
  }
}

// out[e] = sum over blocks b (in order) of part[b][e], e < NPART_ROW: 32 columns x 8 block slices
// per workgroup, each slice's loads in flight together, slices added in slice order
__global__ __launch_bounds__(256) void modal_head_reduce_kernel(const float* __restrict__ part, int nblk,
                                                                float* __restrict__ out) {
  __shared__ float red[8][32];
  const int o = threadIdx.x & 31, sl = threadIdx.x >> 5;
  const int e = min(blockIdx.x * 32 + o, NPART_ROW - 1);
  float s = 0.f;
  for (int b0 = sl; b0 < nblk; b0 += 8 * 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)min(b0 + 8 * u, nblk - 1) * NPART_ROW + e];
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (b0 + 8 * u < nblk) s += v[u];
  }
  red[sl][o] = s;
  __syncthreads();
  if (sl == 0 && blockIdx.x * 32 + o < NPART_ROW) {
    float t = red[0][o];
#pragma unroll
    for (int q = 1; q < 8; ++q) t += red[q][o];
    out[blockIdx.x * 32 + o] = t;
  }
}

bool supported_len(int L) { return L == 20 || L == 16 || L == 10 || L == 8 || L == 5 || L == 4; }

int fill(HeadArgs& a, const float* enc, const float* query, const int64_t* ids, const int64_t* num, int64_t pad_id,
         int64_t n, int L, const float* const* ln, float eps, const float* rows, const float* labels, int H,
         const float* const* mlp, float thr, float wh, float wk, float* out) {
  FR_REQUIRE(n > 0 && supported_len(L), "n_items > 0 and L in {4, 5, 8, 10, 16, 20} required");
  FR_REQUIRE(H >= 1 && H <= HMAX, "1 <= H <= 16 required");
  FR_REQUIRE(enc && query && ids && num && ln && ln[0] && ln[1] && ln[2] && ln[3] && rows && labels && mlp &&
                 mlp[0] && mlp[1] && mlp[2] && mlp[3] && out,
             "null operand");
  a.f.enc = enc; a.f.query = query; a.f.ids = ids; a.f.num = num; a.f.pad_id = pad_id; a.f.n_items = n;
  a.f.ga = ln[0]; a.f.ba = ln[1]; a.f.gb = ln[2]; a.f.bb = ln[3]; a.f.eps = eps;
  a.rows = rows; a.labels = labels; a.H = H;
  a.w1 = mlp[0]; a.b1 = mlp[1]; a.w2 = mlp[2]; a.b2 = mlp[3];
  a.thr = thr; a.wh = wh; a.wk = wk; a.out = out;
  return FR_OK;
}

template <int L>
void launch(const HeadArgs& a, bool backward, hipStream_t s) {
  const unsigned nb = (unsigned)fr::ceil_div(a.f.n_items, WAVES);
  if (backward)
    hipLaunchKernelGGL(modal_head_bwd_kernel<L>, dim3(nb), dim3(NT), 0, s, a);
  else
    hipLaunchKernelGGL(modal_head_fwd_kernel<L>, dim3(nb), dim3(NT), 0, s, a);
}

int dispatch(const HeadArgs& a, int L, bool backward, hipStream_t s) {
  switch (L) {
    case 20: launch<20>(a, backward, s); break;
    case 16: launch<16>(a, backward, s); break;
    case 10: launch<10>(a, backward, s); break;
    case 8: launch<8>(a, backward, s); break;
    case 5: launch<5>(a, backward, s); break;
    default: launch<4>(a, backward, s); break;
  }
  FR_LAUNCH_CHECK();
  return FR_OK;
}

}  // namespace

// HealthRec's loss finalize in one launch (one 256-thread block): the head's finalize (the loss
// terms from fr_modal_head_fwd_items' block partials: head_final), the EmbLoss ingredient norms from
// fr_gather_norms_fwd's partials (norms_final's fixed-order sums), reg = w * (a + (n0 + n1) / B)
// (fr_reg_combine_fwd's arithmetic) and, when acc is given, the step's bookkeeping over the parts
// [mf, health, kd, reg] (fr_step_book's arithmetic and counter advance).
struct LossFin {
  const float* npart; int nnblk;
  const float* emb3; float B, w;
  float *nrm, *reg;
  const float* mf;
  double* acc; int accumulate; int32_t* nan; float* loss;
  int64_t* ctr[8]; int nc;
};

__global__ __launch_bounds__(256) void loss_finalize_kernel(HeadArgs a, int nblk, LossFin f) {
  __shared__ float red[2][256];
  // thread 0's bookkeeping operands (independent of the sums) and every thread's first norm partials
  // are loaded before anything waits: the launch's memory round trips overlap instead of chaining
  int64_t cv[8];
  double av[4];
  float mfv = 0.f;
  const bool book = threadIdx.x == 0 && f.npart && f.acc;
  if (book) {
#pragma unroll
    for (int i = 0; i < 8; ++i) cv[i] = i < f.nc ? f.ctr[i][0] : 0;
    mfv = f.mf[0];
#pragma unroll
    for (int i = 0; i < 4; ++i) av[i] = f.accumulate ? f.acc[i] : 0.0;
  }
  float s0 = 0.f, s1 = 0.f;
  if (f.npart && (int)threadIdx.x < f.nnblk) {
    s0 = f.npart[2 * threadIdx.x];
    s1 = f.npart[2 * threadIdx.x + 1];
  }
  if (a.part && threadIdx.x < 64) head_final(a, nblk, threadIdx.x);  // out[0..2], written by thread 0
  if (!f.npart) return;
  for (int b = threadIdx.x + 256; b < f.nnblk; b += 256) {
    s0 += f.npart[2 * b];
    s1 += f.npart[2 * b + 1];
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
  if (threadIdx.x != 0) return;
  const float n0 = sqrtf(red[0][0]), n1 = sqrtf(red[1][0]);
  f.nrm[0] = n0;
  f.nrm[1] = n1;
  const float reg = f.w * (f.emb3[0] + (n0 + n1) / f.B);
  f.reg[0] = reg;
  if (!book) return;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (i < f.nc) f.ctr[i][0] = cv[i] + 1;  // (distinct counters: checked by the host)
  const float v[4] = {mfv, a.out[0], a.out[1], reg};  // this thread wrote out[0..1] above
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f.acc[i] = f.accumulate ? av[i] + (double)v[i] : (double)v[i];
    s = i == 0 ? v[i] : s + v[i];
  }
  if (s != s) f.nan[0] |= 1;
  if (f.loss) f.loss[0] = s;
}

extern "C" int64_t fr_modal_head_partials(int64_t n_items, int backward) {
  if (n_items <= 0) return 0;
  const int64_t nb = fr::ceil_div(n_items, WAVES);
  return backward ? nb * NPART_ROW : 2 * nb;
}

extern "C" int64_t fr_modal_head_grad_numel(void) { return NPART_ROW; }

extern "C" int fr_modal_head_fwd(const float* d_enc, const float* d_query, const int64_t* d_ids, const int64_t* d_num,
                                 int64_t pad_id, int64_t n_items, int L, const float* const* d_ln, float eps,
                                 const float* d_rows, const float* d_labels, int H, const float* const* d_mlp,
                                 float kd_threshold, float w_health, float w_kd, float* d_out, float* d_partials,
                                 int64_t partial_floats, int32_t* d_ticket, void* stream) {
  HeadArgs a{};
  int rc = fill(a, d_enc, d_query, d_ids, d_num, pad_id, n_items, L, d_ln, eps, d_rows, d_labels, H, d_mlp,
                kd_threshold, w_health, w_kd, d_out);
  if (rc) return rc;
  FR_REQUIRE(d_partials && partial_floats >= fr_modal_head_partials(n_items, 0), "partial buffer too small");
  a.part = d_partials;
  a.ticket = d_ticket;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  rc = dispatch(a, L, false, s);
  if (rc) return rc;
  if (!d_ticket) {
    hipLaunchKernelGGL(modal_head_final_kernel, dim3(1), dim3(64), 0, s, a, (int)fr::ceil_div(n_items, WAVES));
    FR_LAUNCH_CHECK();
  }
  return FR_OK;
}

extern "C" int fr_modal_head_fwd_items(const float* d_enc, const float* d_query, const int64_t* d_ids,
                                       const int64_t* d_num, int64_t pad_id, int64_t n_items, int L,
                                       const float* const* d_ln, float eps, const float* d_rows, const float* d_labels,
                                       int H, const float* const* d_mlp, float kd_threshold, float w_health, float w_kd,
                                       float* d_partials, int64_t partial_floats, void* stream) {
  HeadArgs a{};
  float dummy_out[1];
  int rc = fill(a, d_enc, d_query, d_ids, d_num, pad_id, n_items, L, d_ln, eps, d_rows, d_labels, H, d_mlp,
                kd_threshold, w_health, w_kd, dummy_out);
  if (rc) return rc;
  a.out = nullptr;  // the per-item kernel writes only the block partials
  FR_REQUIRE(d_partials && partial_floats >= fr_modal_head_partials(n_items, 0), "partial buffer too small");
  a.part = d_partials;
  return dispatch(a, L, false, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int fr_healthrec_loss_finalize(const float* d_head_partials, int64_t n_items, float kd_threshold,
                                          float w_health, float w_kd, float* d_out, const float* d_norm_partials,
                                          int64_t n_norm_rows, const float* d_emb3, float B, float w_reg,
                                          float* d_nrm, float* d_reg, const float* d_mf, double* d_acc, int accumulate,
                                          int32_t* d_nan, int64_t* const* d_counters, int n_counters, float* d_loss,
                                          void* stream) {
  FR_REQUIRE(!d_head_partials || (n_items > 0 && d_out), "head finalize needs n_items and out");
  FR_REQUIRE(!d_norm_partials || (n_norm_rows > 0 && d_emb3 && B > 0.f && d_nrm && d_reg), "norms / reg operands");
  FR_REQUIRE(!d_acc || (d_head_partials && d_norm_partials && d_mf && d_nan), "bookkeeping needs every part");
  FR_REQUIRE(n_counters >= 0 && n_counters <= 8 && (n_counters == 0 || d_counters), "0..8 counters");
  HeadArgs a{};
  a.part = const_cast<float*>(d_head_partials);
  a.f.n_items = n_items;
  a.thr = kd_threshold; a.wh = w_health; a.wk = w_kd; a.out = d_out;
  LossFin f{};
  f.npart = d_norm_partials;
  f.nnblk = d_norm_partials ? (int)(fr_gather_norms_partials(n_norm_rows) / 2) : 0;
  f.emb3 = d_emb3; f.B = B; f.w = w_reg; f.nrm = d_nrm; f.reg = d_reg; f.mf = d_mf;
  f.acc = d_acc; f.accumulate = accumulate; f.nan = d_nan; f.loss = d_loss;
  for (int i = 0; i < n_counters; ++i) {
    FR_REQUIRE(d_counters[i] != nullptr, "null counter");
    for (int j = 0; j < i; ++j) FR_REQUIRE(d_counters[j] != d_counters[i], "counters must be distinct");
    f.ctr[i] = d_counters[i];
  }
  f.nc = n_counters;
  hipLaunchKernelGGL(loss_finalize_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a,
                     d_head_partials ? (int)fr::ceil_div(n_items, WAVES) : 0, f);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_modal_head_bwd(const float* d_enc, const float* d_query, const int64_t* d_ids, const int64_t* d_num,
                                 int64_t pad_id, int64_t n_items, int L, const float* const* d_ln, float eps,
                                 const float* d_rows, const float* d_labels, int H, const float* const* d_mlp,
                                 float kd_threshold, float w_health, float w_kd, const float* d_out, const float* d_gh,
                                 const float* d_gk, float* d_denc, float* d_dquery, float* d_drows, float* d_partials,
                                 int64_t partial_floats, void* stream) {
  HeadArgs a{};
  int rc = fill(a, d_enc, d_query, d_ids, d_num, pad_id, n_items, L, d_ln, eps, d_rows, d_labels, H, d_mlp,
                kd_threshold, w_health, w_kd, const_cast<float*>(d_out));
  if (rc) return rc;
  FR_REQUIRE(d_gh && d_gk && d_denc && d_dquery && d_drows && d_partials, "null operand");
  FR_REQUIRE(partial_floats >= fr_modal_head_partials(n_items, 1), "partial buffer too small");
  a.gh = d_gh; a.gk = d_gk; a.f.denc = d_denc; a.f.dquery = d_dquery; a.drows = d_drows; a.part = d_partials;
  return dispatch(a, L, true, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int fr_modal_head_reduce(const float* d_partials, int64_t n_items, float* d_grad, void* stream) {
  FR_REQUIRE(n_items > 0 && d_partials && d_grad, "null operand");
  hipLaunchKernelGGL(modal_head_reduce_kernel, dim3((unsigned)fr::ceil_div(NPART_ROW, 32)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), d_partials, (int)fr::ceil_div(n_items, WAVES), d_grad);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
