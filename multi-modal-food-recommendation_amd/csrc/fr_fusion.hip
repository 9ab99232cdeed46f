// Fused modal fusion of HealthRec (training forward + backward), gfx950.
//
// Replaces, per item i of the 2B batch items (models/cikm_model.py:245-249, 311-369):
//   item_health = target_attention(Q_i, E_i, E_i, key mask)     mm_target_atten    (queries: 2 modal rows)
//   item_mm     = target_attention(E_i, Q_i, Q_i)               ingre_target_atten (queries: L tokens)
//   know_i      = F.normalize(item_mm, dim=1).sum(1) / ingre_num_i
//   hin_i       = F.normalize(item_health, dim=1).mean(1)       (the health MLP's input)
// where Q_i = [image_trs(img_i); text_trs(txt_i)] ([2, 64]), E_i = the encoder output ([L, 64]) and
// target_attention(q, k, v) splits 2 heads of 32 (chunk/cat), applies the module's LayerNorm(32,
// eps 1e-12) to the q and k heads (not v), scores = q k^T / sqrt(32), padded keys replaced by
// -(2^32 - 1) (keep * s + pad * C), softmax over keys, then p v.
//
// torch runs this as ~12 batched 2x20 / 20x2 GEMMs (bmm, ~25 us each at this size) plus ~40
// cat / chunk / LayerNorm / normalize kernels forward and backward.  Here one wave owns one item
// with lane = embedding column (head = lane / 32): LayerNorm statistics and score dot products are
// 32-lane shuffle reductions, every weighted sum is lane-local, nothing is staged through memory.
// Both LayerNorms normalise the same rows, so x^ = (x - mu) * rstd is computed once (equal eps).
// The backward recomputes the forward (a few microseconds) instead of saving activations; LayerNorm
// parameter gradients are per-block partials summed in block order (deterministic).
#include "fr_common.h"

namespace {

constexpr int D = 64, HD = 32;
constexpr int NQ = 2;                 // modal queries per item (image, text)
constexpr int WAVES = 4;              // items per block
constexpr float kScale = 0.17677669529663688f;  // 1/sqrt(32)
constexpr float kMasked = -4294967295.f;         // -(2^32) + 1 (cikm_model.py:356)
constexpr float kNormEps = 1e-12f;               // F.normalize eps
constexpr int NPARAM = 4 * D;         // partials per block: dgamma_a, dbeta_a, dgamma_b, dbeta_b per column

struct FusionArgs {
  const float* enc;      // [n_items, L, 64]
  const float* query;    // [n_items, 2, 64]
  const int64_t* ids;    // [n_items, L] ingredient ids (padded with pad_id)
  const int64_t* num;    // [n_items] ingredient counts
  int64_t pad_id;
  int64_t n_items;
  const float *ga, *ba, *gb, *bb;  // mm_target_atten.ln / ingre_target_atten.ln weight, bias [32]
  float eps;             // LayerNorm eps (both modules)
  // forward outputs
  float* know;           // [n_items, 64]
  float* hin;            // [n_items, 64]
  // backward
  const float* dknow;    // [n_items, 64]
  const float* dhin;     // [n_items, 64]
  float* denc;           // [n_items, L, 64]
  float* dquery;         // [n_items, 2, 64]
  float* part;           // [n_blocks, 4 * 64]
};

__device__ __forceinline__ float hsum(float v) { return group_sum<32>(v); }

// the forward of one item, kept in registers (lane = column c); shared by both kernels
template <int L>
struct ItemFwd {
  float e[L], xe[L], re[L];   // rows of E: value, x^, rstd (uniform per row)
  float q[NQ], xq[NQ], rq[NQ];
  float pa[NQ][L];            // mm_target_atten probabilities (uniform over the head's lanes)
  float pb[L][NQ];            // ingre_target_atten probabilities
  bool keep[L];
  float M[L], H[NQ];          // item_mm column, item_health column
  float ga, ba, gb, bb;

  __device__ __forceinline__ void run(const FusionArgs& a, int64_t item, int c) {
    const int j = c & (HD - 1);
    ga = a.ga[j]; ba = a.ba[j]; gb = a.gb[j]; bb = a.bb[j];
    const float* E = a.enc + item * (L * D);
    const float* Q = a.query + item * (NQ * D);
#pragma unroll
    for (int t = 0; t < L; ++t) {
      e[t] = E[t * D + c];
      keep[t] = a.ids[item * L + t] != a.pad_id;
    }
#pragma unroll
    for (int r = 0; r < NQ; ++r) q[r] = Q[r * D + c];
    // LayerNorm statistics per (row, head): mean and biased variance over the head's 32 columns
#pragma unroll
    for (int t = 0; t < L; ++t) {
      const float mu = hsum(e[t]) * (1.f / HD);
      const float d = e[t] - mu;
      re[t] = rsqrtf(hsum(d * d) * (1.f / HD) + a.eps);
      xe[t] = d * re[t];
    }
#pragma unroll
    for (int r = 0; r < NQ; ++r) {
      const float mu = hsum(q[r]) * (1.f / HD);
      const float d = q[r] - mu;
      rq[r] = rsqrtf(hsum(d * d) * (1.f / HD) + a.eps);
      xq[r] = d * rq[r];
    }
    // mm_target_atten: queries Q (LN a), keys E (LN a), values E; masked softmax over the L keys
#pragma unroll
    for (int r = 0; r < NQ; ++r) {
      const float qa = fmaf(xq[r], ga, ba);
      float mx = -INFINITY;
#pragma unroll
      for (int t = 0; t < L; ++t) {
        const float s = hsum(qa * fmaf(xe[t], ga, ba)) * kScale;
        pa[r][t] = keep[t] ? s : kMasked;
        mx = fmaxf(mx, pa[r][t]);
      }
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < L; ++t) {
        pa[r][t] = expf(pa[r][t] - mx);
        sum += pa[r][t];
      }
      const float inv = 1.f / sum;
      float h = 0.f;
#pragma unroll
      for (int t = 0; t < L; ++t) {
        pa[r][t] *= inv;
        h = fmaf(pa[r][t], e[t], h);
      }
      H[r] = h;
    }
    // ingre_target_atten: queries E (LN b), keys Q (LN b), values Q; softmax over the 2 keys
    const float kb0 = fmaf(xq[0], gb, bb), kb1 = fmaf(xq[1], gb, bb);
#pragma unroll
    for (int t = 0; t < L; ++t) {
      const float qb = fmaf(xe[t], gb, bb);
      const float s0 = hsum(qb * kb0) * kScale, s1 = hsum(qb * kb1) * kScale;
      const float mx = fmaxf(s0, s1);
      const float e0 = expf(s0 - mx), e1 = expf(s1 - mx);
      const float inv = 1.f / (e0 + e1);
      pb[t][0] = e0 * inv;
      pb[t][1] = e1 * inv;
      M[t] = fmaf(pb[t][0], q[0], pb[t][1] * q[1]);
    }
  }
};

template <int L>
__global__ __launch_bounds__(64 * WAVES) void fusion_fwd_kernel(FusionArgs a) {
  const int64_t item = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  const int c = threadIdx.x & 63;
  if (item >= a.n_items) return;  // wave-uniform
  ItemFwd<L> f;
  f.run(a, item, c);
  // know = sum_t normalize(item_mm)[t] / n ;  hin = mean_r normalize(item_health)[r]
  float n2 = 0.f;
#pragma unroll
  for (int t = 0; t < L; ++t) n2 = fmaf(f.M[t], f.M[t], n2);
  const float N = fmaxf(sqrtf(n2), kNormEps);
  float s = 0.f;
#pragma unroll
  for (int t = 0; t < L; ++t) s += f.M[t] / N;
  a.know[item * D + c] = s / (float)a.num[item];
  const float hN = fmaxf(sqrtf(fmaf(f.H[0], f.H[0], f.H[1] * f.H[1])), kNormEps);
  a.hin[item * D + c] = (f.H[0] / hN + f.H[1] / hN) * 0.5f;
}

template <int L>
__global__ __launch_bounds__(64 * WAVES) void fusion_bwd_kernel(FusionArgs a) {
  __shared__ float sp[WAVES][NPARAM];
  const int w = threadIdx.x >> 6, c = threadIdx.x & 63;
  const int64_t item = (int64_t)blockIdx.x * WAVES + w;
  float pg_a = 0.f, pb_a = 0.f, pg_b = 0.f, pb_b = 0.f;
  if (item < a.n_items) {  // wave-uniform
    ItemFwd<L> f;
    f.run(a, item, c);
    const float dk = a.dknow[item * D + c] / (float)a.num[item];
    const float dv = a.dhin[item * D + c] * 0.5f;
    // F.normalize backward (x / max(||x||, eps)): the clamp stops the norm's gradient
    float n2 = 0.f, S = 0.f;
#pragma unroll
    for (int t = 0; t < L; ++t) {
      n2 = fmaf(f.M[t], f.M[t], n2);
      S += f.M[t];
    }
    const float nr = sqrtf(n2);
    const bool clampM = nr <= kNormEps;
    const float N = fmaxf(nr, kNormEps);
    float dM[L];
#pragma unroll
    for (int t = 0; t < L; ++t) dM[t] = clampM ? dk / N : dk / N - f.M[t] * (dk * S) / (N * N * N);
    const float hr = sqrtf(fmaf(f.H[0], f.H[0], f.H[1] * f.H[1]));
    const bool clampH = hr <= kNormEps;
    const float hN = fmaxf(hr, kNormEps);
    float dH[NQ];
#pragma unroll
    for (int r = 0; r < NQ; ++r)
      dH[r] = clampH ? dv / hN : dv / hN - f.H[r] * (dv * (f.H[0] + f.H[1])) / (hN * hN * hN);

    float de[L], dq[NQ], dxe[L], dxq[NQ];
#pragma unroll
    for (int t = 0; t < L; ++t) de[t] = dxe[t] = 0.f;
#pragma unroll
    for (int r = 0; r < NQ; ++r) dq[r] = dxq[r] = 0.f;

    // ingre_target_atten backward (values Q raw; q = LN_b(E), k = LN_b(Q))
    const float kb0 = fmaf(f.xq[0], f.gb, f.bb), kb1 = fmaf(f.xq[1], f.gb, f.bb);
    float dkb0 = 0.f, dkb1 = 0.f;
#pragma unroll
    for (int t = 0; t < L; ++t) {
      dq[0] = fmaf(f.pb[t][0], dM[t], dq[0]);
      dq[1] = fmaf(f.pb[t][1], dM[t], dq[1]);
      const float dp0 = hsum(dM[t] * f.q[0]), dp1 = hsum(dM[t] * f.q[1]);
      const float dot = f.pb[t][0] * dp0 + f.pb[t][1] * dp1;
      const float ds0 = f.pb[t][0] * (dp0 - dot) * kScale, ds1 = f.pb[t][1] * (dp1 - dot) * kScale;
      const float qb = fmaf(f.xe[t], f.gb, f.bb);
      const float dqb = ds0 * kb0 + ds1 * kb1;
      dkb0 = fmaf(ds0, qb, dkb0);
      dkb1 = fmaf(ds1, qb, dkb1);
      dxe[t] = dqb * f.gb;
      pg_b = fmaf(dqb, f.xe[t], pg_b);
      pb_b += dqb;
    }
    dxq[0] = dkb0 * f.gb;
    dxq[1] = dkb1 * f.gb;
    pg_b = fmaf(dkb0, f.xq[0], fmaf(dkb1, f.xq[1], pg_b));
    pb_b += dkb0 + dkb1;

    // mm_target_atten backward (values E raw; q = LN_a(Q), k = LN_a(E); padded keys carry no gradient)
#pragma unroll
    for (int r = 0; r < NQ; ++r) {
      const float qa = fmaf(f.xq[r], f.ga, f.ba);
      float dpa[L];
      float dot = 0.f;
#pragma unroll
      for (int t = 0; t < L; ++t) {
        de[t] = fmaf(f.pa[r][t], dH[r], de[t]);
        dpa[t] = hsum(dH[r] * f.e[t]);
        dot = fmaf(f.pa[r][t], dpa[t], dot);
      }
      float dqa = 0.f;
#pragma unroll
      for (int t = 0; t < L; ++t) {
        const float ds = f.keep[t] ? f.pa[r][t] * (dpa[t] - dot) * kScale : 0.f;
        const float ka = fmaf(f.xe[t], f.ga, f.ba);
        dqa = fmaf(ds, ka, dqa);
        const float dka = ds * qa;
        dxe[t] = fmaf(dka, f.ga, dxe[t]);
        pg_a = fmaf(dka, f.xe[t], pg_a);
        pb_a += dka;
      }
      dxq[r] = fmaf(dqa, f.ga, dxq[r]);
      pg_a = fmaf(dqa, f.xq[r], pg_a);
      pb_a += dqa;
    }

    // LayerNorm backward through the shared x^: dx = rstd * (dx^ - mean(dx^) - x^ mean(dx^ x^))
#pragma unroll
    for (int t = 0; t < L; ++t) {
      const float m1 = hsum(dxe[t]) * (1.f / HD), m2 = hsum(dxe[t] * f.xe[t]) * (1.f / HD);
      de[t] += f.re[t] * (dxe[t] - m1 - f.xe[t] * m2);
      a.denc[item * (L * D) + t * D + c] = de[t];
    }
#pragma unroll
    for (int r = 0; r < NQ; ++r) {
      const float m1 = hsum(dxq[r]) * (1.f / HD), m2 = hsum(dxq[r] * f.xq[r]) * (1.f / HD);
      dq[r] += f.rq[r] * (dxq[r] - m1 - f.xq[r] * m2);
      a.dquery[item * (NQ * D) + r * D + c] = dq[r];
    }
  }
  sp[w][c] = pg_a;
  sp[w][D + c] = pb_a;
  sp[w][2 * D + c] = pg_b;
  sp[w][3 * D + c] = pb_b;
  __syncthreads();
  // block partial, waves in order
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < WAVES; ++k) s += sp[k][threadIdx.x];
  a.part[(int64_t)blockIdx.x * NPARAM + threadIdx.x] = s;
}

// out[k][j] = sum over blocks of part[b][k][j] + part[b][k][j + 32], k = dgamma_a, dbeta_a,
// dgamma_b, dbeta_b.  1024 threads: 128 outputs x 8 block slices (4 loads in flight each), slices
// added in slice order (deterministic).
__global__ __launch_bounds__(1024) void fusion_reduce_kernel(const float* __restrict__ part, int64_t nblk,
                                                             float* __restrict__ out) {
  __shared__ float red[8][4 * HD];
  const int o = threadIdx.x & 127, sl = threadIdx.x >> 7, k = o / HD, j = o % HD;
  float s = 0.f;
  for (int64_t b0 = sl; b0 < nblk; b0 += 32) {
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t b = min(b0 + 8 * u, nblk - 1);
      v[u] = part[b * NPARAM + k * D + j] + part[b * NPARAM + k * D + j + HD];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (b0 + 8 * u < nblk) s += v[u];
  }
  red[sl][o] = s;
  __syncthreads();
  if (sl == 0) {
    float t = red[0][o];
#pragma unroll
    for (int q = 1; q < 8; ++q) t += red[q][o];
    out[o] = t;
  }
}

bool supported_len(int L) { return L == 20 || L == 16 || L == 10 || L == 8 || L == 5 || L == 4; }

template <int L>
void launch(const FusionArgs& a, bool backward, hipStream_t s) {
  const unsigned blocks = (unsigned)fr::ceil_div(a.n_items, WAVES);
  if (backward)
    hipLaunchKernelGGL(fusion_bwd_kernel<L>, dim3(blocks), dim3(64 * WAVES), 0, s, a);
  else
    hipLaunchKernelGGL(fusion_fwd_kernel<L>, dim3(blocks), dim3(64 * WAVES), 0, s, a);
}

int dispatch(const FusionArgs& a, int L, bool backward, hipStream_t s) {
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

int common_args(FusionArgs& a, const float* enc, const float* query, const int64_t* ids, const int64_t* num,
                int64_t pad_id, int64_t n_items, int L, const float* const* ln, float eps) {
  FR_REQUIRE(n_items > 0 && supported_len(L), "n_items > 0 and L in {4, 5, 8, 10, 16, 20} required");
  FR_REQUIRE(enc && query && ids && num && ln && ln[0] && ln[1] && ln[2] && ln[3], "null operand");
  a.enc = enc; a.query = query; a.ids = ids; a.num = num; a.pad_id = pad_id; a.n_items = n_items;
  a.ga = ln[0]; a.ba = ln[1]; a.gb = ln[2]; a.bb = ln[3]; a.eps = eps;
  return FR_OK;
}

}  // namespace

extern "C" int64_t fr_modal_fusion_partials(int64_t n_items) {
  return n_items > 0 ? fr::ceil_div(n_items, WAVES) * NPARAM : 0;
}

extern "C" int fr_modal_fusion_fwd(const float* d_enc, const float* d_query, const int64_t* d_ids,
                                   const int64_t* d_num, int64_t pad_id, int64_t n_items, int L,
                                   const float* const* d_ln, float eps, float* d_know, float* d_hin, void* stream) {
  FusionArgs a{};
  int rc = common_args(a, d_enc, d_query, d_ids, d_num, pad_id, n_items, L, d_ln, eps);
  if (rc) return rc;
  FR_REQUIRE(d_know && d_hin, "null output");
  a.know = d_know; a.hin = d_hin;
  return dispatch(a, L, false, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int fr_modal_fusion_bwd(const float* d_enc, const float* d_query, const int64_t* d_ids,
                                   const int64_t* d_num, int64_t pad_id, int64_t n_items, int L,
                                   const float* const* d_ln, float eps, const float* d_dknow, const float* d_dhin,
                                   float* d_denc, float* d_dquery, float* d_dln, float* d_partials,
                                   int64_t partial_floats, void* stream) {
  FusionArgs a{};
  int rc = common_args(a, d_enc, d_query, d_ids, d_num, pad_id, n_items, L, d_ln, eps);
  if (rc) return rc;
  FR_REQUIRE(d_dknow && d_dhin && d_denc && d_dquery && d_dln && d_partials, "null operand");
  FR_REQUIRE(partial_floats >= fr_modal_fusion_partials(n_items), "partial buffer too small");
  a.dknow = d_dknow; a.dhin = d_dhin; a.denc = d_denc; a.dquery = d_dquery; a.part = d_partials;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  rc = dispatch(a, L, true, s);
  if (rc) return rc;
  hipLaunchKernelGGL(fusion_reduce_kernel, dim3(1), dim3(1024), 0, s, d_partials, fr::ceil_div(n_items, WAVES),
                     d_dln);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
