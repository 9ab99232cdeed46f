// Per-item modal fusion math of HealthRec (models/cikm_model.py:245-249, 311-369), shared by the
// fusion kernels (fr_fusion.hip) and the fused loss head (fr_modal_head.hip).  See fr_fusion.hip for
// the formulas.  One wave owns one item with lane = embedding column (head = lane / 32).
#pragma once
#include "fr_common.h"

namespace {

constexpr int D = 64, HD = 32;
constexpr int NQ = 2;                 // modal queries per item (image, text)
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


// The fusion backward of one item given d know (already divided by num) ``dk`` and d hin (already
// halved) ``dv`` for lane c: d enc / d query written, the four LayerNorm-parameter partial sums
// accumulated (lane c: column c of its head).
template <int L>
__device__ __forceinline__ void fusion_item_bwd(const ItemFwd<L>& f, const FusionArgs& a, int64_t item, int c,
                                                float dk, float dv, float& pg_a, float& pb_a, float& pg_b,
                                                float& pb_b) {
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
  // the L quotients by the same N^3 through one double reciprocal: RN32(x * RN64(1 / y)) is the
  // correctly rounded x / y for every normal quotient (fr_ssl.hip's div_rden), 3 operations each
  const float dkN = dk / N, dkS = dk * S;
  const double rN3 = 1.0 / (double)(N * N * N);
#pragma unroll
  for (int t = 0; t < L; ++t) dM[t] = clampM ? dkN : dkN - (float)((double)(f.M[t] * dkS) * rN3);
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

// know / hin of one item (lane c), from its forward
template <int L>
__device__ __forceinline__ void fusion_item_out(const ItemFwd<L>& f, float num, float& know, float& hin) {
  float n2 = 0.f;
#pragma unroll
  for (int t = 0; t < L; ++t) n2 = fmaf(f.M[t], f.M[t], n2);
  const float N = fmaxf(sqrtf(n2), kNormEps);
  float s = 0.f;
  const double rN = 1.0 / (double)N;  // (the L quotients by N through one double reciprocal, as above)
#pragma unroll
  for (int t = 0; t < L; ++t) s += (float)((double)f.M[t] * rN);
  know = s / num;
  const float hN = fmaxf(sqrtf(fmaf(f.H[0], f.H[0], f.H[1] * f.H[1])), kNormEps);
  hin = (f.H[0] / hN + f.H[1] / hN) * 0.5f;
}

}  // namespace
