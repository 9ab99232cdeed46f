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

#include "fr_fusion_item.h"

namespace {

constexpr int WAVES = 4;              // items per block

template <int L>
__global__ __launch_bounds__(64 * WAVES) void fusion_fwd_kernel(FusionArgs a) {
  const int64_t item = (int64_t)blockIdx.x * WAVES + (threadIdx.x >> 6);
  const int c = threadIdx.x & 63;
  if (item >= a.n_items) return;  // wave-uniform
  ItemFwd<L> f;
  f.run(a, item, c);
  // know = sum_t normalize(item_mm)[t] / n ;  hin = mean_r normalize(item_health)[r]
  float know, hin;
  fusion_item_out(f, (float)a.num[item], know, hin);
  a.know[item * D + c] = know;
  a.hin[item * D + c] = hin;
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
    fusion_item_bwd(f, a, item, c, a.dknow[item * D + c] / (float)a.num[item], a.dhin[item * D + c] * 0.5f,
                    pg_a, pb_a, pg_b, pb_b);
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
