// Fused gather-dot-BPR + EmbLoss (forward and backward).
//
// Replaces, per step:
//   u = U_all[user]; p = I_all[pos]; n = I_all[neg]                 models/lightgcn.py:158-166
//   mf = -log(1e-10 + sigmoid(<u,p> - <u,n>)).mean()                 common/loss.py:32-34
//   reg = (||Ue[user]||_F + ||Ie[pos]||_F + ||Ie[neg]||_F) / B       common/loss.py:45-50
// B x 3 row gathers of d floats, a 16-lane group per triple (float4 per lane, shuffle reduce);
// no MFMA: d=64 dot products are bandwidth work.  Batch reductions are fp64 and fixed-order.
//
// Backward scatters into dense gradient tables.  Default: float atomics (one 256-B row segment
// per wave-instruction, the shape the atomic unit runs at full rate).  deterministic=1: every
// destination row is summed by its first-occurring slot in the reference's autograd order
// (index backward of pos, then of neg, each in batch order), so results are run-to-run identical.
#include "fr_common.h"
#include "fr_bf16.h"

#include <algorithm>
#include <type_traits>

namespace {

constexpr int LPR = 16;  // lanes per triple

struct BprWS {
  float* spos; float* sneg; float* squ; float* sqp; float* sqn;  // [B] each
  float* norms;                                                   // [4]: |U|,|P|,|N|, pad
  uint64_t* keys_u;  // deterministic scatter: (row << 20 | slot) of the user slots, sorted [pow2(B)]
  uint64_t* keys_i;  //   ... of the item slots (pos t -> t, neg t -> B + t), sorted [pow2(2B)]
};

// the deterministic scatter sorts the slot keys of a table in one workgroup's LDS when the larger
// table (2B item slots) fits: 16,384 keys = 128 KB
constexpr int64_t kDetSortMax = 16384;
__host__ __device__ inline int64_t pow2_at_least(int64_t n) {
  int64_t p = 1;
  while (p < n) p <<= 1;
  return p;
}

__host__ __device__ inline BprWS bpr_ws(void* base, int64_t B) {
  char* p = reinterpret_cast<char*>(base);
  auto take = [&](int64_t bytes) { char* r = p; p += (bytes + 255) / 256 * 256; return r; };
  BprWS w;
  w.spos = reinterpret_cast<float*>(take(B * 4));
  w.sneg = reinterpret_cast<float*>(take(B * 4));
  w.squ = reinterpret_cast<float*>(take(B * 4));
  w.sqp = reinterpret_cast<float*>(take(B * 4));
  w.sqn = reinterpret_cast<float*>(take(B * 4));
  w.norms = reinterpret_cast<float*>(take(16));
  const bool sortable = 2 * B <= kDetSortMax;
  w.keys_u = sortable ? reinterpret_cast<uint64_t*>(take(pow2_at_least(B) * 8)) : nullptr;
  w.keys_i = sortable ? reinterpret_cast<uint64_t*>(take(pow2_at_least(2 * B) * 8)) : nullptr;
  return w;
}

inline int64_t bpr_ws_bytes(int64_t B) {
  auto r = [](int64_t b) { return (b + 255) / 256 * 256; };
  const int64_t keys = 2 * B <= kDetSortMax ? r(pow2_at_least(B) * 8) + r(pow2_at_least(2 * B) * 8) : 0;
  return 5 * r(B * 4) + r(16) + keys;
}

__device__ __forceinline__ float4 ld4(const float* base, int64_t row, int64_t ld, int q) {
  return reinterpret_cast<const float4*>(base + row * ld)[q];
}

__global__ __launch_bounds__(256) void bpr_scores_kernel(
    const float* __restrict__ U, int64_t ldu, const float* __restrict__ I, int64_t ldi,
    const float* __restrict__ Ue, int64_t ldue, const float* __restrict__ Ie, int64_t ldie,
    const int64_t* __restrict__ uu, const int64_t* __restrict__ pp, const int64_t* __restrict__ nn,
    int64_t B, int d4, BprWS ws, float* __restrict__ rows_out, int64_t ldr) {
  constexpr int GPB = 256 / LPR;
  const int q0 = threadIdx.x % LPR;
  for (int64_t b = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; b < B;
       b += (int64_t)gridDim.x * GPB) {
    const int64_t u = uu[b], p = pp[b], n = nn[b];
    float sp = 0.f, sn = 0.f, a = 0.f, c = 0.f, e = 0.f;
    for (int q = q0; q < d4; q += LPR) {
      const float4 xu = ld4(U, u, ldu, q), xp = ld4(I, p, ldi, q), xn = ld4(I, n, ldi, q);
      sp += f4_dot(xu, xp);
      sn += f4_dot(xu, xn);
      if (rows_out) {  // [I[pos]; I[neg]] for another consumer of those rows
        reinterpret_cast<float4*>(rows_out + b * ldr)[q] = xp;
        reinterpret_cast<float4*>(rows_out + (B + b) * ldr)[q] = xn;
      }
      if (Ue) {
        const float4 eu = ld4(Ue, u, ldue, q), ep = ld4(Ie, p, ldie, q), en = ld4(Ie, n, ldie, q);
        a += f4_dot(eu, eu);
        c += f4_dot(ep, ep);
        e += f4_dot(en, en);
      }
    }
    sp = group_sum<LPR>(sp);
    sn = group_sum<LPR>(sn);
    a = group_sum<LPR>(a);
    c = group_sum<LPR>(c);
    e = group_sum<LPR>(e);
    if (q0 == 0) {
      ws.spos[b] = sp;
      ws.sneg[b] = sn;
      ws.squ[b] = a;
      ws.sqp[b] = c;
      ws.sqn[b] = e;
    }
  }
}

// one block, fixed-order fp64 reduction -> out[0..4], ws.norms
__global__ __launch_bounds__(1024) void bpr_reduce_kernel(int64_t B, float gamma, int has_emb, float w_emb,
                                                          BprWS ws, float* out) {
  __shared__ double red[4][16];
  double l = 0.0, a = 0.0, c = 0.0, e = 0.0;
  for (int64_t b = threadIdx.x; b < B; b += blockDim.x) {
    const float x = ws.spos[b] - ws.sneg[b];
    const float sg = 1.f / (1.f + expf(-x));
    l += (double)logf(gamma + sg);
    a += ws.squ[b];
    c += ws.sqp[b];
    e += ws.sqn[b];
  }
  l = group_sum_d<64>(l);
  a = group_sum_d<64>(a);
  c = group_sum_d<64>(c);
  e = group_sum_d<64>(e);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { red[0][w] = l; red[1][w] = a; red[2][w] = c; red[3][w] = e; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double s[4] = {0, 0, 0, 0};
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k)
      for (int j = 0; j < 4; ++j) s[j] += red[j][k];
    const float nu = has_emb ? (float)sqrt(s[1]) : 0.f;
    const float np = has_emb ? (float)sqrt(s[2]) : 0.f;
    const float nn = has_emb ? (float)sqrt(s[3]) : 0.f;
    out[0] = (float)(-s[0] / (double)B);
    out[1] = nu;
    out[2] = np;
    out[3] = nn;
    out[4] = w_emb * (((nu + np) + nn) / (float)B);  // (w_emb = 1: the EmbLoss itself, exactly)
    ws.norms[0] = nu;
    ws.norms[1] = np;
    ws.norms[2] = nn;
  }
}

// dL/ds+ for triple b (dL/ds- = -that), with the upstream scale applied
__device__ __forceinline__ float bpr_coef(const BprWS& ws, int64_t b, int64_t B, float gamma, float gmf) {
  const float x = ws.spos[b] - ws.sneg[b];
  const float sg = 1.f / (1.f + expf(-x));
  // d/dx -log(gamma + sigmoid(x)) / B = -sigmoid*(1-sigmoid) / (gamma + sigmoid) / B
  return -gmf / (float)B / (gamma + sg) * (sg * (1.f - sg));
}

__device__ __forceinline__ void atomic_row_add(float* base, int64_t row, int64_t ld, int q, float4 v) {
  float* p = base + row * ld + 4 * q;
  atomicAdd(p + 0, v.x);
  atomicAdd(p + 1, v.y);
  atomicAdd(p + 2, v.z);
  atomicAdd(p + 3, v.w);
}

__global__ __launch_bounds__(256) void bpr_bwd_atomic_kernel(
    const float* __restrict__ U, int64_t ldu, const float* __restrict__ I, int64_t ldi,
    const float* __restrict__ Ue, int64_t ldue, const float* __restrict__ Ie, int64_t ldie,
    const int64_t* __restrict__ uu, const int64_t* __restrict__ pp, const int64_t* __restrict__ nn,
    int64_t B, int d4, float gamma, float gmf, float greg, const float* gscale, float* dU, int64_t lddu,
    float* dI, int64_t lddi, float* dUe, int64_t lddue, float* dIe, int64_t lddie, BprWS ws,
    const float* __restrict__ extra, int64_t ldx) {
  constexpr int GPB = 256 / LPR;
  const int q0 = threadIdx.x % LPR;
  if (gscale) { gmf *= gscale[0]; if (dUe || dIe) greg *= gscale[1]; }
  const float inv_b = 1.f / (float)B;
  const float ru = ws.norms[0] > 0.f ? greg * inv_b / ws.norms[0] : 0.f;
  const float rp = ws.norms[1] > 0.f ? greg * inv_b / ws.norms[1] : 0.f;
  const float rn = ws.norms[2] > 0.f ? greg * inv_b / ws.norms[2] : 0.f;
  for (int64_t b = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; b < B;
       b += (int64_t)gridDim.x * GPB) {
    const int64_t u = uu[b], p = pp[b], n = nn[b];
    const float g = bpr_coef(ws, b, B, gamma, gmf);
    for (int q = q0; q < d4; q += LPR) {
      const float4 xu = ld4(U, u, ldu, q), xp = ld4(I, p, ldi, q), xn = ld4(I, n, ldi, q);
      if (dU) {
        float4 t = f4_scale(g, xp);
        t = f4_fma(-g, xn, t);
        atomic_row_add(dU, u, lddu, q, t);
      }
      if (dI) {
        float4 tp = f4_scale(g, xu), tn = f4_scale(-g, xu);
        if (extra) {  // gradient of the returned item rows [I[pos]; I[neg]] (another consumer of them)
          tp = f4_add(tp, ld4(extra, b, ldx, q));
          tn = f4_add(tn, ld4(extra, B + b, ldx, q));
        }
        atomic_row_add(dI, p, lddi, q, tp);
        atomic_row_add(dI, n, lddi, q, tn);
      }
      if (Ue && dUe) atomic_row_add(dUe, u, lddue, q, f4_scale(ru, ld4(Ue, u, ldue, q)));
      if (Ie && dIe) {
        atomic_row_add(dIe, p, lddie, q, f4_scale(rp, ld4(Ie, p, ldie, q)));
        atomic_row_add(dIe, n, lddie, q, f4_scale(rn, ld4(Ie, n, ldie, q)));
      }
    }
  }
}

// d = 64: one wave per triple, lane = column -- every row update is ONE atomic wave-instruction over
// 256 contiguous bytes (the full-rate shape of the memory-side atomic units; the float4-per-lane form
// above issues four 16-B-strided instructions per four rows).  Same per-element arithmetic.
__global__ __launch_bounds__(256) void bpr_bwd_atomic64_kernel(
    const float* __restrict__ U, int64_t ldu, const float* __restrict__ I, int64_t ldi,
    const float* __restrict__ Ue, int64_t ldue, const float* __restrict__ Ie, int64_t ldie,
    const int64_t* __restrict__ uu, const int64_t* __restrict__ pp, const int64_t* __restrict__ nn,
    int64_t B, float gamma, float gmf, float greg, const float* gscale, float* dU, int64_t lddu,
    float* dI, int64_t lddi, float* dUe, int64_t lddue, float* dIe, int64_t lddie, BprWS ws,
    const float* __restrict__ extra, int64_t ldx) {
  const int lane = threadIdx.x & 63;
  if (gscale) { gmf *= gscale[0]; if (dUe || dIe) greg *= gscale[1]; }
  const float inv_b = 1.f / (float)B;
  const float ru = ws.norms[0] > 0.f ? greg * inv_b / ws.norms[0] : 0.f;
  const float rp = ws.norms[1] > 0.f ? greg * inv_b / ws.norms[1] : 0.f;
  const float rn = ws.norms[2] > 0.f ? greg * inv_b / ws.norms[2] : 0.f;
  for (int64_t b = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6; b < B; b += (int64_t)gridDim.x * 4) {
    const int64_t u = uu[b], p = pp[b], n = nn[b];
    const float g = bpr_coef(ws, b, B, gamma, gmf);
    const float xu = U[u * ldu + lane], xp = I[p * ldi + lane], xn = I[n * ldi + lane];
    if (dU) atomicAdd(dU + u * lddu + lane, fmaf(-g, xn, g * xp));
    if (dI) {
      float tp = g * xu, tn = -g * xu;
      if (extra) {
        tp += extra[b * ldx + lane];
        tn += extra[(B + b) * ldx + lane];
      }
      atomicAdd(dI + p * lddi + lane, tp);
      atomicAdd(dI + n * lddi + lane, tn);
    }
    if (Ue && dUe) atomicAdd(dUe + u * lddue + lane, ru * Ue[u * ldue + lane]);
    if (Ie && dIe) {
      atomicAdd(dIe + p * lddie + lane, rp * Ie[p * ldie + lane]);
      atomicAdd(dIe + n * lddie + lane, rn * Ie[n * ldie + lane]);
    }
  }
}

// The tail of HealthRec's fused propagation backward (fr_graph_bpr_finish): clear the batch rows'
// column-mask bytes (users at u, items at U + pos / U + neg), add the EmbLoss gradient of the ego
// rows (the same per-row terms and float atomics as bpr_bwd_atomic_kernel's dUe / dIe branch, with
// g_reg scaled by d_greg[0]; a null dUe / dIe skips that table) and zero `zero_n` floats at `zero`
// (the padding row).
__global__ __launch_bounds__(256) void graph_bpr_finish_kernel(
    uint8_t* __restrict__ mask, int64_t U, const float* __restrict__ Ue, int64_t ldue,
    const float* __restrict__ Ie, int64_t ldie, const int64_t* __restrict__ uu, const int64_t* __restrict__ pp,
    const int64_t* __restrict__ nn, int64_t B, int d4, float greg, const float* greg_dev, float* dUe,
    int64_t lddue, float* dIe, int64_t lddie, BprWS ws, float* __restrict__ zero, int zero_n,
    uint32_t* __restrict__ bits) {
  constexpr int GPB = 256 / LPR;
  const int q0 = threadIdx.x % LPR;
  if (greg_dev) greg *= greg_dev[0];
  const float inv_b = 1.f / (float)B;
  const float ru = ws.norms[0] > 0.f ? greg * inv_b / ws.norms[0] : 0.f;
  const float rp = ws.norms[1] > 0.f ? greg * inv_b / ws.norms[1] : 0.f;
  const float rn = ws.norms[2] > 0.f ? greg * inv_b / ws.norms[2] : 0.f;
  if (blockIdx.x == 0)
    for (int k = threadIdx.x; k < zero_n; k += 256) zero[k] = 0.f;
  if (d4 == 16) {  // d = 64: one wave per triple, lane = column (one 256-B atomic instruction per row)
    const int lane = threadIdx.x & 63;
    for (int64_t b = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6; b < B; b += (int64_t)gridDim.x * 4) {
      const int64_t u = uu[b], p = pp[b], n = nn[b];
      if (mask && lane == 0) {
        mask[u] = 0;
        mask[U + p] = 0;
        mask[U + n] = 0;
      }
      if (bits && lane == 0) {
        atomicAnd(bits + (u >> 5), ~(1u << (u & 31)));
        atomicAnd(bits + ((U + p) >> 5), ~(1u << ((U + p) & 31)));
        atomicAnd(bits + ((U + n) >> 5), ~(1u << ((U + n) & 31)));
      }
      if (dUe) atomicAdd(dUe + u * lddue + lane, ru * Ue[u * ldue + lane]);
      if (dIe) {
        atomicAdd(dIe + p * lddie + lane, rp * Ie[p * ldie + lane]);
        atomicAdd(dIe + n * lddie + lane, rn * Ie[n * ldie + lane]);
      }
    }
    return;
  }
  for (int64_t b = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; b < B; b += (int64_t)gridDim.x * GPB) {
    const int64_t u = uu[b], p = pp[b], n = nn[b];
    if (mask && q0 == 0) {
      mask[u] = 0;
      mask[U + p] = 0;
      mask[U + n] = 0;
    }
    if (bits && q0 == 0) {
      atomicAnd(bits + (u >> 5), ~(1u << (u & 31)));
      atomicAnd(bits + ((U + p) >> 5), ~(1u << ((U + p) & 31)));
      atomicAnd(bits + ((U + n) >> 5), ~(1u << ((U + n) & 31)));
    }
    for (int q = q0; q < d4; q += LPR) {
      if (dUe) atomic_row_add(dUe, u, lddue, q, f4_scale(ru, ld4(Ue, u, ldue, q)));
      if (dIe) {
        atomic_row_add(dIe, p, lddie, q, f4_scale(rp, ld4(Ie, p, ldie, q)));
        atomic_row_add(dIe, n, lddie, q, f4_scale(rn, ld4(Ie, n, ldie, q)));
      }
    }
  }
}

// Deterministic scatter.  Slots: [0,B) user occurrences, [B,2B) pos, [2B,3B) neg.  The first
// slot of each (table,row) owns it and sums all its contributions in reference order.
__global__ __launch_bounds__(256) void bpr_bwd_det_kernel(
    const float* __restrict__ U, int64_t ldu, const float* __restrict__ I, int64_t ldi,
    const float* __restrict__ Ue, int64_t ldue, const float* __restrict__ Ie, int64_t ldie,
    const int64_t* __restrict__ uu, const int64_t* __restrict__ pp, const int64_t* __restrict__ nn,
    int64_t B, int d4, float gamma, float gmf, float greg, const float* gscale, float* dU, int64_t lddu,
    float* dI, int64_t lddi, float* dUe, int64_t lddue, float* dIe, int64_t lddie, BprWS ws) {
  constexpr int GPB = 256 / LPR;
  const int q0 = threadIdx.x % LPR;
  if (gscale) { gmf *= gscale[0]; if (dUe || dIe) greg *= gscale[1]; }
  const float inv_b = 1.f / (float)B;
  const float ru = ws.norms[0] > 0.f ? greg * inv_b / ws.norms[0] : 0.f;
  const float rp = ws.norms[1] > 0.f ? greg * inv_b / ws.norms[1] : 0.f;
  const float rn = ws.norms[2] > 0.f ? greg * inv_b / ws.norms[2] : 0.f;
  for (int64_t s = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; s < 3 * B;
       s += (int64_t)gridDim.x * GPB) {
    const bool is_user = s < B;
    const int64_t row = is_user ? uu[s] : (s < 2 * B ? pp[s - B] : nn[s - 2 * B]);
    // owner test: no earlier slot of the same table maps to this row (lanes split the scan)
    bool earlier = false;
    if (is_user) {
      for (int64_t t = q0; t < s; t += LPR) earlier |= (uu[t] == row);
    } else {
      for (int64_t t = B + q0; t < s; t += LPR)
        earlier |= ((t < 2 * B ? pp[t - B] : nn[t - 2 * B]) == row);
    }
    // OR across the group
    int e = earlier ? 1 : 0;
#pragma unroll
    for (int off = LPR / 2; off > 0; off >>= 1) e |= __shfl_xor(e, off, LPR);
    if (e) continue;
    for (int q = q0; q < d4; q += LPR) {
      if (is_user) {
        float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f), r4 = g4;
        for (int64_t t = 0; t < B; ++t) {
          if (uu[t] != row) continue;
          const float g = bpr_coef(ws, t, B, gamma, gmf);
          // u grad = dpos * p + dneg * n (mul backward of both scores)
          g4 = f4_add(g4, f4_add(f4_scale(g, ld4(I, pp[t], ldi, q)), f4_scale(-g, ld4(I, nn[t], ldi, q))));
          if (Ue) r4 = f4_add(r4, f4_scale(ru, ld4(Ue, row, ldue, q)));
        }
        if (dU) { float4* o = reinterpret_cast<float4*>(dU + row * lddu) + q; *o = f4_add(*o, g4); }
        if (Ue && dUe) { float4* o = reinterpret_cast<float4*>(dUe + row * lddue) + q; *o = f4_add(*o, r4); }
      } else {
        float4 gp = make_float4(0.f, 0.f, 0.f, 0.f), gn = gp, rp4 = gp, rn4 = gp;
        for (int64_t t = 0; t < B; ++t) {
          const bool mp = pp[t] == row, mn = nn[t] == row;
          if (!mp && !mn) continue;
          const float g = bpr_coef(ws, t, B, gamma, gmf);
          const float4 xu = ld4(U, uu[t], ldu, q);
          if (mp) {
            gp = f4_add(gp, f4_scale(g, xu));
            if (Ie) rp4 = f4_add(rp4, f4_scale(rp, ld4(Ie, row, ldie, q)));
          }
          if (mn) {
            gn = f4_add(gn, f4_scale(-g, xu));
            if (Ie) rn4 = f4_add(rn4, f4_scale(rn, ld4(Ie, row, ldie, q)));
          }
        }
        if (dI) { float4* o = reinterpret_cast<float4*>(dI + row * lddi) + q; *o = f4_add(*o, f4_add(gp, gn)); }
        if (Ie && dIe) {
          float4* o = reinterpret_cast<float4*>(dIe + row * lddie) + q;
          *o = f4_add(*o, f4_add(rp4, rn4));
        }
      }
    }
  }
}


// Deterministic scatter, sorted form (2B <= kDetSortMax): the owner-slot kernel above scans every
// earlier slot and, per owner, every triple -- O(B^2), 19 ms at B = 8192.  Here each table's slot keys
// (row << 20 | slot) are sorted once in LDS (block 0: users, block 1: items; bitonic, 1024 threads),
// then the first slot of each row's run owns the row and sums the run in slot order -- the same
// contributions in the same order as bpr_bwd_det_kernel (bit-identical results), O(B log B).
__global__ __launch_bounds__(1024) void bpr_det_sort_kernel(const int64_t* __restrict__ uu,
                                                            const int64_t* __restrict__ pp,
                                                            const int64_t* __restrict__ nn, int64_t B, BprWS ws) {
  __shared__ uint64_t K[kDetSortMax];
  const bool items = blockIdx.x == 1;
  const int64_t cnt = items ? 2 * B : B;
  const int64_t N = pow2_at_least(cnt);
  for (int64_t k = threadIdx.x; k < N; k += 1024) {
    uint64_t key = ~0ull;  // padding sorts last
    if (k < cnt) {
      const int64_t row = items ? (k < B ? pp[k] : nn[k - B]) : uu[k];
      key = ((uint64_t)row << 20) | (uint64_t)k;
    }
    K[k] = key;
  }
  __syncthreads();
  for (int64_t len = 2; len <= N; len <<= 1) {
    for (int64_t j = len >> 1; j > 0; j >>= 1) {
      for (int64_t k = threadIdx.x; k < N; k += 1024) {
        const int64_t x = k ^ j;
        if (x > k) {
          const uint64_t a = K[k], b = K[x];
          const bool up = (k & len) == 0;
          if ((a > b) == up) {
            K[k] = b;
            K[x] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  uint64_t* out = items ? ws.keys_i : ws.keys_u;
  for (int64_t k = threadIdx.x; k < cnt; k += 1024) out[k] = K[k];
}

__global__ __launch_bounds__(256) void bpr_bwd_det_sorted_kernel(
    const float* __restrict__ U, int64_t ldu, const float* __restrict__ I, int64_t ldi,
    const float* __restrict__ Ue, int64_t ldue, const float* __restrict__ Ie, int64_t ldie,
    const int64_t* __restrict__ uu, const int64_t* __restrict__ pp, const int64_t* __restrict__ nn,
    int64_t B, int d4, float gamma, float gmf, float greg, const float* gscale, float* dU, int64_t lddu,
    float* dI, int64_t lddi, float* dUe, int64_t lddue, float* dIe, int64_t lddie, BprWS ws) {
  constexpr int GPB = 256 / LPR;
  constexpr uint64_t SLOT = (1ull << 20) - 1;
  const int q0 = threadIdx.x % LPR;
  if (gscale) { gmf *= gscale[0]; if (dUe || dIe) greg *= gscale[1]; }
  const float inv_b = 1.f / (float)B;
  const float ru = ws.norms[0] > 0.f ? greg * inv_b / ws.norms[0] : 0.f;
  const float rp = ws.norms[1] > 0.f ? greg * inv_b / ws.norms[1] : 0.f;
  const float rn = ws.norms[2] > 0.f ? greg * inv_b / ws.norms[2] : 0.f;
  for (int64_t s = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; s < 3 * B; s += (int64_t)gridDim.x * GPB) {
    const bool is_user = s < B;
    const uint64_t* keys = is_user ? ws.keys_u : ws.keys_i;
    const int64_t k = is_user ? s : s - B, cnt = is_user ? B : 2 * B;
    const uint64_t row = keys[k] >> 20;
    if (k > 0 && (keys[k - 1] >> 20) == row) continue;  // not the first slot of its row's run
    for (int q = q0; q < d4; q += LPR) {
      if (is_user) {
        float4 g4 = make_float4(0.f, 0.f, 0.f, 0.f), r4 = g4;
        for (int64_t j = k; j < cnt && (keys[j] >> 20) == row; ++j) {
          const int64_t t = (int64_t)(keys[j] & SLOT);
          const float g = bpr_coef(ws, t, B, gamma, gmf);
          g4 = f4_add(g4, f4_add(f4_scale(g, ld4(I, pp[t], ldi, q)), f4_scale(-g, ld4(I, nn[t], ldi, q))));
          if (Ue) r4 = f4_add(r4, f4_scale(ru, ld4(Ue, (int64_t)row, ldue, q)));
        }
        if (dU) { float4* o = reinterpret_cast<float4*>(dU + (int64_t)row * lddu) + q; *o = f4_add(*o, g4); }
        if (Ue && dUe) { float4* o = reinterpret_cast<float4*>(dUe + (int64_t)row * lddue) + q; *o = f4_add(*o, r4); }
      } else {
        float4 gp = make_float4(0.f, 0.f, 0.f, 0.f), gn = gp, rp4 = gp, rn4 = gp;
        for (int64_t j = k; j < cnt && (keys[j] >> 20) == row; ++j) {
          const int64_t sl = (int64_t)(keys[j] & SLOT);
          const bool mp = sl < B;
          const int64_t t = mp ? sl : sl - B;
          const float g = bpr_coef(ws, t, B, gamma, gmf);
          const float4 xu = ld4(U, uu[t], ldu, q);
          if (mp) {
            gp = f4_add(gp, f4_scale(g, xu));
            if (Ie) rp4 = f4_add(rp4, f4_scale(rp, ld4(Ie, (int64_t)row, ldie, q)));
          } else {
            gn = f4_add(gn, f4_scale(-g, xu));
            if (Ie) rn4 = f4_add(rn4, f4_scale(rn, ld4(Ie, (int64_t)row, ldie, q)));
          }
        }
        if (dI) { float4* o = reinterpret_cast<float4*>(dI + (int64_t)row * lddi) + q; *o = f4_add(*o, f4_add(gp, gn)); }
        if (Ie && dIe) {
          float4* o = reinterpret_cast<float4*>(dIe + (int64_t)row * lddie) + q;
          *o = f4_add(*o, f4_add(rp4, rn4));
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// bf16 tables (BASELINE config 5): rows of d bf16, LPR = d/8 lanes x 16 B; fp32 arithmetic.
// Same workspace / reduce kernel / coefficients as the fp32 path.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void ld8(const uint16_t* base, int64_t row, int64_t ld, int q, float* o) {
  fr_unpack8(reinterpret_cast<const uint4*>(base + row * ld)[q], o);
}

template <int L>
__global__ __launch_bounds__(256) void bpr16_scores_kernel(
    const uint16_t* __restrict__ U, int64_t ldu, const uint16_t* __restrict__ I, int64_t ldi,
    const uint16_t* __restrict__ Ue, int64_t ldue, const uint16_t* __restrict__ Ie, int64_t ldie,
    const int64_t* __restrict__ uu, const int64_t* __restrict__ pp, const int64_t* __restrict__ nn,
    int64_t B, int d8, BprWS ws) {
  constexpr int GPB = 256 / L;
  const int q0 = threadIdx.x % L;
  for (int64_t b = (int64_t)blockIdx.x * GPB + threadIdx.x / L; b < B; b += (int64_t)gridDim.x * GPB) {
    const int64_t u = uu[b], p = pp[b], n = nn[b];
    float sp = 0.f, sn = 0.f, a = 0.f, c = 0.f, e = 0.f;
    for (int q = q0; q < d8; q += L) {
      float xu[8], xp[8], xn[8];
      ld8(U, u, ldu, q, xu);
      ld8(I, p, ldi, q, xp);
      ld8(I, n, ldi, q, xn);
      sp += fr_dot8(xu, xp);
      sn += fr_dot8(xu, xn);
      if (Ue) {
        ld8(Ue, u, ldue, q, xu);
        ld8(Ie, p, ldie, q, xp);
        ld8(Ie, n, ldie, q, xn);
        a += fr_dot8(xu, xu);
        c += fr_dot8(xp, xp);
        e += fr_dot8(xn, xn);
      }
    }
    sp = group_sum<L>(sp);
    sn = group_sum<L>(sn);
    a = group_sum<L>(a);
    c = group_sum<L>(c);
    e = group_sum<L>(e);
    if (q0 == 0) {
      ws.spos[b] = sp;
      ws.sneg[b] = sn;
      ws.squ[b] = a;
      ws.sqp[b] = c;
      ws.sqn[b] = e;
    }
  }
}

__device__ __forceinline__ void rmw_add8(uint16_t* base, int64_t row, int64_t ld, int q, const float* g) {
  uint4* o = reinterpret_cast<uint4*>(base + row * ld) + q;
  float cur[8];
  fr_unpack8(*o, cur);
#pragma unroll
  for (int j = 0; j < 8; ++j) cur[j] += g[j];
  *o = fr_pack8(cur);
}

// Deterministic owner-slot scatter (as bpr_bwd_det_kernel): every destination row is summed in
// fp32 by its first slot and added to the bf16 gradient table once (one rounding per row).
template <int L>
__global__ __launch_bounds__(256) void bpr16_bwd_det_kernel(
    const uint16_t* __restrict__ U, int64_t ldu, const uint16_t* __restrict__ I, int64_t ldi,
    const uint16_t* __restrict__ Ue, int64_t ldue, const uint16_t* __restrict__ Ie, int64_t ldie,
    const int64_t* __restrict__ uu, const int64_t* __restrict__ pp, const int64_t* __restrict__ nn,
    int64_t B, int d8, float gamma, float gmf, float greg, const float* gscale, uint16_t* dU,
    uint16_t* dI, uint16_t* dUe, uint16_t* dIe, BprWS ws) {
  constexpr int GPB = 256 / L;
  const int q0 = threadIdx.x % L;
  if (gscale) { gmf *= gscale[0]; greg *= gscale[1]; }
  const float inv_b = 1.f / (float)B;
  const float ru = ws.norms[0] > 0.f ? greg * inv_b / ws.norms[0] : 0.f;
  const float rp = ws.norms[1] > 0.f ? greg * inv_b / ws.norms[1] : 0.f;
  const float rn = ws.norms[2] > 0.f ? greg * inv_b / ws.norms[2] : 0.f;
  for (int64_t s = (int64_t)blockIdx.x * GPB + threadIdx.x / L; s < 3 * B; s += (int64_t)gridDim.x * GPB) {
    const bool is_user = s < B;
    const int64_t row = is_user ? uu[s] : (s < 2 * B ? pp[s - B] : nn[s - 2 * B]);
    bool earlier = false;
    if (is_user) {
      for (int64_t t = q0; t < s; t += L) earlier |= (uu[t] == row);
    } else {
      for (int64_t t = B + q0; t < s; t += L) earlier |= ((t < 2 * B ? pp[t - B] : nn[t - 2 * B]) == row);
    }
    int e = earlier ? 1 : 0;
#pragma unroll
    for (int off = L / 2; off > 0; off >>= 1) e |= __shfl_xor(e, off, L);
    if (e) continue;
    for (int q = q0; q < d8; q += L) {
      float g8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, r8[8] = {0, 0, 0, 0, 0, 0, 0, 0}, x[8], y[8];
      if (is_user) {
        int cnt = 0;
        for (int64_t t = 0; t < B; ++t) {
          if (uu[t] != row) continue;
          const float g = bpr_coef(ws, t, B, gamma, gmf);
          ld8(I, pp[t], ldi, q, x);
          ld8(I, nn[t], ldi, q, y);
#pragma unroll
          for (int j = 0; j < 8; ++j) g8[j] += g * x[j] + (-g) * y[j];
          ++cnt;
        }
        if (dU) rmw_add8(dU, row, ldu, q, g8);
        if (Ue && dUe) {
          ld8(Ue, row, ldue, q, x);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            for (int k = 0; k < cnt; ++k) r8[j] += ru * x[j];
          rmw_add8(dUe, row, ldue, q, r8);
        }
      } else {
        int cp = 0, cn = 0;
        for (int64_t t = 0; t < B; ++t) {
          const bool mp = pp[t] == row, mn = nn[t] == row;
          if (!mp && !mn) continue;
          const float g = bpr_coef(ws, t, B, gamma, gmf);
          ld8(U, uu[t], ldu, q, x);
#pragma unroll
          for (int j = 0; j < 8; ++j) g8[j] += (mp ? g * x[j] : 0.f) + (mn ? -g * x[j] : 0.f);
          cp += mp;
          cn += mn;
        }
        if (dI) rmw_add8(dI, row, ldi, q, g8);
        if (Ie && dIe) {
          ld8(Ie, row, ldie, q, x);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            float a = 0.f, b = 0.f;
            for (int k = 0; k < cp; ++k) a += rp * x[j];
            for (int k = 0; k < cn; ++k) b += rn * x[j];
            r8[j] = a + b;
          }
          rmw_add8(dIe, row, ldie, q, r8);
        }
      }
    }
  }
}
}  // namespace

extern "C" int64_t fr_bpr_workspace(int64_t B) { return B > 0 ? bpr_ws_bytes(B) : 0; }

static int bpr_check(const float* U, int64_t ldu, const float* I, int64_t ldi, const float* Ue,
                     int64_t ldue, const float* Ie, int64_t ldie, const int64_t* u, const int64_t* p,
                     const int64_t* n, int64_t B, int d, void* ws, int64_t wsb) {
  FR_REQUIRE(B >= 1, "B must be >= 1");
  FR_REQUIRE(d >= 4 && d % 4 == 0, "d must be a positive multiple of 4");
  FR_REQUIRE(U && I && u && p && n, "null table/index");
  FR_REQUIRE(fr::aligned16(U) && fr::aligned16(I) && ldu % 4 == 0 && ldi % 4 == 0 && ldu >= d && ldi >= d,
             "U/I must be 16-B aligned with ld % 4 == 0");
  FR_REQUIRE((Ue == nullptr) == (Ie == nullptr), "Ue and Ie must both be given or both null");
  FR_REQUIRE(!Ue || (fr::aligned16(Ue) && fr::aligned16(Ie) && ldue % 4 == 0 && ldie % 4 == 0 &&
                     ldue >= d && ldie >= d),
             "Ue/Ie must be 16-B aligned with ld % 4 == 0");
  FR_REQUIRE(ws && wsb >= bpr_ws_bytes(B) && fr::aligned16(ws), "workspace too small");
  return FR_OK;
}

extern "C" int fr_bpr_fwd(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
                          const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
                          const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B, int d,
                          float gamma, float* d_out, void* d_workspace, int64_t workspace_bytes,
                          void* stream) {
  return fr_bpr_fwd_rows(d_U, ldu, d_I, ldi, d_Ue, ldue, d_Ie, ldie, d_u, d_p, d_n, B, d, gamma, d_out, nullptr, 0,
                         d_workspace, workspace_bytes, stream);
}

extern "C" int fr_bpr_fwd_rows(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
                               const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
                               const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B, int d,
                               float gamma, float* d_out, float* d_rows, int64_t ld_rows, void* d_workspace,
                               int64_t workspace_bytes, void* stream) {
  return fr_bpr_fwd_ex(d_U, ldu, d_I, ldi, d_Ue, ldue, d_Ie, ldie, d_u, d_p, d_n, B, d, gamma, 1.f, d_out, d_rows,
                       ld_rows, d_workspace, workspace_bytes, stream);
}

extern "C" int fr_bpr_fwd_ex(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
                             const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
                             const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B, int d,
                             float gamma, float w_emb, float* d_out, float* d_rows, int64_t ld_rows,
                             void* d_workspace, int64_t workspace_bytes, void* stream) {
  int rc = bpr_check(d_U, ldu, d_I, ldi, d_Ue, ldue, d_Ie, ldie, d_u, d_p, d_n, B, d, d_workspace,
                     workspace_bytes);
  if (rc) return rc;
  FR_REQUIRE(d_out, "out null");
  FR_REQUIRE(!d_rows || (fr::aligned16(d_rows) && ld_rows >= d && ld_rows % 4 == 0), "rows output [2B, d] unaligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  BprWS w = bpr_ws(d_workspace, B);
  const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(B, 256 / LPR), 4096);
  hipLaunchKernelGGL(bpr_scores_kernel, dim3(blocks), dim3(256), 0, s, d_U, ldu, d_I, ldi, d_Ue, ldue,
                     d_Ie, ldie, d_u, d_p, d_n, B, d / 4, w, d_rows, ld_rows);
  FR_LAUNCH_CHECK();
  hipLaunchKernelGGL(bpr_reduce_kernel, dim3(1), dim3(1024), 0, s, B, gamma, d_Ue ? 1 : 0, w_emb, w, d_out);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

static int bpr_bwd_impl(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi, const float* d_Ue,
                        int64_t ldue, const float* d_Ie, int64_t ldie, const int64_t* d_u, const int64_t* d_p,
                        const int64_t* d_n, int64_t B, int d, float gamma, float g_mf, float g_reg,
                        const float* d_gscale, float* d_dU, float* d_dI, float* d_dUe, float* d_dIe,
                        int deterministic, const float* d_extra, int64_t ldx, void* d_workspace,
                        int64_t workspace_bytes, void* stream) {
  int rc = bpr_check(d_U, ldu, d_I, ldi, d_Ue, ldue, d_Ie, ldie, d_u, d_p, d_n, B, d, d_workspace,
                     workspace_bytes);
  if (rc) return rc;
  for (const float* g : {d_dU, d_dI, d_dUe, d_dIe}) FR_REQUIRE(!g || fr::aligned16(g), "grad unaligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  BprWS w = bpr_ws(d_workspace, B);
  // gradient tables share the leading dimension of their forward tables
  if (deterministic && w.keys_u) {
    hipLaunchKernelGGL(bpr_det_sort_kernel, dim3(2), dim3(1024), 0, s, d_u, d_p, d_n, B, w);
    FR_LAUNCH_CHECK();
    const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(3 * B, 256 / LPR), 4096);
    hipLaunchKernelGGL(bpr_bwd_det_sorted_kernel, dim3(blocks), dim3(256), 0, s, d_U, ldu, d_I, ldi, d_Ue,
                       ldue, d_Ie, ldie, d_u, d_p, d_n, B, d / 4, gamma, g_mf, g_reg, d_gscale, d_dU,
                       ldu, d_dI, ldi, d_dUe, ldue, d_dIe, ldie, w);
  } else if (deterministic) {
    const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(3 * B, 256 / LPR), 4096);
    hipLaunchKernelGGL(bpr_bwd_det_kernel, dim3(blocks), dim3(256), 0, s, d_U, ldu, d_I, ldi, d_Ue,
                       ldue, d_Ie, ldie, d_u, d_p, d_n, B, d / 4, gamma, g_mf, g_reg, d_gscale, d_dU,
                       ldu, d_dI, ldi, d_dUe, ldue, d_dIe, ldie, w);
  } else if (d == 64) {
    const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(B, 4), 4096);
    hipLaunchKernelGGL(bpr_bwd_atomic64_kernel, dim3(blocks), dim3(256), 0, s, d_U, ldu, d_I, ldi, d_Ue,
                       ldue, d_Ie, ldie, d_u, d_p, d_n, B, gamma, g_mf, g_reg, d_gscale, d_dU,
                       ldu, d_dI, ldi, d_dUe, ldue, d_dIe, ldie, w, d_extra, ldx);
  } else {
    const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(B, 256 / LPR), 4096);
    hipLaunchKernelGGL(bpr_bwd_atomic_kernel, dim3(blocks), dim3(256), 0, s, d_U, ldu, d_I, ldi, d_Ue,
                       ldue, d_Ie, ldie, d_u, d_p, d_n, B, d / 4, gamma, g_mf, g_reg, d_gscale, d_dU,
                       ldu, d_dI, ldi, d_dUe, ldue, d_dIe, ldie, w, d_extra, ldx);
  }
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_bpr_bwd(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
                          const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
                          const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B, int d,
                          float gamma, float g_mf, float g_reg, const float* d_gscale, float* d_dU,
                          float* d_dI, float* d_dUe, float* d_dIe, int deterministic,
                          void* d_workspace, int64_t workspace_bytes, void* stream) {
  return bpr_bwd_impl(d_U, ldu, d_I, ldi, d_Ue, ldue, d_Ie, ldie, d_u, d_p, d_n, B, d, gamma, g_mf, g_reg, d_gscale,
                      d_dU, d_dI, d_dUe, d_dIe, deterministic, nullptr, 0, d_workspace, workspace_bytes, stream);
}

extern "C" int fr_bpr_bwd_ex(const float* d_U, int64_t ldu, const float* d_I, int64_t ldi,
                             const float* d_Ue, int64_t ldue, const float* d_Ie, int64_t ldie,
                             const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B, int d,
                             float gamma, float g_mf, float g_reg, const float* d_gscale, float* d_dU,
                             float* d_dI, float* d_dUe, float* d_dIe, const float* d_extra_i, int64_t ld_extra,
                             void* d_workspace, int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(d_extra_i && d_dI && fr::aligned16(d_extra_i) && ld_extra >= d && ld_extra % 4 == 0,
             "extra item-row gradient [2B, d] (16-B aligned) and dI required");
  return bpr_bwd_impl(d_U, ldu, d_I, ldi, d_Ue, ldue, d_Ie, ldie, d_u, d_p, d_n, B, d, gamma, g_mf, g_reg, d_gscale,
                      d_dU, d_dI, d_dUe, d_dIe, 0, d_extra_i, ld_extra, d_workspace, workspace_bytes, stream);
}

extern "C" int fr_graph_bpr_finish(uint8_t* d_mask, int64_t U, const float* d_Ue, int64_t ldue, const float* d_Ie,
                                   int64_t ldie, const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B,
                                   int d, float g_reg, const float* d_greg, float* d_dUe, float* d_dIe,
                                   float* d_zero, int zero_n, uint32_t* d_bits, void* d_workspace,
                                   int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(B >= 1 && d >= 4 && d % 4 == 0 && U >= 0 && zero_n >= 0, "bad sizes");
  FR_REQUIRE(d_Ue && d_Ie && d_u && d_p && d_n && (zero_n == 0 || d_zero), "null argument");
  FR_REQUIRE(fr::aligned16(d_Ue) && fr::aligned16(d_Ie) && (!d_dUe || fr::aligned16(d_dUe)) &&
                 (!d_dIe || fr::aligned16(d_dIe)) && ldue % 4 == 0 && ldie % 4 == 0 && ldue >= d && ldie >= d,
             "tables must be 16-B aligned with ld % 4 == 0");
  FR_REQUIRE(d_workspace && workspace_bytes >= bpr_ws_bytes(B) && fr::aligned16(d_workspace), "workspace too small");
  BprWS w = bpr_ws(d_workspace, B);
  const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(B, d == 64 ? 4 : 256 / LPR), 4096);
  hipLaunchKernelGGL(graph_bpr_finish_kernel, dim3(blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), d_mask,
                     U, d_Ue, ldue, d_Ie, ldie, d_u, d_p, d_n, B, d / 4, g_reg, d_greg, d_dUe, ldue, d_dIe, ldie, w,
                     d_zero, zero_n, d_bits);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

// ---- bf16 entry points -----------------------------------------------------------------------
static int bpr16_check(const uint16_t* U, int64_t ldu, const uint16_t* I, int64_t ldi, const uint16_t* Ue,
                       int64_t ldue, const uint16_t* Ie, int64_t ldie, const int64_t* u, const int64_t* p,
                       const int64_t* n, int64_t B, int d, void* ws, int64_t wsb) {
  FR_REQUIRE(B >= 1, "B must be >= 1");
  FR_REQUIRE(d >= 8 && d % 8 == 0, "d must be a positive multiple of 8");
  FR_REQUIRE(U && I && u && p && n, "null table/index");
  auto ok = [d](const uint16_t* t, int64_t ld) { return fr::aligned16(t) && ld % 8 == 0 && ld >= d; };
  FR_REQUIRE(ok(U, ldu) && ok(I, ldi), "U/I must be 16-B aligned with ld % 8 == 0");
  FR_REQUIRE((Ue == nullptr) == (Ie == nullptr), "Ue and Ie must both be given or both null");
  FR_REQUIRE(!Ue || (ok(Ue, ldue) && ok(Ie, ldie)), "Ue/Ie must be 16-B aligned with ld % 8 == 0");
  FR_REQUIRE(ws && wsb >= bpr_ws_bytes(B) && fr::aligned16(ws), "workspace too small");
  return FR_OK;
}

template <class F>
static void bpr16_dispatch(int d8, F&& f) {
  if (d8 >= 32) f(std::integral_constant<int, 32>{});
  else if (d8 >= 16) f(std::integral_constant<int, 16>{});
  else if (d8 >= 8) f(std::integral_constant<int, 8>{});
  else if (d8 >= 4) f(std::integral_constant<int, 4>{});
  else if (d8 >= 2) f(std::integral_constant<int, 2>{});
  else f(std::integral_constant<int, 1>{});
}

extern "C" int fr_bpr_fwd_bf16(const uint16_t* d_U, int64_t ldu, const uint16_t* d_I, int64_t ldi,
                               const uint16_t* d_Ue, int64_t ldue, const uint16_t* d_Ie, int64_t ldie,
                               const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B, int d,
                               float gamma, float* d_out, void* d_workspace, int64_t workspace_bytes,
                               void* stream) {
  int rc = bpr16_check(d_U, ldu, d_I, ldi, d_Ue, ldue, d_Ie, ldie, d_u, d_p, d_n, B, d, d_workspace,
                       workspace_bytes);
  if (rc) return rc;
  FR_REQUIRE(d_out, "out null");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  BprWS w = bpr_ws(d_workspace, B);
  bpr16_dispatch(d / 8, [&](auto L) {
    constexpr int LL = decltype(L)::value;
    const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(B, 256 / LL), 4096);
    hipLaunchKernelGGL(bpr16_scores_kernel<LL>, dim3(blocks), dim3(256), 0, s, d_U, ldu, d_I, ldi, d_Ue, ldue,
                       d_Ie, ldie, d_u, d_p, d_n, B, d / 8, w);
  });
  FR_LAUNCH_CHECK();
  hipLaunchKernelGGL(bpr_reduce_kernel, dim3(1), dim3(1024), 0, s, B, gamma, d_Ue ? 1 : 0, 1.f, w, d_out);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_bpr_bwd_bf16(const uint16_t* d_U, int64_t ldu, const uint16_t* d_I, int64_t ldi,
                               const uint16_t* d_Ue, int64_t ldue, const uint16_t* d_Ie, int64_t ldie,
                               const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B, int d,
                               float gamma, float g_mf, float g_reg, const float* d_gscale, uint16_t* d_dU,
                               uint16_t* d_dI, uint16_t* d_dUe, uint16_t* d_dIe, void* d_workspace,
                               int64_t workspace_bytes, void* stream) {
  int rc = bpr16_check(d_U, ldu, d_I, ldi, d_Ue, ldue, d_Ie, ldie, d_u, d_p, d_n, B, d, d_workspace,
                       workspace_bytes);
  if (rc) return rc;
  for (const uint16_t* g : {d_dU, d_dI, d_dUe, d_dIe}) FR_REQUIRE(!g || fr::aligned16(g), "grad unaligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  BprWS w = bpr_ws(d_workspace, B);
  bpr16_dispatch(d / 8, [&](auto L) {
    constexpr int LL = decltype(L)::value;
    const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(3 * B, 256 / LL), 4096);
    hipLaunchKernelGGL(bpr16_bwd_det_kernel<LL>, dim3(blocks), dim3(256), 0, s, d_U, ldu, d_I, ldi, d_Ue, ldue,
                       d_Ie, ldie, d_u, d_p, d_n, B, d / 8, gamma, g_mf, g_reg, d_gscale, d_dU, d_dI, d_dUe,
                       d_dIe, w);
  });
  FR_LAUNCH_CHECK();
  return FR_OK;
}
