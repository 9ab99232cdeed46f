// Per-user ranking metrics of the evaluation the trainer runs every epoch, on the device.
//
// Replaces the host loop of Trainer._valid_by_user_epoch (FoodRec/common/trainer.py:231-282) over
// EvalByUserDataloader's candidate lists (utils/dataloader.py:228-302): for each user, with the
// candidate scores pr (the npos positives first, then the negatives)
//     order = np.argsort(pr)[::-1];  metrics_by_user(order[:k], range(npos)), k = 10, 20  (:55-69)
//     get_auc_fast(range(npos), pr, neg_num)                                             (:49-52)
// One wave per user; the candidates sit in registers (lane l holds elements l, l + 64, ...).
//   * top-(K+1) by K+1 rounds of a wave-wide argmax; bit t of hits[u] says whether rank t (< K) is a
//     positive.  The metrics' float64 arithmetic (log2 discounts in rank order, recall, NDCG) is
//     left to the host, which evaluates the reference's formulas on the hit masks bit for bit.
//   * numpy's argsort (introsort) breaks ties in an order no kernel reproduces, so a user whose
//     K+1 largest scores are not strictly decreasing, who has a NaN score, or more candidates than
//     the registers hold is flagged (flags[u] != 0) and ranked by the host's numpy path instead;
//     ties below rank K+1 change nothing.
//   * auc[u] = sum over positives p of #{negatives j : pr[j] < pr[p]} (strict, order-free: exact).
// Latency-bound (~K rounds of ~40 instructions per user), a few hundred microseconds for 68,768
// Allrecipes test users against seconds for the host loop.
#include "fr_common.h"

namespace {

constexpr int PER_LANE = 32;             // candidates per user held in registers: 64 x 32 = 2048
constexpr int KMAX = 31;                  // hit mask bits

__device__ __forceinline__ float wave_max(float v) {
  v = fmaxf(v, dpp_mov<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmaxf(v, dpp_mov<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmaxf(v, dpp_mov<0x141>(v));  // row_half_mirror
  v = fmaxf(v, dpp_mov<0x140>(v));  // row_mirror
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
  const auto t = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(t[0]), __uint_as_float(t[1]));
}

__device__ __forceinline__ int wave_sum_i(int v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(256) void rank_metrics_kernel(const float* __restrict__ scores,
                                                           const int64_t* __restrict__ off,
                                                           const int32_t* __restrict__ npos, int64_t U, int K,
                                                           uint32_t* __restrict__ hits, int64_t* __restrict__ auc,
                                                           uint8_t* __restrict__ flags) {
  const int64_t u = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (u >= U) return;
  const int lane = threadIdx.x & 63;
  const int64_t o = off[u];
  const int n = (int)(off[u + 1] - o);
  const int np = npos[u];
  if (n > 64 * PER_LANE || np <= 0 || np > n) {  // host path (reference semantics for odd users)
    if (lane == 0) {
      flags[u] = 2;
      hits[u] = 0;
      auc[u] = 0;
    }
    return;
  }
  float v[PER_LANE];
  uint32_t valid = 0;
  bool nan = false;
#pragma unroll
  for (int k = 0; k < PER_LANE; ++k) {
    const int idx = lane + 64 * k;
    v[k] = idx < n ? scores[o + idx] : -INFINITY;
    valid |= (uint32_t)(idx < n) << k;
    nan |= v[k] != v[k];
  }
  // AUC: every positive's score against this lane's negatives (index >= np)
  int cnt = 0;
  for (int p = 0; p < np; ++p) {
    const float pv = scores[o + p];  // the same address in every lane: one broadcast load
#pragma unroll
    for (int k = 0; k < PER_LANE; ++k) cnt += (((valid >> k) & 1u) && lane + 64 * k >= np && v[k] < pv) ? 1 : 0;
  }
  const int64_t auc_u = wave_sum_i(cnt);
  // top-(K+1): rounds of wave argmax over the unselected candidates
  const int rounds = min(n, K + 1);
  uint32_t sel = 0, hit = 0;
  bool tie = false;
  float prev = INFINITY;
  for (int t = 0; t < rounds; ++t) {
    float bv = -INFINITY;
    int bk = -1;
#pragma unroll
    for (int k = 0; k < PER_LANE; ++k) {
      const bool live = ((valid & ~sel) >> k) & 1u;
      if (live && (bk < 0 || v[k] > bv)) {
        bv = v[k];
        bk = k;
      }
    }
    const float m = wave_max(bk >= 0 ? bv : -INFINITY);
    const uint64_t win = __ballot(bk >= 0 && bv == m);
    const int wl = __ffsll((unsigned long long)win) - 1;  // one of the lanes holding the maximum
    const int wk = __shfl(bk, wl);
    if (lane == wl) sel |= 1u << bk;
    if (t < K && wl + 64 * wk < np) hit |= 1u << t;
    tie |= !(m < prev);  // equal to the previous round's value (or a NaN): tie order matters
    prev = m;
  }
  const bool any_nan = __ballot(nan) != 0;  // every lane votes (a ballot under lane == 0 sees lane 0 only)
  if (lane == 0) {
    hits[u] = hit;
    auc[u] = auc_u;
    flags[u] = (uint8_t)((tie || any_nan) ? 1 : 0);
  }
}

// Candidate scores of the evaluation, fused: score[e] = <U[uid[s]], I[items[e]]> for e in segment s
// = [off[s], off[s + 1]) (the graph models' inference_fast, torch.mul(user[u], item[i]).sum(1), over
// EvalByUserDataloader's back-to-back per-user lists).  One wave per segment: 16-lane groups hold
// the user row as one float4 per lane (d = 64) and take 4 candidates per round, each group loading
// its candidate's item row as 16 float4 (256 contiguous bytes) and reducing by DPP; two rounds in
// flight.  No [n, 64] gathers are materialised (torch: two gathers, a product, a reduction).
constexpr int SC_WAVES = 4;
__global__ __launch_bounds__(64 * SC_WAVES) void score_segments_kernel(
    const float* __restrict__ U, int64_t ldu, const float* __restrict__ I, int64_t ldi, const int64_t* __restrict__ uid,
    const int64_t* __restrict__ off, int64_t nseg, const int64_t* __restrict__ items, float* __restrict__ out) {
  const int64_t s = (int64_t)blockIdx.x * SC_WAVES + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (s >= nseg) return;
  const int lane = threadIdx.x & 63, g = lane >> 4, j = lane & 15;
  const float4 u4 = *reinterpret_cast<const float4*>(U + uid[s] * ldu + 4 * j);
  const int64_t e0 = off[s], e1 = off[s + 1];
  for (int64_t e = e0 + g; e < e1; e += 8) {
    const int64_t ea = e, eb = e + 4;
    const bool hb = eb < e1;
    const int64_t ia = items[ea], ib = hb ? items[eb] : ia;
    const float4 a4 = *reinterpret_cast<const float4*>(I + ia * ldi + 4 * j);
    const float4 b4 = *reinterpret_cast<const float4*>(I + ib * ldi + 4 * j);
    const float sa = group_sum<16>(fmaf(u4.w, a4.w, fmaf(u4.z, a4.z, fmaf(u4.y, a4.y, u4.x * a4.x))));
    const float sb = group_sum<16>(fmaf(u4.w, b4.w, fmaf(u4.z, b4.z, fmaf(u4.y, b4.y, u4.x * b4.x))));
    if (j == 0) {
      out[ea] = sa;
      if (hb) out[eb] = sb;
    }
  }
}

}  // namespace

extern "C" int fr_score_segments(const float* d_user, int64_t ld_user, const float* d_item, int64_t ld_item,
                                 const int64_t* d_uid, const int64_t* d_offsets, int64_t n_seg, const int64_t* d_items,
                                 int d, float* d_out, void* stream) {
  FR_REQUIRE(d == 64, "d = 64 (16 lanes x float4 per row)");
  FR_REQUIRE(n_seg >= 0 && ld_user >= d && ld_item >= d && ld_user % 4 == 0 && ld_item % 4 == 0,
             "n_seg >= 0, row strides >= d and multiples of 4");
  if (n_seg == 0) return FR_OK;
  FR_REQUIRE(d_user && d_item && d_uid && d_offsets && d_items && d_out && fr::aligned16(d_user) &&
                 fr::aligned16(d_item),
             "null or unaligned operand");
  hipLaunchKernelGGL(score_segments_kernel, dim3((unsigned)fr::ceil_div(n_seg, SC_WAVES)), dim3(64 * SC_WAVES), 0,
                     reinterpret_cast<hipStream_t>(stream), d_user, ld_user, d_item, ld_item, d_uid, d_offsets, n_seg,
                     d_items, d_out);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_rank_metrics(const float* d_scores, const int64_t* d_offsets, const int32_t* d_npos, int64_t n_users,
                               int k, uint32_t* d_hits, int64_t* d_auc, uint8_t* d_flags, void* stream) {
  FR_REQUIRE(n_users >= 0 && k >= 1 && k <= KMAX, "n_users >= 0, 1 <= k <= 31");
  if (n_users == 0) return FR_OK;
  FR_REQUIRE(d_scores && d_offsets && d_npos && d_hits && d_auc && d_flags, "null argument");
  hipLaunchKernelGGL(rank_metrics_kernel, dim3((unsigned)fr::ceil_div(n_users, 4)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), d_scores, d_offsets, d_npos, n_users, k, d_hits, d_auc,
                     d_flags);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_rank_capacity(void) { return 64 * PER_LANE; }
