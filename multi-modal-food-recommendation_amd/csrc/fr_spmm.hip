// CSR SpMM with fused LightGCN layer epilogue — the propagation hot op.
//
// Replaces torch.sparse.mm(norm_adj, X) (+ the layer mean torch.stack(..).mean(1)) at
// models/lightgcn.py:136-144, models/cikm_model.py:187-190,199-202, models/pricai_modelx.py:183-226.
//
// Layout / mapping (MI355X, wave64):
//   * a row of X is d fp32 = d/4 float4; a "group" of LPR = d/4 lanes owns one work unit
//     (d=64 -> 16 lanes, 4 units per wave).  One wave-instruction of the gather moves 4 whole
//     256-B rows = 1 KiB, the widest coalesced access (16 B/lane).
//   * the group loads LPR (col,val) pairs with one coalesced load each, then broadcasts edge k
//     to all its lanes in-register (DPP row_newbcast for LPR=16, ds_bpermute otherwise) and
//     issues LPR independent row gathers before consuming any -> LPR x 1 KiB in flight / wave.
//   * heavy rows are split into units of <= chunk edges (nnz balance, host planner below);
//     their partial sums go to a workspace slab and a fix-up kernel adds them in chunk order,
//     so the result is deterministic (no float atomics).
//   * epilogue fuses the layer mean: Y2 = alpha*acc + beta1*A1 + beta2*A2, optional raw Y1.
//
// Algorithmic bytes per launch: 8(N+1) + nnz*(4+4) + nnz*d*4 + N*d*4 (+ epilogue
// addend reads / extra writes), used by bench.py for roofline.achieved.
#include "fr_common.h"

#include <algorithm>
#include <vector>

namespace {

template <int LPR, int K>
__device__ __forceinline__ int bcast_i(int v) {
  if constexpr (LPR == 16) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xf, 0xf, false);  // row_newbcast:K
  } else {
    const int lane = threadIdx.x & 63;
    return __shfl(v, (lane & ~(LPR - 1)) | K, 64);
  }
}

template <int LPR, int K>
__device__ __forceinline__ float bcast_f(float v) {
  return __int_as_float(bcast_i<LPR, K>(__float_as_int(v)));
}

// A row table whose rows [0, split) live at lo (stride ld) and rows [split, n) at hi (stride ldh,
// row r at hi + (r - split) * ldh); hi == nullptr: every row at lo.  Lets a propagation read its
// ego table as [user table ; item table] and write its gradient into the parameters' own buffers
// (no concatenation, no split copies).
struct Tab {
  const float* lo; int64_t ld;
  const float* hi; int64_t ldh;
};

__device__ __forceinline__ const float* tab_row(const Tab& t, int64_t r, int64_t split) {
  return (t.hi != nullptr && r >= split) ? t.hi + (r - split) * t.ldh : t.lo + r * t.ld;
}

struct Epi {
  Tab Y1;
  Tab Y2; float alpha;
  Tab A1; float beta1;
  Tab A2; float beta2;
  int64_t split;
  const uint8_t* a1_gate;  // A1 row r is read only where a1_gate[r] != 0 (else it counts as zero)
};

// write one row's result (float4 slot q of row r) through the fused epilogue
__device__ __forceinline__ void epilogue(const Epi& ep, int64_t r, int q, float4 acc) {
  if (ep.Y1.lo) reinterpret_cast<float4*>(const_cast<float*>(tab_row(ep.Y1, r, ep.split)))[q] = acc;
  if (ep.Y2.lo) {
    float4 o = f4_scale(ep.alpha, acc);
    if (ep.A1.lo && (ep.a1_gate == nullptr || ep.a1_gate[r] != 0))
      o = f4_fma(ep.beta1, reinterpret_cast<const float4*>(tab_row(ep.A1, r, ep.split))[q], o);
    if (ep.A2.lo) o = f4_fma(ep.beta2, reinterpret_cast<const float4*>(tab_row(ep.A2, r, ep.split))[q], o);
    reinterpret_cast<float4*>(const_cast<float*>(tab_row(ep.Y2, r, ep.split)))[q] = o;
  }
}

// X operand of the gather: [lo ; hi] split at `split` (SPLIT), columns masked by cmask (MASK:
// an edge whose column has cmask == 0 is skipped -- its row of X is known to be zero).
struct XSrc {
  const float4* lo; int64_t ld4;
  const float4* hi; int64_t ldh4;
  int64_t split;
  const uint8_t* cmask;
};

// a zero row for masked-out edges (d <= 1024 -> at most 256 float4); zero-initialised at load
__device__ float4 g_zero_row[256];


// Gather-accumulate edges [e0, e1) of one unit into acc (slot q of an LPR-lane group).
// Rows wider than LPR float4 slots are handled by the caller's group-uniform slot loop.
// Plain tables broadcast the edge's column and address X from it; split tables (SPLIT) and masked
// gathers (MASK) resolve every lane's row address once, before the broadcasts, as a float4 offset
// from xs.lo (the hi table, or the zero row of a masked-out edge, expressed relative to lo), so the
// 16 gathers of a batch stay branch-free.
template <int LPR, bool SPLIT, bool MASK>
__device__ __forceinline__ float4 gather_unit(const int32_t* __restrict__ col,
                                              const float* __restrict__ val, const XSrc& xs,
                                              int64_t e0, int64_t e1, int lig, int q) {
  // lig = lane index inside the group (edge slot of the cooperative col/val load),
  // q   = float4 slot of the row this lane gathers
  constexpr bool OFF = SPLIT || MASK;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t e = e0; e < e1; e += LPR) {
    const int64_t my = e + lig;
    const int64_t last = e1 - 1;
    // lanes past the unit's end re-point at its last edge (cache hit) with weight 0
    const int c = __builtin_nontemporal_load(col + (my < e1 ? my : last));
    float v = my < e1 ? __builtin_nontemporal_load(val + my) : 0.f;
    int64_t off = 0;  // float4 offset of this lane's X row from xs.lo (OFF mode)
    if constexpr (OFF) {
      if constexpr (SPLIT) {
        off = c >= xs.split ? (xs.hi - xs.lo) + ((int64_t)c - xs.split) * xs.ldh4 : (int64_t)c * xs.ld4;
      } else {
        off = (int64_t)c * xs.ld4;
      }
      if constexpr (MASK) {
        // one mask load per lane, then a group-uniform skip of batches that reach no marked row;
        // the remaining masked-out edges read the (cached) zero row with weight 0
        const bool m = my < e1 && xs.cmask[c] != 0;
        const uint64_t bal = __ballot(m);
        const int gbase = (threadIdx.x & 63) & ~(LPR - 1);
        const uint64_t gmask = LPR >= 64 ? ~0ull : ((1ull << LPR) - 1ull);
        if (((bal >> gbase) & gmask) == 0) continue;
        if (!m) {
          v = 0.f;
          off = g_zero_row - xs.lo;
        }
      }
    }
    const int off_lo = (int)(uint32_t)(uint64_t)off, off_hi = (int)(uint32_t)((uint64_t)off >> 32);
    constexpr int NB = LPR < 16 ? LPR : 16;
    float4 x[NB];
    float w[NB];
#define FR_GATHER(K)                                                                        \
    if constexpr ((K) < LPR) {                                                              \
      w[(K)] = bcast_f<LPR, (K)>(v);                                                        \
      if constexpr (OFF) {                                                                  \
        const uint64_t ok = (uint64_t)(uint32_t)bcast_i<LPR, (K)>(off_lo) |                 \
                            ((uint64_t)(uint32_t)bcast_i<LPR, (K)>(off_hi) << 32);          \
        x[(K)] = xs.lo[(int64_t)ok + q];                                                    \
      } else {                                                                              \
        const int ck = bcast_i<LPR, (K)>(c);                                                \
        x[(K)] = xs.lo[(int64_t)ck * xs.ld4 + q];                                           \
      }                                                                                     \
    }
    FR_GATHER(0) FR_GATHER(1) FR_GATHER(2) FR_GATHER(3)
    FR_GATHER(4) FR_GATHER(5) FR_GATHER(6) FR_GATHER(7)
    FR_GATHER(8) FR_GATHER(9) FR_GATHER(10) FR_GATHER(11)
    FR_GATHER(12) FR_GATHER(13) FR_GATHER(14) FR_GATHER(15)
#undef FR_GATHER
#pragma unroll
    for (int k = 0; k < (LPR < 16 ? LPR : 16); ++k) acc = f4_fma(w[k], x[k], acc);
    if constexpr (LPR > 16) {
      // wider groups: remaining broadcasts through ds_bpermute in a runtime loop
      for (int k = 16; k < LPR; ++k) {
        const int lane = threadIdx.x & 63;
        const int src = (lane & ~(LPR - 1)) | k;
        const float wk = __shfl(v, src, 64);
        if constexpr (OFF) {
          const uint64_t ok = (uint64_t)(uint32_t)__shfl(off_lo, src, 64) |
                              ((uint64_t)(uint32_t)__shfl(off_hi, src, 64) << 32);
          acc = f4_fma(wk, xs.lo[(int64_t)ok + q], acc);
        } else {
          const int ck = __shfl(c, src, 64);
          acc = f4_fma(wk, xs.lo[(int64_t)ck * xs.ld4 + q], acc);
        }
      }
    }
  }
  return acc;
}

template <int LPR, bool SPLIT, bool MASK>
__global__ __launch_bounds__(256) void spmm_units_kernel(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const int2* __restrict__ units, int64_t n_units,
    int64_t n_plain, int chunk, XSrc xs, int d4, Epi ep,
    float4* __restrict__ partial, int64_t row_lo, int64_t row_hi) {
  constexpr int GPB = 256 / LPR;  // groups per block
  const int q0 = threadIdx.x % LPR;
  const int grp = threadIdx.x / LPR;
  for (int64_t u = (int64_t)blockIdx.x * GPB + grp; u < n_units; u += (int64_t)gridDim.x * GPB) {
    const int2 unit = units[u];
    if (unit.x < row_lo || unit.x >= row_hi) continue;  // row range (group-uniform)
    const int64_t rs = rowptr[unit.x];
    const int64_t e0 = rs + (int64_t)unit.y * chunk;
    const int64_t e1 = min(rowptr[unit.x + 1], e0 + (int64_t)chunk);
    // group-uniform slot loop: every lane of the group takes part in the broadcasts
    for (int qb = 0; qb < d4; qb += LPR) {
      const int q = qb + q0;
      const float4 acc = gather_unit<LPR, SPLIT, MASK>(col, val, xs, e0, e1, q0, q < d4 ? q : d4 - 1);
      if (q < d4) {
        if (u < n_plain) {
          epilogue(ep, unit.x, q, acc);
        } else {
          partial[(u - n_plain) * d4 + q] = acc;
        }
      }
    }
  }
}

// Fix-up for split rows: sum the row's chunk partials in order, then the epilogue.
template <int LPR>
__global__ __launch_bounds__(256) void spmm_fixup_kernel(const int3* __restrict__ split_rows,
                                                         int64_t n_split, int d4, Epi ep,
                                                         const float4* __restrict__ partial, int64_t row_lo,
                                                         int64_t row_hi) {
  constexpr int GPB = 256 / LPR;
  const int q0 = threadIdx.x % LPR;
  const int grp = threadIdx.x / LPR;
  for (int64_t s = (int64_t)blockIdx.x * GPB + grp; s < n_split; s += (int64_t)gridDim.x * GPB) {
    const int3 sr = split_rows[s];
    if (sr.x < row_lo || sr.x >= row_hi) continue;
    for (int q = q0; q < d4; q += LPR) {
      float4 acc = partial[(int64_t)sr.y * d4 + q];
      for (int k = 1; k < sr.z; ++k) acc = f4_add(acc, partial[((int64_t)sr.y + k) * d4 + q]);
      epilogue(ep, sr.x, q, acc);
    }
  }
}

// Row-list mode: only the rows named by `rl` (up to three id segments, each shifted by its
// offset; duplicates allowed -- they write identical values) are computed, one 1024-thread
// workgroup per listed row: the row's 16-edge batches are dealt round-robin to the 64 lane groups
// and the 64 group partials are summed in group order (deterministic; the summation order differs
// from the full launch's, so rows agree with it to fp32 rounding).  A heavy row (an item with
// thousands of users) costs a few batches per group instead of a serial chain.
struct RowList {
  const int64_t* ids[3];
  int64_t n[3];
  int64_t off[3];
};

constexpr int kRowThreads = 1024;

template <int LPR, bool SPLIT>
__global__ __launch_bounds__(kRowThreads) void spmm_rows_kernel(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, RowList rl, XSrc xs, int d4, Epi ep) {
  static_assert(LPR == 16, "row-list mode is built for d = 64 (16 lanes x float4)");
  constexpr int GPB = kRowThreads / LPR;
  __shared__ float4 slots[GPB][LPR];
  const int q0 = threadIdx.x % LPR;
  const int grp = threadIdx.x / LPR;
  int64_t idx = blockIdx.x;
  int seg = 0;
  while (seg < 3 && idx >= rl.n[seg]) idx -= rl.n[seg++];
  if (seg >= 3 || rl.ids[seg][idx] < 0) return;  // a negative id: no row (e.g. a batch user owned elsewhere)
  const int64_t row = rl.ids[seg][idx] + rl.off[seg];
  const int64_t rs = rowptr[row], re = rowptr[row + 1];
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t e0 = rs + (int64_t)grp * LPR; e0 < re; e0 += (int64_t)GPB * LPR) {
    const int64_t e1 = e0 + LPR < re ? e0 + LPR : re;
    acc = f4_add(acc, gather_unit<LPR, SPLIT, false>(col, val, xs, e0, e1, q0, q0));
  }
  slots[grp][q0] = acc;
  __syncthreads();
  if (grp == 0) {
    float4 t = slots[0][q0];
    for (int g = 1; g < GPB; ++g) t = f4_add(t, slots[g][q0]);
    epilogue(ep, row, q0, t);
  }
}

// mask[row] = value at the listed rows; with Z, also Z[row][0..d) = 0 (16 lanes x float4 per row);
// with bits, bit `row` of the bitmask set (value != 0) or cleared
__global__ __launch_bounds__(256) void rows_mark_kernel(uint8_t* __restrict__ mask, RowList rl, int64_t total,
                                                        uint8_t value, float4* __restrict__ Z, int64_t ldz4, int d4,
                                                        uint32_t* __restrict__ bits) {
  const int per = Z ? 16 : 1;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total * per; i += (int64_t)gridDim.x * 256) {
    int64_t idx = i / per;
    const int q = (int)(i % per);
    int seg = 0;
    while (idx >= rl.n[seg]) idx -= rl.n[seg++];
    if (rl.ids[seg][idx] < 0) continue;  // negative ids name no row
    const int64_t row = rl.ids[seg][idx] + rl.off[seg];
    if (q == 0) mask[row] = value;
    if (q == 0 && bits) {
      if (value) atomicOr(bits + (row >> 5), 1u << (row & 31));
      else atomicAnd(bits + (row >> 5), ~(1u << (row & 31)));
    }
    if (Z)
      for (int c = q; c < d4; c += 16) Z[row * ldz4 + c] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}


// ---------------------------------------------------------------------------------------------
// Sparse-upstream mode (fr_spmm_sparse_upstream): Y2 = alpha * A X + beta1 * gate(X) where X is
// non-zero only at the rows set in a bitmask (the batch rows of a propagation's upstream
// gradient; the rest of X is never read).  One workgroup per 64 consecutive rows:
//   * the bitmask is staged in LDS;
//   * the block's edge range is scanned in coalesced 1024-edge rounds; the edges whose column is
//     marked ("hits") are compacted in edge order (wave ballots + a prefix over the 16 wave-slices
//     of the round), so the hit list is sorted by row;
//   * each 16-lane group (float4 column slot per lane) walks a contiguous slice of the hits,
//     gathers X at the hit columns (four in flight), sums each row's run in registers and adds it
//     to the block's LDS row accumulator once per run -- LDS float atomics per run, not per hit
//     (a per-hit add serialises: consecutive hits share a row);
//   * every row is written once: alpha * acc + beta1 * X (X read at marked rows only).
// Work: one column + value load per edge, one 256-B gather per hit.  A row split over group slices
// or rounds gets several adds in a run-to-run variable order (the deterministic mode keeps the
// column-masked gather).  d = 64.
constexpr int kSpRows = 64;
// bit 0: a plan block of more than kSpRows rows (or outside [0, n_rows)); bit 1: a block whose edge
// range leaves its rows.  Set by spmm_sparse_kernel, read and cleared by fr_spmm_plan_status.
__device__ unsigned int g_sparse_plan_status;
constexpr int kSpRound = 1024;
constexpr int kSpStageWords = 1024;  // bitmask staged in LDS (dynamic, ceil(n / 32) words): up to 32,768 rows

// GBITS: the bitmask is read from global memory (L2-resident: ceil(n / 32) words, 1.4 MB at 11M
// rows) instead of being staged in LDS -- graphs beyond 32,768 rows (HealthRec UI, config 4).
// UNGATED (a rectangular slice: the bitmask marks X's rows, i.e. columns, not output rows): A1 is
// read at every output row.
// BLOCKS (a row-block plan, fr_spmm_sparse_upstream*_blocks): block b covers rows
// [blocks[4b], blocks[4b+1]) and edges [blocks[4b+2], blocks[4b+3]) -- at most 64 rows of a bounded
// edge count, or one CHUNK of a heavy row (Zipf item rows: up to 434k edges at config 4, which a
// 64-row block would scan alone in hundreds of rounds).  A chunk adds alpha * its partial into the
// row atomically; the row's own term (beta1 * A1 or 0) is written first by sparse_split_init_kernel.
template <bool GBITS, bool UNGATED = false>
__global__ __launch_bounds__(256) void spmm_sparse_kernel(const int64_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ col,
                                                          const float* __restrict__ val, int64_t n_rows,
                                                          const uint32_t* __restrict__ bits, int nwords,
                                                          const float4* __restrict__ X, int64_t ldx4, Epi ep,
                                                          const int64_t* __restrict__ blocks = nullptr,
                                                          float4* __restrict__ zero4 = nullptr, int64_t zero_n4 = 0) {
  constexpr int KS = kSpRound / 256;  // edges per thread per round
  extern __shared__ uint32_t sbits_dyn[];
  const uint32_t* sbits = GBITS ? bits : sbits_dyn;
  __shared__ float4 acc[kSpRows][16];
  __shared__ int64_t srp[kSpRows + 1];
  __shared__ int hit_c[kSpRound];    // the edge's column
  __shared__ short hit_e[kSpRound];  // its offset in the round
  __shared__ float hit_v[kSpRound];  // its value
  __shared__ int cnt[KS * 4];        // hits per (k, wave) slice of the round
  const int t = threadIdx.x, q = t & 15, lane = t & 63, wave = t >> 6;
  // side job (fr_spmm_sparse_upstream_zero): zero a contiguous region for the next kernel on the
  // stream -- HealthRec's d ingre rows, which the RI backward's list scatter then accumulates into --
  // instead of a memset launch of its own between the two
  for (int64_t k = (int64_t)blockIdx.x * 256 + t; k < zero_n4; k += (int64_t)gridDim.x * 256)
    zero4[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int64_t r0 = blocks ? blocks[4 * (int64_t)blockIdx.x] : (int64_t)blockIdx.x * kSpRows;
  const int64_t r1 = blocks ? blocks[4 * (int64_t)blockIdx.x + 1] : min<int64_t>(r0 + kSpRows, n_rows);
  // a plan block must fit the LDS row accumulator (kSpRows rows) and the adjacency's rows: anything
  // else is refused here (block-uniform, before any LDS index depends on it) and reported through
  // g_sparse_plan_status (fr_spmm_plan_status), never computed into a wrong row
  if (r0 < 0 || r1 < r0 || r1 - r0 > kSpRows || r1 > n_rows) {
    if (t == 0) atomicOr(&g_sparse_plan_status, 1u);
    return;
  }
  const int nr = (int)(r1 - r0);
  if constexpr (!GBITS) {  // stage the bitmask: 16-B loads, all in flight before the LDS stores
    const int n4 = nwords >> 2;
    const uint4* b4 = reinterpret_cast<const uint4*>(bits);
#pragma unroll 8
    for (int w = t; w < n4; w += 256) reinterpret_cast<uint4*>(sbits_dyn)[w] = b4[w];
    if (t < (nwords & 3)) sbits_dyn[(n4 << 2) + t] = bits[(n4 << 2) + t];
  }
  for (int i = t; i < kSpRows * 16; i += 256) acc[i >> 4][i & 15] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int i = t; i <= nr; i += 256) srp[i] = rowptr[r0 + i];
  __syncthreads();
  const int64_t e0 = blocks ? blocks[4 * (int64_t)blockIdx.x + 2] : srp[0];
  const int64_t e1 = blocks ? blocks[4 * (int64_t)blockIdx.x + 3] : srp[nr];
  const bool chunk = e0 != srp[0] || e1 != srp[nr];  // part of one heavy row (block-uniform)
  if (e0 < srp[0] || e1 > srp[nr] || e1 < e0 || (chunk && nr != 1)) {  // edges outside the block's rows
    if (t == 0) atomicOr(&g_sparse_plan_status, 2u);
    return;
  }
  for (int64_t base = e0; base < e1; base += kSpRound) {
    // scan: coalesced column and value loads (edge base + k * 256 + t), hit flags by wave ballot
    int cs[KS];
    float vs[KS];
    uint64_t bal[KS];
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int64_t e = base + k * 256 + t;
      cs[k] = e < e1 ? __builtin_nontemporal_load(col + e) : -1;
      vs[k] = e < e1 ? __builtin_nontemporal_load(val + e) : 0.f;
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      const int c = cs[k];
      bal[k] = __ballot(c >= 0 && ((sbits[c >> 5] >> (c & 31)) & 1u));
      if (lane == 0) cnt[k * 4 + wave] = __popcll(bal[k]);
    }
    __syncthreads();
    // ordered compaction: slice (k, wave) starts after every earlier slice's hits
    int nh = 0, off[KS];
#pragma unroll
    for (int j = 0; j < KS * 4; ++j) {
      const int cj = cnt[j];
#pragma unroll
      for (int k = 0; k < KS; ++k)
        if (j == k * 4 + wave) off[k] = nh;
      nh += cj;
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) {
      if ((bal[k] >> lane) & 1ull) {
        const int slot = off[k] + __builtin_amdgcn_mbcnt_hi((uint32_t)(bal[k] >> 32),
                                                            __builtin_amdgcn_mbcnt_lo((uint32_t)bal[k], 0u));
        hit_c[slot] = cs[k];
        hit_e[slot] = (short)(k * 256 + t);
        hit_v[slot] = vs[k];
      }
    }
    __syncthreads();
    // accumulate: group g walks hits [g nh / 16, (g + 1) nh / 16) in row order
    const int g = t >> 4;
    const int h_lo = (g * nh) >> 4, h_hi = ((g + 1) * nh) >> 4;
    if (h_lo < h_hi) {
      int rl = 0;
      {  // row of the first hit: srp[rl] <= e < srp[rl + 1]
        const int64_t e = base + hit_e[h_lo];
        int hi = nr;
        while (hi - rl > 1) {
          const int mid = (rl + hi) >> 1;
          if (srp[mid] <= e) rl = mid; else hi = mid;
        }
      }
      int cur = rl;
      float4 sum = make_float4(0.f, 0.f, 0.f, 0.f);
      for (int h0 = h_lo; h0 < h_hi; h0 += 4) {
        float4 x[4];
        float v[4];
        int eo[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int h = min(h0 + j, h_hi - 1);
          eo[j] = hit_e[h];
          v[j] = hit_v[h];
          x[j] = X[(int64_t)hit_c[h] * ldx4 + q];
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          if (h0 + j < h_hi) {
            const int64_t e = base + eo[j];
            while (srp[rl + 1] <= e) ++rl;
            if (rl != cur) {
              float* a = reinterpret_cast<float*>(&acc[cur][q]);
              atomicAdd(a + 0, sum.x);
              atomicAdd(a + 1, sum.y);
              atomicAdd(a + 2, sum.z);
              atomicAdd(a + 3, sum.w);
              sum = make_float4(0.f, 0.f, 0.f, 0.f);
              cur = rl;
            }
            sum = f4_fma(v[j], x[j], sum);
          }
        }
      }
      float* a = reinterpret_cast<float*>(&acc[cur][q]);
      atomicAdd(a + 0, sum.x);
      atomicAdd(a + 1, sum.y);
      atomicAdd(a + 2, sum.z);
      atomicAdd(a + 3, sum.w);
    }
    __syncthreads();
  }
  if (chunk) {  // the row's own term is already in Y2 (sparse_split_init_kernel)
    if (t < 16) {
      float* y = const_cast<float*>(tab_row(ep.Y2, r0, ep.split)) + 4 * q;
      const float4 o = f4_scale(ep.alpha, acc[0][q]);
      atomicAdd(y + 0, o.x);
      atomicAdd(y + 1, o.y);
      atomicAdd(y + 2, o.z);
      atomicAdd(y + 3, o.w);
    }
    return;
  }
  // write every row: Y2 = alpha * acc + beta1 * A1 (A1 read only at marked rows)
  for (int i = t; i < nr * 16; i += 256) {
    const int rl = i >> 4;
    const int64_t r = r0 + rl;
    float4 o = f4_scale(ep.alpha, acc[rl][q]);
    if (ep.A1.lo && (UNGATED || ((sbits[r >> 5] >> (r & 31)) & 1u)))
      o = f4_fma(ep.beta1, reinterpret_cast<const float4*>(tab_row(ep.A1, r, ep.split))[q], o);
    reinterpret_cast<float4*>(const_cast<float*>(tab_row(ep.Y2, r, ep.split)))[q] = o;
  }
}

// ---------------------------------------------------------------------------------------------
// Pipelined plain mode (d = 64, every row a plain unit, no column mask; X one table or split): the shape of
// HealthRec's RI propagation (65,617 rows of <= 45 edges).  There a group's unit is one batch of
// <= 16 edges and the general kernel pays four dependent memory trips per row (unit entry ->
// rowptr -> col / val -> gathers, then the epilogue addends); here a 16-lane group walks rows
// r, r + G, ... with the next row's rowptr pair, the current row's epilogue addends and the next
// batch's col / val all issued before the current batch's 16 gathers are consumed, so a row costs
// about one exposed trip.  Edge order and FMA order are those of gather_unit (bit-identical rows).
__device__ __forceinline__ void load_batch(const int32_t* __restrict__ col, const float* __restrict__ val, int64_t e,
                                           int64_t e1, int lig, int& c, float& v) {
  const int64_t my = e + lig;
  c = my < e1 ? __builtin_nontemporal_load(col + my) : 0;  // lanes past the end: row 0, weight 0
  v = my < e1 ? __builtin_nontemporal_load(val + my) : 0.f;
}

template <bool SPLIT>
__global__ __launch_bounds__(256) void spmm_plain16_kernel(const int64_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ col,
                                                           const float* __restrict__ val, int64_t row_lo,
                                                           int64_t n_rows, XSrc xs, Epi ep) {
  // rows [row_lo, n_rows), walked from the last row down: the bipartite item-side graphs keep
  // their heavier side rows (ingredients, clusters) at the end, so these start first and the
  // light item rows fill the tail
  constexpr int LPR = 16, GPB = 256 / LPR;
  const int q = threadIdx.x % LPR;
  const int64_t G = (int64_t)gridDim.x * GPB, n = n_rows - row_lo;
  int64_t j = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR;
  if (j >= n) return;
  int64_t r = n_rows - 1 - j;
  int64_t e0 = rowptr[r], e1 = rowptr[r + 1];
  int c;
  float v;
  load_batch(col, val, e0, e1, q, c, v);
  const bool has_a1 = ep.Y2.lo && ep.A1.lo, has_a2 = ep.Y2.lo && ep.A2.lo;
  while (true) {
    const int64_t jn = j + G, rn = n_rows - 1 - jn;
    const bool more = jn < n;
    int64_t ne0 = 0, ne1 = 0;
    if (more) {
      ne0 = rowptr[rn];
      ne1 = rowptr[rn + 1];
    }
    float4 a1 = make_float4(0.f, 0.f, 0.f, 0.f), a2 = a1;
    if (has_a1 && (ep.a1_gate == nullptr || ep.a1_gate[r] != 0))
      a1 = reinterpret_cast<const float4*>(tab_row(ep.A1, r, ep.split))[q];
    if (has_a2) a2 = reinterpret_cast<const float4*>(tab_row(ep.A2, r, ep.split))[q];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t e = e0; e < e1; e += LPR) {
      float4 x[LPR];
      float w[LPR];
      // SPLIT: each lane's X row as a float4 offset from xs.lo (the hi table relative to it), the
      // 64-bit offsets broadcast in two halves (as gather_unit's OFF mode)
      int64_t off = 0;
      if constexpr (SPLIT)
        off = c >= xs.split ? (xs.hi - xs.lo) + ((int64_t)c - xs.split) * xs.ldh4 : (int64_t)c * xs.ld4;
      const int off_lo = (int)(uint32_t)(uint64_t)off, off_hi = (int)(uint32_t)((uint64_t)off >> 32);
#define FR_PG(K)                                                                           \
      {                                                                                    \
        w[(K)] = bcast_f<LPR, (K)>(v);                                                     \
        if constexpr (SPLIT) {                                                             \
          const uint64_t ok = (uint64_t)(uint32_t)bcast_i<LPR, (K)>(off_lo) |              \
                              ((uint64_t)(uint32_t)bcast_i<LPR, (K)>(off_hi) << 32);       \
          x[(K)] = xs.lo[(int64_t)ok + q];                                                 \
        } else {                                                                           \
          const int ck = bcast_i<LPR, (K)>(c);                                             \
          x[(K)] = xs.lo[(int64_t)ck * xs.ld4 + q];                                        \
        }                                                                                  \
      }
      FR_PG(0) FR_PG(1) FR_PG(2) FR_PG(3) FR_PG(4) FR_PG(5) FR_PG(6) FR_PG(7)
      FR_PG(8) FR_PG(9) FR_PG(10) FR_PG(11) FR_PG(12) FR_PG(13) FR_PG(14) FR_PG(15)
#undef FR_PG
      // the next batch of this row, else the next row's first batch, in flight during the gathers
      if (e + LPR < e1) load_batch(col, val, e + LPR, e1, q, c, v);
      else if (more) load_batch(col, val, ne0, ne1, q, c, v);
#pragma unroll
      for (int k = 0; k < LPR; ++k) acc = f4_fma(w[k], x[k], acc);
    }
    if (e0 == e1 && more) load_batch(col, val, ne0, ne1, q, c, v);  // empty row
    if (ep.Y1.lo) reinterpret_cast<float4*>(const_cast<float*>(tab_row(ep.Y1, r, ep.split)))[q] = acc;
    if (ep.Y2.lo) {
      float4 o = f4_scale(ep.alpha, acc);
      if (has_a1) o = f4_fma(ep.beta1, a1, o);
      if (has_a2) o = f4_fma(ep.beta2, a2, o);
      reinterpret_cast<float4*>(const_cast<float*>(tab_row(ep.Y2, r, ep.split)))[q] = o;
    }
    if (!more) break;
    j = jn;
    r = rn;
    e0 = ne0;
    e1 = ne1;
  }
}

// Row-list walk (fr_spmm_csr_list): the rows list[0 .. *count) only, the count read on the device (a
// list built by an earlier launch, e.g. fr_rows_frontier).  Each 16-lane group takes rows j, j + G,
// ...; per row the same 16-edge batches and FMA order as spmm_plain16_kernel (rows bit-identical).
template <bool SPLIT>
__global__ __launch_bounds__(256) void spmm_list16_kernel(const int64_t* __restrict__ rowptr,
                                                          const int32_t* __restrict__ col,
                                                          const float* __restrict__ val,
                                                          const int32_t* __restrict__ list,
                                                          const int32_t* __restrict__ d_count, XSrc xs, Epi ep) {
  constexpr int LPR = 16, GPB = 256 / LPR;
  const int q = threadIdx.x % LPR;
  const int64_t n = d_count[0];
  const int64_t G = (int64_t)gridDim.x * GPB;
  const bool has_a1 = ep.Y2.lo && ep.A1.lo, has_a2 = ep.Y2.lo && ep.A2.lo;
  for (int64_t j = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR; j < n; j += G) {
    const int64_t r = list[j];
    const int64_t e0 = rowptr[r], e1 = rowptr[r + 1];
    int c;
    float v;
    load_batch(col, val, e0, e1, q, c, v);
    float4 a1 = make_float4(0.f, 0.f, 0.f, 0.f), a2 = a1;
    if (has_a1) a1 = reinterpret_cast<const float4*>(tab_row(ep.A1, r, ep.split))[q];
    if (has_a2) a2 = reinterpret_cast<const float4*>(tab_row(ep.A2, r, ep.split))[q];
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int64_t e = e0; e < e1; e += LPR) {
      float4 x[LPR];
      float w[LPR];
      int64_t off = 0;
      if constexpr (SPLIT)
        off = c >= xs.split ? (xs.hi - xs.lo) + ((int64_t)c - xs.split) * xs.ldh4 : (int64_t)c * xs.ld4;
      const int off_lo = (int)(uint32_t)(uint64_t)off, off_hi = (int)(uint32_t)((uint64_t)off >> 32);
#define FR_PG(K)                                                                           \
      {                                                                                    \
        w[(K)] = bcast_f<LPR, (K)>(v);                                                     \
        if constexpr (SPLIT) {                                                             \
          const uint64_t ok = (uint64_t)(uint32_t)bcast_i<LPR, (K)>(off_lo) |              \
                              ((uint64_t)(uint32_t)bcast_i<LPR, (K)>(off_hi) << 32);       \
          x[(K)] = xs.lo[(int64_t)ok + q];                                                 \
        } else {                                                                           \
          const int ck = bcast_i<LPR, (K)>(c);                                             \
          x[(K)] = xs.lo[(int64_t)ck * xs.ld4 + q];                                        \
        }                                                                                  \
      }
      FR_PG(0) FR_PG(1) FR_PG(2) FR_PG(3) FR_PG(4) FR_PG(5) FR_PG(6) FR_PG(7)
      FR_PG(8) FR_PG(9) FR_PG(10) FR_PG(11) FR_PG(12) FR_PG(13) FR_PG(14) FR_PG(15)
#undef FR_PG
      if (e + LPR < e1) load_batch(col, val, e + LPR, e1, q, c, v);
#pragma unroll
      for (int k = 0; k < LPR; ++k) acc = f4_fma(w[k], x[k], acc);
    }
    if (ep.Y1.lo) reinterpret_cast<float4*>(const_cast<float*>(tab_row(ep.Y1, r, ep.split)))[q] = acc;
    if (ep.Y2.lo) {
      float4 o = f4_scale(ep.alpha, acc);
      if (has_a1) o = f4_fma(ep.beta1, a1, o);
      if (has_a2) o = f4_fma(ep.beta2, a2, o);
      reinterpret_cast<float4*>(const_cast<float*>(tab_row(ep.Y2, r, ep.split)))[q] = o;
    }
  }
}

// fr_spmm_list_scatter: Y[c - split] += alpha * A[r][c] * X[r] for the listed rows r (count read on the
// device) and their columns c >= split -- the transpose product A^T X restricted to the side rows, for
// an X that is zero outside the list (A symmetric: the side rows' gather becomes the listed rows'
// scatter, work proportional to the listed rows' degrees).  One wave per listed row, lane = column:
// each edge is one 256-B float-atomic wave instruction; the row's edges are read 64 at a time
// (coalesced) and broadcast from their lanes.
__global__ __launch_bounds__(256) void list_scatter_kernel(const int64_t* __restrict__ rowptr,
                                                           const int32_t* __restrict__ col,
                                                           const float* __restrict__ val,
                                                           const int32_t* __restrict__ list,
                                                           const int32_t* __restrict__ d_count, int64_t split,
                                                           const float* __restrict__ X, int64_t ldx,
                                                           float* __restrict__ Y, int64_t ldy, float alpha) {
  const int lane = threadIdx.x & 63;
  const int64_t n = d_count[0];
  const int64_t W = (int64_t)gridDim.x * 4;
  for (int64_t j = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); j < n; j += W) {
    const int64_t r = list[j];
    const float x = alpha * X[r * ldx + lane];
    const int64_t e0 = rowptr[r], e1 = rowptr[r + 1];
    for (int64_t e = e0; e < e1; e += 64) {
      const int m = (int)min((int64_t)64, e1 - e);
      const int cl = lane < m ? col[e + lane] : 0;
      const float vl = lane < m ? val[e + lane] : 0.f;
      for (int k = 0; k < m; ++k) {
        const int64_t c = (int64_t)__builtin_amdgcn_readlane(cl, k);
        const float v = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, vl), k));
        if (c >= split) atomicAdd(Y + (c - split) * ldy + lane, v * x);
      }
    }
  }
}

// fr_rows_frontier: mark[i] = 1 for the item columns of the batch users' rows of a [users | items]
// adjacency (columns U + i) and for the batch items; count reset for the compaction.  One wave per
// batch triple.
__global__ __launch_bounds__(256) void frontier_mark_kernel(const int64_t* __restrict__ rowptr,
                                                            const int32_t* __restrict__ col, int64_t U, int64_t I,
                                                            const int64_t* __restrict__ uu,
                                                            const int64_t* __restrict__ pp,
                                                            const int64_t* __restrict__ nn, int64_t B,
                                                            uint8_t* __restrict__ mark, int32_t* __restrict__ count) {
  const int lane = threadIdx.x & 63;
  const int64_t b = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 6;
  if (blockIdx.x == 0 && threadIdx.x == 0) count[0] = 0;
  if (b >= B) return;
  const int64_t u = uu[b];
  for (int64_t e = rowptr[u] + lane; e < rowptr[u + 1]; e += 64) {
    const int64_t i = (int64_t)col[e] - U;
    if (i >= 0 && i < I) mark[i] = 1;
  }
  if (lane == 0) {
    if (pp[b] >= 0 && pp[b] < I) mark[pp[b]] = 1;
    if (nn[b] >= 0 && nn[b] < I) mark[nn[b]] = 1;
  }
}

// the marked items appended to list (order: arbitrary -- each listed row is computed on its own) and
// unmarked for the next step.  Each thread takes 4 marks (one 32-bit load), the block scans its
// counts (wave shuffles + LDS) and takes its list range with ONE atomic: a 1024-item block per
// atomic instead of a wave per atomic (the counter is the serialisation point).
constexpr int kCompactItems = 1024;
__global__ __launch_bounds__(256) void frontier_compact_kernel(uint8_t* __restrict__ mark, int64_t I,
                                                               int32_t* __restrict__ list, int32_t* __restrict__ count) {
  __shared__ int wsum[4];
  __shared__ int base_s;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t i0 = (int64_t)blockIdx.x * kCompactItems + 4 * t;
  uint32_t m = 0;
  if (i0 + 3 < I) {
    m = *reinterpret_cast<const uint32_t*>(mark + i0);  // (mark 4-B aligned: host check)
  } else {
    for (int k = 0; k < 4; ++k)
      if (i0 + k < I && mark[i0 + k]) m |= 1u << (8 * k);
  }
  int c = 0;
  for (int k = 0; k < 4; ++k) c += ((m >> (8 * k)) & 0xffu) != 0;
  int x = c;  // inclusive wave scan
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  if (t == 0) {
    const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    base_s = tot ? atomicAdd(count, tot) : 0;
  }
  __syncthreads();
  int off = base_s + x - c;
  for (int k = 0; k < w; ++k) off += wsum[k];
  if (m == 0) return;
  for (int k = 0; k < 4; ++k)
    if ((m >> (8 * k)) & 0xffu) list[off++] = (int32_t)(i0 + k);
  if (i0 + 3 < I) {
    *reinterpret_cast<uint32_t*>(mark + i0) = 0u;
  } else {
    for (int k = 0; k < 4; ++k)
      if (i0 + k < I) mark[i0 + k] = 0;
  }
}

template <int LPR, bool SPLIT, bool MASK>
hipError_t launch_units(const int64_t* rowptr, const int32_t* col, const float* val,
                        const fr_spmm_plan* plan, const XSrc& xs, int d4, const Epi& ep,
                        float4* partial, hipStream_t s, int64_t row_lo, int64_t row_hi) {
  constexpr int GPB = 256 / LPR;
  int64_t blocks = fr::ceil_div(plan->n_units, GPB);
  blocks = std::min<int64_t>(blocks, (int64_t)fr::kNumCU * 64);
  hipLaunchKernelGGL((spmm_units_kernel<LPR, SPLIT, MASK>), dim3((unsigned)blocks), dim3(256), 0, s, rowptr, col,
                     val, reinterpret_cast<const int2*>(plan->d_units), plan->n_units,
                     plan->n_plain, plan->chunk, xs, d4, ep, partial, row_lo, row_hi);
  return hipGetLastError();
}

template <int LPR>
hipError_t launch_spmm(const int64_t* rowptr, const int32_t* col, const float* val, int64_t n_rows,
                       const fr_spmm_plan* plan, const XSrc& xs, int d, const Epi& ep,
                       float4* partial, hipStream_t s, int64_t row_lo, int64_t row_hi) {
  constexpr int GPB = 256 / LPR;
  const int d4 = d / 4;
  const bool split = xs.hi != nullptr, mask = xs.cmask != nullptr;
  if constexpr (LPR == 16) {
    // every row one plain unit, in row order (the planner's plain units are the rows of degree <=
    // chunk, ascending): the pipelined row walk, ~2 rows per group
    if (!mask && d4 == 16 && plan->n_split == 0 && plan->n_units == n_rows && plan->n_plain == n_rows) {
      if (row_hi <= row_lo) return hipSuccess;
      const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(row_hi - row_lo, 2 * GPB),
                                                                    (int64_t)fr::kNumCU * 16));
      if (split)
        hipLaunchKernelGGL(spmm_plain16_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, rowptr, col, val,
                           row_lo, row_hi, xs, ep);
      else
        hipLaunchKernelGGL(spmm_plain16_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, rowptr, col, val,
                           row_lo, row_hi, xs, ep);
      return hipGetLastError();
    }
  }
  if (plan->n_units > 0) {
    hipError_t e;
    if (split && mask) e = launch_units<LPR, true, true>(rowptr, col, val, plan, xs, d4, ep, partial, s, row_lo, row_hi);
    else if (split) e = launch_units<LPR, true, false>(rowptr, col, val, plan, xs, d4, ep, partial, s, row_lo, row_hi);
    else if (mask) e = launch_units<LPR, false, true>(rowptr, col, val, plan, xs, d4, ep, partial, s, row_lo, row_hi);
    else e = launch_units<LPR, false, false>(rowptr, col, val, plan, xs, d4, ep, partial, s, row_lo, row_hi);
    if (e != hipSuccess) return e;
  }
  if (plan->n_split > 0) {
    int64_t blocks = std::min<int64_t>(fr::ceil_div(plan->n_split, GPB), (int64_t)fr::kNumCU * 16);
    hipLaunchKernelGGL(spmm_fixup_kernel<LPR>, dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<const int3*>(plan->d_split_rows), plan->n_split, d4, ep,
                       partial, row_lo, row_hi);
    return hipGetLastError();
  }
  return hipSuccess;
}

}  // namespace

extern "C" int64_t fr_spmm_workspace(const fr_spmm_plan* plan, int d) {
  if (!plan) return 0;
  return (plan->n_units - plan->n_plain) * (int64_t)d * 4 + 256;
}

extern "C" int fr_spmm_plan_host(const int64_t* rowptr, int64_t n_rows, int32_t chunk,
                                 int32_t* units, int64_t* n_units, int64_t* n_plain,
                                 int32_t* split_rows, int64_t* n_split) {
  FR_REQUIRE(rowptr && units && n_units && n_plain && split_rows && n_split, "null argument");
  FR_REQUIRE(chunk > 0, "chunk must be > 0");
  FR_REQUIRE(n_rows >= 0 && n_rows < (int64_t)INT32_MAX, "n_rows out of int32 range");
  int64_t nu = 0;
  for (int64_t r = 0; r < n_rows; ++r) {
    const int64_t deg = rowptr[r + 1] - rowptr[r];
    FR_REQUIRE(deg >= 0, "rowptr must be non-decreasing");
    if (deg <= chunk) {
      units[2 * nu] = (int32_t)r;
      units[2 * nu + 1] = 0;
      ++nu;
    }
  }
  *n_plain = nu;
  int64_t ns = 0, first = 0;
  for (int64_t r = 0; r < n_rows; ++r) {
    const int64_t deg = rowptr[r + 1] - rowptr[r];
    if (deg > chunk) {
      const int64_t nc = fr::ceil_div(deg, chunk);
      FR_REQUIRE(nc < INT32_MAX && first + nc < INT32_MAX, "too many split chunks");
      for (int64_t k = 0; k < nc; ++k) {
        units[2 * nu] = (int32_t)r;
        units[2 * nu + 1] = (int32_t)k;
        ++nu;
      }
      split_rows[3 * ns] = (int32_t)r;
      split_rows[3 * ns + 1] = (int32_t)first;
      split_rows[3 * ns + 2] = (int32_t)nc;
      first += nc;
      ++ns;
    }
  }
  *n_units = nu;
  *n_split = ns;
  return FR_OK;
}

namespace {

Tab host_tab(const fr_tab* t) {
  if (t == nullptr || t->lo == nullptr) return Tab{nullptr, 0, nullptr, 0};
  return Tab{t->lo, t->ld_lo, t->hi, t->ld_hi};
}

bool tab_ok(const fr_tab* t, int d) {
  if (t == nullptr || t->lo == nullptr) return true;
  if (!(t->ld_lo >= d && t->ld_lo % 4 == 0 && fr::aligned16(t->lo))) return false;
  return t->hi == nullptr || (t->ld_hi >= d && t->ld_hi % 4 == 0 && fr::aligned16(t->hi));
}

bool tab_touches(const fr_tab* t, const void* p) {
  return t != nullptr && p != nullptr && (t->lo == p || t->hi == p);
}

int spmm_impl(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
              const fr_spmm_plan* plan, int64_t split, const fr_tab* X, int d, const fr_tab* Y1,
              const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1, const fr_tab* A2, float beta2,
              const uint8_t* col_mask, const fr_rowlist* rows, const uint8_t* a1_gate, void* d_workspace,
              int64_t workspace_bytes, void* stream, const char* who, int64_t row_lo = 0,
              int64_t row_hi = -1) {
  FR_REQUIRE(plan != nullptr, "plan is null");
  FR_REQUIRE(d > 0 && d % 4 == 0 && d <= 1024, "d must be a positive multiple of 4, <= 1024");
  FR_REQUIRE(n_rows >= 0, "n_rows < 0");
  if (n_rows == 0) return FR_OK;
  FR_REQUIRE(d_rowptr && X && X->lo, "rowptr/X null");
  FR_REQUIRE((Y1 && Y1->lo) || (Y2 && Y2->lo), "no output requested");
  FR_REQUIRE(plan->n_units == 0 || (plan->d_units && d_col && d_val), "plan/col/val null");
  FR_REQUIRE(plan->n_split == 0 || plan->d_split_rows, "split_rows null");
  FR_REQUIRE(plan->chunk > 0, "plan chunk must be > 0");
  FR_REQUIRE(tab_ok(X, d), "X must be 16-B aligned, ld % 4 == 0, ld >= d");
  FR_REQUIRE(tab_ok(Y1, d) && tab_ok(Y2, d) && tab_ok(A1, d) && tab_ok(A2, d), "bad Y1/Y2/A1/A2 table");
  FR_REQUIRE(split >= 0, "split < 0");
  if (row_hi < 0) row_hi = n_rows;
  FR_REQUIRE(row_lo >= 0 && row_lo <= row_hi && row_hi <= n_rows, "row range out of [0, n_rows]");
  FR_REQUIRE(rows == nullptr || (row_lo == 0 && row_hi == n_rows), "a row list takes no row range");
  for (const fr_tab* y : {Y1, Y2})
    FR_REQUIRE(!(y && (tab_touches(y, X->lo) || tab_touches(y, X->hi))), "outputs must not alias X");
  const int64_t need = fr_spmm_workspace(plan, d);
  FR_REQUIRE(rows != nullptr || plan->n_split == 0 ||
             (d_workspace && workspace_bytes >= need && fr::aligned16(d_workspace)),
             "workspace too small (need " + std::to_string(need) + " bytes)");
  Epi ep{host_tab(Y1), host_tab(Y2), alpha, host_tab(A1), beta1, host_tab(A2), beta2,
         split, a1_gate};
  XSrc xs{reinterpret_cast<const float4*>(X->lo), X->ld_lo >> 2, reinterpret_cast<const float4*>(X->hi),
          X->hi ? (X->ld_hi >> 2) : 0, X->hi ? split : INT64_MAX, col_mask};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float4* partial = reinterpret_cast<float4*>(d_workspace);
  const int d4 = d / 4;
  hipError_t e = hipSuccess;
  if (rows != nullptr) {
    FR_REQUIRE(d4 == 16, "row-list mode supports d = 64");
    FR_REQUIRE(col_mask == nullptr, "row-list mode takes no column mask");
    RowList rl{};
    int64_t total = 0;
    for (int k = 0; k < 3; ++k) {
      FR_REQUIRE(rows->n[k] >= 0 && (rows->n[k] == 0 || rows->ids[k]), "bad row segment");
      rl.ids[k] = rows->ids[k];
      rl.n[k] = rows->n[k];
      rl.off[k] = rows->off[k];
      total += rows->n[k];
    }
    if (total == 0) return FR_OK;
    if (xs.hi) {
      hipLaunchKernelGGL((spmm_rows_kernel<16, true>), dim3((unsigned)total), dim3(kRowThreads), 0, s, d_rowptr,
                         d_col, d_val, rl, xs, d4, ep);
    } else {
      hipLaunchKernelGGL((spmm_rows_kernel<16, false>), dim3((unsigned)total), dim3(kRowThreads), 0, s, d_rowptr,
                         d_col, d_val, rl, xs, d4, ep);
    }
    e = hipGetLastError();
  } else if (d4 >= 64) {
    e = launch_spmm<64>(d_rowptr, d_col, d_val, n_rows, plan, xs, d, ep, partial, s, row_lo, row_hi);
  } else if (d4 >= 32) {
    e = (d4 == 32) ? launch_spmm<32>(d_rowptr, d_col, d_val, n_rows, plan, xs, d, ep, partial, s, row_lo, row_hi)
                   : launch_spmm<16>(d_rowptr, d_col, d_val, n_rows, plan, xs, d, ep, partial, s, row_lo, row_hi);
  } else if (d4 >= 16) {
    e = launch_spmm<16>(d_rowptr, d_col, d_val, n_rows, plan, xs, d, ep, partial, s, row_lo, row_hi);
  } else if (d4 >= 8) {
    e = launch_spmm<8>(d_rowptr, d_col, d_val, n_rows, plan, xs, d, ep, partial, s, row_lo, row_hi);
  } else if (d4 >= 4) {
    e = launch_spmm<4>(d_rowptr, d_col, d_val, n_rows, plan, xs, d, ep, partial, s, row_lo, row_hi);
  } else {
    e = launch_spmm<1>(d_rowptr, d_col, d_val, n_rows, plan, xs, d, ep, partial, s, row_lo, row_hi);
  }
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string(who) + ": " + hipGetErrorString(e));
  return FR_OK;
}

}  // namespace

extern "C" int fr_spmm_csr(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                           int64_t n_rows, const fr_spmm_plan* plan, const float* d_X, int64_t ldx,
                           int d, float* d_Y1, int64_t ldy1, float* d_Y2, int64_t ldy2,
                           float alpha, const float* d_A1, int64_t lda1, float beta1,
                           const float* d_A2, int64_t lda2, float beta2, void* d_workspace,
                           int64_t workspace_bytes, void* stream) {
  const fr_tab X{d_X, ldx, nullptr, 0}, Y1{d_Y1, ldy1, nullptr, 0}, Y2{d_Y2, ldy2, nullptr, 0};
  const fr_tab A1{d_A1, lda1, nullptr, 0}, A2{d_A2, lda2, nullptr, 0};
  return spmm_impl(d_rowptr, d_col, d_val, n_rows, plan, 0, &X, d, &Y1, &Y2, alpha, &A1, beta1, &A2, beta2,
                   nullptr, nullptr, nullptr, d_workspace, workspace_bytes, stream, "fr_spmm_csr");
}

extern "C" int fr_spmm_csr_ex(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                              const fr_spmm_plan* plan, int64_t split, const fr_tab* X, int d, const fr_tab* Y1,
                              const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1, const fr_tab* A2,
                              float beta2, const uint8_t* d_col_mask, const fr_rowlist* rows,
                              const uint8_t* d_a1_gate, void* d_workspace, int64_t workspace_bytes, void* stream) {
  return spmm_impl(d_rowptr, d_col, d_val, n_rows, plan, split, X, d, Y1, Y2, alpha, A1, beta1, A2, beta2,
                   d_col_mask, rows, d_a1_gate, d_workspace, workspace_bytes, stream, "fr_spmm_csr_ex");
}

extern "C" int fr_spmm_csr_range(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                                 const fr_spmm_plan* plan, int64_t split, const fr_tab* X, int d, const fr_tab* Y1,
                                 const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1, const fr_tab* A2,
                                 float beta2, int64_t row_lo, int64_t row_hi, void* d_workspace,
                                 int64_t workspace_bytes, void* stream) {
  return spmm_impl(d_rowptr, d_col, d_val, n_rows, plan, split, X, d, Y1, Y2, alpha, A1, beta1, A2, beta2, nullptr,
                   nullptr, nullptr, d_workspace, workspace_bytes, stream, "fr_spmm_csr_range", row_lo, row_hi);
}

extern "C" int fr_rows_mark(uint8_t* d_mask, const fr_rowlist* rows, uint8_t value, void* stream) {
  return fr_rows_mark_zero(d_mask, rows, value, nullptr, 0, 0, nullptr, stream);
}

extern "C" int fr_rows_mark_zero(uint8_t* d_mask, const fr_rowlist* rows, uint8_t value, float* d_Z, int64_t ldz, int d,
                                 uint32_t* d_bits, void* stream) {
  FR_REQUIRE(d_mask != nullptr && rows != nullptr, "null argument");
  FR_REQUIRE(!d_Z || (d > 0 && d % 4 == 0 && ldz >= d && ldz % 4 == 0 && fr::aligned16(d_Z)),
             "Z must be 16-B aligned with d % 4 == 0 and ld >= d");
  RowList rl{};
  int64_t total = 0;
  for (int k = 0; k < 3; ++k) {
    FR_REQUIRE(rows->n[k] >= 0 && (rows->n[k] == 0 || rows->ids[k]), "bad row segment");
    rl.ids[k] = rows->ids[k];
    rl.n[k] = rows->n[k];
    rl.off[k] = rows->off[k];
    total += rows->n[k];
  }
  if (total == 0) return FR_OK;
  const int64_t work = total * (d_Z ? 16 : 1);
  const int64_t blocks = std::min<int64_t>(fr::ceil_div(work, (int64_t)256), (int64_t)fr::kNumCU * 4);
  hipLaunchKernelGGL(rows_mark_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     d_mask, rl, total, value, reinterpret_cast<float4*>(d_Z), ldz / 4, d / 4, d_bits);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

// ---------------------------------------------------------------------------------------------
// Scatter form of the sparse upstream (fr_spmm_scatter_upstream), for a SYMMETRIC adjacency:
// Y2 = alpha A X + beta1 gate(X) with X non-zero only at the listed rows.  Since A[c][r] = A[r][c],
// row r's contribution to every output row c is on r's own CSR row, so the work is proportional to
// the listed rows' degrees instead of a scan of every edge:
//   1. every row of Y2 = beta1 X[r] where mask[r] != 0, else 0 (the dense write the output needs);
//   2. one wave per listed occurrence; the first occurrence of a row claims it by clearing its bit
//      in the bitmask, then adds alpha A[r][c] X[r] to Y2[c] for each edge of row r, lane = column
//      (one 256-B float-atomic wave instruction per edge).
// Run-to-run variable summation order (float atomics): the non-deterministic mode's UI backward.
__global__ __launch_bounds__(256) void scatter_init_kernel(int64_t n_rows, const uint8_t* __restrict__ mask,
                                                           const float4* __restrict__ X, int64_t ldx4, Tab Y,
                                                           int64_t split, float beta1) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n_rows * 16; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i >> 4;
    const int q = (int)(i & 15);
    const float4 v = mask[r] ? f4_scale(beta1, X[r * ldx4 + q]) : make_float4(0.f, 0.f, 0.f, 0.f);
    reinterpret_cast<float4*>(const_cast<float*>(tab_row(Y, r, split)))[q] = v;
  }
}

__global__ __launch_bounds__(256) void scatter_edges_kernel(const int64_t* __restrict__ rowptr,
                                                            const int32_t* __restrict__ col,
                                                            const float* __restrict__ val, RowList rl, int64_t total,
                                                            uint32_t* __restrict__ bits, const float* __restrict__ X,
                                                            int64_t ldx, Tab Y, int64_t split, float alpha) {
  const int lane = threadIdx.x & 63;
  const int64_t idx0 = (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if (idx0 >= total) return;
  int64_t idx = idx0;
  int seg = 0;
  while (idx >= rl.n[seg]) idx -= rl.n[seg++];
  if (rl.ids[seg][idx] < 0) return;
  const int64_t row = rl.ids[seg][idx] + rl.off[seg];
  uint32_t old = 0;
  if (lane == 0) old = atomicAnd(bits + (row >> 5), ~(1u << (row & 31)));
  old = __builtin_amdgcn_readfirstlane(old);
  if (!((old >> (row & 31)) & 1u)) return;  // an earlier occurrence owns the row
  const float x = alpha * X[row * ldx + lane];
  const int64_t rs = rowptr[row], re = rowptr[row + 1];
  for (int64_t e = rs; e < re; e += 4) {
    int c[4];
    float v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c[k] = e + k < re ? col[e + k] : -1;
      v[k] = e + k < re ? val[e + k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (c[k] >= 0) atomicAdd(const_cast<float*>(tab_row(Y, c[k], split)) + lane, v[k] * x);
  }
}

extern "C" int fr_spmm_scatter_upstream(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                        int64_t n_rows, const uint8_t* d_mask, uint32_t* d_bits,
                                        const fr_rowlist* rows, const float* d_X, int64_t ldx, int64_t split,
                                        const fr_tab* Y2, float alpha, float beta1, void* stream) {
  FR_REQUIRE(n_rows >= 0 && n_rows < (int64_t)INT32_MAX, "n_rows out of range");
  if (n_rows == 0) return FR_OK;
  FR_REQUIRE(d_rowptr && d_col && d_val && d_mask && d_bits && rows && d_X && Y2 && Y2->lo, "null operand");
  FR_REQUIRE(ldx >= 64 && ldx % 4 == 0 && fr::aligned16(d_X) && tab_ok(Y2, 64),
             "X / Y2 must be 16-B aligned fp32 [*, 64] tables");
  FR_REQUIRE(!(tab_touches(Y2, d_X)), "Y2 must not alias X");
  RowList rl{};
  int64_t total = 0;
  for (int k = 0; k < 3; ++k) {
    FR_REQUIRE(rows->n[k] >= 0 && (rows->n[k] == 0 || rows->ids[k]), "bad row segment");
    rl.ids[k] = rows->ids[k];
    rl.n[k] = rows->n[k];
    rl.off[k] = rows->off[k];
    total += rows->n[k];
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const Tab Y = host_tab(Y2);
  const int64_t blocks = std::min<int64_t>(fr::ceil_div(n_rows * 16, (int64_t)256), (int64_t)fr::kNumCU * 8);
  hipLaunchKernelGGL(scatter_init_kernel, dim3((unsigned)blocks), dim3(256), 0, s, n_rows, d_mask,
                     reinterpret_cast<const float4*>(d_X), ldx / 4, Y, split, beta1);
  FR_LAUNCH_CHECK();
  if (total == 0) return FR_OK;
  hipLaunchKernelGGL(scatter_edges_kernel, dim3((unsigned)fr::ceil_div(total, (int64_t)4)), dim3(256), 0, s,
                     d_rowptr, d_col, d_val, rl, total, d_bits, d_X, ldx, Y, split, alpha);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

// the rows split into chunks by a block plan: Y2[r] = beta1 * A1[r] (A1 read where r is marked, or
// always for a rectangular slice), else 0 -- the term the chunks then add onto
__global__ __launch_bounds__(256) void sparse_split_init_kernel(const int64_t* __restrict__ rows, int64_t n,
                                                                const uint32_t* __restrict__ bits, bool ungated,
                                                                Epi ep) {
  const int64_t i = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int q = threadIdx.x & 15;
  if (i >= n) return;
  const int64_t r = rows[i];
  float4 o = make_float4(0.f, 0.f, 0.f, 0.f);
  if (ep.A1.lo && (ungated || ((bits[r >> 5] >> (r & 31)) & 1u)))
    o = f4_scale(ep.beta1, reinterpret_cast<const float4*>(tab_row(ep.A1, r, ep.split))[q]);
  reinterpret_cast<float4*>(const_cast<float*>(tab_row(ep.Y2, r, ep.split)))[q] = o;
}

static hipError_t sparse_blocks_launch(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                       int64_t n_rows, const uint32_t* d_bits, int nwords, const float* d_X,
                                       int64_t ldx, const Epi& ep, bool ungated, const int64_t* d_blocks,
                                       int64_t n_blocks, const int64_t* d_split_rows, int64_t n_split_rows,
                                       hipStream_t s, float* d_zero = nullptr, int64_t zero_floats = 0) {
  if (n_split_rows > 0)
    hipLaunchKernelGGL(sparse_split_init_kernel, dim3((unsigned)fr::ceil_div(n_split_rows, (int64_t)16)), dim3(256),
                       0, s, d_split_rows, n_split_rows, d_bits, ungated, ep);
  if (ungated)
    hipLaunchKernelGGL((spmm_sparse_kernel<true, true>), dim3((unsigned)n_blocks), dim3(256), 0, s, d_rowptr, d_col,
                       d_val, n_rows, d_bits, nwords, reinterpret_cast<const float4*>(d_X), ldx / 4, ep, d_blocks,
                       reinterpret_cast<float4*>(d_zero), zero_floats / 4);
  else
    hipLaunchKernelGGL((spmm_sparse_kernel<true, false>), dim3((unsigned)n_blocks), dim3(256), 0, s, d_rowptr, d_col,
                       d_val, n_rows, d_bits, nwords, reinterpret_cast<const float4*>(d_X), ldx / 4, ep, d_blocks,
                       reinterpret_cast<float4*>(d_zero), zero_floats / 4);
  return hipGetLastError();
}

static int sparse_zero_check(const float* d_zero, int64_t zero_floats) {
  FR_REQUIRE(zero_floats >= 0 && zero_floats % 4 == 0 && (zero_floats == 0 || (d_zero && fr::aligned16(d_zero))),
             "zero region: 16-B aligned, a multiple of 4 floats");
  return FR_OK;
}

static int sparse_upstream_blocks_impl(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                       int64_t n_rows, int64_t n_cols, int ungated, const uint32_t* d_bits,
                                       const float* d_X, int64_t ldx, int64_t split, const fr_tab* Y2, float alpha,
                                       const fr_tab* A1, float beta1, const int64_t* d_blocks, int64_t n_blocks,
                                       const int64_t* d_split_rows, int64_t n_split_rows, float* d_zero,
                                       int64_t zero_floats, void* stream);

extern "C" int fr_spmm_sparse_upstream_blocks(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                              int64_t n_rows, int64_t n_cols, int ungated, const uint32_t* d_bits,
                                              const float* d_X, int64_t ldx, int64_t split, const fr_tab* Y2,
                                              float alpha, const fr_tab* A1, float beta1, const int64_t* d_blocks,
                                              int64_t n_blocks, const int64_t* d_split_rows, int64_t n_split_rows,
                                              void* stream) {
  return sparse_upstream_blocks_impl(d_rowptr, d_col, d_val, n_rows, n_cols, ungated, d_bits, d_X, ldx, split, Y2,
                                     alpha, A1, beta1, d_blocks, n_blocks, d_split_rows, n_split_rows, nullptr, 0,
                                     stream);
}

extern "C" int fr_spmm_sparse_upstream_blocks_zero(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                                   int64_t n_rows, int64_t n_cols, int ungated, const uint32_t* d_bits,
                                                   const float* d_X, int64_t ldx, int64_t split, const fr_tab* Y2,
                                                   float alpha, const fr_tab* A1, float beta1, const int64_t* d_blocks,
                                                   int64_t n_blocks, const int64_t* d_split_rows, int64_t n_split_rows,
                                                   float* d_zero, int64_t zero_floats, void* stream) {
  return sparse_upstream_blocks_impl(d_rowptr, d_col, d_val, n_rows, n_cols, ungated, d_bits, d_X, ldx, split, Y2,
                                     alpha, A1, beta1, d_blocks, n_blocks, d_split_rows, n_split_rows, d_zero,
                                     zero_floats, stream);
}

static int sparse_upstream_blocks_impl(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                       int64_t n_rows, int64_t n_cols, int ungated, const uint32_t* d_bits,
                                       const float* d_X, int64_t ldx, int64_t split, const fr_tab* Y2, float alpha,
                                       const fr_tab* A1, float beta1, const int64_t* d_blocks, int64_t n_blocks,
                                       const int64_t* d_split_rows, int64_t n_split_rows, float* d_zero,
                                       int64_t zero_floats, void* stream) {
  if (int rc = sparse_zero_check(d_zero, zero_floats)) return rc;
  FR_REQUIRE(n_rows >= 0 && n_rows < (int64_t)INT32_MAX && n_cols >= 0 && n_cols < (int64_t)INT32_MAX,
             "n_rows / n_cols out of range");
  if (n_rows == 0) return FR_OK;
  FR_REQUIRE(d_rowptr && d_col && d_val && d_bits && d_X && Y2 && Y2->lo, "null operand");
  FR_REQUIRE(d_blocks && n_blocks > 0 && n_blocks < (int64_t)INT32_MAX, "block plan required");
  FR_REQUIRE(n_split_rows == 0 || d_split_rows, "split-row list missing");
  FR_REQUIRE(ungated || n_cols == n_rows, "the gated form needs a square adjacency");
  FR_REQUIRE(fr::aligned16(d_bits), "bits must be 16-B aligned");
  FR_REQUIRE(ldx >= 64 && ldx % 4 == 0 && fr::aligned16(d_X) && tab_ok(Y2, 64) && tab_ok(A1, 64),
             "X / Y2 / A1 must be 16-B aligned fp32 [*, 64] tables");
  FR_REQUIRE(!(tab_touches(Y2, d_X)), "Y2 must not alias X");
  Epi ep{Tab{nullptr, 0, nullptr, 0}, host_tab(Y2), alpha, host_tab(A1), beta1, Tab{nullptr, 0, nullptr, 0}, 0.f,
         ungated ? 0 : split, nullptr};
  const int nwords = (int)fr::ceil_div(std::max<int64_t>(n_cols, 1), 32);
  const hipError_t e = sparse_blocks_launch(d_rowptr, d_col, d_val, n_rows, d_bits, nwords, d_X, ldx, ep, ungated != 0,
                                            d_blocks, n_blocks, d_split_rows, n_split_rows,
                                            reinterpret_cast<hipStream_t>(stream), d_zero, zero_floats);
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_spmm_sparse_upstream_blocks: ") + hipGetErrorString(e));
  return FR_OK;
}

extern "C" int fr_spmm_sparse_block_rows(void) { return kSpRows; }

extern "C" int fr_spmm_plan_status(int clear) {
  unsigned int v = 0;
  FR_HIP_CHECK(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_sparse_plan_status), sizeof(v)));
  if (clear && v) {
    const unsigned int z = 0;
    FR_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_sparse_plan_status), &z, sizeof(z)));
  }
  return (int)v;
}

extern "C" int fr_spmm_sparse_upstream_rect(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                            int64_t n_rows, int64_t n_cols, const uint32_t* d_bits, const float* d_X,
                                            int64_t ldx, const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1,
                                            void* stream) {
  FR_REQUIRE(n_rows >= 0 && n_rows < (int64_t)INT32_MAX && n_cols >= 0 && n_cols < (int64_t)INT32_MAX,
             "n_rows / n_cols out of range");
  if (n_rows == 0) return FR_OK;
  FR_REQUIRE(d_rowptr && d_col && d_val && d_bits && d_X && Y2 && Y2->lo, "null operand");
  FR_REQUIRE(fr::aligned16(d_bits), "bits must be 16-B aligned");
  FR_REQUIRE(ldx >= 64 && ldx % 4 == 0 && fr::aligned16(d_X) && tab_ok(Y2, 64) && tab_ok(A1, 64),
             "X / Y2 / A1 must be 16-B aligned fp32 [*, 64] tables");
  FR_REQUIRE(!(tab_touches(Y2, d_X)), "Y2 must not alias X");
  Epi ep{Tab{nullptr, 0, nullptr, 0}, host_tab(Y2), alpha, host_tab(A1), beta1, Tab{nullptr, 0, nullptr, 0}, 0.f,
         0, nullptr};
  const int nwords = (int)fr::ceil_div(std::max<int64_t>(n_cols, 1), 32);
  hipLaunchKernelGGL((spmm_sparse_kernel<true, true>), dim3((unsigned)fr::ceil_div(n_rows, kSpRows)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), d_rowptr, d_col, d_val, n_rows, d_bits, nwords,
                     reinterpret_cast<const float4*>(d_X), ldx / 4, ep);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_spmm_sparse_upstream_zero(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                            int64_t n_rows, const uint32_t* d_bits, const float* d_X, int64_t ldx,
                                            int64_t split, const fr_tab* Y2, float alpha, const fr_tab* A1,
                                            float beta1, float* d_zero, int64_t zero_floats, void* stream);

extern "C" int fr_spmm_sparse_upstream(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                       int64_t n_rows, const uint32_t* d_bits, const float* d_X, int64_t ldx,
                                       int64_t split, const fr_tab* Y2, float alpha, const fr_tab* A1, float beta1,
                                       void* stream) {
  return fr_spmm_sparse_upstream_zero(d_rowptr, d_col, d_val, n_rows, d_bits, d_X, ldx, split, Y2, alpha, A1, beta1,
                                      nullptr, 0, stream);
}

extern "C" int fr_spmm_sparse_upstream_zero(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                            int64_t n_rows, const uint32_t* d_bits, const float* d_X, int64_t ldx,
                                            int64_t split, const fr_tab* Y2, float alpha, const fr_tab* A1,
                                            float beta1, float* d_zero, int64_t zero_floats, void* stream) {
  if (int rc = sparse_zero_check(d_zero, zero_floats)) return rc;
  FR_REQUIRE(n_rows >= 0 && n_rows < (int64_t)INT32_MAX, "n_rows out of range");
  if (n_rows == 0) return FR_OK;
  FR_REQUIRE(d_rowptr && d_col && d_val && d_bits && d_X && Y2 && Y2->lo, "null operand");
  FR_REQUIRE(fr::aligned16(d_bits), "bits must be 16-B aligned");
  FR_REQUIRE(ldx >= 64 && ldx % 4 == 0 && fr::aligned16(d_X) && tab_ok(Y2, 64) && tab_ok(A1, 64),
             "X / Y2 / A1 must be 16-B aligned fp32 [*, 64] tables");
  FR_REQUIRE(!(tab_touches(Y2, d_X)), "Y2 must not alias X");
  Epi ep{Tab{nullptr, 0, nullptr, 0}, host_tab(Y2), alpha, host_tab(A1), beta1, Tab{nullptr, 0, nullptr, 0}, 0.f,
         split, nullptr};
  const int nwords = (int)fr::ceil_div(n_rows, 32);
  const dim3 grid((unsigned)fr::ceil_div(n_rows, kSpRows));
  // bitmask staged in LDS only while it is small next to a block's edge range: each of the
  // ceil(n / 64) blocks would copy all of it (HealthRec's UI graph: 14.3 KB per block against ~6 KB
  // of col / val; the L1-resident global lookups are 4.4 us faster per launch there)
  float4* z4 = reinterpret_cast<float4*>(d_zero);
  if (nwords <= kSpStageWords)
    hipLaunchKernelGGL(spmm_sparse_kernel<false>, grid, dim3(256), (size_t)nwords * sizeof(uint32_t),
                       reinterpret_cast<hipStream_t>(stream), d_rowptr, d_col, d_val, n_rows, d_bits, nwords,
                       reinterpret_cast<const float4*>(d_X), ldx / 4, ep, nullptr, z4, zero_floats / 4);
  else
    hipLaunchKernelGGL(spmm_sparse_kernel<true>, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), d_rowptr,
                       d_col, d_val, n_rows, d_bits, nwords, reinterpret_cast<const float4*>(d_X), ldx / 4, ep, nullptr,
                       z4, zero_floats / 4);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_rows_frontier(const int64_t* d_rowptr, const int32_t* d_col, int64_t U, int64_t I,
                                const int64_t* d_u, const int64_t* d_p, const int64_t* d_n, int64_t B, uint8_t* d_mark,
                                int32_t* d_list, int32_t* d_count, void* stream) {
  FR_REQUIRE(U >= 0 && I > 0 && I < (int64_t)INT32_MAX && B >= 1, "bad sizes");
  FR_REQUIRE(d_rowptr && d_col && d_u && d_p && d_n && d_mark && d_list && d_count, "null argument");
  FR_REQUIRE((reinterpret_cast<uintptr_t>(d_mark) & 3u) == 0, "mark must be 4-B aligned");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(frontier_mark_kernel, dim3((unsigned)fr::ceil_div(B, (int64_t)4)), dim3(256), 0, s, d_rowptr,
                     d_col, U, I, d_u, d_p, d_n, B, d_mark, d_count);
  FR_LAUNCH_CHECK();
  hipLaunchKernelGGL(frontier_compact_kernel, dim3((unsigned)fr::ceil_div(I, (int64_t)kCompactItems)), dim3(256), 0, s, d_mark,
                     I, d_list, d_count);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_spmm_csr_list(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val, int64_t n_rows,
                                int64_t split, const fr_tab* X, const fr_tab* Y1, const fr_tab* Y2, float alpha,
                                const fr_tab* A1, float beta1, const fr_tab* A2, float beta2, const int32_t* d_list,
                                const int32_t* d_count, int64_t max_rows, void* stream) {
  FR_REQUIRE(n_rows >= 0 && max_rows >= 0 && max_rows <= n_rows, "bad sizes");
  if (max_rows == 0) return FR_OK;
  FR_REQUIRE(d_rowptr && d_col && d_val && X && X->lo && d_list && d_count, "null argument");
  FR_REQUIRE((Y1 && Y1->lo) || (Y2 && Y2->lo), "no output requested");
  FR_REQUIRE(tab_ok(X, 64) && tab_ok(Y1, 64) && tab_ok(Y2, 64) && tab_ok(A1, 64) && tab_ok(A2, 64),
             "tables must be 16-B aligned fp32 [*, 64] (d = 64)");
  for (const fr_tab* y : {Y1, Y2})
    FR_REQUIRE(!(y && (tab_touches(y, X->lo) || tab_touches(y, X->hi))), "outputs must not alias X");
  Epi ep{host_tab(Y1), host_tab(Y2), alpha, host_tab(A1), beta1, host_tab(A2), beta2, split, nullptr};
  XSrc xs{reinterpret_cast<const float4*>(X->lo), X->ld_lo >> 2, reinterpret_cast<const float4*>(X->hi),
          X->hi ? (X->ld_hi >> 2) : 0, X->hi ? split : INT64_MAX, nullptr};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(max_rows, 16), (int64_t)fr::kNumCU * 8));
  if (xs.hi)
    hipLaunchKernelGGL(spmm_list16_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, d_rowptr, d_col, d_val,
                       d_list, d_count, xs, ep);
  else
    hipLaunchKernelGGL(spmm_list16_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, d_rowptr, d_col, d_val,
                       d_list, d_count, xs, ep);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_spmm_list_scatter(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                    int64_t n_rows, int64_t split, const int32_t* d_list, const int32_t* d_count,
                                    int64_t max_rows, const float* d_X, int64_t ldx, float* d_Y, int64_t ldy,
                                    float alpha, int zero_first, void* stream) {
  FR_REQUIRE(n_rows >= 0 && n_rows < (int64_t)INT32_MAX && split >= 0 && split <= n_rows && max_rows >= 0 &&
                 max_rows <= n_rows,
             "bad sizes");
  FR_REQUIRE(d_rowptr && d_col && d_val && d_list && d_count && d_X && d_Y, "null argument");
  FR_REQUIRE(ldx >= 64 && ldy >= 64, "X / Y must be fp32 [*, 64] tables");
  const float* y_end = d_Y + (n_rows - split) * ldy;
  FR_REQUIRE(!(d_X < y_end && d_Y < d_X + max_rows * ldx), "Y must not alias X");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (zero_first && n_rows > split) {
    if (ldy == 64) {
      FR_HIP_CHECK(hipMemsetAsync(d_Y, 0, (size_t)(n_rows - split) * 64 * sizeof(float), s));
    } else {
      FR_HIP_CHECK(hipMemset2DAsync(d_Y, (size_t)ldy * sizeof(float), 0, 64 * sizeof(float),
                                    (size_t)(n_rows - split), s));
    }
  }
  if (max_rows == 0) return FR_OK;
  const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(max_rows, 4), (int64_t)fr::kNumCU * 8));
  hipLaunchKernelGGL(list_scatter_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_rowptr, d_col, d_val, d_list,
                     d_count, split, d_X, ldx, d_Y, ldy, alpha);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
