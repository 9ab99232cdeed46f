// Embedding-table backward (row gather -> row scatter-add) for gfx950.
//
//   dW[r, :] = sum over positions i with idx[i] == r (r != padding_idx) of G[i, :]
//
// The reference's gathers ``ingr_all[ingredients]`` (cikm_model.py:230), ``ingre_embedding(...)``
// with padding_idx (cikm_model.py:67-68, 270-271) and the trainable feature tables
// ``image_embedding``/``text_embedding`` (cikm_model.py:83-87) all back-propagate through this.
// torch's sort/unique_by_key path costs ~10 launches per call; here:
//
// Batches of <= 4096 ids take a sort-free owner pass (emb_owner_scan/sum_kernel); larger ones:
//   1. histogram of rows + zero fill of the dense gradient (one grid-stride kernel; the wave's
//      most frequent candidate row -- the padding row of ingredient lists -- is aggregated with a
//      ballot so the hot counter sees one atomic per wave),
//   2. exclusive scan of the counts (one block) -> bucket starts, per-row fill cursors,
//   3. placement of positions into buckets,
//   4. ordering of each bucket by position: <= 32 entries with an in-register bitonic network,
//      larger buckets with an LDS bitmap over positions (popcount ranks; exact, no comparisons),
//   5. segmented sum over the position-ordered slots in fixed chunks of kChunk slots: segments
//      complete inside a chunk are written straight to dW, the (at most two) cut segments of a
//      chunk go to partial slots,
//   6. fix-up: each row cut by chunk boundaries is summed from its partials in chunk order.
//
// Every step is deterministic: the result depends only on (idx, G), never on scheduling.  No
// step's launch shape depends on device data, so the whole chain captures into a HIP graph.
#include "fr_common.h"

#include <algorithm>

namespace {

constexpr int kSmall = 32;    // buckets up to this size are ordered in registers by one thread
constexpr int kChunk = 16;    // sorted slots per segmented-sum chunk (one 16-slot batch)
constexpr int LPR = 16;       // lanes per group = one DPP row; each lane owns one float4 column
constexpr int GPB = 256 / LPR;
constexpr int64_t kMaxPositions = 1 << 18;  // LDS bitmap of step 4: n/32 words <= 32 KiB

// Status bits (cursor[R+1]): a step found device data inconsistent with the launch (an index out
// of range) and skipped the access instead of faulting.  Zero after every well-formed call.
enum : int { kBadScan = 1, kBadPlace = 2, kBadSmall = 4, kBadBig = 8, kBadSegsum = 16, kBadFixup = 32 };

struct EmbWS {
  int32_t* cursor;  // [R+2]: counts, then fill cursors; [R] = number of big buckets; [R+1] = status
  int32_t* start;   // [R+1]: bucket starts, start[R] = number of valid positions
  int32_t* sorted;  // [n]  : positions grouped by row, ascending inside a row
  int32_t* big;     // [n/(kSmall+1)+1]: rows whose bucket exceeds kSmall
  float4* pf;       // [nchunks*d4]: the chunk's first segment when it began in an earlier chunk
  float4* pl;       // [nchunks*d4]: the chunk's last segment when it continues past the chunk
  int32_t* nxt;     // [n]  : owner path: next position with the same row (-1: none)
  int32_t* own;     // [n]  : owner path: 1 when no earlier position has the row
};

inline int64_t r256(int64_t b) { return (b + 255) / 256 * 256; }

__host__ __device__ inline int64_t n_chunks(int64_t n) { return (n + kChunk - 1) / kChunk; }

inline EmbWS emb_ws(void* base, int64_t n, int64_t R, int d) {
  char* p = reinterpret_cast<char*>(base);
  auto take = [&](int64_t bytes) { char* r = p; p += r256(bytes); return r; };
  EmbWS w;
  w.cursor = reinterpret_cast<int32_t*>(take((R + 2) * 4));
  w.start = reinterpret_cast<int32_t*>(take((R + 1) * 4));
  w.sorted = reinterpret_cast<int32_t*>(take(std::max<int64_t>(n, 1) * 4));
  w.big = reinterpret_cast<int32_t*>(take((n / (kSmall + 1) + 1) * 4));
  w.pf = reinterpret_cast<float4*>(take(n_chunks(n) * (d / 4) * 16));
  w.pl = reinterpret_cast<float4*>(take(n_chunks(n) * (d / 4) * 16));
  w.nxt = reinterpret_cast<int32_t*>(take(std::max<int64_t>(n, 1) * 4));
  w.own = reinterpret_cast<int32_t*>(take(std::max<int64_t>(n, 1) * 4));
  return w;
}

inline int64_t emb_ws_bytes(int64_t n, int64_t R, int d) {
  return r256((R + 2) * 4) + r256((R + 1) * 4) + r256(std::max<int64_t>(n, 1) * 4) + r256((n / (kSmall + 1) + 1) * 4) +
         2 * r256(n_chunks(n) * (d / 4) * 16) + 2 * r256(std::max<int64_t>(n, 1) * 4);
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, __shfl_xor(v, off, 64));
  return v;
}

// row of position i, or -1 when i is out of range / the padding row / an invalid id
__device__ __forceinline__ int emb_key(const int64_t* idx, int64_t i, int64_t n, int64_t R, int64_t pad) {
  if (i >= n) return -1;
  const int64_t r = idx[i];
  return (r >= 0 && r < R && r != pad) ? (int)r : -1;
}

// 0. zero the counters (a kernel, not hipMemsetAsync: a captured memset node is not relied on to
//    be ordered before the histogram's atomics on graph replay)
__global__ __launch_bounds__(256) void emb_clear_kernel(int32_t* __restrict__ p, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = 0;
}

// 1. histogram + zero fill of dW
__global__ __launch_bounds__(256) void emb_hist_zero_kernel(const int64_t* __restrict__ idx, int64_t n,
                                                            int64_t R, int64_t pad, int32_t* __restrict__ cnt,
                                                            float4* __restrict__ out, int64_t ldo4, int d4) {
  const int lane = threadIdx.x & 63;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  // wave-uniform trip count (nth is a multiple of 64), so the ballots see every lane
  for (int64_t i0 = tid - lane; i0 < n; i0 += nth) {
    int key = emb_key(idx, i0 + lane, n, R, pad);
    const int m = wave_max(key);
    const uint64_t mask = __ballot(key == m && m >= 0);
    const int c = __popcll(mask);
    if (c > 1) {
      if (lane == __ffsll((unsigned long long)mask) - 1) atomicAdd(&cnt[m], c);
      if (key == m) key = -1;
    }
    if (key >= 0) atomicAdd(&cnt[key], 1);
  }
  const int64_t total4 = out ? R * d4 : 0;  // compact (row-gradient) mode: no dense table to clear
  for (int64_t e = tid; e < total4; e += nth) {
    const int64_t r = e / d4;
    out[r * ldo4 + (e - r * d4)] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// block-wide exclusive scan of one int per thread (1024 threads); returns the exclusive prefix,
// *total = block sum.  `sh` holds >= 16 ints.
__device__ __forceinline__ int block_excl_scan_1024(int v, int* sh, int* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) sh[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    int run = 0;
    for (int w = 0; w < 16; ++w) { const int t = sh[w]; sh[w] = run; run += t; }
    sh[16] = run;
  }
  __syncthreads();
  const int res = sh[wid] + inc - v;
  *total = sh[16];
  __syncthreads();
  return res;
}

// 2. scan counts -> start[], cursors; list big buckets.  One block; rows pass through LDS in
//    tiles of 8192 (coalesced global loads/stores, each thread scans 8 consecutive LDS entries).
constexpr int kScanTile = 8192;

__device__ __forceinline__ int scan_pad(int i) { return i + (i >> 5); }  // LDS bank-conflict padding

__global__ __launch_bounds__(1024) void emb_scan_kernel(int32_t* __restrict__ cursor, int64_t R,
                                                        int32_t* __restrict__ start, int32_t* __restrict__ big,
                                                        int64_t big_cap) {
  __shared__ int tile[kScanTile + kScanTile / 32];
  __shared__ int sh[17];
  const int t = threadIdx.x;
  int carry = 0;
  for (int64_t base = 0; base < R; base += kScanTile) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = j * 1024 + t;
      tile[scan_pad(i)] = (base + i < R) ? cursor[base + i] : 0;
    }
    __syncthreads();
    int c[8];
    int sum = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) { c[j] = tile[scan_pad(t * 8 + j)]; sum += c[j]; }
    int tot;
    int off = carry + block_excl_scan_1024(sum, sh, &tot);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      tile[scan_pad(t * 8 + j)] = off;
      const int64_t row = base + t * 8 + j;
      if (c[j] > kSmall && row < R) {
        const int b = atomicAdd(&cursor[R], 1);
        if (b < big_cap) big[b] = (int)row;
        else atomicOr(&cursor[R + 1], kBadScan);
      }
      off += c[j];
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = j * 1024 + t;
      if (base + i < R) {
        const int v = tile[scan_pad(i)];
        start[base + i] = v;
        cursor[base + i] = v;
      }
    }
    carry += tot;
    __syncthreads();
  }
  if (t == 0) start[R] = carry;
}

// Small batches (n <= kOwnerMax, e.g. 2B item ids into a 45k-row feature table): no sort.
//   scan: one thread per position (all ids staged in LDS) finds whether it owns its row (no earlier
//         position has it) and the next position with the same row;
//   sum:  one thread per (owning position, float4 column) adds the row's positions along that
//         chain, in ascending position order, and writes dW[r] (dense mode, zero-filled by the
//         previous launch) or the compact slot rows[i] with rmap[r] = i (row-gradient mode, the
//         form fr_adam_step_rows consumes; rmap was filled with -1 by the previous launch).
constexpr int kOwnerMax = 4096;

__global__ __launch_bounds__(256) void emb_rmap_fill_kernel(int32_t* __restrict__ rmap, int64_t R) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < R; i += (int64_t)gridDim.x * blockDim.x)
    rmap[i] = -1;
}

// Row-gradient mode for up to kOneBlock positions: the owner pass in ONE workgroup (replaces the
// rmap fill, status clear and owner scan launches of the owner path; emb_owner_sum_kernel then sums):
//   1. status = 0; rmap[0 .. R) = -1 (stores drained before the barrier, so the owners' later
//      rmap stores land after them);
//   2. keys (row << 12 | position; invalid rows and the padding row -> max) bitonic-sorted in LDS:
//      equal rows become runs in ascending position;
//   3. per sorted element: own[pos] = first of its run (then rmap[row] = pos), nxt[pos] = the next
//      position of the run or -1 -- the chains emb_owner_sum_kernel walks, as the owner scan builds.
constexpr int kOneBlock = 1024;  // one key per thread
constexpr int kOneThreads = 1024;

__device__ __forceinline__ uint64_t shfl_xor_u64(uint64_t v, int m) {
  const int lo = __shfl_xor((int)(uint32_t)v, m, 64), hi = __shfl_xor((int)(uint32_t)(v >> 32), m, 64);
  return ((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo;
}

__global__ __launch_bounds__(kOneThreads) void emb_owner_one_kernel(const int64_t* __restrict__ idx, int n, int64_t R,
                                                                    int64_t pad, int32_t* __restrict__ nxt,
                                                                    int32_t* __restrict__ own,
                                                                    int32_t* __restrict__ rmap,
                                                                    int32_t* __restrict__ status) {
  __shared__ uint64_t key[kOneBlock];
  const int t = threadIdx.x;
  if (t == 0) status[0] = 0;
  for (int64_t r = t; r < R; r += kOneThreads) rmap[r] = -1;
  int np2 = 1;
  while (np2 < n) np2 <<= 1;
  const int rk = emb_key(idx, t, n, R, pad);
  uint64_t v = (t < n && rk >= 0) ? (((uint64_t)rk << 12) | (uint64_t)t) : ~0ull;
  // bitonic sort, one key per thread: partner distances below 64 exchange in registers (lane
  // shuffles), the larger ones through LDS
  for (int k = 2; k <= np2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      uint64_t o;
      if (j >= 64) {  // block-uniform
        key[t] = v;
        __syncthreads();
        o = key[t ^ j];
        __syncthreads();
      } else {
        o = shfl_xor_u64(v, j);
      }
      const bool keep_min = ((t & j) == 0) == ((t & k) == 0);
      v = keep_min ? (o < v ? o : v) : (o > v ? o : v);
    }
  }
  key[t] = v;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the rmap fill has reached L2
  __syncthreads();
  if (t < n) {
    if (v != ~0ull) {  // invalid / padding positions sort last: no owner, no chain
      const int pos = (int)(v & 0xFFF);
      const bool first = t == 0 || (key[t - 1] >> 12) != (v >> 12);
      const bool more = t + 1 < n && key[t + 1] != ~0ull && (key[t + 1] >> 12) == (v >> 12);
      own[pos] = first ? 1 : 0;
      nxt[pos] = more ? (int32_t)(key[t + 1] & 0xFFF) : -1;
      if (first) rmap[v >> 12] = pos;
    }
    if (rk < 0) own[t] = 0;  // a position with an invalid row is never an owner
  }
}

// one wave per position: lanes compare 256 ids per step (4 x 64, ballots), stopping once an earlier
// duplicate and the next duplicate are both found
constexpr int kScanPerWave = 1;

__global__ __launch_bounds__(256) void emb_owner_scan_kernel(const int64_t* __restrict__ idx, int64_t n, int64_t R,
                                                             int64_t pad, int32_t* __restrict__ nxt,
                                                             int32_t* __restrict__ own, int32_t* __restrict__ rmap) {
  __shared__ int ids[kOwnerMax];
  for (int64_t i = threadIdx.x; i < n; i += 256) ids[i] = emb_key(idx, i, n, R, pad);
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int i0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * kScanPerWave;
  for (int i = i0; i < min<int64_t>(i0 + kScanPerWave, n); ++i) {  // wave-uniform
    const int r = ids[i];
    bool before = false;
    int next = -1;
    if (r >= 0) {
      for (int j0 = 0; j0 < n; j0 += 256) {
        int v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + 64 * u + lane;
          v[u] = j < n ? ids[j] : -1;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + 64 * u + lane;
          const bool m = v[u] == r;
          before |= __ballot(m && j < i) != 0ull;
          const uint64_t after = __ballot(m && j > i);
          if (next < 0 && after) next = j0 + 64 * u + __ffsll((unsigned long long)after) - 1;
        }
        if (before && next >= 0) break;
      }
    }
    if (lane == 0) {
      nxt[i] = next;
      own[i] = (r >= 0 && !before) ? 1 : 0;
      if (r >= 0 && !before && rmap) rmap[r] = i;
    }
  }
}

__global__ __launch_bounds__(256) void emb_owner_sum_kernel(const int64_t* __restrict__ idx, int64_t n,
                                                            const int32_t* __restrict__ nxt,
                                                            const int32_t* __restrict__ own,
                                                            const float4* __restrict__ G4, int64_t ldg4, int d4,
                                                            float4* __restrict__ out, int64_t ldo4, int compact) {
  const int64_t total = n * d4;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / d4;
    const int q = (int)(e - i * d4);
    if (!own[i]) continue;
    float4 acc = f4_add(make_float4(0.f, 0.f, 0.f, 0.f), G4[i * ldg4 + q]);
    for (int j = nxt[i]; j >= 0; j = nxt[j]) acc = f4_add(acc, G4[(int64_t)j * ldg4 + q]);
    out[(compact ? i : idx[i]) * ldo4 + q] = acc;
  }
}

// 3. placement (the wave's hot row takes one cursor atomic and ranks by lane)
__global__ __launch_bounds__(256) void emb_place_kernel(const int64_t* __restrict__ idx, int64_t n, int64_t R,
                                                        int64_t pad, int32_t* __restrict__ cursor,
                                                        int32_t* __restrict__ sorted) {
  const int lane = threadIdx.x & 63;
  const int64_t tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nth = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = tid - lane; i0 < n; i0 += nth) {
    const int64_t i = i0 + lane;
    int key = emb_key(idx, i, n, R, pad);
    const int m = wave_max(key);
    const uint64_t mask = __ballot(key == m && m >= 0);
    const int c = __popcll(mask);
    if (c > 1) {
      const int leader = __ffsll((unsigned long long)mask) - 1;
      int base = 0;
      if (lane == leader) base = atomicAdd(&cursor[m], c);
      base = __shfl(base, leader, 64);
      if (key == m) {
        const int slot = base + __popcll(mask & ((1ull << lane) - 1));
        if (slot >= 0 && slot < n) sorted[slot] = (int)i;
        else atomicOr(&cursor[R + 1], kBadPlace);
        key = -1;
      }
    }
    if (key >= 0) {
      const int slot = atomicAdd(&cursor[key], 1);
      if (slot >= 0 && slot < n) sorted[slot] = (int)i;
      else atomicOr(&cursor[R + 1], kBadPlace);
    }
  }
}

// 4a. small buckets: in-register bitonic network (fully unrolled, compile-time indices)
__global__ __launch_bounds__(256) void emb_sort_small_kernel(const int32_t* __restrict__ start, int64_t R,
                                                             int64_t n, int32_t* __restrict__ sorted,
                                                             int32_t* __restrict__ status) {
  for (int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x) {
    const int s = start[r], c = start[r + 1] - s;
    if (c < 2 || c > kSmall) continue;
    if (s < 0 || s + c > n) { atomicOr(status, kBadSmall); continue; }
    int v[kSmall];
#pragma unroll
    for (int j = 0; j < kSmall; ++j) v[j] = j < c ? sorted[s + j] : INT32_MAX;
#pragma unroll
    for (int k = 2; k <= kSmall; k <<= 1) {
#pragma unroll
      for (int j = k >> 1; j > 0; j >>= 1) {
#pragma unroll
        for (int i = 0; i < kSmall; ++i) {
          const int l = i ^ j;
          if (l > i) {
            const int a = v[i], b = v[l];
            const bool up = (i & k) == 0;
            if ((a > b) == up) { v[i] = b; v[l] = a; }
          }
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kSmall; ++j)
      if (j < c) sorted[s + j] = v[j];
  }
}

// 4b. big buckets: one block each; positions are distinct in [0, n), so an LDS bitmap over them
//     plus popcount prefix sums yields the ascending order directly.
__global__ __launch_bounds__(256) void emb_sort_big_kernel(int32_t* __restrict__ cursor_tail, int64_t n,
                                                           int64_t R, const int32_t* __restrict__ big,
                                                           const int32_t* __restrict__ start,
                                                           int32_t* __restrict__ sorted) {
  extern __shared__ uint32_t bm[];
  __shared__ int sh[5];
  if ((int)blockIdx.x >= cursor_tail[0]) return;  // block-uniform
  const int r = big[blockIdx.x];
  if (r < 0 || r >= R) { if (threadIdx.x == 0) atomicOr(&cursor_tail[1], kBadBig); return; }
  const int s = start[r], e = start[r + 1];
  if (s < 0 || e > n || s > e) { if (threadIdx.x == 0) atomicOr(&cursor_tail[1], kBadBig); return; }
  const int words = (int)((n + 31) / 32);
  for (int w = threadIdx.x; w < words; w += 256) bm[w] = 0u;
  __syncthreads();
  for (int k = s + threadIdx.x; k < e; k += 256) {
    const int p = sorted[k];
    if (p >= 0 && p < n) atomicOr(&bm[p >> 5], 1u << (p & 31));
    else atomicOr(&cursor_tail[1], kBadBig);
  }
  __syncthreads();
  const int per = (words + 255) / 256;
  const int w0 = threadIdx.x * per, w1 = min(words, w0 + per);
  int local = 0;
  for (int w = w0; w < w1; ++w) local += __popc(bm[w]);
  // 256-thread exclusive scan (4 waves)
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int inc = local;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const int t = __shfl_up(inc, off, 64);
    if (lane >= off) inc += t;
  }
  if (lane == 63) sh[wid] = inc;
  __syncthreads();
  int off = inc - local;
  for (int w = 0; w < wid; ++w) off += sh[w];
  for (int w = w0; w < w1; ++w) {
    uint32_t bits = bm[w];
    while (bits) {
      const int b = __ffs(bits) - 1;
      if (s + off < e) sorted[s + off] = w * 32 + b;
      else atomicOr(&cursor_tail[1], kBadBig);
      ++off;
      bits &= bits - 1u;
    }
  }
}

template <int K>
__device__ __forceinline__ int row_bcast(int v) {
  return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xf, 0xf, false);  // row_newbcast:K
}

// 5. segmented sum over the position-ordered slots, one 16-lane group per (chunk, 64-column slice)
__global__ __launch_bounds__(256) void emb_segsum_kernel(const int64_t* __restrict__ idx,
                                                         const int32_t* __restrict__ sorted,
                                                         const int32_t* __restrict__ start, int64_t R,
                                                         int64_t nchunks, const float4* __restrict__ G4,
                                                         int64_t ldg4, int d4, float4* __restrict__ out,
                                                         int64_t ldo4, float4* __restrict__ pf,
                                                         float4* __restrict__ pl, int64_t n,
                                                         int32_t* __restrict__ status, int32_t* __restrict__ rmap) {
  const int lig = threadIdx.x % LPR;
  const int64_t c = (int64_t)blockIdx.x * GPB + threadIdx.x / LPR;
  const int q = blockIdx.y * LPR + lig;
  const bool qok = q < d4;
  int total = start[R];
  if (total < 0 || total > n) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) atomicOr(status, kBadSegsum);
    total = total < 0 ? 0 : (int)n;
  }
  const int64_t k0 = c * kChunk;
  if (c >= nchunks || k0 >= total) return;  // group-uniform
  const int64_t k1 = min((int64_t)total, k0 + kChunk);
  const int64_t cend = k0 + kChunk;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  int cur = -1, cs = 0, ce = 0;
  auto flush = [&]() {
    if (cs >= k0 && ce <= cend && rmap && lig == 0 && blockIdx.y == 0) rmap[cur] = sorted[cs];
    if (!qok) return;
    // row-gradient mode: the row's slot is its first (smallest) position, sorted[bucket start]
    if (cs >= k0 && ce <= cend) out[(rmap ? (int64_t)sorted[cs] : (int64_t)cur) * ldo4 + q] = acc;
    else if (cs < k0) pf[c * d4 + q] = acc;
    else pl[c * d4 + q] = acc;
  };
  for (int64_t kb = k0; kb < k1; kb += LPR) {
    // each lane fetches one slot's (position, row, bucket bounds); DPP broadcasts them
    const int64_t my = kb + lig;
    int p = my < k1 ? sorted[my] : -1;
    if (p >= n) { atomicOr(status, kBadSegsum); p = -1; }
    int r = p >= 0 ? (int)idx[p] : -1;
    if (r >= R) { atomicOr(status, kBadSegsum); r = -1; }
    const int rs = r >= 0 ? start[r] : 0;
    const int re = r >= 0 ? start[r + 1] : 0;
    int rr[LPR], ss[LPR], ee[LPR];
    float4 x[LPR];
#define FR_EMB_BCAST(K)                                                                   \
    {                                                                                     \
      const int pk = row_bcast<K>(p);                                                     \
      rr[K] = row_bcast<K>(r);                                                            \
      ss[K] = row_bcast<K>(rs);                                                           \
      ee[K] = row_bcast<K>(re);                                                           \
      x[K] = (pk >= 0 && qok) ? G4[(int64_t)pk * ldg4 + q] : make_float4(0.f, 0.f, 0.f, 0.f); \
    }
    FR_EMB_BCAST(0) FR_EMB_BCAST(1) FR_EMB_BCAST(2) FR_EMB_BCAST(3)
    FR_EMB_BCAST(4) FR_EMB_BCAST(5) FR_EMB_BCAST(6) FR_EMB_BCAST(7)
    FR_EMB_BCAST(8) FR_EMB_BCAST(9) FR_EMB_BCAST(10) FR_EMB_BCAST(11)
    FR_EMB_BCAST(12) FR_EMB_BCAST(13) FR_EMB_BCAST(14) FR_EMB_BCAST(15)
#undef FR_EMB_BCAST
#pragma unroll
    for (int k = 0; k < LPR; ++k) {
      if (rr[k] < 0) break;  // past the chunk's last slot (uniform across the group)
      if (rr[k] != cur) {
        if (cur >= 0) flush();
        cur = rr[k]; cs = ss[k]; ce = ee[k];
        acc = make_float4(0.f, 0.f, 0.f, 0.f);
      }
      acc = f4_add(acc, x[k]);
    }
  }
  if (cur >= 0) flush();
}

// 6. rows cut by chunk boundaries: the block of the chunk where such a row begins sums its
//    partials (first piece, then pf of every following chunk it covers) in a fixed order.
__global__ __launch_bounds__(256) void emb_fixup_kernel(const int64_t* __restrict__ idx,
                                                        const int32_t* __restrict__ sorted,
                                                        const int32_t* __restrict__ start, int64_t R, int d4,
                                                        float4* __restrict__ out, int64_t ldo4,
                                                        const float4* __restrict__ pf,
                                                        const float4* __restrict__ pl, int64_t n,
                                                        int64_t nchunks, int32_t* __restrict__ status,
                                                        int32_t* __restrict__ rmap) {
  __shared__ float4 red[GPB][LPR];
  const int lig = threadIdx.x % LPR, g = threadIdx.x / LPR;
  const int q = blockIdx.y * LPR + lig;
  const bool qok = q < d4;
  const int total = start[R];
  const int64_t c = blockIdx.x;
  const int64_t k0 = c * kChunk;
  if (total < 0 || total > n) {  // reported by segsum; nothing here is trustworthy
    if (threadIdx.x == 0) atomicOr(status, kBadFixup);
    return;
  }
  if (k0 >= total) return;  // block-uniform
  const int64_t klast = min((int64_t)total, k0 + kChunk) - 1;
  const int p = sorted[klast];
  const int r = (p >= 0 && p < n) ? (int)idx[p] : -1;
  if (r < 0 || r >= R) { if (threadIdx.x == 0) atomicOr(status, kBadFixup); return; }
  const int64_t s = start[r], e = start[r + 1];
  if (!(e > k0 + kChunk && s >= k0)) return;  // no row starts here and crosses the chunk end
  const int64_t clast = (e - 1) / kChunk;
  if (clast >= nchunks) { if (threadIdx.x == 0) atomicOr(status, kBadFixup); return; }
  // pieces: j = 0 -> pl[c] (the row starts inside chunk c), j >= 1 -> pf[c + j]
  const int64_t np = clast - c + 1;
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  if (qok) {
    for (int64_t j = g; j < np; j += GPB) {
      const float4 v = j == 0 ? pl[c * d4 + q] : pf[(c + j) * d4 + q];
      acc = f4_add(acc, v);
    }
  }
  red[g][lig] = acc;
  __syncthreads();
  if (g == 0 && rmap && lig == 0 && blockIdx.y == 0) rmap[r] = sorted[s];
  if (g == 0 && qok) {
    float4 t = red[0][lig];
#pragma unroll
    for (int k = 1; k < GPB; ++k) t = f4_add(t, red[k][lig]);
    out[(rmap ? (int64_t)sorted[s] : (int64_t)r) * ldo4 + q] = t;
  }
}

}  // namespace

extern "C" int64_t fr_embedding_bwd_workspace(int64_t n, int64_t num_rows, int d) {
  if (n < 0 || num_rows < 0 || d <= 0) return 0;
  return emb_ws_bytes(n, num_rows, d);
}

extern "C" int64_t fr_embedding_bwd_status_offset(int64_t num_rows) { return (num_rows + 1) * 4; }

namespace {

// dense mode: out = dW [R, ldo], rmap == null.  row-gradient mode: out = compact rows [n, ldo],
// rmap = [R] row -> slot map.  Same sums, same order, in both modes.
int emb_bwd_impl(const int64_t* d_idx, int64_t n, const float* d_grad, int64_t ldg, int d, int64_t R,
                 int64_t padding_idx, float* d_out, int64_t ldo, int32_t* rmap, void* d_workspace, hipStream_t s) {
  const int d4 = d / 4;
  EmbWS w = emb_ws(d_workspace, n, R, d);
  float4* out4 = reinterpret_cast<float4*>(d_out);
  if (rmap && n > 0 && n <= kOneBlock) {  // one workgroup: fill, sort, owners; then the chain sums
    hipLaunchKernelGGL(emb_owner_one_kernel, dim3(1), dim3(kOneThreads), 0, s, d_idx, (int)n, R, padding_idx, w.nxt,
                       w.own, rmap, w.cursor + R + 1);
    FR_LAUNCH_CHECK();
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(n * d4, 256), (int64_t)fr::kNumCU * 8));
    hipLaunchKernelGGL(emb_owner_sum_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_idx, n, w.nxt, w.own,
                       reinterpret_cast<const float4*>(d_grad), ldg / 4, d4, out4, ldo / 4, 1);
    FR_LAUNCH_CHECK();
    return FR_OK;
  }
  if (rmap) {
    hipLaunchKernelGGL(emb_rmap_fill_kernel, dim3((unsigned)std::min<int64_t>(fr::ceil_div(R, 256), 1024)), dim3(256),
                       0, s, rmap, R);
    FR_LAUNCH_CHECK();
  }
  if (n <= kOwnerMax) {  // owner scan + chain sums: no counting sort
    if (!rmap) {  // zero fill of the dense table
      const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(R * d4, 256), (int64_t)fr::kNumCU * 8));
      hipLaunchKernelGGL(emb_hist_zero_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_idx, (int64_t)0, R,
                         padding_idx, w.cursor, out4, ldo / 4, d4);
      FR_LAUNCH_CHECK();
    }
    hipLaunchKernelGGL(emb_clear_kernel, dim3(1), dim3(256), 0, s, w.cursor + R + 1, (int64_t)1);  // status = 0
    FR_LAUNCH_CHECK();
    if (n > 0) {
      hipLaunchKernelGGL(emb_owner_scan_kernel, dim3((unsigned)fr::ceil_div(n, 4 * kScanPerWave)), dim3(256), 0, s,
                         d_idx, n, R, padding_idx, w.nxt, w.own, rmap);
      FR_LAUNCH_CHECK();
      const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(n * d4, 256), (int64_t)fr::kNumCU * 8));
      hipLaunchKernelGGL(emb_owner_sum_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_idx, n, w.nxt, w.own,
                         reinterpret_cast<const float4*>(d_grad), ldg / 4, d4, out4, ldo / 4, rmap ? 1 : 0);
      FR_LAUNCH_CHECK();
    }
    return FR_OK;
  }
  hipLaunchKernelGGL(emb_clear_kernel, dim3((unsigned)std::min<int64_t>(fr::ceil_div(R + 1, 256), 1024)), dim3(256), 0,
                     s, w.cursor, R + 2);
  FR_LAUNCH_CHECK();
  {
    const int64_t work = std::max<int64_t>(n, rmap ? 0 : R * d4);
    const int64_t blocks = std::max<int64_t>(1, std::min<int64_t>(fr::ceil_div(work, 256), (int64_t)fr::kNumCU * 8));
    hipLaunchKernelGGL(emb_hist_zero_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_idx, n, R, padding_idx,
                       w.cursor, rmap ? nullptr : out4, ldo / 4, d4);
    FR_LAUNCH_CHECK();
  }
  hipLaunchKernelGGL(emb_scan_kernel, dim3(1), dim3(1024), 0, s, w.cursor, R, w.start, w.big,
                     n / (kSmall + 1) + 1);
  FR_LAUNCH_CHECK();
  {
    const int64_t blocks = std::min<int64_t>(fr::ceil_div(n, 256), (int64_t)fr::kNumCU * 8);
    hipLaunchKernelGGL(emb_place_kernel, dim3((unsigned)blocks), dim3(256), 0, s, d_idx, n, R, padding_idx,
                       w.cursor, w.sorted);
    FR_LAUNCH_CHECK();
  }
  {
    const int64_t blocks = std::min<int64_t>(fr::ceil_div(R, 256), (int64_t)fr::kNumCU * 8);
    hipLaunchKernelGGL(emb_sort_small_kernel, dim3((unsigned)blocks), dim3(256), 0, s, w.start, R, n, w.sorted,
                       w.cursor + R + 1);
    FR_LAUNCH_CHECK();
  }
  {
    const int64_t max_big = n / (kSmall + 1);
    if (max_big > 0) {
      const size_t lds = (size_t)fr::ceil_div(n, 32) * 4;
      hipLaunchKernelGGL(emb_sort_big_kernel, dim3((unsigned)max_big), dim3(256), lds, s, w.cursor + R, n, R,
                         w.big, w.start, w.sorted);
      FR_LAUNCH_CHECK();
    }
  }
  const int64_t nch = n_chunks(n);
  const unsigned slices = (unsigned)fr::ceil_div(d4, LPR);
  hipLaunchKernelGGL(emb_segsum_kernel, dim3((unsigned)fr::ceil_div(nch, GPB), slices), dim3(256), 0, s, d_idx,
                     w.sorted, w.start, R, nch, reinterpret_cast<const float4*>(d_grad), ldg / 4, d4, out4, ldo / 4,
                     w.pf, w.pl, n, w.cursor + R + 1, rmap);
  FR_LAUNCH_CHECK();
  hipLaunchKernelGGL(emb_fixup_kernel, dim3((unsigned)nch, slices), dim3(256), 0, s, d_idx, w.sorted, w.start, R,
                     d4, out4, ldo / 4, w.pf, w.pl, n, nch, w.cursor + R + 1, rmap);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

}  // namespace

extern "C" int fr_embedding_bwd(const int64_t* d_idx, int64_t n, const float* d_grad, int64_t ldg, int d,
                                int64_t num_rows, int64_t padding_idx, float* d_out, int64_t ldo,
                                void* d_workspace, int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(n >= 0 && n <= kMaxPositions, "n out of range [0, 2^18]");
  FR_REQUIRE(num_rows > 0 && num_rows < INT32_MAX, "num_rows out of range");
  FR_REQUIRE(d > 0 && d % 4 == 0, "d must be a positive multiple of 4");
  FR_REQUIRE(ldo >= d && ldo % 4 == 0 && d_out && fr::aligned16(d_out), "bad output table");
  FR_REQUIRE(n == 0 || (d_idx && d_grad && ldg >= d && ldg % 4 == 0 && fr::aligned16(d_grad)),
             "bad grad / index arguments");
  FR_REQUIRE(d_workspace && fr::aligned16(d_workspace) && workspace_bytes >= emb_ws_bytes(n, num_rows, d),
             "workspace too small");
  return emb_bwd_impl(d_idx, n, d_grad, ldg, d, num_rows, padding_idx, d_out, ldo, nullptr, d_workspace,
                      reinterpret_cast<hipStream_t>(stream));
}

extern "C" int64_t fr_embedding_rowgrad_workspace(int64_t n, int64_t num_rows, int d) {
  return fr_embedding_bwd_workspace(n, num_rows, d);
}

extern "C" int fr_embedding_rowgrad(const int64_t* d_idx, int64_t n, const float* d_grad, int64_t ldg, int d,
                                    int64_t num_rows, int64_t padding_idx, int32_t* d_rmap, float* d_rows,
                                    void* d_workspace, int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(n >= 0 && n <= kMaxPositions, "n out of range [0, 2^18]");
  FR_REQUIRE(num_rows > 0 && num_rows < INT32_MAX && d_rmap, "bad row map");
  FR_REQUIRE(d > 0 && d % 4 == 0, "d must be a positive multiple of 4");
  FR_REQUIRE(n == 0 || (d_idx && d_grad && d_rows && ldg >= d && ldg % 4 == 0 && fr::aligned16(d_grad) &&
                        fr::aligned16(d_rows)),
             "bad grad / index / row arguments");
  FR_REQUIRE(d_workspace && fr::aligned16(d_workspace) && workspace_bytes >= emb_ws_bytes(n, num_rows, d),
             "workspace too small");
  return emb_bwd_impl(d_idx, n, d_grad, ldg, d, num_rows, padding_idx, d_rows, d, d_rmap, d_workspace,
                      reinterpret_cast<hipStream_t>(stream));
}

// ---------------------------------------------------------------------------------------------
// Atomic scatter-add (run-to-run order of float additions not fixed; the deterministic counting
// sort above is the engine's `deterministic` mode).  dW must hold the values to add onto (zeros
// for a plain embedding gradient).  d = 64: one wave per position, lane = column, so each
// position is ONE atomic wave-instruction over 256 contiguous bytes of its row (the shape the
// memory-side atomic units run at full rate; four float4 lanes-per-row groups per instruction,
// 16-B strided, ran ~5x slower); a wave's 32 indices come in one load and are broadcast by
// readlane, and four gradient rows are loaded before their atomics are issued.  Positions of the
// `hot` row (HealthRec's ingredient padding id: about half of the 2B x 20 positions) are summed in
// registers, then across the workgroup in LDS, and added with one atomic row update per workgroup.
// Two launches (zero fill + this) replace the eight of the sort path.
namespace {

constexpr int kAtomWaves = 4;          // 256 threads
constexpr int kAtomPerWave = 16;       // consecutive positions per wave -> 64 positions per block

__device__ __forceinline__ int64_t readlane64(int64_t v, int k) {
  const int lo = __builtin_amdgcn_readlane((int)(uint32_t)(uint64_t)v, k);
  const int hi = __builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), k);
  return (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint64_t)(uint32_t)lo);
}

// One wave per 16 consecutive positions: the ids in lanes 0-15, then all 16 gradient rows loaded
// before the first atomic (one memory round trip per wave: the scatter runs in the step's tail,
// where a chain of dependent load rounds is what made it slow), then one 256-B float-atomic wave
// instruction per position.  Positions at ``hot`` (the padding row, most of the ids) are summed in
// registers and added with one atomic per block.
__global__ __launch_bounds__(256) void emb_atomic_kernel(const int64_t* __restrict__ idx, int64_t n,
                                                         const float* __restrict__ G, int64_t ldg, int64_t R,
                                                         int64_t pad, int64_t hot, float* __restrict__ dW,
                                                         int64_t lddw) {
  __shared__ float hot_part[kAtomWaves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t base = ((int64_t)blockIdx.x * kAtomWaves + wv) * kAtomPerWave;
  const int64_t my_r = (lane < kAtomPerWave && base + lane < n) ? idx[base + lane] : -1;
  int64_t r[kAtomPerWave];
  float g[kAtomPerWave];
#pragma unroll
  for (int u = 0; u < kAtomPerWave; ++u) {
    r[u] = readlane64(my_r, u);  // wave-uniform; -1 past n
    if (!(r[u] >= 0 && r[u] < R && r[u] != pad)) r[u] = -1;
    g[u] = r[u] >= 0 ? __builtin_nontemporal_load(G + (base + u) * ldg + lane) : 0.f;
  }
  // every row arrived before the first atomic: the waits the compiler would place inside the
  // branchy atomic loop are vmcnt(0), which also waits for the atomics already issued
#pragma unroll
  for (int u = 0; u < kAtomPerWave; ++u) asm volatile("" : "+v"(g[u]));
  float h = 0.f;
#pragma unroll
  for (int u = 0; u < kAtomPerWave; ++u) {
    if (r[u] < 0) continue;
    if (r[u] == hot) h += g[u];
    else atomicAdd(dW + r[u] * lddw + lane, g[u]);
  }
  if (hot < 0 || hot >= R) return;  // block-uniform
  hot_part[wv][lane] = h;
  __syncthreads();
  if (wv == 0) {
    float t = hot_part[0][lane];
    for (int w2 = 1; w2 < kAtomWaves; ++w2) t += hot_part[w2][lane];
    if (__ballot(t != 0.f)) atomicAdd(dW + hot * lddw + lane, t);
  }
}

// fr_norms_bwd_coef + fr_embedding_bwd_atomic in one launch (HealthRec's deferred ingredient rows):
// the row of position i is G[i] + c_i E[i], c_i = [ids[i] != pad] gn[h] / nrm[h] with h the
// position's half (vector_norm's backward, zero where the norm is zero), scattered as above
__global__ __launch_bounds__(256) void norms_scatter_kernel(const int64_t* __restrict__ idx, int64_t n, int64_t half,
                                                            int64_t pad, const float* __restrict__ G,
                                                            const float* __restrict__ E,
                                                            const float* __restrict__ gn, int64_t gn_stride,
                                                            const float* __restrict__ nrm, int64_t R, int64_t hot,
                                                            float* __restrict__ dW, int64_t lddw) {
  __shared__ float hot_part[kAtomWaves][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float c0 = nrm[0] > 0.f ? gn[0] / nrm[0] : 0.f;
  const float c1 = nrm[1] > 0.f ? gn[gn_stride] / nrm[1] : 0.f;
  const int64_t base = ((int64_t)blockIdx.x * kAtomWaves + wv) * kAtomPerWave;
  const int64_t my_i = (lane < kAtomPerWave && base + lane < n) ? idx[base + lane] : -1;
  int64_t r[kAtomPerWave];
  float g[kAtomPerWave], e[kAtomPerWave];
#pragma unroll
  for (int u = 0; u < kAtomPerWave; ++u) {
    const int64_t id = readlane64(my_i, u);  // wave-uniform; -1 past n
    r[u] = (id >= 0 && id < R) ? id : -1;
    const int64_t off = (base + u) * 64 + lane;
    g[u] = r[u] >= 0 ? __builtin_nontemporal_load(G + off) : 0.f;
    e[u] = (r[u] >= 0 && id != pad) ? __builtin_nontemporal_load(E + off) : 0.f;
  }
#pragma unroll
  for (int u = 0; u < kAtomPerWave; ++u) asm volatile("" : "+v"(g[u]), "+v"(e[u]));
  float h = 0.f;
#pragma unroll
  for (int u = 0; u < kAtomPerWave; ++u) {
    if (r[u] < 0) continue;
    const float c = r[u] == pad ? 0.f : (base + u < half ? c0 : c1);
    const float v = fmaf(c, e[u], g[u]);  // the bits norms_bwd_kernel writes
    if (r[u] == hot) h += v;
    else atomicAdd(dW + r[u] * lddw + lane, v);
  }
  if (hot < 0 || hot >= R) return;  // block-uniform
  hot_part[wv][lane] = h;
  __syncthreads();
  if (wv == 0) {
    float t = hot_part[0][lane];
    for (int w2 = 1; w2 < kAtomWaves; ++w2) t += hot_part[w2][lane];
    if (__ballot(t != 0.f)) atomicAdd(dW + hot * lddw + lane, t);
  }
}

}  // namespace

extern "C" int fr_embedding_bwd_atomic(const int64_t* d_idx, int64_t n, const float* d_grad, int64_t ldg, int d,
                                       int64_t num_rows, int64_t padding_idx, int64_t hot_row, float* d_out,
                                       int64_t ldo, void* stream) {
  FR_REQUIRE(d == 64, "the atomic scatter is built for d = 64");
  FR_REQUIRE(n >= 0 && num_rows >= 1, "bad sizes");
  if (n == 0) return FR_OK;
  FR_REQUIRE(d_idx && d_grad && d_out, "null argument");
  FR_REQUIRE(ldg >= d && ldg % 4 == 0 && fr::aligned16(d_grad) && ldo >= d && ldo % 4 == 0 && fr::aligned16(d_out),
             "grad / out must be 16-B aligned with ld % 4 == 0");
  const int64_t per_block = (int64_t)kAtomWaves * kAtomPerWave;
  const int64_t blocks = fr::ceil_div(n, per_block);
  FR_REQUIRE(blocks < (int64_t)INT32_MAX, "too many positions");
  hipLaunchKernelGGL(emb_atomic_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     d_idx, n, d_grad, ldg, num_rows, padding_idx, hot_row, d_out, ldo);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_norms_bwd_scatter(const int64_t* d_ids, int64_t n, int64_t half, int64_t pad, const float* d_g,
                                    const float* d_e, const float* d_gn, int64_t gn_stride, const float* d_nrm,
                                    int64_t num_rows, int64_t hot_row, float* d_out, int64_t ldo, void* stream) {
  FR_REQUIRE(n >= 0 && half >= 0 && half <= n && num_rows >= 1, "bad sizes");
  if (n == 0) return FR_OK;
  FR_REQUIRE(d_ids && d_g && d_e && d_gn && d_nrm && d_out, "null operand");
  FR_REQUIRE(ldo >= 64 && ldo % 4 == 0 && fr::aligned16(d_out), "out: 64-wide rows, ld % 4 == 0, 16-B aligned");
  const int64_t per_block = (int64_t)kAtomWaves * kAtomPerWave;
  const int64_t blocks = fr::ceil_div(n, per_block);
  FR_REQUIRE(blocks < (int64_t)INT32_MAX, "too many positions");
  hipLaunchKernelGGL(norms_scatter_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     d_ids, n, half, pad, d_g, d_e, d_gn, gn_stride, d_nrm, num_rows, hot_row, d_out, ldo);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
