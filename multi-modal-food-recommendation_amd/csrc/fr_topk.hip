// Full-sort top-k: user x item scores on the matrix cores, fused with the top-k selection.
//
// Replaces, for a batch of users, full_sort_predict's  scores = user_all[u] @ item_all.T
// (common/abstract_recommender.py:39-50, the MMRec dense form) followed by
// torch.topk(scores, max(topk)) in Trainer.evaluate (common/trainer.py:476-503) and
// TopKEvaluator.collect (utils/topk_evaluator.py:45-66), optionally masking each user's training
// items first (the MMRec full-sort convention), and the hit test `i in pos_items` of
// TopKEvaluator.evaluate (topk_evaluator.py:104-107).  The [users x items] score matrix is never
// written: at 32k users x 1M items it would be 128 GB of fp32.
//
// GEMM (every kernel below): a workgroup = 8 waves x 32 users = 256 users x an item range (split).
//   * MFMA with A = a 32-item tile (LDS) and B = the wave's 32 users (VGPRs for the whole kernel):
//     bf16 tables -> v_mfma_f32_32x32x16_bf16 (fp32 accumulate); fp32 tables ->
//     v_mfma_f32_32x32x2_f32 (exact fp32 products).  The 32x32 accumulator has the user on the
//     lane (col = lane & 31) and 16 items in registers, so selection is lane-local.
//   * item tiles: global -> registers (one tile ahead) -> LDS (double buffer) with a 16-B chunk
//     XOR swizzle (conflict-free ds_read_b128 A fragments); item rows read once per workgroup.
//   * XCD-aware block order: workgroups of one XCD take consecutive (user tile, split) ids, so
//     the user tiles sharing an item range share that XCD's L2.
// Selection, for large item counts (exact for any data):
//   1. LIST kernel on a sparse strided sub-sample (every s0-th item, s0 = 16 s): exact per-user
//      top-k -> T0_u = its k-th best admissible score, a lower bound of the k-th best overall.
//   2. APPEND kernel over the sample (every s-th item, s <= 16) against T0_u, then MERGE -> T_u =
//      the sample's k-th best admissible score (~k*16 candidates per user; a user whose regions
//      overflow keeps T0_u, looser but still a lower bound).  (Round 5 took T_u from a LIST pass
//      over a 64-stride sample: its per-lane insertions cost more than these two launches.)
//   3. APPEND kernel over all items: the GEMM plus a compare against T_u; the few scores >= T_u
//      (expected ~k*s per user) are appended to per-(user, split, lane-half) regions.
//   4. MERGE: per user, the top-k of its admissible candidates by (score desc, item id asc); the
//      exclusion (history mask) is tested here, once per candidate, off the GEMM's path.
//   A region that overflows its capacity (adversarial score orders) flags its user; flagged users
//   are recomputed by the LIST kernel over all items and merged again (launches that exit at once
//   when nothing is flagged), so the result never depends on the data's order.
// LIST kernel: each lane keeps a PRIVATE sorted top-k (64-bit keys in registers) of the items it
// sees, updated by bubble passes in which every lane with a candidate inserts at once.  Small
// item counts use it directly (one pass + merge).
// Order is total and deterministic: score descending, item id ascending on ties (the order of a
// stable descending argsort), independent of tiling, splits and sampling.
#include "fr_bf16.h"

#include <algorithm>
#include <cmath>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kUsersPerWG = kWaves * 32;
constexpr int kTile = 32;      // items per staged tile
constexpr int kKMax = 32;      // largest k
constexpr int kAppendDepth = 2;  // APPEND's register stages of item tiles (1 or 2)
#ifndef FR_TOPK_PIPE
#define FR_TOPK_PIPE 1
#endif
// APPEND: the candidate masks of tile t - 1 are formed between tile t's MFMAs (the matrix pipe
// runs while the VALU compares), only the rare append passes stay outside the MFMA stream
constexpr bool kAppendPipe = FR_TOPK_PIPE != 0;
#ifndef FR_TOPK_PRETEST
#define FR_TOPK_PRETEST 1
#endif
// APPEND: only the max of each block's 16 scores between the MFMAs; the candidate bits and the
// append passes only for the blocks where some lane's max reaches the threshold
constexpr bool kAppendPretest = FR_TOPK_PRETEST != 0;
#ifndef FR_TOPK_RING
#define FR_TOPK_RING 2
#endif
// APPEND's LDS ring of staged item tiles: 2 (one barrier per tile) or 4 (two tiles per barrier)
constexpr int kAppendRing = FR_TOPK_RING;

template <typename T, int D, int NB = 1>
struct Cfg {
  static constexpr int RB = D * (int)sizeof(T);           // bytes per row
  static constexpr int CPR = RB / 16;                       // 16-B chunks per row
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int KS = BF ? D / 16 : D / 2;            // MFMA k-steps
  static constexpr int TILE = kTile * NB;                   // items per staged tile (NB 32-item blocks)
  static constexpr int STAGE = TILE * RB;                   // bytes per staged tile
  static constexpr int G = CPR >= 16 ? 1 : 16 / CPR;        // rows sharing one 256-B bank row
  static constexpr int SWM = (CPR >= 16 ? 16 : CPR) - 1;
  static constexpr int CH = (TILE * CPR + kThreads - 1) / kThreads;  // staged chunks per thread
  static constexpr int LDS = 2 * STAGE;
};

template <typename T, int D>
__device__ __forceinline__ int swz(int r, int c) {
  using C = Cfg<T, D>;
  return c ^ ((r / C::G) & C::SWM);
}

// Entries are ordered by the 64-bit key (ordered score bits << 32 | ~item): higher score first,
// lower item id first on ties.
// fp32 -> uint32 preserving order (larger float -> larger uint; -0 < +0, NaN above +inf)
__device__ __forceinline__ uint32_t fr_ord(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
__device__ __forceinline__ float fr_unord(uint32_t o) {
  return __uint_as_float((o & 0x80000000u) ? (o & 0x7fffffffu) : ~o);
}

// byte offset, in a staged tile, of lane (r, h)'s A fragment for k-step s (bf16: chunk 2s+h;
// fp32: 4 k-steps per chunk, lane half h holds the upper half of k)
template <typename T, int D>
__device__ __forceinline__ int a_off(int r, int h, int s) {
  using C = Cfg<T, D>;
  return (r * C::CPR + swz<T, D>(r, C::BF ? 2 * s + h : h * (C::CPR / 2) + s)) * 16;
}

__device__ __forceinline__ bool in_csr_row(const int32_t* __restrict__ col, int64_t lo, int64_t hi, int64_t key) {
  const int64_t end = hi;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if ((int64_t)col[mid] < key) lo = mid + 1;
    else hi = mid;
  }
  return lo < end && (int64_t)col[lo] == key;
}

__device__ __forceinline__ uint32_t bloom_hash(int64_t key) { return ((uint32_t)key * 0x9E3779B1u) >> 25; }

// Per-lane exclusion test: a 128-bit Bloom signature of the user's row (registers) screens every
// candidate; only signature hits (the row's items + ~15% false positives) bisect the CSR row.
struct Excl {
  uint32_t w0, w1, w2, w3;
  int64_t lo, hi, base;
  const int32_t* col;
  __device__ void init(const int64_t* __restrict__ ptr, const int32_t* __restrict__ c, int64_t b, int64_t row) {
    w0 = w1 = w2 = w3 = 0u;
    col = c;
    base = b;
    lo = hi = 0;
    if (!ptr) return;
    lo = ptr[row];
    hi = ptr[row + 1];
    for (int64_t e = lo; e < hi; ++e) {
      const uint32_t hsh = bloom_hash(c[e]);
      const uint32_t bit = 1u << (hsh & 31u);
      const uint32_t w = hsh >> 5;
      w0 |= w == 0 ? bit : 0u;
      w1 |= w == 1 ? bit : 0u;
      w2 |= w == 2 ? bit : 0u;
      w3 |= w == 3 ? bit : 0u;
    }
  }
  __device__ __forceinline__ bool test(int64_t item) const {
    if (lo == hi) return false;
    const int64_t key = base + item;
    const uint32_t hsh = bloom_hash(key);
    const uint32_t w = hsh >> 5;
    const uint32_t word = w == 0 ? w0 : (w == 1 ? w1 : (w == 2 ? w2 : w3));
    if (!((word >> (hsh & 31u)) & 1u)) return false;
    return in_csr_row(col, lo, hi, key);
  }
};

struct ScoreArgs {
  const void* Uq; int64_t ldu; int64_t n_users; const int32_t* urows; const int32_t* d_nu;
  const void* It; int64_t ldi; int64_t n_items; int64_t item_mul;   // tile item i = item id i * item_mul
  const int64_t* uid; const int64_t* ex_ptr; const int32_t* ex_col; int64_t ex_base;
  int k; int n_splits; int64_t span; int n_utiles;
  float* ls; int32_t* li;                                           // LIST: [slot][split][half][k]
  const float* thr; int cap; float* cs; int32_t* ci; int32_t* cc;   // APPEND: [slot][split][half][cap], counts
};

// kGmax: per lane 8 running maxima (score, item) -- one per pair of score positions (j, j + 8) of the
// MFMA fragment -- over the lane's share of the items (APPEND's staging and schedule, no selection
// passes): distinct items whose merged k-th best is a lower bound of the user's k-th best
enum { kList = 0, kAppend = 1, kGmax = 2 };

template <typename T, int D, int KC, int MODE, int NB>
__global__ __launch_bounds__(kThreads) void topk_score_kernel(ScoreArgs a) {
  using C = Cfg<T, D, NB>;
  constexpr bool STREAM = MODE != kList;  // APPEND / GMAX: register-held staging, pipelined epilogue
  constexpr int RING = STREAM ? kAppendRing : 2;
  __shared__ __attribute__((aligned(16))) char smem[RING * C::STAGE];

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;
  const int64_t n_users = a.d_nu ? (int64_t)*a.d_nu : a.n_users;

  // XCD-aware bijective remap (blocks are dispatched round-robin over the 8 XCDs)
  const int total = a.n_utiles * a.n_splits;
  const int b = blockIdx.x, xcd = b & 7, q8 = total >> 3, r8 = total & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int ut = wg % a.n_utiles, sp = wg / a.n_utiles;
  if ((int64_t)ut * kUsersPerWG >= n_users) return;  // whole workgroup idle (device-sized grids)

  const int64_t slot = (int64_t)ut * kUsersPerWG + wave * 32 + r;
  const bool uvalid = slot < n_users;
  const int64_t urow = uvalid ? (a.urows ? (int64_t)a.urows[slot] : slot) : 0;
  const int64_t i_lo = (int64_t)sp * a.span;
  const int64_t i_hi = min(a.n_items, i_lo + a.span);
  const int n_tiles = (int)((i_hi - i_lo + C::TILE - 1) / C::TILE);
  const T* __restrict__ It = reinterpret_cast<const T*>(a.It);
  const int64_t ldi = a.ldi;

  // exclusion: tested at insertion by the LIST kernel; the APPEND kernel leaves it to the merge
  Excl ex;
  ex.init(MODE == kList ? a.ex_ptr : nullptr, a.ex_col, a.ex_base, a.uid ? a.uid[urow] : urow);

  // B operand: this lane's user, held for the whole kernel
  typedef typename std::conditional<C::BF, bf16x8, float4>::type BFrag;
  constexpr int NBF = C::BF ? C::KS : C::KS / 4;
  BFrag bf[NBF];
#pragma unroll
  for (int s = 0; s < NBF; ++s) {
    if constexpr (C::BF) {
      bf[s] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const uint16_t*>(a.Uq) + urow * a.ldu + 16 * s + 8 * h);
    } else {
      bf[s] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(a.Uq) + urow * a.ldu + h * (D / 2) + 4 * s);
    }
  }
  // make the compiler itself retire these loads here (an asm that reads them), so its counted
  // waits inside the tile loop only ever cover the item-tile prefetch
#pragma unroll
  for (int s = 0; s < NBF; ++s) asm volatile("" ::"v"(__builtin_bit_cast(i32x4, bf[s])));
  // APPEND: this user's threshold and this lane's region
  const float thr_u = MODE == kAppend && uvalid ? a.thr[slot] : -INFINITY;
  // (read by an asm too: the counted waits are placed by the compiler, which does not see the
  // vmcnt(0) below -- without this it waits for every load in flight, the item-tile prefetch
  // included, before the threshold's first use in each pass of the tile loop)
  asm volatile("" ::"v"(thr_u));
  const int64_t region = (slot * a.n_splits + sp) * 2 + h;
  int cnt = 0;

  // the B-fragment / exclusion-row / threshold loads retire here, so the loop's counted waits
  // only ever cover the item-tile prefetch
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // LIST: lane-private list of KC 64-bit keys (ordered score bits << 32 | ~item: larger key =
  // better entry; keys are unique since item ids differ), sorted descending.  The first KC - k
  // entries are sentinels (~0, above every real key), so the k live entries are
  // key[KC-k .. KC-1]; empty live entries hold 0.
  uint64_t key[KC];
#pragma unroll
  for (int q = 0; q < KC; ++q) key[q] = q < KC - a.k ? ~0ull : 0ull;

  // item tiles: global -> registers (one tile ahead) -> LDS (double buffer, swizzled chunks).
  // APPEND keeps each staged chunk's row, LDS offset and global source (advanced one tile of rows
  // per step) in registers; the register-heavy LIST kernel recomputes them per tile.
  constexpr int NSH = STREAM ? C::CH : 1;
  int srow[NSH], sdst[NSH];
  const char* ssrc[NSH];
#pragma unroll
  for (int c = 0; c < NSH; ++c) {
    const int x = tid + c * kThreads;
    const int row = x / C::CPR, cc = x % C::CPR;
    srow[c] = x < C::TILE * C::CPR ? row : 1 << 30;  // rows past the tile are never stored
    sdst[c] = (row * C::CPR + swz<T, D>(row, cc)) * 16;
    ssrc[c] = reinterpret_cast<const char*>(It) + (i_lo * ldi) * (int64_t)sizeof(T) + cc * 16;
  }
  const uint32_t row_bytes = (uint32_t)(ldi * (int64_t)sizeof(T));
  const int n_split = (int)(i_hi - i_lo);
#define FR_LOAD_TILE(T_, S_)                                                                        \
  _Pragma("unroll") for (int c = 0; c < C::CH; ++c) {                                               \
    if constexpr (STREAM) {                                                                         \
      /* unconditional (rows past the split re-read its last row; their scores are dropped): */     \
      /* with no load skipped on any path the compiler's counted waits stay exact */                \
      const int rr = min((T_) * C::TILE + min(srow[c], C::TILE - 1), n_split - 1);                 \
      S_[c] = __builtin_bit_cast(uint4, *reinterpret_cast<const i32x4*>(ssrc[c] + (uint64_t)(uint32_t)rr * row_bytes)); \
    } else {                                                                                        \
      const int x = tid + c * kThreads;                                                             \
      S_[c] = make_uint4(0, 0, 0, 0);                                                               \
      if (x < C::TILE * C::CPR) {                                                                   \
        const int row = x / C::CPR, cc = x % C::CPR;                                                \
        const int64_t item = i_lo + (int64_t)(T_) * C::TILE + row;                                  \
        if (item < i_hi)                                                                            \
          S_[c] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(It) +               \
                                                   (item * ldi) * (int64_t)sizeof(T) + cc * 16);    \
      }                                                                                             \
    }                                                                                               \
  }
#define FR_STORE_TILE(BUF_, S_)                                                                     \
  _Pragma("unroll") for (int c = 0; c < C::CH; ++c) {                                               \
    if constexpr (STREAM) {                                                                         \
      if (srow[c] < C::TILE) *reinterpret_cast<uint4*>(smem + (BUF_) * C::STAGE + sdst[c]) = S_[c];  \
    } else {                                                                                        \
      const int x = tid + c * kThreads;                                                             \
      if (x < C::TILE * C::CPR) {                                                                   \
        const int row = x / C::CPR, cc = x % C::CPR;                                                \
        *reinterpret_cast<uint4*>(smem + (BUF_) * C::STAGE + (row * C::CPR + swz<T, D>(row, cc)) * 16) = S_[c];  \
      }                                                                                             \
    }                                                                                               \
  }
  // A-fragment LDS offsets of this lane (row r of each 32-item block, chunk 2s+h): held in
  // registers by the APPEND kernel, recomputed per use by the register-heavy LIST kernel
  constexpr int NA = C::BF ? C::KS : C::KS / 4;
  constexpr int NAH = STREAM ? NA : 1;
  int aoff[NAH];
#pragma unroll
  for (int s = 0; s < NAH; ++s) aoff[s] = a_off<T, D>(r, h, s);
#define FR_AOFF(S_) (STREAM ? aoff[STREAM ? (S_) : 0] : a_off<T, D>(r, h, (S_)))

  // register stages of the item tiles: APPEND keeps two (the global loads of tile t + 3 are issued
  // after tile t's barrier and have two tiles of MFMA work to land in), LIST one (its key lists
  // hold the registers)
  constexpr int DEPTH = STREAM ? kAppendDepth : 1;
  uint4 stgA[C::CH], stgB[DEPTH == 2 ? C::CH : 1];
  // GMAX: this lane's 8 running maxima, group g = positions g and g + 8 of every 32-item block's
  // fragment: the score and 2 q + (position g + 8), q the block's index in the split (the item of
  // position j is i_lo + 32 q + 4h + (j&3) + 8(j>>2)); -1: none
  float gmx[MODE == kGmax ? 8 : 1];
  int32_t gq[MODE == kGmax ? 8 : 1];
#pragma unroll
  for (int g = 0; g < (MODE == kGmax ? 8 : 1); ++g) { gmx[g] = -INFINITY; gq[g] = -1; }
  if constexpr (STREAM) {
    if (n_tiles <= 0) {  // an empty split: no rows to clamp to
      if (uvalid) {
        if constexpr (MODE == kAppend) a.cc[region] = 0;
        else
#pragma unroll
          for (int g = 0; g < 8; ++g) { a.ls[region * 8 + g] = -INFINITY; a.li[region * 8 + g] = INT32_MAX; }
      }
      return;
    }
    if constexpr (RING == 4) {  // tiles 0, 1 staged; 2, 3 in registers
      FR_LOAD_TILE(0, stgA)
      FR_LOAD_TILE(1, stgB)
      FR_STORE_TILE(0, stgA)
      FR_STORE_TILE(1, stgB)
      __syncthreads();
      FR_LOAD_TILE(2, stgA)
      FR_LOAD_TILE(3, stgB)
    } else {
      FR_LOAD_TILE(0, stgA)
      FR_STORE_TILE(0, stgA)
      __syncthreads();
      FR_LOAD_TILE(1, stgA)
      if constexpr (DEPTH == 2) { FR_LOAD_TILE(2, stgB) }
    }
  } else {
    if (n_tiles > 0) {
      FR_LOAD_TILE(0, stgA)
      FR_STORE_TILE(0, stgA)
    }
    __syncthreads();
    if (n_tiles > 1) { FR_LOAD_TILE(1, stgA) }
  }
  // APPEND: the threshold of an invalid slot is NaN (no score passes any compare)
  const float wv = uvalid ? thr_u : __builtin_nanf("");
  // this lane's candidate bits of one block's 16 scores (branch-free: VALU only)
  auto cand_mask = [&](const f32x16& av) __attribute__((always_inline)) {
    uint32_t m = 0u;
#pragma unroll
    for (int j = 0; j < 16; ++j) m |= av[j] >= wv ? (1u << j) : 0u;
    return m;
  };
  // the largest of a block's 16 scores (v_max3 tree; a NaN score drops out -- it never passes the
  // threshold compare either)
  auto max16 = [&](const f32x16& av) __attribute__((always_inline)) {
    float m0 = fmaxf(fmaxf(av[0], av[1]), av[2]), m1 = fmaxf(fmaxf(av[3], av[4]), av[5]);
    float m2 = fmaxf(fmaxf(av[6], av[7]), av[8]), m3 = fmaxf(fmaxf(av[9], av[10]), av[11]);
    float m4 = fmaxf(fmaxf(av[12], av[13]), av[14]);
    return fmaxf(fmaxf(fmaxf(m0, m1), m2), fmaxf(fmaxf(m3, m4), av[15]));
  };
  // selection of one block (scores av, items ib + (j&3) + 8(j>>2)) given its candidate bits
  auto select_block = [&](const f32x16& av, uint32_t mask, const int64_t ib, const float wf)
                          __attribute__((always_inline)) {
    {  // the split's last block: drop items past its end -- a 32-bit offset mask (no 64-bit compares
       // per position: if-converted, those cost ~50 VALU per block on every block)
      const int64_t left = i_hi - ib;  // items of the block from this lane's first offset on
      const uint32_t vb = left >= 32 ? 0xffffffffu : (left <= 0 ? 0u : (1u << (int)left) - 1u);
      const uint32_t jm = (vb & 0xfu) | ((vb >> 4) & 0xf0u) | ((vb >> 8) & 0xf00u) | ((vb >> 12) & 0xf000u);
      mask &= jm;  // position j <-> offset (j & 3) + 8 (j >> 2)
    }
    if (!uvalid) mask = 0u;
    // every lane handles its next candidate in the same pass
    while (__ballot(mask != 0u)) {
      const bool act = mask != 0u;
      const int j = act ? __builtin_ctz(mask) : 0;
      mask &= mask - 1u;
      const float v0 = (j & 1) ? av[1] : av[0], v1 = (j & 1) ? av[3] : av[2];
      const float v2 = (j & 1) ? av[5] : av[4], v3 = (j & 1) ? av[7] : av[6];
      const float v4 = (j & 1) ? av[9] : av[8], v5 = (j & 1) ? av[11] : av[10];
      const float v6 = (j & 1) ? av[13] : av[12], v7 = (j & 1) ? av[15] : av[14];
      const float w0 = (j & 2) ? v1 : v0, w1 = (j & 2) ? v3 : v2, w2 = (j & 2) ? v5 : v4, w3 = (j & 2) ? v7 : v6;
      const float x0 = (j & 4) ? w1 : w0, x1 = (j & 4) ? w3 : w2;
      const float sc = (j & 8) ? x1 : x0;
      const int64_t item = (ib + (j & 3) + 8 * (j >> 2)) * a.item_mul;
      if constexpr (MODE == kList) {
        const uint64_t kk = ((uint64_t)fr_ord(sc) << 32) | (uint32_t)(~(uint32_t)item);
        if (act && kk > key[KC - 1] && !ex.test(item)) {
          // one bubble pass: the new key sinks to its place, the old minimum falls off the end
          uint64_t x = kk;
#pragma unroll
          for (int q = 0; q < KC; ++q) {
            const uint64_t cur = key[q];
            const bool gt = x > cur;
            key[q] = gt ? x : cur;
            x = gt ? cur : x;
          }
        }
      } else {
        if (act) {
          if (cnt < a.cap) {
            a.cs[region * a.cap + cnt] = sc;
            a.ci[region * a.cap + cnt] = (int32_t)item;
          }
          ++cnt;
        }
      }
    }
  };
  constexpr bool PIPE = STREAM && kAppendPipe;
  static_assert(MODE != kGmax || PIPE, "the position maxima are folded between the MFMAs only");
  // GMAX: fold one block's scores into the running maxima (strict >: the first -- lowest -- item
  // keeps a tie; NaN never enters); `live` (wave-uniform) false skips the block
  auto gmax_fold = [&](const f32x16& av, const int q, const bool live) __attribute__((always_inline)) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const bool hi = av[g + 8] > av[g];  // (a tie keeps the lower item)
      const float m = hi ? av[g + 8] : av[g];
      const bool up = live && m > gmx[g];
      gmx[g] = up ? m : gmx[g];
      gq[g] = up ? 2 * q + (hi ? 1 : 0) : gq[g];
    }
  };
  // the same with the split's end checked (its last real tile): positions past it take no part
  auto gmax_fold_tail = [&](const f32x16& av, const int q) __attribute__((always_inline)) {
    const int lim = (int)(i_hi - i_lo - 32 * (int64_t)q - 4 * h);  // items of the block this lane may take
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const float lo_v = (g & 3) + 8 * (g >> 2) < lim ? av[g] : -INFINITY;
      const bool hi = (g & 3) + 8 * (g >> 2) + 16 < lim && av[g + 8] > lo_v;
      const float m = hi ? av[g + 8] : lo_v;
      const bool up = m > gmx[g];
      gmx[g] = up ? m : gmx[g];
      gq[g] = up ? 2 * q + (hi ? 1 : 0) : gq[g];
    }
  };
  // one tile: its scores from LDS buffer t & 1 into `acc` -- with PIPE the previous tile's scores
  // (`prev`) are selected after them, their masks formed between the MFMAs; without, this tile's
  // own -- then the next tile (in `cur`) into the other buffer, and `cur` refilled DEPTH + 1 ahead
  auto tile_step = [&](const int t, uint4 (&cur)[C::CH], f32x16 (&acc)[NB], const f32x16 (&prev)[NB])
                       __attribute__((always_inline)) {
    // ---- scores of this tile on the matrix cores (NB independent 32-item blocks)
    const char* abuf = smem + (t & (RING - 1)) * C::STAGE;
#pragma unroll
    for (int bb = 0; bb < NB; ++bb)
#pragma unroll
      for (int j = 0; j < 16; ++j) acc[bb][j] = 0.f;
    uint32_t pmask[NB];
    bool pany[NB];  // APPEND pre-test: this lane's block holds a score >= the threshold
    if constexpr (C::BF) {
      // the tile's A fragments are read ahead of the MFMA chains that consume them in order
      bf16x8 af[NB][C::KS];
#pragma unroll
      for (int s = 0; s < C::KS; ++s)
#pragma unroll
        for (int bb = 0; bb < NB; ++bb)
          af[bb][s] = *reinterpret_cast<const bf16x8*>(abuf + bb * 32 * C::RB + FR_AOFF(s));
#pragma unroll
      for (int s = 0; s < C::KS; ++s)
#pragma unroll
        for (int bb = 0; bb < NB; ++bb)
          acc[bb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[bb][s], bf[s], acc[bb], 0, 0, 0);
      if constexpr (PIPE && MODE == kAppend && kAppendPretest) {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) pany[bb] = max16(prev[bb]) >= wv;
      } else if constexpr (PIPE && MODE == kAppend) {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) pmask[bb] = cand_mask(prev[bb]);
      }
      if constexpr (PIPE && MODE == kGmax) {  // (the previous tile is never the split's last here)
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) gmax_fold(prev[bb], (t - 1) * NB + bb, t - 1 < n_tiles - 1);
      }
      // schedule: 4 LDS reads ahead, then MFMA / next read interleaved (3-4 reads in flight);
      // PIPE: the previous tile's compares spread over the MFMA slots
      constexpr int NM = NB * C::KS;
      constexpr int VPM = PIPE ? (NB * (MODE == kAppend && kAppendPretest ? 10 : 40) + NM - 1) / NM : 0;  // VALU per MFMA slot
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
#pragma unroll
      for (int s = 0; s < NM - 4; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        if constexpr (VPM > 0) __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if constexpr (VPM > 0) __builtin_amdgcn_sched_group_barrier(0x002, VPM, 0);
      }
    } else {
#pragma unroll
      for (int sg = 0; sg < C::KS / 4; ++sg) {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) {
          const float4 af = *reinterpret_cast<const float4*>(abuf + bb * 32 * C::RB + FR_AOFF(sg));
          acc[bb] = __builtin_amdgcn_mfma_f32_32x32x2f32(af.x, bf[sg].x, acc[bb], 0, 0, 0);
          acc[bb] = __builtin_amdgcn_mfma_f32_32x32x2f32(af.y, bf[sg].y, acc[bb], 0, 0, 0);
          acc[bb] = __builtin_amdgcn_mfma_f32_32x32x2f32(af.z, bf[sg].z, acc[bb], 0, 0, 0);
          acc[bb] = __builtin_amdgcn_mfma_f32_32x32x2f32(af.w, bf[sg].w, acc[bb], 0, 0, 0);
        }
      }
      if constexpr (PIPE && MODE == kAppend && kAppendPretest) {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) pany[bb] = max16(prev[bb]) >= wv;
      } else if constexpr (PIPE && MODE == kAppend) {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) pmask[bb] = cand_mask(prev[bb]);
      }
      if constexpr (PIPE && MODE == kGmax) {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) gmax_fold(prev[bb], (t - 1) * NB + bb, t - 1 < n_tiles - 1);
      }
    }
#pragma unroll
    for (int bb = 0; bb < NB; ++bb) {
      if constexpr (PIPE && MODE == kGmax) {
        // (folded between the MFMAs)
      } else if constexpr (PIPE && kAppendPretest) {
        // the previous tile's block bb, only when some lane's pre-test passed (t - 1 < 0: NaN scores)
        if (__ballot(pany[bb]))
          select_block(prev[bb], cand_mask(prev[bb]), i_lo + (int64_t)(t - 1) * C::TILE + bb * 32 + 4 * h, wv);
      } else if constexpr (PIPE) {
        // the previous tile's block bb (t - 1 < 0: its scores are NaN, no bit set)
        select_block(prev[bb], pmask[bb], i_lo + (int64_t)(t - 1) * C::TILE + bb * 32 + 4 * h, wv);
      } else {
        // ---- this lane's 16 scores of block bb: user `slot`, items ib + (j&3) + 8(j>>2) + 4h
        const int64_t ib = i_lo + (int64_t)t * C::TILE + bb * 32 + 4 * h;
        float wf;
        if constexpr (MODE == kList) {
          const uint32_t wsc = (uint32_t)(key[KC - 1] >> 32);
          wf = wsc < 0x00800000u ? -INFINITY : fr_unord(wsc);  // the list's worst score (empty: -inf)
        } else {
          wf = thr_u;
        }
        const f32x16 av = acc[bb];
        uint32_t mask = 0u;
#pragma unroll
        for (int j = 0; j < 16; ++j) mask |= av[j] >= wf ? (1u << j) : 0u;
        select_block(av, mask, ib, wf);
      }
    }
    if constexpr (RING == 2) {
      // ---- next tile into the other buffer; prefetch DEPTH + 1 tiles ahead into the freed stage
      // (APPEND: unconditionally -- past the last tile the stores go to a buffer no one reads again
      // and the loads re-read the split's last row)
      if (STREAM || t + 1 < n_tiles) { FR_STORE_TILE((t + 1) & 1, cur) }
      __syncthreads();
      if (STREAM || t + 1 + DEPTH < n_tiles) { FR_LOAD_TILE(t + 1 + DEPTH, cur) }
    }
  };
  f32x16 accX[NB], accY[PIPE ? NB : 1];
  if constexpr (PIPE) {
#pragma unroll
    for (int bb = 0; bb < NB; ++bb)
#pragma unroll
      for (int j = 0; j < 16; ++j) accY[bb][j] = __builtin_nanf("");
  }
  if constexpr (DEPTH == 2) {
    // an odd tile count runs one tile past the split: all its items are dropped by the i_hi test
    int t = 0;
    for (; t < n_tiles; t += 2) {
      if constexpr (PIPE) {
        tile_step(t, stgA, accX, accY);
        tile_step(t + 1, stgB, accY, accX);
      } else {
        tile_step(t, stgA, accX, accX);
        tile_step(t + 1, stgB, accX, accX);
      }
      if constexpr (RING == 4) {
        // tiles t + 2, t + 3 into the buffers tiles t - 2, t - 1 left (every wave passed the
        // previous barrier after computing them), then one barrier for both, then the next pair
        FR_STORE_TILE((t + 2) & 3, stgA)
        FR_STORE_TILE((t + 3) & 3, stgB)
        __syncthreads();
        FR_LOAD_TILE(t + 4, stgA)
        FR_LOAD_TILE(t + 5, stgB)
      }
    }
    if constexpr (PIPE && MODE == kGmax) {
      // the split's last real tile n_tiles - 1 (in accY if the count is even, else in accX: the
      // extra tile's scores in accY are dropped), folded with its end checked
      const int q0 = (n_tiles - 1) * NB;
      if (n_tiles & 1) {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) gmax_fold_tail(accX[bb], q0 + bb);
      } else {
#pragma unroll
        for (int bb = 0; bb < NB; ++bb) gmax_fold_tail(accY[bb], q0 + bb);
      }
    } else if constexpr (PIPE) {  // the last tile (t - 1)
#pragma unroll
      for (int bb = 0; bb < NB; ++bb)
        select_block(accY[bb], cand_mask(accY[bb]), i_lo + (int64_t)(t - 1) * C::TILE + bb * 32 + 4 * h, wv);
    }
  } else {
    for (int t = 0; t < n_tiles; ++t) tile_step(t, stgA, accX, accX);
  }
#undef FR_LOAD_TILE
#undef FR_STORE_TILE
#undef FR_AOFF

  if (!uvalid) return;
  if constexpr (MODE == kList) {
    // list (slot, split, half): k unsorted entries, decoded back to (score, item)
    const int64_t o = region * (int64_t)a.k - (KC - a.k);
#pragma unroll
    for (int q = 0; q < KC; ++q) {
      if (q >= KC - a.k) {
        const uint64_t kk = key[q];
        const bool empty = kk < (1ull << 32);
        a.ls[o + q] = empty ? -INFINITY : fr_unord((uint32_t)(kk >> 32));
        a.li[o + q] = empty ? INT32_MAX : (int32_t)(~(uint32_t)kk);
      }
    }
  } else if constexpr (MODE == kGmax) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {
      const int j = g + 8 * (gq[g] & 1);
      a.ls[region * 8 + g] = gmx[g];
      a.li[region * 8 + g] = gq[g] < 0 ? INT32_MAX
                                       : (int32_t)((i_lo + 32 * (int64_t)(gq[g] >> 1) + 4 * h + (j & 3) + 8 * (j >> 2)) * a.item_mul);
    }
  } else {
    a.cc[region] = cnt;
  }
}

struct MergeArgs {
  const float* ps; const int32_t* pi; const int32_t* cnt;   // regions (cnt null: every region holds k)
  int cap; int n_regions;
  int64_t n_users; const int32_t* d_nu; const int32_t* urows;  // slot -> output row
  int k; const int64_t* uid; const int64_t* t_ptr; const int32_t* t_col; int64_t t_base;
  float* out_s; int64_t* out_i; uint8_t* hits;
  float* thr_out;                                              // write the k-th best score only
  const int64_t* ex_ptr; const int32_t* ex_col; int64_t ex_base;  // exclusion applied here (APPEND input)
  int32_t* flag_list; int32_t* flag_cnt;                      // overflowed users -> exact recompute
  const float* thr_fb;  // threshold stage: an overflowed user keeps this (looser) lower bound instead
};

// One wave per user: each lane streams a strided share of the user's candidates (all regions,
// concatenated through a prefix sum of their counts in LDS; kMergeBatch loads in flight per lane)
// into a private sorted register list (bubble insertion, as the LIST kernel), then k rounds of a
// wave arg-max over the lanes' list heads emit the top-k in order (the winner lane pops its
// head); finally the hit flags against the user's held-out CSR row.
constexpr int kMergeBatch = 8;
constexpr int kMergeMaxRegions = 128;  // 2 x the largest split count
template <int KC>
__global__ __launch_bounds__(256) void topk_merge_kernel(MergeArgs a) {
  __shared__ int pre_all[4][kMergeMaxRegions + 1];
  const int lane = threadIdx.x & 63;
  int* pre = pre_all[threadIdx.x >> 6];
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t n_users = a.d_nu ? (int64_t)*a.d_nu : a.n_users;
  if (u >= n_users) return;
  const int64_t orow = a.urows ? (int64_t)a.urows[u] : u;
  const int64_t base = u * (int64_t)a.n_regions * a.cap;
  // region counts -> exclusive prefix (pre[g] = first candidate of region g, pre[n_regions] = total)
  bool over = false;
  int carry = 0;
  for (int g0 = 0; g0 < a.n_regions; g0 += 64) {
    const int g = g0 + lane;
    int c = g < a.n_regions ? (a.cnt ? a.cnt[u * a.n_regions + g] : a.cap) : 0;
    over |= c > a.cap;
    c = min(c, a.cap);
    int incl = c;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const int o = __shfl_up(incl, off, 64);
      if (lane >= off) incl += o;
    }
    if (g < a.n_regions) pre[g + 1] = carry + incl;
    carry += __shfl(incl, 63, 64);
  }
  if (lane == 0) pre[0] = 0;
  if (a.cnt && __ballot(over)) {
    if (lane == 0) {
      if (a.thr_fb) a.thr_out[orow] = a.thr_fb[orow];
      else a.flag_list[atomicAdd(a.flag_cnt, 1)] = (int32_t)orow;
    }
    return;
  }
  const int total = carry;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  Excl ex;
  ex.init(a.ex_ptr, a.ex_col, a.ex_base, a.uid ? a.uid[orow] : orow);
  uint64_t key[KC];
#pragma unroll
  for (int q = 0; q < KC; ++q) key[q] = 0ull;
  int g = 0;  // this lane's current region (its candidate indices only grow)
  for (int e0 = 0; e0 < total; e0 += 64 * kMergeBatch) {
    int ci[kMergeBatch];
    float cs[kMergeBatch];
#pragma unroll
    for (int b = 0; b < kMergeBatch; ++b) {
      const int e = e0 + 64 * b + lane;
      ci[b] = INT32_MAX;
      cs[b] = 0.f;
      if (e < total) {
        while (pre[g + 1] <= e) ++g;
        const int64_t o = base + (int64_t)g * a.cap + (e - pre[g]);
        ci[b] = a.pi[o];
        cs[b] = a.ps[o];
      }
    }
#pragma unroll
    for (int b = 0; b < kMergeBatch; ++b) {
      const int i = ci[b];
      if (i == INT32_MAX) continue;
      const uint64_t kk = ((uint64_t)fr_ord(cs[b]) << 32) | (uint32_t)(~(uint32_t)i);
      if (kk > key[KC - 1] && !ex.test(i)) {
        uint64_t x = kk;
#pragma unroll
        for (int q = 0; q < KC; ++q) {
          const uint64_t cur = key[q];
          const bool gt = x > cur;
          key[q] = gt ? x : cur;
          x = gt ? cur : x;
        }
      }
    }
  }
  for (int j = 0; j < a.k; ++j) {
    uint64_t best = key[0];
    int bl = lane;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const uint64_t ob = __shfl_xor(best, off, 64);
      const int ol = __shfl_xor(bl, off, 64);
      if (ob > best) {
        best = ob;
        bl = ol;
      }
    }
    if (lane == bl) {  // pop the head
#pragma unroll
      for (int q = 0; q < KC - 1; ++q) key[q] = key[q + 1];
      key[KC - 1] = 0ull;
    }
    const bool valid = best != 0ull;
    const float bs = valid ? fr_unord((uint32_t)(best >> 32)) : -INFINITY;
    const int bi = valid ? (int)(~(uint32_t)best) : -1;
    if (lane == 0) {
      if (a.thr_out) {
        if (j == a.k - 1) a.thr_out[orow] = bs;
      } else {
        a.out_s[orow * a.k + j] = bs;
        a.out_i[orow * a.k + j] = (int64_t)bi;
        if (a.hits) {
          bool hit = false;
          if (valid) {
            const int64_t row = a.uid ? a.uid[orow] : orow;
            hit = in_csr_row(a.t_col, a.t_ptr[row], a.t_ptr[row + 1], a.t_base + bi);
          }
          a.hits[orow * a.k + j] = hit ? 1 : 0;
        }
      }
    }
  }
}

hipError_t launch_merge(const MergeArgs& m, unsigned blocks, hipStream_t s) {
  if (m.n_regions > kMergeMaxRegions) return hipErrorInvalidValue;  // (split_plan keeps <= 64 splits)
  auto kern = m.k <= 10 ? topk_merge_kernel<10> : (m.k <= 20 ? topk_merge_kernel<20> : topk_merge_kernel<32>);
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, s, m);
  return hipGetLastError();
}

__global__ void topk_zero_kernel(int32_t* p) {
  if (threadIdx.x == 0) p[0] = 0;
}

template <typename T, int D, int MODE>
hipError_t launch_score_t(const ScoreArgs& a, hipStream_t s) {
  void (*kern)(ScoreArgs);
  if constexpr (MODE == kAppend) {
    kern = topk_score_kernel<T, D, 1, kAppend, 2>;
  } else if constexpr (MODE == kGmax) {
    kern = topk_score_kernel<T, D, 1, kGmax, 2>;
  } else {
    kern = a.k <= 10 ? topk_score_kernel<T, D, 10, kList, 1>
                     : (a.k <= 20 ? topk_score_kernel<T, D, 20, kList, 1> : topk_score_kernel<T, D, 32, kList, 1>);
  }
  hipLaunchKernelGGL(kern, dim3((unsigned)(a.n_utiles * a.n_splits)), dim3(kThreads), 0, s, a);
  return hipGetLastError();
}

template <int MODE>
hipError_t launch_score(int dtype, int d, const ScoreArgs& a, hipStream_t s) {
  if (dtype == FR_BF16) {
    if (d == 256) return launch_score_t<uint16_t, 256, MODE>(a, s);
    if (d == 128) return launch_score_t<uint16_t, 128, MODE>(a, s);
    return launch_score_t<uint16_t, 64, MODE>(a, s);
  }
  if (d == 128) return launch_score_t<float, 128, MODE>(a, s);
  return launch_score_t<float, 64, MODE>(a, s);
}

void split_plan(int64_t n_users, int64_t n_items, int* n_splits, int64_t* span) {
  const int64_t n_utiles = fr::ceil_div(n_users, kUsersPerWG);
  int64_t ns = std::max<int64_t>(1, fr::ceil_div(2 * fr::kNumCU, n_utiles));
  ns = std::min<int64_t>(ns, 64);
  ns = std::min<int64_t>(ns, std::max<int64_t>(1, n_items / (8 * kTile)));  // >= 8 blocks per split
  int64_t sp = fr::align_up(fr::ceil_div(n_items, ns), 2 * kTile);
  *span = sp;
  *n_splits = (int)fr::ceil_div(n_items, sp);
}

constexpr int64_t kSampledMinItems = 32768;  // below this: one exact LIST pass
#ifndef FR_TOPK_SUB
#define FR_TOPK_SUB 16
#endif
constexpr int64_t kSubRatio = FR_TOPK_SUB;   // sub-sample stride / sample stride
#ifndef FR_TOPK_GMAX
#define FR_TOPK_GMAX 1
#endif
// thresholds from the sample's per-lane position maxima (one GMAX pass + merge) instead of the
// two-level LIST / APPEND scheme
constexpr bool kTopkGmax = FR_TOPK_GMAX != 0;
#ifndef FR_TOPK_GSPLIT
#define FR_TOPK_GSPLIT 1
#endif
constexpr int kGmaxSplitMul = FR_TOPK_GSPLIT;  // the GMAX pass's splits: the plan's times this (<= 64)
#ifndef FR_TOPK_SCAP
#define FR_TOPK_SCAP 16
#endif
constexpr int64_t kSampleStrideCap = FR_TOPK_SCAP;  // the sample's stride at >= 1M items

// The launch plan and the workspace carve-up (identical in the size query and the call).
struct Plan {
  bool sampled, gmax;
  int64_t stride, n_sample, stride0, n_sub;
  int ns0, ns1, ns2, cap1, cap;
  int64_t span0, span1, span2;
  int64_t off_l0, off_thr1, off_cs1, off_ci1, off_cc1, off_g;
  int64_t off_l1, off_thr, off_cs, off_ci, off_cc, off_flag, off_l2, total;
};

// region capacity: candidates per user ~ NegBinomial(k, 1/ratio) (mean k * ratio) over n_regions;
// room for ~4x the mean plus the long tail of small k (overflow only costs time)
int region_cap(int k, int64_t ratio, int n_regions) {
  return (int)std::min<int64_t>(1 << 16, std::max<int64_t>(256, (4 * k + 32) * ratio / n_regions));
}

Plan make_plan(int64_t n_users, int64_t n_items, int k) {
  Plan p{};
  p.sampled = n_items >= kSampledMinItems;
  split_plan(n_users, n_items, &p.ns2, &p.span2);
  auto take = [&](int64_t bytes) { const int64_t o = p.total; p.total += fr::align_up(bytes, 256); return o; };
  if (!p.sampled) {
    p.off_l1 = take(n_users * p.ns2 * 2 * (int64_t)k * 8);
    return p;
  }
  // thresholds in two levels: the exact top-k of a sub-sample (every stride0-th item, LIST) bounds
  // an APPEND pass over the sample (every stride-th item) whose merged top-k gives the threshold of
  // the APPEND pass over all items (~k * stride candidates per user)
  p.stride = std::min<int64_t>(kSampleStrideCap, std::max<int64_t>(2, n_items * kSampleStrideCap / (16 * 65536)));
  p.n_sample = fr::ceil_div(n_items, p.stride);
  p.stride0 = p.stride * kSubRatio;
  p.n_sub = fr::ceil_div(n_items, p.stride0);
  split_plan(n_users, p.n_sub, &p.ns0, &p.span0);
  split_plan(n_users, p.n_sample, &p.ns1, &p.span1);
  p.cap1 = region_cap(k, kSubRatio, 2 * p.ns1);
  p.cap = region_cap(k, p.stride, 2 * p.ns2);
  const int64_t nreg1 = n_users * p.ns1 * 2;
  // the position-group maxima need enough entries per user (16 per split) to bound the k-th best
  // tightly; with few splits (>= 128k users) the two-level scheme is kept
  p.gmax = kTopkGmax && 16 * p.ns1 >= 3 * k;
  if (p.gmax && kGmaxSplitMul > 1) {  // more splits: more maxima per user (a tighter bound)
    const int64_t ns = std::min<int64_t>(64, (int64_t)p.ns1 * kGmaxSplitMul);
    p.span1 = fr::align_up(fr::ceil_div(p.n_sample, ns), 2 * kTile);
    p.ns1 = (int)fr::ceil_div(p.n_sample, p.span1);
  }
  const int64_t nreg1g = n_users * p.ns1 * 2;
  if (p.gmax) {
    p.off_g = take(nreg1g * 8 * 8);  // [region][8] scores, then [region][8] items
  } else {
    p.off_l0 = take(n_users * p.ns0 * 2 * (int64_t)k * 8);
    p.off_thr1 = take(n_users * 4);
    p.off_cs1 = take(nreg1 * p.cap1 * 4);
    p.off_ci1 = take(nreg1 * p.cap1 * 4);
    p.off_cc1 = take(nreg1 * 4);
  }
  p.off_thr = take(n_users * 4);
  const int64_t nreg = n_users * p.ns2 * 2;
  p.off_cs = take(nreg * p.cap * 4);
  p.off_ci = take(nreg * p.cap * 4);
  p.off_cc = take(nreg * 4);
  p.off_flag = take((n_users + 1) * 4);
  p.off_l2 = take(n_users * p.ns2 * 2 * (int64_t)k * 8);
  p.off_l1 = p.off_l2;  // (unused)
  return p;
}

}  // namespace

extern "C" int64_t fr_topk_workspace(int64_t n_users, int64_t n_items, int k) {
  if (n_users <= 0 || n_items <= 0 || k <= 0) return 0;
  return make_plan(n_users, n_items, k).total + 256;
}

extern "C" int fr_topk_scores(const void* d_U, int64_t ldu, int64_t n_users, const void* d_I, int64_t ldi,
                              int64_t n_items, int d, int dtype, int k, const int64_t* d_uid,
                              const int64_t* d_ex_ptr, const int32_t* d_ex_col, int64_t ex_base,
                              const int64_t* d_test_ptr, const int32_t* d_test_col, int64_t test_base,
                              float* d_out_scores, int64_t* d_out_items, uint8_t* d_hits, void* d_workspace,
                              int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(n_users >= 0 && n_items >= 0, "negative size");
  if (n_users == 0) return FR_OK;
  FR_REQUIRE(n_items > 0 && n_items < INT32_MAX, "n_items out of range");
  FR_REQUIRE(n_users < INT32_MAX / 2, "n_users out of range");
  FR_REQUIRE(k >= 1 && k <= kKMax, "k must be in [1, 32]");
  FR_REQUIRE(d_U && d_I && d_out_scores && d_out_items, "null pointer");
  FR_REQUIRE(!d_ex_ptr || d_ex_col, "exclusion CSR incomplete");
  FR_REQUIRE(!d_hits || (d_test_ptr && d_test_col), "hits need the held-out CSR");
  FR_REQUIRE(dtype == FR_BF16 || dtype == FR_F32, "dtype must be FR_F32 or FR_BF16");
  if (dtype == FR_BF16) FR_REQUIRE(d == 64 || d == 128 || d == 256, "bf16 supports d in {64, 128, 256}");
  else FR_REQUIRE(d == 64 || d == 128, "fp32 supports d in {64, 128}");
  const int es = dtype == FR_BF16 ? 2 : 4;
  FR_REQUIRE(fr::aligned16(d_U) && fr::aligned16(d_I) && (ldu * es) % 16 == 0 && (ldi * es) % 16 == 0 &&
                 ldu >= d && ldi >= d,
             "tables must be 16-B aligned with 16-B row strides");
  const int64_t need = fr_topk_workspace(n_users, n_items, k);
  FR_REQUIRE(d_workspace && workspace_bytes >= need && fr::aligned16(d_workspace),
             "workspace too small (need " + std::to_string(need) + " bytes)");
  const Plan p = make_plan(n_users, n_items, k);
  char* ws = reinterpret_cast<char*>(d_workspace);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const int n_utiles = (int)fr::ceil_div(n_users, kUsersPerWG);
  const unsigned merge_blocks = (unsigned)fr::ceil_div(n_users, 4);

  ScoreArgs sa{};
  sa.Uq = d_U; sa.ldu = ldu; sa.n_users = n_users;
  sa.uid = d_uid; sa.ex_ptr = d_ex_ptr; sa.ex_col = d_ex_col; sa.ex_base = ex_base;
  sa.k = k; sa.n_utiles = n_utiles;
  MergeArgs ma{};
  ma.n_users = n_users; ma.k = k; ma.uid = d_uid;
  ma.t_ptr = d_test_ptr; ma.t_col = d_test_col; ma.t_base = test_base;
  ma.out_s = d_out_scores; ma.out_i = d_out_items; ma.hits = d_hits;
  hipError_t e;

  // exact LIST pass over `items` (stride item_mul) then a merge into the outputs or thresholds.
  // A threshold pass leaves the exclusion to its merge: the k-th best admissible entry of the
  // union of the lanes' unfiltered top-k lists is still k admissible items' worst -- a lower bound
  // of the user's k-th best admissible score (-inf if fewer remain) -- and the LIST kernel then
  // never stalls its wave on a candidate's CSR-row bisection.
  auto list_pass = [&](const void* It, int64_t ld, int64_t n_it, int64_t mul, int ns, int64_t span, char* lists,
                       const int32_t* urows, const int32_t* d_nu, float* thr_out) -> hipError_t {
    ScoreArgs l = sa;
    l.It = It; l.ldi = ld; l.n_items = n_it; l.item_mul = mul; l.n_splits = ns; l.span = span;
    l.urows = urows; l.d_nu = d_nu;
    if (thr_out) l.ex_ptr = nullptr;
    l.ls = reinterpret_cast<float*>(lists);
    l.li = reinterpret_cast<int32_t*>(lists + n_users * ns * 2 * (int64_t)k * 4);
    hipError_t err = launch_score<kList>(dtype, d, l, s);
    if (err != hipSuccess) return err;
    MergeArgs m = ma;
    m.ps = l.ls; m.pi = l.li; m.cnt = nullptr; m.cap = k; m.n_regions = 2 * ns;
    m.d_nu = d_nu; m.urows = urows; m.thr_out = thr_out;
    if (thr_out) { m.ex_ptr = d_ex_ptr; m.ex_col = d_ex_col; m.ex_base = ex_base; }
    return launch_merge(m, merge_blocks, s);
  };

  if (!p.sampled) {
    e = list_pass(d_I, ldi, n_items, 1, p.ns2, p.span2, ws + p.off_l1, nullptr, nullptr, nullptr);
    if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
    return FR_OK;
  }
  FR_REQUIRE(ldi * p.stride0 * es < INT32_MAX, "item row stride too large for the sampled passes");
  float* thr = reinterpret_cast<float*>(ws + p.off_thr);
  int32_t* flag_cnt = reinterpret_cast<int32_t*>(ws + p.off_flag);
  int32_t* flag_list = flag_cnt + 1;
  if (p.gmax) {
    // 1-2. the sample's per-lane position-group maxima (distinct items: 8 per lane, split and half),
    //      merged into their k-th best admissible score -- a lower bound of the user's k-th best
    //      (-inf if fewer remain), within ~k^2 / (2 * entries) ranks of the sample's exact one
    ScoreArgs gs = sa;
    gs.It = d_I; gs.ldi = ldi * p.stride; gs.n_items = p.n_sample; gs.item_mul = p.stride;
    gs.n_splits = p.ns1; gs.span = p.span1;
    const int64_t nreg1 = n_users * p.ns1 * 2;
    gs.ls = reinterpret_cast<float*>(ws + p.off_g);
    gs.li = reinterpret_cast<int32_t*>(ws + p.off_g + nreg1 * 8 * 4);
    e = launch_score<kGmax>(dtype, d, gs, s);
    if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
    MergeArgs mg = ma;
    mg.ps = gs.ls; mg.pi = gs.li; mg.cnt = nullptr; mg.cap = 8; mg.n_regions = 2 * p.ns1;
    mg.ex_ptr = d_ex_ptr; mg.ex_col = d_ex_col; mg.ex_base = ex_base;
    mg.thr_out = thr;
    e = launch_merge(mg, merge_blocks, s);
    if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
  } else {
  float* thr1 = reinterpret_cast<float*>(ws + p.off_thr1);
  // 1. a lower bound of every user's k-th best: the exact top-k of every stride0-th item
  e = list_pass(d_I, ldi * p.stride0, p.n_sub, p.stride0, p.ns0, p.span0, ws + p.off_l0, nullptr, nullptr, thr1);
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
  // 2. the sample's scores above it, merged into its exact top-k: the threshold (an overflowed user
  //    keeps the sub-sample's bound -- looser, still below its k-th best)
  ScoreArgs as = sa;
  as.It = d_I; as.ldi = ldi * p.stride; as.n_items = p.n_sample; as.item_mul = p.stride;
  as.n_splits = p.ns1; as.span = p.span1;
  as.thr = thr1; as.cap = p.cap1;
  as.cs = reinterpret_cast<float*>(ws + p.off_cs1);
  as.ci = reinterpret_cast<int32_t*>(ws + p.off_ci1);
  as.cc = reinterpret_cast<int32_t*>(ws + p.off_cc1);
  e = launch_score<kAppend>(dtype, d, as, s);
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
  MergeArgs mt = ma;
  mt.ps = as.cs; mt.pi = as.ci; mt.cnt = as.cc; mt.cap = p.cap1; mt.n_regions = 2 * p.ns1;
  mt.ex_ptr = d_ex_ptr; mt.ex_col = d_ex_col; mt.ex_base = ex_base;
  mt.thr_out = thr; mt.thr_fb = thr1;
  e = launch_merge(mt, merge_blocks, s);
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
  }
  // 3. all items: GEMM + threshold, candidates appended
  ScoreArgs ap = sa;
  ap.It = d_I; ap.ldi = ldi; ap.n_items = n_items; ap.item_mul = 1; ap.n_splits = p.ns2; ap.span = p.span2;
  ap.thr = thr; ap.cap = p.cap;
  ap.cs = reinterpret_cast<float*>(ws + p.off_cs);
  ap.ci = reinterpret_cast<int32_t*>(ws + p.off_ci);
  ap.cc = reinterpret_cast<int32_t*>(ws + p.off_cc);
  e = launch_score<kAppend>(dtype, d, ap, s);
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
  // 4. merge the candidates; overflowed users are listed for the exact pass
  hipLaunchKernelGGL(topk_zero_kernel, dim3(1), dim3(64), 0, s, flag_cnt);
  FR_LAUNCH_CHECK();
  MergeArgs mc = ma;
  mc.ps = ap.cs; mc.pi = ap.ci; mc.cnt = ap.cc; mc.cap = p.cap; mc.n_regions = 2 * p.ns2;
  mc.flag_list = flag_list; mc.flag_cnt = flag_cnt;
  mc.ex_ptr = d_ex_ptr; mc.ex_col = d_ex_col; mc.ex_base = ex_base;
  e = launch_merge(mc, merge_blocks, s);
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
  // 5. exact LIST pass + merge for the flagged users (grid sized for all; exits when none)
  e = list_pass(d_I, ldi, n_items, 1, p.ns2, p.span2, ws + p.off_l2, flag_list, flag_cnt, nullptr);
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
  return FR_OK;
}
