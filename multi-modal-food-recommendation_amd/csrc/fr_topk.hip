// Full-sort top-k: user x item scores on the matrix cores, fused with a running per-user top-k.
//
// Replaces, for a batch of users, full_sort_predict's  scores = user_all[u] @ item_all.T
// (common/abstract_recommender.py:39-50, the MMRec dense form) followed by
// torch.topk(scores, max(topk)) in Trainer.evaluate (common/trainer.py:476-503) and
// TopKEvaluator.collect (utils/topk_evaluator.py:45-66), optionally masking each user's training
// items first (the MMRec full-sort convention), and the hit test `i in pos_items` of
// TopKEvaluator.evaluate (topk_evaluator.py:104-107).  The [users x items] score matrix is never
// written: at 32k users x 1M items it would be 128 GB of fp32.
//
// Score kernel (per workgroup: 8 waves x 32 users = 256 users, an item range of the split):
//   * MFMA with A = a 32-item tile (from LDS) and B = the wave's 32 users (held in VGPRs for the
//     whole kernel): bf16 tables -> v_mfma_f32_32x32x16_bf16 (K = 16 per instruction, fp32
//     accumulate); fp32 tables -> v_mfma_f32_32x32x2_f32 (exact fp32 products, K = 2).
//   * the 32x32 accumulator has the user on the lane (col = lane & 31) and 16 items in the
//     registers, so each lane filters its own user's scores against that user's current k-th
//     best (a register), and only candidates touch the user's sorted top-k list in LDS.
//   * item tiles are staged global -> registers -> LDS (double buffer, one barrier per tile) with
//     a 16-B chunk XOR swizzle so the A-fragment ds_read_b128 of 16 lanes hits 16 distinct bank
//     slots; item rows are read once per workgroup (256 users), users once per kernel.
//   * order is total and deterministic: score descending, item id ascending on ties (the order
//     of a stable descending argsort), independent of tiling and split count.
//   * XCD-aware block order: the workgroups of one XCD take consecutive (user tile, split)
//     ids, so the user tiles sharing an item range share that XCD's L2.
// Merge kernel: one wave per user merges the splits' sorted lists (k rounds of a wave arg-max)
// and flags hits against the user's held-out items.
#include "fr_bf16.h"

#include <algorithm>
#include <cmath>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kWaves = 8;
constexpr int kThreads = kWaves * 64;
constexpr int kUsersPerWG = kWaves * 32;
constexpr int kTile = 32;      // items per staged tile
constexpr int kKMax = 32;      // largest k

template <typename T, int D>
struct Cfg {
  static constexpr int RB = D * (int)sizeof(T);           // bytes per row
  static constexpr int CPR = RB / 16;                       // 16-B chunks per row
  static constexpr bool BF = sizeof(T) == 2;
  static constexpr int KS = BF ? D / 16 : D / 2;            // MFMA k-steps
  static constexpr int STAGE = kTile * RB;                  // bytes per staged tile
  static constexpr int G = CPR >= 16 ? 1 : 16 / CPR;        // rows sharing one 256-B bank row
  static constexpr int SWM = (CPR >= 16 ? 16 : CPR) - 1;
  static constexpr int CH = (kTile * CPR + kThreads - 1) / kThreads;  // staged chunks per thread
  static constexpr int LDS = 2 * STAGE + kUsersPerWG * kKMax * 8;
};

template <typename T, int D>
__device__ __forceinline__ int swz(int r, int c) {
  using C = Cfg<T, D>;
  return c ^ ((r / C::G) & C::SWM);
}

__device__ __forceinline__ bool better(float s, int i, float t, int ti) {
  return s > t || (s == t && i < ti);
}

__device__ __forceinline__ bool excluded(const int64_t* __restrict__ ex_ptr, const int32_t* __restrict__ ex_col,
                                         int64_t ex_base, int64_t urow, int64_t item) {
  if (!ex_ptr) return false;
  int64_t lo = ex_ptr[urow], hi = ex_ptr[urow + 1];
  const int64_t key = ex_base + item;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int64_t v = ex_col[mid];
    if (v < key) lo = mid + 1;
    else hi = mid;
  }
  return lo < ex_ptr[urow + 1] && (int64_t)ex_col[lo] == key;
}

template <typename T, int D>
__global__ __launch_bounds__(kThreads) void topk_score_kernel(
    const T* __restrict__ Uq, int64_t ldu, int64_t n_users, const T* __restrict__ It, int64_t ldi,
    int64_t n_items, const int64_t* __restrict__ uid, const int64_t* __restrict__ ex_ptr,
    const int32_t* __restrict__ ex_col, int64_t ex_base, int k, int n_splits, int64_t span, int n_utiles,
    float* __restrict__ out_s, int32_t* __restrict__ out_i) {
  using C = Cfg<T, D>;
  __shared__ __attribute__((aligned(16))) char smem[C::LDS];
  float* tks = reinterpret_cast<float*>(smem + 2 * C::STAGE);
  int* tki = reinterpret_cast<int*>(tks + kUsersPerWG * kKMax);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int r = lane & 31, h = lane >> 5;

  // XCD-aware bijective remap (blocks are dispatched round-robin over the 8 XCDs)
  const int total = n_utiles * n_splits;
  const int b = blockIdx.x, xcd = b & 7, q8 = total >> 3, r8 = total & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (b >> 3);
  const int ut = wg % n_utiles, sp = wg / n_utiles;

  const int64_t myu = (int64_t)ut * kUsersPerWG + wave * 32 + r;
  const bool uvalid = myu < n_users;
  const int64_t urow = uvalid ? myu : 0;
  const int64_t exrow = uid ? uid[urow] : urow;
  const int64_t i_lo = (int64_t)sp * span;
  const int64_t i_hi = min(n_items, i_lo + span);
  const int n_tiles = (int)((i_hi - i_lo + kTile - 1) / kTile);

  // B operand: this lane's user, held for the whole kernel
  typedef typename std::conditional<C::BF, bf16x8, float4>::type BFrag;
  constexpr int NB = C::BF ? C::KS : C::KS / 4;
  BFrag bf[NB];
#pragma unroll
  for (int s = 0; s < NB; ++s) {
    if constexpr (C::BF) {
      bf[s] = *reinterpret_cast<const bf16x8*>(reinterpret_cast<const uint16_t*>(Uq) + urow * ldu + 16 * s + 8 * h);
    } else {
      bf[s] = *reinterpret_cast<const float4*>(reinterpret_cast<const float*>(Uq) + urow * ldu + h * (D / 2) + 4 * s);
    }
  }

  // top-k list of this lane's user (both lane halves initialise half of it)
  const int lbase = (wave * 32 + r) * kKMax;
  for (int j = h; j < kKMax; j += 2) {
    tks[lbase + j] = -INFINITY;
    tki[lbase + j] = INT32_MAX;
  }
  float thr = -INFINITY;
  int thr_i = INT32_MAX;

  uint4 stg[C::CH];
  auto load_tile = [&](int t) {
#pragma unroll
    for (int c = 0; c < C::CH; ++c) {
      const int x = tid + c * kThreads;
      stg[c] = make_uint4(0, 0, 0, 0);
      if (x < kTile * C::CPR) {
        const int row = x / C::CPR, cc = x % C::CPR;
        const int64_t item = i_lo + (int64_t)t * kTile + row;
        if (item < i_hi)
          stg[c] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(It) + (item * ldi) * (int64_t)sizeof(T) +
                                                   cc * 16);
      }
    }
  };
  auto store_tile = [&](int buf) {
    char* base = smem + buf * C::STAGE;
#pragma unroll
    for (int c = 0; c < C::CH; ++c) {
      const int x = tid + c * kThreads;
      if (x < kTile * C::CPR) {
        const int row = x / C::CPR, cc = x % C::CPR;
        *reinterpret_cast<uint4*>(base + (row * C::CPR + swz<T, D>(row, cc)) * 16) = stg[c];
      }
    }
  };

  if (n_tiles > 0) {
    load_tile(0);
    store_tile(0);
  }
  __syncthreads();
  if (n_tiles > 1) load_tile(1);

  for (int t = 0; t < n_tiles; ++t) {
    const char* abuf = smem + (t & 1) * C::STAGE;
    f32x16 acc;
#pragma unroll
    for (int j = 0; j < 16; ++j) acc[j] = 0.f;
    if constexpr (C::BF) {
#pragma unroll
      for (int s = 0; s < C::KS; ++s) {
        const bf16x8 a = *reinterpret_cast<const bf16x8*>(abuf + (r * C::CPR + swz<T, D>(r, 2 * s + h)) * 16);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, bf[s], acc, 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int sg = 0; sg < C::KS / 4; ++sg) {
        const float4 a = *reinterpret_cast<const float4*>(abuf + (r * C::CPR + swz<T, D>(r, h * (C::CPR / 2) + sg)) * 16);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.x, bf[sg].x, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.y, bf[sg].y, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.z, bf[sg].z, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.w, bf[sg].w, acc, 0, 0, 0);
      }
    }
    // this lane's 16 scores: user myu, items ib + (j&3) + 8(j>>2) + 4h
    const int64_t ib = i_lo + (int64_t)t * kTile + 4 * h;
    bool cand = false;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t item = ib + (j & 3) + 8 * (j >> 2);
      cand |= (item < i_hi) && better(acc[j], (int)item, thr, thr_i);
    }
    cand = cand && uvalid;
    if (__ballot(cand)) {
      for (int hh = 0; hh < 2; ++hh) {
        if (cand && h == hh) {
#pragma unroll
          for (int j = 0; j < 16; ++j) {
            const int64_t item = ib + (j & 3) + 8 * (j >> 2);
            const float s = acc[j];
            if (item < i_hi && better(s, (int)item, thr, thr_i) && !excluded(ex_ptr, ex_col, ex_base, exrow, item)) {
              int pos = k - 1;
              while (pos > 0) {
                const float ps = tks[lbase + pos - 1];
                const int pi = tki[lbase + pos - 1];
                if (better(ps, pi, s, (int)item)) break;
                tks[lbase + pos] = ps;
                tki[lbase + pos] = pi;
                --pos;
              }
              tks[lbase + pos] = s;
              tki[lbase + pos] = (int)item;
              thr = tks[lbase + k - 1];
              thr_i = tki[lbase + k - 1];
            }
          }
        }
        // the list is private to this wave: program order makes the other half see the inserts
        thr = tks[lbase + k - 1];
        thr_i = tki[lbase + k - 1];
      }
    }
    if (t + 1 < n_tiles) store_tile((t + 1) & 1);
    __syncthreads();
    if (t + 2 < n_tiles) load_tile(t + 2);
  }

  if (uvalid) {
    const int64_t o = (myu * n_splits + sp) * (int64_t)k;
    for (int j = h; j < k; j += 2) {
      out_s[o + j] = tks[lbase + j];
      out_i[o + j] = tki[lbase + j];
    }
  }
}

// One wave per user: k rounds of a wave arg-max over the heads of the n_splits sorted lists.
__global__ __launch_bounds__(256) void topk_merge_kernel(
    const float* __restrict__ ps, const int32_t* __restrict__ pi, int64_t n_users, int n_splits, int k,
    const int64_t* __restrict__ uid, const int64_t* __restrict__ t_ptr, const int32_t* __restrict__ t_col,
    int64_t t_base, float* __restrict__ out_s, int64_t* __restrict__ out_i, uint8_t* __restrict__ hits) {
  const int lane = threadIdx.x & 63;
  const int64_t u = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (u >= n_users) return;
  const int64_t base = u * n_splits * (int64_t)k;
  int hp = 0;
  for (int j = 0; j < k; ++j) {
    float s = -INFINITY;
    int i = INT32_MAX;
    if (lane < n_splits && hp < k) {
      s = ps[base + (int64_t)lane * k + hp];
      i = pi[base + (int64_t)lane * k + hp];
    }
    float bs = s;
    int bi = i, bl = lane;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
      const float os = __shfl_xor(bs, off, 64);
      const int oi = __shfl_xor(bi, off, 64);
      const int ol = __shfl_xor(bl, off, 64);
      if (better(os, oi, bs, bi) || (os == bs && oi == bi && ol < bl)) {
        bs = os;
        bi = oi;
        bl = ol;
      }
    }
    if (lane == bl) ++hp;
    if (lane == 0) {
      const bool valid = bi != INT32_MAX;
      out_s[u * k + j] = valid ? bs : -INFINITY;
      out_i[u * k + j] = valid ? (int64_t)bi : -1;
      if (hits) hits[u * k + j] = valid && excluded(t_ptr, t_col, t_base, uid ? uid[u] : u, bi) ? 1 : 0;
    }
  }
}

template <typename T, int D>
hipError_t launch_score(const void* Uq, int64_t ldu, int64_t n_users, const void* It, int64_t ldi, int64_t n_items,
                        const int64_t* uid, const int64_t* ex_ptr, const int32_t* ex_col, int64_t ex_base, int k,
                        int n_splits, int64_t span, float* ps, int32_t* pi, hipStream_t s) {
  const int n_utiles = (int)fr::ceil_div(n_users, kUsersPerWG);
  hipLaunchKernelGGL((topk_score_kernel<T, D>), dim3((unsigned)(n_utiles * n_splits)), dim3(kThreads), 0, s,
                     reinterpret_cast<const T*>(Uq), ldu, n_users, reinterpret_cast<const T*>(It), ldi, n_items, uid,
                     ex_ptr, ex_col, ex_base, k, n_splits, span, n_utiles, ps, pi);
  return hipGetLastError();
}

void split_plan(int64_t n_users, int64_t n_items, int* n_splits, int64_t* span) {
  const int64_t n_utiles = fr::ceil_div(n_users, kUsersPerWG);
  int64_t ns = std::max<int64_t>(1, fr::ceil_div(2 * fr::kNumCU, n_utiles));
  ns = std::min<int64_t>(ns, 64);
  ns = std::min<int64_t>(ns, std::max<int64_t>(1, n_items / (4 * kTile)));  // >= 4 tiles per split
  int64_t sp = fr::align_up(fr::ceil_div(n_items, ns), kTile);
  *span = sp;
  *n_splits = (int)fr::ceil_div(n_items, sp);
}

}  // namespace

extern "C" int64_t fr_topk_workspace(int64_t n_users, int64_t n_items, int k) {
  if (n_users <= 0 || n_items <= 0 || k <= 0) return 0;
  int ns;
  int64_t span;
  split_plan(n_users, n_items, &ns, &span);
  return n_users * ns * (int64_t)k * 8 + 256;
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
  FR_REQUIRE(k >= 1 && k <= kKMax, "k must be in [1, 32]");
  FR_REQUIRE(d_U && d_I && d_out_scores && d_out_items, "null pointer");
  FR_REQUIRE(!d_ex_ptr || d_ex_col, "exclusion CSR incomplete");
  FR_REQUIRE(!d_hits || (d_test_ptr && d_test_col), "hits need the held-out CSR");
  FR_REQUIRE(dtype == FR_BF16 || dtype == FR_F32, "dtype must be FR_F32 or FR_BF16");
  const int es = dtype == FR_BF16 ? 2 : 4;
  FR_REQUIRE(fr::aligned16(d_U) && fr::aligned16(d_I) && (ldu * es) % 16 == 0 && (ldi * es) % 16 == 0 &&
                 ldu >= d && ldi >= d,
             "tables must be 16-B aligned with 16-B row strides");
  const int64_t need = fr_topk_workspace(n_users, n_items, k);
  FR_REQUIRE(d_workspace && workspace_bytes >= need && fr::aligned16(d_workspace),
             "workspace too small (need " + std::to_string(need) + " bytes)");
  int ns;
  int64_t span;
  split_plan(n_users, n_items, &ns, &span);
  float* ps = reinterpret_cast<float*>(d_workspace);
  int32_t* pi = reinterpret_cast<int32_t*>(ps + n_users * ns * (int64_t)k);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e;
  if (dtype == FR_BF16) {
    if (d == 256) e = launch_score<uint16_t, 256>(d_U, ldu, n_users, d_I, ldi, n_items, d_uid, d_ex_ptr, d_ex_col, ex_base, k, ns, span, ps, pi, s);
    else if (d == 128) e = launch_score<uint16_t, 128>(d_U, ldu, n_users, d_I, ldi, n_items, d_uid, d_ex_ptr, d_ex_col, ex_base, k, ns, span, ps, pi, s);
    else if (d == 64) e = launch_score<uint16_t, 64>(d_U, ldu, n_users, d_I, ldi, n_items, d_uid, d_ex_ptr, d_ex_col, ex_base, k, ns, span, ps, pi, s);
    else return fr::fail(FR_ENOTSUP, "fr_topk_scores: bf16 supports d in {64, 128, 256}");
  } else {
    if (d == 64) e = launch_score<float, 64>(d_U, ldu, n_users, d_I, ldi, n_items, d_uid, d_ex_ptr, d_ex_col, ex_base, k, ns, span, ps, pi, s);
    else if (d == 128) e = launch_score<float, 128>(d_U, ldu, n_users, d_I, ldi, n_items, d_uid, d_ex_ptr, d_ex_col, ex_base, k, ns, span, ps, pi, s);
    else return fr::fail(FR_ENOTSUP, "fr_topk_scores: fp32 supports d in {64, 128}");
  }
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_topk_scores: ") + hipGetErrorString(e));
  hipLaunchKernelGGL(topk_merge_kernel, dim3((unsigned)fr::ceil_div(n_users, 4)), dim3(256), 0, s, ps, pi, n_users,
                     ns, k, d_uid, d_test_ptr, d_test_col, test_base, d_out_scores, d_out_items, d_hits);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
