// Negative sampling on the device for interaction graphs too large for host-side exclusion lists
// (BASELINE config 4: 10M users x 1M items x 200M interactions).
//
// Semantics of the reference's TrainDataLoader.get_random_neg (utils/dataloader.py:145-151): an item
// id uniform over [0, n_items), redrawn while it is one of user u's training items.  The exclusion
// set is the user's row of the bipartite adjacency already resident in HBM (columns = item node ids
// item_base + i, sorted), searched by bisection -- no extra memory.  Draws come from a counter-based
// generator (splitmix64 of seed, triple index, attempt), so a step is reproducible from its seed and
// needs no device RNG state.  After max_tries rejections the last draw is kept (a user who has
// interacted with nearly every item).
#include "fr_common.h"

#include <algorithm>

namespace {

__device__ __forceinline__ uint64_t splitmix64(uint64_t z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__device__ __forceinline__ bool row_contains(const int32_t* __restrict__ col, int64_t lo, int64_t hi, int32_t key) {
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    const int32_t v = col[mid];
    if (v == key) return true;
    if (v < key) lo = mid + 1;
    else hi = mid;
  }
  return false;
}

__global__ __launch_bounds__(256) void neg_csr_kernel(const int64_t* __restrict__ rowptr,
                                                      const int32_t* __restrict__ col,
                                                      const int64_t* __restrict__ users, int64_t B, int64_t n_users,
                                                      int64_t n_items, int64_t item_base, uint64_t seed,
                                                      int max_tries, int64_t* __restrict__ out) {
  const int64_t b = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const int64_t u = users[b];
  const bool valid = u >= 0 && u < n_users;
  const int64_t lo = valid ? rowptr[u] : 0, hi = valid ? rowptr[u + 1] : 0;
  int64_t cand = 0;
  for (int t = 0; t < max_tries; ++t) {
    const uint64_t r = splitmix64(seed ^ splitmix64(((uint64_t)b << 20) ^ (uint64_t)t));
    // multiply-shift maps the top 32 bits uniformly onto [0, n_items) (n_items < 2^31)
    cand = (int64_t)(((r >> 32) * (uint64_t)n_items) >> 32);
    if (!row_contains(col, lo, hi, (int32_t)(item_base + cand))) break;
  }
  out[b] = cand;
}

}  // namespace

extern "C" int fr_sample_negatives_csr(const int64_t* d_rowptr, const int32_t* d_col, int64_t n_users,
                                       const int64_t* d_users, int64_t B, int64_t n_items, int64_t item_base,
                                       uint64_t seed, int max_tries, int64_t* d_out, void* stream) {
  FR_REQUIRE(B >= 0 && n_users > 0 && n_items > 0 && n_items < INT32_MAX && max_tries >= 1, "bad sizes");
  FR_REQUIRE(item_base >= 0 && item_base + n_items < INT32_MAX, "item node ids must fit int32");
  if (B == 0) return FR_OK;
  FR_REQUIRE(d_rowptr && d_col && d_users && d_out, "null pointer");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(neg_csr_kernel, dim3((unsigned)fr::ceil_div(B, 256)), dim3(256), 0, s, d_rowptr, d_col, d_users, B,
                     n_users, n_items, item_base, seed, max_tries, d_out);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
