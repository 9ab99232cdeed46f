// Host-side negative sampler: numpy's legacy MT19937 stream and masked-rejection bounded ints,
// exclusion by binary search in per-user sorted CSR lists (reference utils/dataloader.py:40-48,
// 145-151).  Host code only (no HIP): also built with -fsanitize=address,undefined (make asan).
#include <algorithm>
#include <cstdint>
#include <string>
#include <vector>

#include "fr_engine.h"

namespace fr {
void set_error(const std::string& msg);  // fr_error.cpp
}  // namespace fr

// ------------------------------------------------------------------------------------------
// MT19937 exactly as numpy's legacy RandomState (randomkit / numpy/random/src/mt19937).
// ------------------------------------------------------------------------------------------
namespace {

constexpr int kN = 624;
constexpr int kM = 397;
constexpr uint32_t kMatrixA = 0x9908b0dfu;
constexpr uint32_t kUpper = 0x80000000u;
constexpr uint32_t kLower = 0x7fffffffu;

struct MT {
  uint32_t* key;
  int32_t* pos;

  void gen() {
    int i;
    uint32_t y;
    for (i = 0; i < kN - kM; ++i) {
      y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + kM] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    for (; i < kN - 1; ++i) {
      y = (key[i] & kUpper) | (key[i + 1] & kLower);
      key[i] = key[i + (kM - kN)] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    }
    y = (key[kN - 1] & kUpper) | (key[0] & kLower);
    key[kN - 1] = key[kM - 1] ^ (y >> 1) ^ (-(y & 1u) & kMatrixA);
    *pos = 0;
  }

  uint32_t next32() {
    if (*pos >= kN) gen();
    uint32_t y = key[(*pos)++];
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
  }

  uint64_t next64() {
    const uint64_t hi = next32();
    return (hi << 32) | next32();
  }

  // RandomState.randint(high) for 0 < high: masked rejection sampling on [0, high-1]
  // (numpy/random/_bounded_integers.pyx.in: _rand_int64 -> random_bounded_uint64_fill, use_masked)
  int64_t bounded(uint64_t rng) {
    if (rng == 0) return 0;
    uint64_t mask = rng;
    mask |= mask >> 1;
    mask |= mask >> 2;
    mask |= mask >> 4;
    mask |= mask >> 8;
    mask |= mask >> 16;
    mask |= mask >> 32;
    if (rng <= 0xffffffffull) {
      if (rng == 0xffffffffull) return (int64_t)next32();
      const uint32_t m32 = (uint32_t)mask;
      uint32_t v;
      while ((v = (next32() & m32)) > (uint32_t)rng) {
      }
      return (int64_t)v;
    }
    uint64_t v;
    while ((v = (next64() & mask)) > rng) {
    }
    return (int64_t)v;
  }
};

inline bool in_sorted(const int64_t* items, int64_t lo, int64_t hi, int64_t x) {
  return std::binary_search(items + lo, items + hi, x);
}

}  // namespace

extern "C" int fr_sampler_randint(uint32_t* mt_key, int32_t* mt_pos, int64_t high, int64_t n,
                                  int64_t* out) {
  if (!mt_key || !mt_pos || (n > 0 && !out) || high <= 0 || n < 0) {
    fr::set_error("fr_sampler_randint: bad argument");
    return FR_EINVAL;
  }
  MT mt{mt_key, mt_pos};
  for (int64_t i = 0; i < n; ++i) out[i] = mt.bounded((uint64_t)(high - 1));
  return FR_OK;
}

static int sampler_negatives(uint32_t* mt_key, int32_t* mt_pos, int64_t num_items, const int64_t* users_all,
                             int64_t n_pairs, const int64_t* perm, int64_t n, int64_t n_users,
                             const int64_t* excl_ptr, const int64_t* excl_items, const int64_t* excl2_ptr,
                             const int64_t* excl2_items, int64_t* out_neg);

extern "C" int fr_sampler_negatives(uint32_t* mt_key, int32_t* mt_pos, int64_t num_items,
                                    const int64_t* users, int64_t n, int64_t n_users, const int64_t* excl_ptr,
                                    const int64_t* excl_items, const int64_t* excl2_ptr,
                                    const int64_t* excl2_items, int64_t* out_neg) {
  return sampler_negatives(mt_key, mt_pos, num_items, users, n, nullptr, n, n_users, excl_ptr, excl_items, excl2_ptr,
                           excl2_items, out_neg);
}

extern "C" int fr_sampler_negatives_perm(uint32_t* mt_key, int32_t* mt_pos, int64_t num_items,
                                         const int64_t* users, int64_t n_pairs, const int64_t* perm, int64_t n,
                                         int64_t n_users, const int64_t* excl_ptr, const int64_t* excl_items,
                                         const int64_t* excl2_ptr, const int64_t* excl2_items, int64_t* out_neg) {
  if (!perm && n > 0) {
    fr::set_error("fr_sampler_negatives_perm: null perm");
    return FR_EINVAL;
  }
  return sampler_negatives(mt_key, mt_pos, num_items, users, n_pairs, perm, n, n_users, excl_ptr, excl_items,
                           excl2_ptr, excl2_items, out_neg);
}

namespace {

// a CSR row pointer of n_users + 1 entries: starts at 0 and never decreases (so every row's items lie
// inside the [0, ptr[n_users]) items array the caller passed)
bool valid_rowptr(const int64_t* ptr, int64_t n_users) {
  if (ptr[0] != 0) return false;
  for (int64_t u = 0; u < n_users; ++u)
    if (ptr[u + 1] < ptr[u]) return false;
  return true;
}

// true when the user's exclusions (both lists together, any order, duplicates allowed) contain every
// item of [0, num_items): the rejection loop would never end (the reference's loops forever too)
bool covers_every_item(const int64_t* a, int64_t la, const int64_t* b, int64_t lb, int64_t num_items) {
  if (la + lb < num_items) return false;  // pigeonhole: the common case costs one comparison
  std::vector<int64_t> v;
  v.reserve((size_t)(la + lb));
  for (int64_t i = 0; i < la; ++i)
    if (a[i] >= 0 && a[i] < num_items) v.push_back(a[i]);
  for (int64_t i = 0; i < lb; ++i)
    if (b[i] >= 0 && b[i] < num_items) v.push_back(b[i]);
  std::sort(v.begin(), v.end());
  return (int64_t)(std::unique(v.begin(), v.end()) - v.begin()) == num_items;
}

}  // namespace

static int sampler_negatives(uint32_t* mt_key, int32_t* mt_pos, int64_t num_items, const int64_t* users_all,
                             int64_t n_pairs, const int64_t* perm, int64_t n, int64_t n_users,
                             const int64_t* excl_ptr, const int64_t* excl_items, const int64_t* excl2_ptr,
                             const int64_t* excl2_items, int64_t* out_neg) {
  if (!mt_key || !mt_pos || num_items <= 0 || n < 0 || n_pairs < 0 || n_users < 0 ||
      (n > 0 && (!users_all || !out_neg)) || !excl_ptr || !excl_items || (excl2_ptr && !excl2_items)) {
    fr::set_error("fr_sampler_negatives: bad argument");
    return FR_EINVAL;
  }
  if (!valid_rowptr(excl_ptr, n_users) || (excl2_ptr && !valid_rowptr(excl2_ptr, n_users))) {
    fr::set_error("fr_sampler_negatives: exclusion row pointers must start at 0 and not decrease");
    return FR_EINVAL;
  }
  // users[k] = users_all[perm[k]] (the epoch's permutation order) or users_all[k]; every id (and
  // permutation entry) is range-checked before it is used, the prefetch lookahead's included
  struct Users {
    const int64_t* a;
    const int64_t* p;
    int64_t n_pairs, n_users;
    // the user id of draw k, or -1 when perm[k] or the id is out of range
    int64_t operator[](int64_t k) const {
      const int64_t j = p ? p[k] : k;
      if (j < 0 || j >= n_pairs) return -1;
      const int64_t u = a[j];
      return (u >= 0 && u < n_users) ? u : -1;
    }
  } users{users_all, perm, n_pairs, n_users};
  MT mt{mt_key, mt_pos};
  const uint64_t rng = (uint64_t)(num_items - 1);
  // the loop is bound by the cache misses of its exclusion-list lookups (users in permutation order):
  // the row pointers are prefetched kPf2 users ahead and the lists' first lines kPf1 ahead (results
  // unchanged: the draws and tests are the same, in the same order)
  constexpr int64_t kPf1 = 8, kPf2 = 16;
  for (int64_t k = 0; k < n; ++k) {
    if (perm && k + kPf2 + 8 < n) {
      const int64_t j = perm[k + kPf2 + 8];
      if (j >= 0 && j < n_pairs) __builtin_prefetch(users_all + j);
    }
    if (k + kPf2 < n) {
      const int64_t v = users[k + kPf2];
      if (v >= 0) {
        __builtin_prefetch(excl_ptr + v);
        if (excl2_ptr) __builtin_prefetch(excl2_ptr + v);
      }
    }
    if (k + kPf1 < n) {
      const int64_t v = users[k + kPf1];
      if (v >= 0) {
        const int64_t* ea = excl_items + excl_ptr[v];
        __builtin_prefetch(ea);
        __builtin_prefetch(ea + 8);
        if (excl2_ptr) __builtin_prefetch(excl2_items + excl2_ptr[v]);
      }
    }
    const int64_t u = users[k];
    if (u < 0) {
      fr::set_error(perm && (perm[k] < 0 || perm[k] >= n_pairs)
                        ? "fr_sampler_negatives: permutation entry outside the users array"
                        : "fr_sampler_negatives: user id outside [0, n_users)");
      return FR_ERANGE;
    }
    const int64_t a0 = excl_ptr[u], a1 = excl_ptr[u + 1];
    const int64_t b0 = excl2_ptr ? excl2_ptr[u] : 0, b1 = excl2_ptr ? excl2_ptr[u + 1] : 0;
    if (covers_every_item(excl_items + a0, a1 - a0, excl2_ptr ? excl2_items + b0 : nullptr, b1 - b0, num_items)) {
      fr::set_error("fr_sampler_negatives: user excludes every item");
      return FR_ERANGE;
    }
    int64_t neg;
    for (;;) {
      neg = mt.bounded(rng);
      if (in_sorted(excl_items, a0, a1, neg)) continue;
      if (excl2_ptr && in_sorted(excl2_items, b0, b1, neg)) continue;
      break;
    }
    out_neg[k] = neg;
  }
  return FR_OK;
}
