// Library-level exports: version, error reporting, device query and the host-side negative
// sampler (numpy legacy MT19937 stream, reference utils/dataloader.py:40-48,145-151).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>

#include "fr_engine.h"

namespace fr {
thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace fr

extern "C" int fr_version(void) { return 1; }

extern "C" const char* fr_last_error(void) { return fr::g_last_error.c_str(); }

extern "C" int fr_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

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
                             const int64_t* perm, int64_t n, const int64_t* excl_ptr, const int64_t* excl_items,
                             const int64_t* excl2_ptr, const int64_t* excl2_items, int64_t* out_neg);

extern "C" int fr_sampler_negatives(uint32_t* mt_key, int32_t* mt_pos, int64_t num_items,
                                    const int64_t* users, int64_t n, const int64_t* excl_ptr,
                                    const int64_t* excl_items, const int64_t* excl2_ptr,
                                    const int64_t* excl2_items, int64_t* out_neg) {
  return sampler_negatives(mt_key, mt_pos, num_items, users, nullptr, n, excl_ptr, excl_items, excl2_ptr, excl2_items,
                           out_neg);
}

extern "C" int fr_sampler_negatives_perm(uint32_t* mt_key, int32_t* mt_pos, int64_t num_items,
                                         const int64_t* users, const int64_t* perm, int64_t n,
                                         const int64_t* excl_ptr, const int64_t* excl_items,
                                         const int64_t* excl2_ptr, const int64_t* excl2_items, int64_t* out_neg) {
  if (!perm && n > 0) {
    fr::set_error("fr_sampler_negatives_perm: null perm");
    return FR_EINVAL;
  }
  return sampler_negatives(mt_key, mt_pos, num_items, users, perm, n, excl_ptr, excl_items, excl2_ptr, excl2_items,
                           out_neg);
}

static int sampler_negatives(uint32_t* mt_key, int32_t* mt_pos, int64_t num_items, const int64_t* users_all,
                             const int64_t* perm, int64_t n, const int64_t* excl_ptr, const int64_t* excl_items,
                             const int64_t* excl2_ptr, const int64_t* excl2_items, int64_t* out_neg) {
  if (!mt_key || !mt_pos || num_items <= 0 || n < 0 || (n > 0 && (!users_all || !out_neg)) ||
      !excl_ptr || !excl_items) {
    fr::set_error("fr_sampler_negatives: bad argument");
    return FR_EINVAL;
  }
  // users[k] = users_all[perm[k]] (the epoch's permutation order) or users_all[k]
  struct Users {
    const int64_t* a;
    const int64_t* p;
    int64_t operator[](int64_t k) const { return p ? a[p[k]] : a[k]; }
  } users{users_all, perm};
  MT mt{mt_key, mt_pos};
  const uint64_t rng = (uint64_t)(num_items - 1);
  // the loop is bound by the cache misses of its exclusion-list lookups (users in permutation order):
  // the row pointers are prefetched kPf2 users ahead and the lists' first lines kPf1 ahead (results
  // unchanged: the draws and tests are the same, in the same order)
  constexpr int64_t kPf1 = 8, kPf2 = 16;
  for (int64_t k = 0; k < n; ++k) {
    if (perm && k + kPf2 + 8 < n) __builtin_prefetch(users_all + perm[k + kPf2 + 8]);
    if (k + kPf2 < n && users[k + kPf2] >= 0) {
      __builtin_prefetch(excl_ptr + users[k + kPf2]);
      if (excl2_ptr) __builtin_prefetch(excl2_ptr + users[k + kPf2]);
    }
    if (k + kPf1 < n && users[k + kPf1] >= 0) {
      const int64_t v = users[k + kPf1];
      const int64_t* ea = excl_items + excl_ptr[v];
      __builtin_prefetch(ea);
      __builtin_prefetch(ea + 8);
      if (excl2_ptr) __builtin_prefetch(excl2_items + excl2_ptr[v]);
    }
    const int64_t u = users[k];
    if (u < 0) {
      fr::set_error("fr_sampler_negatives: negative user id");
      return FR_ERANGE;
    }
    const int64_t a0 = excl_ptr[u], a1 = excl_ptr[u + 1];
    const int64_t b0 = excl2_ptr ? excl2_ptr[u] : 0, b1 = excl2_ptr ? excl2_ptr[u + 1] : 0;
    // a user whose exclusions cover every item would loop forever in the reference too
    if ((a1 - a0) >= num_items && std::is_sorted(excl_items + a0, excl_items + a1)) {
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
