// Batch assembly for the training step: the triple batch and the [pos; neg] item-side features in
// one launch.
//
// Replaces, per step, TrainDataLoader.__getitem__ x B + default_collate (utils/dataloader.py:50-115)
// as the engine runs them on the device: the DeviceFeed gathers of (u, pos, neg) from the epoch's
// staged permutation and negatives (4 index_select + 1 add), then the LazyBatch gathers of the
// item features of [pos; neg] (torch.cat + ingredient codes / counts / health multi-hot gathers)
// and HealthRec's key-padding mask (codes == pad) as the additive float mask the encoder takes.  Ten small launches -> one.
//
// Mapping: one thread per (batch row j in [0, 2B), column c in [0, W)), W = max(L, H, 1); every
// thread resolves its row's item id itself (two cached loads), so there is no cross-block
// dependency.  Column 0 also writes the row's scalars (item id, count, u / pos / neg).
// HBM bytes per launch: ~2B (L*8 + L + 8 + H*4) written + the same gathered -- a few hundred KB;
// latency-bound, not a roofline kernel.
#include "fr_common.h"

#include <algorithm>

namespace {

struct FeedArgs {
  // feed mode (perm != nullptr): batch `cursor` of the staged epoch
  const int64_t* perm;    // [E] sample order
  const int64_t* users;   // [E] positive-list users
  const int64_t* items;   // [E] positive-list items
  const int64_t* negs;    // [E] negatives in sample order
  const int64_t* cursor;  // device batch index
  int64_t* u;             // [B] out (feed mode)
  int64_t* p;             // [B] out (feed mode) / in (plain mode)
  int64_t* n;             // [B] out (feed mode) / in (plain mode)
  // item-side features of rows [p ; n]
  const int64_t* codes;   // [I, L]
  const int64_t* nums;    // [I]
  const float* health;    // [I, H] or null
  int64_t n_items;
  int L, H, W;
  int64_t pad;            // padding ingredient id (mask = codes == pad)
  int64_t* pn;            // [2B]
  int64_t* out_codes;     // [2B, L]
  int64_t* out_nums;      // [2B]
  float* out_health;      // [2B, H] or null
  float* out_kpm;         // [2B, L] additive key mask (-inf at padding, 0 elsewhere) or null
  int32_t* err;           // sticky flag: set to 1 when an item id was out of range (or null)
};

__global__ __launch_bounds__(256) void feed_batch_kernel(FeedArgs a, int64_t B) {
  const int64_t total = 2 * B * a.W;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t j = t / a.W;
    const int c = (int)(t - j * a.W);
    const bool is_pos = j < B;
    const int64_t i = is_pos ? j : j - B;
    int64_t item, user = 0;
    if (a.perm) {
      const int64_t pos = a.cursor[0] * B + i;
      if (is_pos) {
        const int64_t k = a.perm[pos];
        item = a.items[k];
        user = a.users[k];
      } else {
        item = a.negs[pos];
      }
    } else {
      item = is_pos ? a.p[i] : a.n[i];
    }
    // ids come from the sampler (valid by construction); a corrupt id must not fault the GPU: it is
    // replaced by item 0 in EVERY output (p / n included, so they agree with pn and the features)
    // and reported through the sticky flag the trainer reads at epoch end
    if (item < 0 || item >= a.n_items) {
      item = 0;
      if (c == 0 && a.err) atomicOr(a.err, 1);
    }
    if (a.perm && c == 0) {
      if (is_pos) {
        a.u[i] = user;
        a.p[i] = item;
      } else {
        a.n[i] = item;
      }
    }
    if (c == 0) {
      a.pn[j] = item;
      a.out_nums[j] = a.nums[item];
    }
    if (c < a.L) {
      const int64_t code = a.codes[item * a.L + c];
      a.out_codes[j * a.L + c] = code;
      if (a.out_kpm) a.out_kpm[j * a.L + c] = code == a.pad ? -INFINITY : 0.f;
    }
    if (a.health && c < a.H) a.out_health[j * a.H + c] = a.health[item * a.H + c];
  }
}

}  // namespace

extern "C" int fr_feed_batch(const int64_t* d_perm, const int64_t* d_users, const int64_t* d_items,
                             const int64_t* d_negs, const int64_t* d_cursor, int64_t B, int64_t* d_u, int64_t* d_p,
                             int64_t* d_n, const int64_t* d_codes, int L, const int64_t* d_nums, const float* d_health,
                             int H, int64_t n_items, int64_t pad, int64_t* d_pn, int64_t* d_out_codes,
                             int64_t* d_out_nums, float* d_out_health, float* d_out_kpm, int32_t* d_err,
                             void* stream) {
  FR_REQUIRE(B >= 1 && L >= 1 && L <= 1024 && H >= 0 && H <= 1024 && n_items >= 1, "bad sizes");
  FR_REQUIRE(d_p && d_n && d_codes && d_nums && d_pn && d_out_codes && d_out_nums, "null argument");
  FR_REQUIRE(!d_perm || (d_users && d_items && d_negs && d_cursor && d_u), "feed mode needs perm/users/items/negs/"
             "cursor/u");
  FR_REQUIRE((d_health == nullptr) == (d_out_health == nullptr) && (H == 0) == (d_health == nullptr),
             "health table and output go together (H > 0)");
  FeedArgs a{d_perm, d_users, d_items, d_negs, d_cursor, d_u, d_p, d_n, d_codes, d_nums, d_health, n_items, L, H,
             L > H ? L : (H > 0 ? H : 1), pad, d_pn, d_out_codes, d_out_nums, d_out_health, d_out_kpm, d_err};
  const int64_t total = 2 * B * a.W;
  const int64_t blocks = std::min<int64_t>(fr::ceil_div(total, (int64_t)256), (int64_t)fr::kNumCU * 8);
  hipLaunchKernelGGL(feed_batch_kernel, dim3((unsigned)blocks), dim3(256), 0, reinterpret_cast<hipStream_t>(stream),
                     a, B);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
