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

struct Epi {
  float* Y1; int64_t ldy1;
  float* Y2; int64_t ldy2; float alpha;
  const float* A1; int64_t lda1; float beta1;
  const float* A2; int64_t lda2; float beta2;
};

// write one row's result (float4 slot q of row r) through the fused epilogue
__device__ __forceinline__ void epilogue(const Epi& ep, int64_t r, int q, float4 acc) {
  if (ep.Y1) reinterpret_cast<float4*>(ep.Y1 + r * ep.ldy1)[q] = acc;
  if (ep.Y2) {
    float4 o = f4_scale(ep.alpha, acc);
    if (ep.A1) o = f4_fma(ep.beta1, reinterpret_cast<const float4*>(ep.A1 + r * ep.lda1)[q], o);
    if (ep.A2) o = f4_fma(ep.beta2, reinterpret_cast<const float4*>(ep.A2 + r * ep.lda2)[q], o);
    reinterpret_cast<float4*>(ep.Y2 + r * ep.ldy2)[q] = o;
  }
}

// Gather-accumulate edges [e0, e1) of one unit into acc (slot q of an LPR-lane group).
// Rows wider than LPR float4 slots are handled by the caller's group-uniform slot loop.
template <int LPR>
__device__ __forceinline__ float4 gather_unit(const int32_t* __restrict__ col,
                                              const float* __restrict__ val,
                                              const float4* __restrict__ X4, int64_t ldx4,
                                              int64_t e0, int64_t e1, int lig, int q) {
  // lig = lane index inside the group (edge slot of the cooperative col/val load),
  // q   = float4 slot of the row this lane gathers
  float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t e = e0; e < e1; e += LPR) {
    const int64_t my = e + lig;
    const int64_t last = e1 - 1;
    // lanes past the unit's end re-point at its last edge (cache hit) with weight 0
    const int c = __builtin_nontemporal_load(col + (my < e1 ? my : last));
    const float v = my < e1 ? __builtin_nontemporal_load(val + my) : 0.f;
    constexpr int NB = LPR < 16 ? LPR : 16;
    float4 x[NB];
    float w[NB];
#define FR_GATHER(K)                                                         \
    if constexpr ((K) < LPR) {                                               \
      const int ck = bcast_i<LPR, (K)>(c);                                   \
      w[(K)] = bcast_f<LPR, (K)>(v);                                         \
      x[(K)] = X4[(int64_t)ck * ldx4 + q];                                   \
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
        const int ck = __shfl(c, src, 64);
        const float wk = __shfl(v, src, 64);
        acc = f4_fma(wk, X4[(int64_t)ck * ldx4 + q], acc);
      }
    }
  }
  return acc;
}

template <int LPR>
__global__ __launch_bounds__(256) void spmm_units_kernel(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const float* __restrict__ val, const int2* __restrict__ units, int64_t n_units,
    int64_t n_plain, int chunk, const float* __restrict__ X, int64_t ldx, int d4, Epi ep,
    float4* __restrict__ partial) {
  constexpr int GPB = 256 / LPR;  // groups per block
  const int q0 = threadIdx.x % LPR;
  const int grp = threadIdx.x / LPR;
  const float4* X4 = reinterpret_cast<const float4*>(X);
  const int64_t ldx4 = ldx >> 2;
  for (int64_t u = (int64_t)blockIdx.x * GPB + grp; u < n_units; u += (int64_t)gridDim.x * GPB) {
    const int2 unit = units[u];
    const int64_t rs = rowptr[unit.x];
    const int64_t e0 = rs + (int64_t)unit.y * chunk;
    const int64_t e1 = min(rowptr[unit.x + 1], e0 + (int64_t)chunk);
    // group-uniform slot loop: every lane of the group takes part in the broadcasts
    for (int qb = 0; qb < d4; qb += LPR) {
      const int q = qb + q0;
      const float4 acc = gather_unit<LPR>(col, val, X4, ldx4, e0, e1, q0, q < d4 ? q : d4 - 1);
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
                                                         const float4* __restrict__ partial) {
  constexpr int GPB = 256 / LPR;
  const int q0 = threadIdx.x % LPR;
  const int grp = threadIdx.x / LPR;
  for (int64_t s = (int64_t)blockIdx.x * GPB + grp; s < n_split; s += (int64_t)gridDim.x * GPB) {
    const int3 sr = split_rows[s];
    for (int q = q0; q < d4; q += LPR) {
      float4 acc = partial[(int64_t)sr.y * d4 + q];
      for (int k = 1; k < sr.z; ++k) acc = f4_add(acc, partial[((int64_t)sr.y + k) * d4 + q]);
      epilogue(ep, sr.x, q, acc);
    }
  }
}

template <int LPR>
hipError_t launch_spmm(const int64_t* rowptr, const int32_t* col, const float* val,
                       const fr_spmm_plan* plan, const float* X, int64_t ldx, int d, const Epi& ep,
                       float4* partial, hipStream_t s) {
  constexpr int GPB = 256 / LPR;
  const int d4 = d / 4;
  if (plan->n_units > 0) {
    int64_t blocks = fr::ceil_div(plan->n_units, GPB);
    blocks = std::min<int64_t>(blocks, (int64_t)fr::kNumCU * 64);
    hipLaunchKernelGGL(spmm_units_kernel<LPR>, dim3((unsigned)blocks), dim3(256), 0, s, rowptr, col,
                       val, reinterpret_cast<const int2*>(plan->d_units), plan->n_units,
                       plan->n_plain, plan->chunk, X, ldx, d4, ep, partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (plan->n_split > 0) {
    int64_t blocks = std::min<int64_t>(fr::ceil_div(plan->n_split, GPB), (int64_t)fr::kNumCU * 16);
    hipLaunchKernelGGL(spmm_fixup_kernel<LPR>, dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<const int3*>(plan->d_split_rows), plan->n_split, d4, ep,
                       partial);
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

extern "C" int fr_spmm_csr(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                           int64_t n_rows, const fr_spmm_plan* plan, const float* d_X, int64_t ldx,
                           int d, float* d_Y1, int64_t ldy1, float* d_Y2, int64_t ldy2,
                           float alpha, const float* d_A1, int64_t lda1, float beta1,
                           const float* d_A2, int64_t lda2, float beta2, void* d_workspace,
                           int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(plan != nullptr, "plan is null");
  FR_REQUIRE(d > 0 && d % 4 == 0 && d <= 1024, "d must be a positive multiple of 4, <= 1024");
  FR_REQUIRE(n_rows >= 0, "n_rows < 0");
  if (n_rows == 0) return FR_OK;
  FR_REQUIRE(d_rowptr && d_X, "rowptr/X null");
  FR_REQUIRE(d_Y1 || d_Y2, "no output requested");
  FR_REQUIRE(plan->n_units == 0 || (plan->d_units && d_col && d_val), "plan/col/val null");
  FR_REQUIRE(plan->n_split == 0 || plan->d_split_rows, "split_rows null");
  FR_REQUIRE(plan->chunk > 0, "plan chunk must be > 0");
  FR_REQUIRE(ldx >= d && ldx % 4 == 0 && fr::aligned16(d_X), "X must be 16-B aligned, ldx%4==0");
  FR_REQUIRE(!d_Y1 || (ldy1 >= d && ldy1 % 4 == 0 && fr::aligned16(d_Y1)), "bad Y1");
  FR_REQUIRE(!d_Y2 || (ldy2 >= d && ldy2 % 4 == 0 && fr::aligned16(d_Y2)), "bad Y2");
  FR_REQUIRE(!d_A1 || (lda1 >= d && lda1 % 4 == 0 && fr::aligned16(d_A1)), "bad A1");
  FR_REQUIRE(!d_A2 || (lda2 >= d && lda2 % 4 == 0 && fr::aligned16(d_A2)), "bad A2");
  FR_REQUIRE(d_Y1 != d_X && d_Y2 != d_X, "outputs must not alias X");
  const int64_t need = fr_spmm_workspace(plan, d);
  FR_REQUIRE(plan->n_split == 0 || (d_workspace && workspace_bytes >= need && fr::aligned16(d_workspace)),
             "workspace too small (need " + std::to_string(need) + " bytes)");
  Epi ep{d_Y1, ldy1, d_Y2, ldy2, alpha, d_A1, lda1, beta1, d_A2, lda2, beta2};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float4* partial = reinterpret_cast<float4*>(d_workspace);
  const int d4 = d / 4;
  hipError_t e;
  if (d4 >= 64) {
    e = launch_spmm<64>(d_rowptr, d_col, d_val, plan, d_X, ldx, d, ep, partial, s);
  } else if (d4 >= 32) {
    e = (d4 == 32) ? launch_spmm<32>(d_rowptr, d_col, d_val, plan, d_X, ldx, d, ep, partial, s)
                   : launch_spmm<16>(d_rowptr, d_col, d_val, plan, d_X, ldx, d, ep, partial, s);
  } else if (d4 >= 16) {
    e = launch_spmm<16>(d_rowptr, d_col, d_val, plan, d_X, ldx, d, ep, partial, s);
  } else if (d4 >= 8) {
    e = launch_spmm<8>(d_rowptr, d_col, d_val, plan, d_X, ldx, d, ep, partial, s);
  } else if (d4 >= 4) {
    e = launch_spmm<4>(d_rowptr, d_col, d_val, plan, d_X, ldx, d, ep, partial, s);
  } else {
    e = launch_spmm<1>(d_rowptr, d_col, d_val, plan, d_X, ldx, d, ep, partial, s);
  }
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_spmm_csr: ") + hipGetErrorString(e));
  return FR_OK;
}
