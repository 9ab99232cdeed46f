// CSR SpMM over bf16 tables with fp32 accumulation — BASELINE config 5 (d=256 bf16 embeddings).
//
// Same operator as fr_spmm_csr (torch.sparse.mm(norm_adj, X) + the layer mean,
// models/lightgcn.py:136-144) and the same work plan (units of <= chunk edges, split rows summed
// in chunk order by a fix-up kernel: deterministic).  X, Y1, Y2, A1, A2 are bf16; the edge
// values, the accumulator and the epilogue arithmetic are fp32, rounded once to bf16 (RNE).
//
// Mapping (wave64): a group of LPR = d/8 lanes owns one work unit, each lane 8 bf16 (16 B) of the
// row, so one wave-instruction of the gather moves 64 x 16 B = 1 KiB (two 512-B rows at d=256).
// Edge metadata is loaded 16 edges at a time by the lanes of every 16-lane DPP row of the group
// (all rows of a group load the same 16 (col,val) pairs: L1 hits) and broadcast in-register with
// row_newbcast, so a group issues 16 independent row gathers before consuming any.  Groups of
// fewer than 16 lanes (d < 128) broadcast with ds_bpermute.
//
// Algorithmic bytes per launch (SURVEY 8(d) with s=2): 8(N+1) + 8 nnz + 2d nnz + 2d N per row
// output written / addend read.
#include "fr_bf16.h"

#include <algorithm>

namespace {

template <int LPR, int K>
__device__ __forceinline__ int bc16_i(int v) {
  if constexpr (LPR >= 16) {
    return __builtin_amdgcn_update_dpp(0, v, 0x150 + K, 0xf, 0xf, false);  // row_newbcast:K
  } else {
    const int lane = threadIdx.x & 63;
    return __shfl(v, (lane & ~(LPR - 1)) | K, 64);
  }
}

struct Epi16 {
  uint4* Y1; int64_t ldy1;  // leading dimensions in uint4 units (8 bf16)
  uint4* Y2; int64_t ldy2; float alpha;
  const uint4* A1; int64_t lda1; float beta1;
  const uint4* A2; int64_t lda2; float beta2;
};

__device__ __forceinline__ void epilogue16(const Epi16& ep, int64_t r, int q, const float* acc) {
  if (ep.Y1) ep.Y1[r * ep.ldy1 + q] = fr_pack8(acc);
  if (ep.Y2) {
    float o[8], a[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = ep.alpha * acc[j];
    if (ep.A1) {
      fr_unpack8(ep.A1[r * ep.lda1 + q], a);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaf(ep.beta1, a[j], o[j]);
    }
    if (ep.A2) {
      fr_unpack8(ep.A2[r * ep.lda2 + q], a);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fmaf(ep.beta2, a[j], o[j]);
    }
    ep.Y2[r * ep.ldy2 + q] = fr_pack8(o);
  }
}

template <int LPR>
__device__ __forceinline__ void gather_unit16(const int32_t* __restrict__ col, const float* __restrict__ val,
                                              const uint4* __restrict__ X8, int64_t ldx8, int64_t e0,
                                              int64_t e1, int q, float* acc) {
  constexpr int EB = LPR >= 16 ? 16 : LPR;  // edges per batch
  const int lane = threadIdx.x & 63;
  const int lig = lane & (EB - 1);
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  for (int64_t e = e0; e < e1; e += EB) {
    const int64_t my = e + lig;
    const int c = __builtin_nontemporal_load(col + (my < e1 ? my : e1 - 1));
    const float v = my < e1 ? __builtin_nontemporal_load(val + my) : 0.f;
    uint4 x[EB];
    float w[EB];
#define FR_G16(K)                                                      \
    if constexpr ((K) < EB) {                                          \
      const int ck = bc16_i<LPR, (K)>(c);                              \
      w[(K)] = __int_as_float(bc16_i<LPR, (K)>(__float_as_int(v)));    \
      x[(K)] = X8[(int64_t)ck * ldx8 + q];                             \
    }
    FR_G16(0) FR_G16(1) FR_G16(2) FR_G16(3) FR_G16(4) FR_G16(5) FR_G16(6) FR_G16(7)
    FR_G16(8) FR_G16(9) FR_G16(10) FR_G16(11) FR_G16(12) FR_G16(13) FR_G16(14) FR_G16(15)
#undef FR_G16
#pragma unroll
    for (int k = 0; k < EB; ++k) {
      float xf[8];
      fr_unpack8(x[k], xf);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(w[k], xf[j], acc[j]);
    }
  }
}

template <int LPR>
__global__ __launch_bounds__(256) void spmm16_units_kernel(
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col, const float* __restrict__ val,
    const int2* __restrict__ units, int64_t n_units, int64_t n_plain, int chunk,
    const uint4* __restrict__ X8, int64_t ldx8, int d8, Epi16 ep, float4* __restrict__ partial) {
  constexpr int GPB = 256 / LPR;
  const int q0 = threadIdx.x % LPR;
  const int grp = threadIdx.x / LPR;
  for (int64_t u = (int64_t)blockIdx.x * GPB + grp; u < n_units; u += (int64_t)gridDim.x * GPB) {
    const int2 unit = units[u];
    const int64_t rs = rowptr[unit.x];
    const int64_t e0 = rs + (int64_t)unit.y * chunk;
    const int64_t e1 = min(rowptr[unit.x + 1], e0 + (int64_t)chunk);
    for (int qb = 0; qb < d8; qb += LPR) {  // group-uniform slot loop
      const int q = qb + q0;
      float acc[8];
      gather_unit16<LPR>(col, val, X8, ldx8, e0, e1, q < d8 ? q : d8 - 1, acc);
      if (q < d8) {
        if (u < n_plain) {
          epilogue16(ep, unit.x, q, acc);
        } else {
          float4* pp = partial + ((u - n_plain) * d8 + q) * 2;
          pp[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
          pp[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
        }
      }
    }
  }
}

__global__ __launch_bounds__(256) void spmm16_fixup_kernel(const int3* __restrict__ split_rows, int64_t n_split,
                                                           int d8, Epi16 ep, const float4* __restrict__ partial) {
  const int64_t total = n_split * d8;
  for (int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int64_t s = t / d8;
    const int q = (int)(t % d8);
    const int3 sr = split_rows[s];
    const float4* p = partial + ((int64_t)sr.y * d8 + q) * 2;
    float4 a = p[0], b = p[1];
    for (int k = 1; k < sr.z; ++k) {
      p += (int64_t)d8 * 2;
      a = f4_add(a, p[0]);
      b = f4_add(b, p[1]);
    }
    const float acc[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    epilogue16(ep, sr.x, q, acc);
  }
}

template <int LPR>
hipError_t launch16(const int64_t* rowptr, const int32_t* col, const float* val, const fr_spmm_plan* plan,
                    const uint4* X8, int64_t ldx8, int d8, const Epi16& ep, float4* partial, hipStream_t s) {
  constexpr int GPB = 256 / LPR;
  if (plan->n_units > 0) {
    const int64_t blocks = std::min<int64_t>(fr::ceil_div(plan->n_units, GPB), (int64_t)fr::kNumCU * 64);
    hipLaunchKernelGGL(spmm16_units_kernel<LPR>, dim3((unsigned)blocks), dim3(256), 0, s, rowptr, col, val,
                       reinterpret_cast<const int2*>(plan->d_units), plan->n_units, plan->n_plain, plan->chunk,
                       X8, ldx8, d8, ep, partial);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (plan->n_split > 0) {
    const int64_t blocks = std::min<int64_t>(fr::ceil_div(plan->n_split * d8, 256), (int64_t)fr::kNumCU * 16);
    hipLaunchKernelGGL(spmm16_fixup_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                       reinterpret_cast<const int3*>(plan->d_split_rows), plan->n_split, d8, ep, partial);
    return hipGetLastError();
  }
  return hipSuccess;
}

inline bool ok_tab(const void* p, int64_t ld, int d) { return !p || (ld >= d && ld % 8 == 0 && fr::aligned16(p)); }

}  // namespace

extern "C" int64_t fr_spmm_bf16_workspace(const fr_spmm_plan* plan, int d) {
  if (!plan) return 0;
  return (plan->n_units - plan->n_plain) * (int64_t)d * 4 + 256;
}

extern "C" int fr_spmm_csr_bf16(const int64_t* d_rowptr, const int32_t* d_col, const float* d_val,
                                int64_t n_rows, const fr_spmm_plan* plan, const uint16_t* d_X, int64_t ldx,
                                int d, uint16_t* d_Y1, int64_t ldy1, uint16_t* d_Y2, int64_t ldy2,
                                float alpha, const uint16_t* d_A1, int64_t lda1, float beta1,
                                const uint16_t* d_A2, int64_t lda2, float beta2, void* d_workspace,
                                int64_t workspace_bytes, void* stream) {
  FR_REQUIRE(plan != nullptr, "plan is null");
  FR_REQUIRE(d > 0 && d % 8 == 0 && d <= 2048, "d must be a positive multiple of 8, <= 2048");
  FR_REQUIRE(n_rows >= 0, "n_rows < 0");
  if (n_rows == 0) return FR_OK;
  FR_REQUIRE(d_rowptr && d_X, "rowptr/X null");
  FR_REQUIRE(d_Y1 || d_Y2, "no output requested");
  FR_REQUIRE(plan->n_units == 0 || (plan->d_units && d_col && d_val), "plan/col/val null");
  FR_REQUIRE(plan->n_split == 0 || plan->d_split_rows, "split_rows null");
  FR_REQUIRE(plan->chunk > 0, "plan chunk must be > 0");
  FR_REQUIRE(ok_tab(d_X, ldx, d), "X must be 16-B aligned with ldx % 8 == 0");
  FR_REQUIRE(ok_tab(d_Y1, ldy1, d) && ok_tab(d_Y2, ldy2, d), "bad Y1/Y2 (16-B aligned, ld % 8 == 0)");
  FR_REQUIRE(ok_tab(d_A1, lda1, d) && ok_tab(d_A2, lda2, d), "bad A1/A2 (16-B aligned, ld % 8 == 0)");
  FR_REQUIRE(d_Y1 != d_X && d_Y2 != d_X, "outputs must not alias X");
  const int64_t need = fr_spmm_bf16_workspace(plan, d);
  FR_REQUIRE(plan->n_split == 0 || (d_workspace && workspace_bytes >= need && fr::aligned16(d_workspace)),
             "workspace too small (need " + std::to_string(need) + " bytes)");
  auto u4 = [](const uint16_t* p) { return reinterpret_cast<uint4*>(const_cast<uint16_t*>(p)); };
  Epi16 ep{u4(d_Y1), ldy1 / 8, u4(d_Y2), ldy2 / 8, alpha, u4(d_A1), lda1 / 8, beta1, u4(d_A2), lda2 / 8, beta2};
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  float4* partial = reinterpret_cast<float4*>(d_workspace);
  const uint4* X8 = u4(d_X);
  const int d8 = d / 8;
  hipError_t e;
  if (d8 >= 32) {
    e = launch16<32>(d_rowptr, d_col, d_val, plan, X8, ldx / 8, d8, ep, partial, s);
  } else if (d8 >= 16) {
    e = launch16<16>(d_rowptr, d_col, d_val, plan, X8, ldx / 8, d8, ep, partial, s);
  } else if (d8 >= 8) {
    e = launch16<8>(d_rowptr, d_col, d_val, plan, X8, ldx / 8, d8, ep, partial, s);
  } else if (d8 >= 4) {
    e = launch16<4>(d_rowptr, d_col, d_val, plan, X8, ldx / 8, d8, ep, partial, s);
  } else if (d8 >= 2) {
    e = launch16<2>(d_rowptr, d_col, d_val, plan, X8, ldx / 8, d8, ep, partial, s);
  } else {
    e = launch16<1>(d_rowptr, d_col, d_val, plan, X8, ldx / 8, d8, ep, partial, s);
  }
  if (e != hipSuccess) return fr::fail(FR_EHIP, std::string("fr_spmm_csr_bf16: ") + hipGetErrorString(e));
  return FR_OK;
}
