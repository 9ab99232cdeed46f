// Multi-tensor fused Adam — replaces torch.optim.Adam.step (common/trainer.py:143-144,224).
//
// One launch updates up to kMaxTensors parameter tensors (pointers travel in the kernel
// argument block, no device-side descriptor table, so the call is graph-capturable).
// Per element, in torch's single-tensor order (torch/optim/adam.py _single_tensor_adam):
//   g  = grad (+ wd * p)
//   m  = fma(1-b1, g - m, m)                       exp_avg.lerp_(grad, 1-beta1)
//   v  = fma((1-b2) * g, g, v * b2)                exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2)
//   p  = p + (-step_size * m) / (sqrt(v) / bc2_sqrt + eps)
// The fused/unfused choice of each step was matched element-for-element against torch-CPU's
// Adam on MI355X (m and v bit-identical; p differs by <= 1 ulp on ~0.1% of elements).
// 28 B of HBM traffic per parameter (p,m,v read+write, g read): HBM-bound, float4 vectorised.
#include "fr_common.h"
#include "fr_bf16.h"

#include <algorithm>
#include <cmath>

namespace {

constexpr int kMaxTensors = 48;  // AdamArgs = 48 x 68 B + 8 B < the 4 KiB kernel-argument limit
constexpr int kChunk = 8192;  // elements per (tensor, chunk) work item
constexpr int kAdamBlocks = fr::kNumCU * 5;  // persistent grid: 5 blocks/CU = the 84-VGPR occupancy

struct AdamArgs {
  float* p[kMaxTensors];
  const float* g[kMaxTensors];
  float* m[kMaxTensors];
  float* v[kMaxTensors];
  int64_t* step[kMaxTensors];   // device step counters (device-scalar mode) or null
  int64_t numel[kMaxTensors];
  int32_t blk_start[kMaxTensors + 1];
  int32_t vec4[kMaxTensors];
  // row-gradient tensors (rmap != null): the parameter is a [R, 2^rshift] table whose gradient is
  // g[r] = rmap[r] >= 0 ? G[rmap[r]] : 0 (compact rows from fr_embedding_rowgrad)
  const int32_t* rmap[kMaxTensors];
  int32_t rshift[kMaxTensors];
  unsigned* ticket;  // device-scalar mode: the caller's 9-word arrival counters (last_block)
  int n;
};

struct AdamHyper {
  double lr, beta1_d, beta2_d;  // device-scalar mode recomputes neg_step / bc2_sqrt from these
  const double* d_lr;       // device lr (device-scalar mode) or null
  float w1;         // 1 - beta1
  float beta2;
  float one_m_b2;   // 1 - beta2
  float neg_step;   // -lr / bias_correction1
  float bc2_sqrt;
  float eps;
  float wd;
};

__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamHyper& h) {
  if (h.wd != 0.f) g = __fadd_rn(g, __fmul_rn(h.wd, p));
  m = fmaf(h.w1, __fsub_rn(g, m), m);
  v = fmaf(__fmul_rn(h.one_m_b2, g), g, __fmul_rn(v, h.beta2));
  const float denom = __fadd_rn(__fdiv_rn(sqrt_rn(v), h.bc2_sqrt), h.eps);
  p = __fadd_rn(p, __fdiv_rn(__fmul_rn(h.neg_step, m), denom));
}

typedef float fv4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float4 nt_load4(const float* p) {
  const fv4 v = __builtin_nontemporal_load(reinterpret_cast<const fv4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ void nt_store4(float* p, float4 v) {
  fv4 w = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(w, reinterpret_cast<fv4*>(p));
}
// The fp32 update streams (adam_kernel) choose by launch size: ordinary loads / stores up to
// kTemporalBytes of state -- at HealthRec's shape (8.9M parameters, 249 MB per launch, within the
// 256 MB MALL) the launch measured 43.5 us against 52.5 us with the non-temporal hints
// (tools/bench_adam.py; 0.708 / 0.713 -> 0.706 / 0.710 ms per step) -- and the non-temporal hints
// beyond (config 4's 19.7 GB launch: 37.5 / 37.8 ms per step with them, 37.8 / 38.4 without).
constexpr int64_t kTemporalBytes = 512ll << 20;
template <bool NT>
__device__ __forceinline__ float4 ld4t(const float* p) {
  if constexpr (NT) return nt_load4(p);
  else return *reinterpret_cast<const float4*>(p);
}
template <bool NT>
__device__ __forceinline__ void st4t(float* p, float4 v) {
  if constexpr (NT) nt_store4(p, v);
  else *reinterpret_cast<float4*>(p) = v;
}

template <bool NT>
__device__ __forceinline__ void adam4(float* P, const float* G, float* M, float* V, int64_t i, const AdamHyper& h,
                                      float4& p, float4& g, float4& m, float4& v) {
  adam_elem(p.x, g.x, m.x, v.x, h);
  adam_elem(p.y, g.y, m.y, v.y, h);
  adam_elem(p.z, g.z, m.z, v.z, h);
  adam_elem(p.w, g.w, m.w, v.w, h);
  st4t<NT>(P + i, p);
  st4t<NT>(M + i, m);
  st4t<NT>(V + i, v);
}

// Device-scalar mode bumps the step counters in the launch itself: every block derives its
// scalars from step + 1, and the block that arrives last (every other block has finished, so has
// read the counters) writes step + 1 back.  Arrival is two-level so that hundreds of blocks do not
// serialise on one atomic word: block b takes a ticket on shard b % 8 (the blocks of one XCD), the
// last arrival of a shard takes a ticket on the top word, the last of those is the grid's last.
// Each last arrival resets its word for the next launch.  The words belong to the caller (one set
// per optimiser and kernel kind, fr_adam_step_dev's d_ticket): launches that share a set must run
// one at a time, which launches of one optimiser do on its stream; two optimisers stepping on two
// streams (or concurrent branches of a captured graph) use their own sets.  (1-D grids.)

__device__ __forceinline__ bool last_block(unsigned* ticket) {
  __shared__ bool last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned G = gridDim.x, sh = blockIdx.x % 8;
    const unsigned in_shard = (G + 7 - sh) / 8, shards = G < 8 ? G : 8;
    bool top = atomicAdd(&ticket[sh], 1u) == in_shard - 1;
    if (top) atomicExch(&ticket[sh], 0u);
    last = top && atomicAdd(&ticket[8], 1u) == shards - 1;
    if (last) atomicExch(&ticket[8], 0u);
  }
  __syncthreads();
  return last;
}

// Persistent grid over the launch's (tensor, chunk) list; the step-dependent scalars are derived
// once per tensor a block meets.  Each thread keeps two float4 quartets (p, g, m, v) in flight.
template <bool ROWS, bool NT>
__global__ __launch_bounds__(256) void adam_kernel(AdamArgs a, AdamHyper h, const int32_t* skip) {
  if (skip && *skip) return;
  const int total = a.blk_start[a.n];
  int t = 0, cur = -1;
  for (int c = blockIdx.x; c < total; c += gridDim.x) {
    while (t + 1 < a.n && c >= a.blk_start[t + 1]) ++t;
    if (t != cur) {
      cur = t;
      if (a.step[t]) {
        // step-dependent scalars from device memory (graph-replayable); same double arithmetic
        // as the host path / torch's Python scalars
        const double st = (double)(a.step[t][0] + 1);  // this step (the counter is bumped at the end)
        const double lr = h.d_lr ? h.d_lr[0] : h.lr;
        const double bc1 = 1.0 - pow(h.beta1_d, st);
        const double bc2 = 1.0 - pow(h.beta2_d, st);
        h.neg_step = (float)(-(lr / bc1));
        h.bc2_sqrt = (float)sqrt(bc2);
      }
    }
    const int64_t base = (int64_t)(c - a.blk_start[t]) * kChunk;
    const int64_t end = min(base + (int64_t)kChunk, a.numel[t]);
    float* __restrict__ P = a.p[t];
    const float* __restrict__ G = a.g[t];
    float* __restrict__ M = a.m[t];
    float* __restrict__ V = a.v[t];
    if constexpr (ROWS) {  // row gradient: p, m, v streamed; g from the compact rows of this step's batch
      const int32_t* __restrict__ rm = a.rmap[t];
      const int sh = a.rshift[t];
      const int64_t cmask = ((int64_t)1 << sh) - 1;
      auto grad4 = [&](int64_t i) {
        const int32_t slot = rm[i >> sh];
        return slot >= 0 ? *reinterpret_cast<const float4*>(G + ((int64_t)slot << sh) + (i & cmask))
                         : make_float4(0.f, 0.f, 0.f, 0.f);
      };
      constexpr int64_t kStride = 4 * 256;
      int64_t i = base + 4 * threadIdx.x;
      for (; i + kStride < end; i += 2 * kStride) {  // two quartets in flight (end - base is a multiple of 4)
        const int64_t i1 = i + kStride;
        float4 p0 = ld4t<NT>(P + i), m0 = ld4t<NT>(M + i), v0 = ld4t<NT>(V + i), g0 = grad4(i);
        float4 p1 = ld4t<NT>(P + i1), m1 = ld4t<NT>(M + i1), v1 = ld4t<NT>(V + i1), g1 = grad4(i1);
        adam4<NT>(P, G, M, V, i, h, p0, g0, m0, v0);
        adam4<NT>(P, G, M, V, i1, h, p1, g1, m1, v1);
      }
      for (; i < end; i += kStride) {
        float4 p0 = ld4t<NT>(P + i), m0 = ld4t<NT>(M + i), v0 = ld4t<NT>(V + i), g0 = grad4(i);
        adam4<NT>(P, G, M, V, i, h, p0, g0, m0, v0);
      }
    } else if (a.vec4[t]) {
      constexpr int64_t kStride = 4 * 256;
      int64_t i = base + 4 * threadIdx.x;
      for (; i + kStride + 3 < end; i += 2 * kStride) {
        float4 p0 = ld4t<NT>(P + i), g0 = ld4t<NT>(G + i), m0 = ld4t<NT>(M + i), v0 = ld4t<NT>(V + i);
        const int64_t i1 = i + kStride;
        float4 p1 = ld4t<NT>(P + i1), g1 = ld4t<NT>(G + i1), m1 = ld4t<NT>(M + i1), v1 = ld4t<NT>(V + i1);
        adam4<NT>(P, G, M, V, i, h, p0, g0, m0, v0);
        adam4<NT>(P, G, M, V, i1, h, p1, g1, m1, v1);
      }
      for (; i + 3 < end; i += kStride) {
        float4 p0 = ld4t<NT>(P + i), g0 = ld4t<NT>(G + i), m0 = ld4t<NT>(M + i), v0 = ld4t<NT>(V + i);
        adam4<NT>(P, G, M, V, i, h, p0, g0, m0, v0);
      }
      // scalar tail of the last chunk (numel % 4)
      const int64_t tail0 = base + ((end - base) / 4) * 4;
      for (int64_t k = tail0 + threadIdx.x; k < end; k += blockDim.x) adam_elem(P[k], G[k], M[k], V[k], h);
    } else {
      for (int64_t k = base + threadIdx.x; k < end; k += blockDim.x) adam_elem(P[k], G[k], M[k], V[k], h);
    }
  }
  if (a.step[0] && last_block(a.ticket) && threadIdx.x < a.n && a.step[threadIdx.x])
    a.step[threadIdx.x][0] += 1;
}


// Mixed precision (BASELINE config 5): bf16 parameter + bf16 gradient, fp32 master copy and
// fp32 exp_avg / exp_avg_sq.  The update is adam_elem on the master; the bf16 parameter the
// SpMM reads is the master rounded to nearest even.  30 B per parameter.
__global__ __launch_bounds__(256) void adam_bf16_kernel(uint4* __restrict__ P16, float* __restrict__ W,
                                                        const uint4* __restrict__ G16, float* __restrict__ M,
                                                        float* __restrict__ V, int64_t n8, int64_t* step,
                                                        AdamHyper h, const int32_t* skip) {
  if (skip && *skip) return;
  if (step) {
    const double st = (double)step[0];
    const double lr = h.d_lr ? h.d_lr[0] : h.lr;
    h.neg_step = (float)(-(lr / (1.0 - pow(h.beta1_d, st))));
    h.bc2_sqrt = (float)sqrt(1.0 - pow(h.beta2_d, st));
  }
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    float g[8], w[8], m[8], v[8];
    fr_unpack8(G16[i], g);
    const float4* W4 = reinterpret_cast<const float4*>(W) + 2 * i;
    const float4* M4 = reinterpret_cast<const float4*>(M) + 2 * i;
    const float4* V4 = reinterpret_cast<const float4*>(V) + 2 * i;
    const float4 w0 = nt_load4(reinterpret_cast<const float*>(W4)), w1 = nt_load4(reinterpret_cast<const float*>(W4 + 1));
    const float4 m0 = nt_load4(reinterpret_cast<const float*>(M4)), m1 = nt_load4(reinterpret_cast<const float*>(M4 + 1));
    const float4 v0 = nt_load4(reinterpret_cast<const float*>(V4)), v1 = nt_load4(reinterpret_cast<const float*>(V4 + 1));
    w[0] = w0.x; w[1] = w0.y; w[2] = w0.z; w[3] = w0.w; w[4] = w1.x; w[5] = w1.y; w[6] = w1.z; w[7] = w1.w;
    m[0] = m0.x; m[1] = m0.y; m[2] = m0.z; m[3] = m0.w; m[4] = m1.x; m[5] = m1.y; m[6] = m1.z; m[7] = m1.w;
    v[0] = v0.x; v[1] = v0.y; v[2] = v0.z; v[3] = v0.w; v[4] = v1.x; v[5] = v1.y; v[6] = v1.z; v[7] = v1.w;
#pragma unroll
    for (int j = 0; j < 8; ++j) adam_elem(w[j], g[j], m[j], v[j], h);
    float* Wo = W + 8 * i;
    float* Mo = M + 8 * i;
    float* Vo = V + 8 * i;
    nt_store4(Wo, make_float4(w[0], w[1], w[2], w[3]));
    nt_store4(Wo + 4, make_float4(w[4], w[5], w[6], w[7]));
    nt_store4(Mo, make_float4(m[0], m[1], m[2], m[3]));
    nt_store4(Mo + 4, make_float4(m[4], m[5], m[6], m[7]));
    nt_store4(Vo, make_float4(v[0], v[1], v[2], v[3]));
    nt_store4(Vo + 4, make_float4(v[4], v[5], v[6], v[7]));
    P16[i] = fr_pack8(w);
  }
}

__global__ void adam_bf16_step_inc_kernel(int64_t* step, const int32_t* skip) {
  if (skip && *skip) return;
  if (threadIdx.x == 0) step[0] += 1;
}

// ---- Deferred zero-gradient steps for row-gradient tables ("lazy rows", exact) ----------------
// torch's Adam updates every row of a table each step, also rows whose gradient is zero.  For such
// a row the step only decays (m, v) and moves p by the step's (neg_step, bc2_sqrt); those two
// scalars depend on the step index and lr alone.  The lazy form records them per step in a ring
// (hist[s % cap]) and keeps last[r] = the step row r is current through.  A row that receives a
// gradient at step t first replays steps last[r]+1 .. t-1 with g = 0 (adam_elem, the same float
// operations as the dense kernel), then applies step t; untouched rows are not read.  A flush
// replays every row up to the current step.  Results are bit-identical to the dense update at
// every flush point; HBM traffic per step is 24 B per parameter of the TOUCHED rows only.
// The host flushes before any full-table read and at least every cap-1 steps.
constexpr int kMaxLazy = 16;

struct LazyArgs {
  float* p[kMaxLazy];
  const float* g[kMaxLazy];
  float* m[kMaxLazy];
  float* v[kMaxLazy];
  int64_t* step[kMaxLazy];
  const int32_t* rmap[kMaxLazy];
  int32_t* last[kMaxLazy];
  float* hist[kMaxLazy];      // [cap][4]: (neg_step, bc2_sqrt, double 1 / bc2_sqrt) of step s at s % cap
  const int64_t* ids[kMaxLazy];  // step: the ids whose rows carry a gradient (duplicates allowed)
  int64_t nrows[kMaxLazy];
  int32_t rshift[kMaxLazy];   // row width = 1 << rshift
  int32_t row_start[kMaxLazy + 1];  // flush: prefix over rows; step: prefix over ids
  int32_t cap;
  int n;
};

// (neg_step, bc2_sqrt) of step st: the values the history ring keeps for it
__device__ __forceinline__ float2 lazy_scalars(const AdamHyper& h, int64_t st) {
  const double lr = h.d_lr ? h.d_lr[0] : h.lr;
  const double bc1 = 1.0 - pow(h.beta1_d, (double)st);
  const double bc2 = 1.0 - pow(h.beta2_d, (double)st);
  return make_float2((float)(-(lr / bc1)), (float)sqrt(bc2));
}

__global__ void adam_lazy_inc_kernel(LazyArgs a, AdamHyper h, const int32_t* skip) {
  const int t = threadIdx.x;
  if (t >= a.n) return;
  // the skip flag, the step and the device lr loaded together (one memory round trip, not three)
  const int32_t sk = skip ? *skip : 0;
  const int64_t st = a.step[t][0] + 1;
  AdamHyper hh = h;
  if (h.d_lr) {
    hh.lr = h.d_lr[0];
    hh.d_lr = nullptr;
  }
  if (sk) return;
  a.step[t][0] = st;
  const float2 e = lazy_scalars(hh, st);
  float* hp = a.hist[t] + 4 * (st % a.cap);  // kHist = 4: neg_step, bc2_sqrt, RN64(1 / bc2_sqrt)
  hp[0] = e.x;
  hp[1] = e.y;
  *reinterpret_cast<double*>(hp + 2) = 1.0 / (double)e.y;
}


// ---- deferred zero-gradient steps, bit-identical to adam_elem(g = 0) and cheaper ---------------
// History ring entry of step s (4 floats at hist + 4 (s % cap)): neg_step, bc2_sqrt (the fp32 scalars
// adam_elem uses) and, as a double in floats 2-3, RN64(1 / bc2_sqrt) for the division below.
constexpr int kHist = 4;
// With g = 0 (and no weight decay) a step is  m = fma(w1, -m, m);  v = v * beta2;
// p += (neg_step * m) / (sqrt_rn(v) / bc2_sqrt + eps).  The division by the step's constant bc2_sqrt
// is done as RN32(double(s) * RN64(1 / bc2_sqrt)): the double product is within 2^-52 (relative) of
// s / bc2_sqrt, and a quotient of two fp32 numbers lies at least 2^-49 (relative) from every fp32
// rounding boundary (it is never a midpoint: that would need a 25-bit odd significand dividing a
// 24-bit one), so the rounded result equals the correctly rounded fp32 quotient (s >= sqrt of the
// smallest subnormal, so the quotient is a normal number).  One double reciprocal per step, shared
// by all of a lane's elements; the elementwise products and sums on packed-fp32 ops.
typedef float pf2 __attribute__((ext_vector_type(2)));
constexpr int KC = 2;  // float4 chunks of a row a lane replays together (replay_row)

// Correctly rounded a / b without the range handling of the general expansion: the compiler's fp32
// division is v_div_scale (x2), v_rcp, the Newton / Markstein fma chain, v_div_fmas, v_div_fixup;
// for |a| in {0} U [2^-40, 2^40] and b in [2^-40, 2^40] the scale steps are the identity (no
// exponent gap >= 96, no denormal operand or result) and the fix-up passes the value through, so the
// fma chain alone returns the same bits.  Callers guarantee the range (replay_row's row check).
__device__ __forceinline__ float div_rn_inrange(float a, float b) {
  const float y0 = __builtin_amdgcn_rcpf(b);
  const float e = fmaf(-b, y0, 1.0f);
  const float y1 = fmaf(e, y0, y0);
  const float q0 = a * y1;
  const float r0 = fmaf(-b, q0, a);
  const float q1 = fmaf(r0, y1, q0);
  const float r1 = fmaf(-b, q1, a);
  return fmaf(r1, y1, q1);
}

// Correctly rounded sqrt for x in {0} U [2^-96, inf): v_sqrt_f32 (1 ulp) + the residual selection of
// sqrt_rn without its small-input scaling
__device__ __forceinline__ float sqrt_rn_inrange(float x) {
  float s = __builtin_amdgcn_sqrtf(x);
  const float s_dn = __int_as_float(__float_as_int(s) - 1);
  const float s_up = __int_as_float(__float_as_int(s) + 1);
  const float r_dn = fmaf(-s_dn, s, x);
  const float r_up = fmaf(-s_up, s, x);
  s = (r_dn <= 0.f) ? s_dn : s;
  return (r_up > 0.f) ? s_up : s;
}

template <bool INRANGE>
__device__ __forceinline__ void zero_step2(float& p0, float& p1, float& m0, float& m1, float& v0, float& v1, float ns,
                                           double rc, const AdamHyper& h) {
#pragma clang fp contract(off)
  pf2 m = {m0, m1}, v = {v0, v1};
  const pf2 w1 = {h.w1, h.w1}, b2 = {h.beta2, h.beta2};
  m = __builtin_elementwise_fma(w1, -m, m);
  v = v * b2;
  const float r0 = INRANGE ? sqrt_rn_inrange(v.x) : sqrt_rn(v.x), r1 = INRANGE ? sqrt_rn_inrange(v.y) : sqrt_rn(v.y);
  const float q0 = (float)((double)r0 * rc), q1 = (float)((double)r1 * rc);
  const pf2 den = pf2{q0, q1} + pf2{h.eps, h.eps};
  const pf2 u = pf2{ns, ns} * m;
  const pf2 d = INRANGE ? pf2{div_rn_inrange(u.x, den.x), div_rn_inrange(u.y, den.y)}
                        : pf2{__fdiv_rn(u.x, den.x), __fdiv_rn(u.y, den.y)};
  const pf2 p = pf2{p0, p1} + d;
  p0 = p.x; p1 = p.y; m0 = m.x; m1 = m.y; v0 = v.x; v1 = v.y;
}

// Zero steps [s0, s1) on KC float4 chunks of a lane (ring index of s0 = i0)
template <bool INRANGE>
__device__ __forceinline__ void zero_steps(float4 (&p)[KC], float4 (&m)[KC], float4 (&v)[KC],
                                           const float* __restrict__ hist, int cap, int i0, int64_t s0, int64_t s1,
                                           const AdamHyper& h) {
  int idx = i0;
  for (int64_t s = s0; s < s1; ++s) {
    const float* e = hist + kHist * idx;
    const float ns = e[0];
    const double rc = *reinterpret_cast<const double*>(e + 2);
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      zero_step2<INRANGE>(p[c].x, p[c].y, m[c].x, m[c].y, v[c].x, v[c].y, ns, rc, h);
      zero_step2<INRANGE>(p[c].z, p[c].w, m[c].z, m[c].w, v[c].z, v[c].w, ns, rc, h);
    }
    if (++idx == cap) idx = 0;
  }
}

// Range bounds for the in-range sqrt / division forms over zero steps [s0, s1) (wave-uniform, once
// per row): m and v only decay over zero steps (|m| by 1 - w1, v by beta2 per step, each rounding
// within 2^-24 relative), so with m_keep / v_keep = half the decay over n steps, bounds at the start
// cover every step; |neg_step| by the replayed entries' min / max, 1 / bc2_sqrt by their max.
struct ReplayRange {
  float ns_lo, ns_hi, m_keep, v_keep;
  bool ok;
};

__device__ __forceinline__ ReplayRange replay_range(const float* __restrict__ hist, int cap, int i0, int64_t s0,
                                                    int64_t s1, const AdamHyper& h) {
  ReplayRange r{INFINITY, 0.f, 0.f, 0.f, false};
  double rc_hi = 0.0;
  int idx = i0;
  for (int64_t s = s0; s < s1; ++s) {
    const float* e = hist + kHist * idx;
    r.ns_lo = fminf(r.ns_lo, fabsf(e[0]));
    r.ns_hi = fmaxf(r.ns_hi, fabsf(e[0]));
    rc_hi = fmax(rc_hi, *reinterpret_cast<const double*>(e + 2));
    if (++idx == cap) idx = 0;
  }
  const float n = (float)(s1 - s0);
  r.m_keep = 0.5f * __builtin_amdgcn_exp2f(n * __builtin_amdgcn_logf(1.0f - h.w1));
  r.v_keep = 0.5f * __builtin_amdgcn_exp2f(n * __builtin_amdgcn_logf(h.beta2));
  r.ok = h.eps >= 0x1p-40f && h.eps <= 1.0f && rc_hi <= 0x1p+10 && r.ns_hi <= 0x1p+10f && r.m_keep > 0.f &&
         r.v_keep > 0.f;
  return r;
}

// Wave-uniform: do these chunks keep u = neg_step * m in {0} U [2^-40, 2^40], v in {0} U [2^-96, 2^50]
// (so den = sqrt(v) / bc2_sqrt + eps lies in [2^-40, 2^40]) at every replayed step?
__device__ __forceinline__ bool chunks_in_range(const float4 (&m)[KC], const float4 (&v)[KC], const ReplayRange& r) {
  bool ok = r.ok;
#pragma unroll
  for (int c = 0; c < KC; ++c) {
    const float mm[4] = {m[c].x, m[c].y, m[c].z, m[c].w}, vv[4] = {v[c].x, v[c].y, v[c].z, v[c].w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const float am = fabsf(mm[k]);
      ok &= (am == 0.f) | ((am * r.m_keep * r.ns_lo >= 0x1p-40f) & (am * r.ns_hi <= 0x1p+30f));
      ok &= ((vv[k] == 0.f) | (vv[k] * r.v_keep >= 0x1p-96f)) & (vv[k] <= 0x1p+50f);
    }
  }
  return __all(ok);
}

// one row of `width` floats at P / M / V, lane-strided float4 chunks: zero steps [s0, s1), then (G
// non-null) step `st` with gradient row G.  Steps run in the outer loop over up to KC of the lane's
// chunks held in registers, so a step's history entry is read once per KC chunks; its ring index
// advances by one per step (no division), and s0 / s1 are wave-uniform (scalar loop).

__device__ __forceinline__ void replay_row(float* __restrict__ P, float* __restrict__ M, float* __restrict__ V,
                                           const float* __restrict__ G, int width, int lane,
                                           const float* __restrict__ hist, int cap, int64_t s0, int64_t s1,
                                           int64_t st, const AdamHyper& h) {
  s0 = __builtin_amdgcn_readfirstlane((int)s0);  // step indices fit in int32 (the last[] entries do)
  s1 = __builtin_amdgcn_readfirstlane((int)s1);
  const int i0 = s0 < s1 ? (int)(s0 % cap) : 0;
  const ReplayRange rr = (s0 < s1 && h.wd == 0.f) ? replay_range(hist, cap, i0, s0, s1, h) : ReplayRange{};
  for (int q0 = 4 * lane; q0 < width; q0 += 4 * 64 * KC) {
    float4 p[KC], m[KC], v[KC];
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int q = q0 + 4 * 64 * c;
      if (q < width) {
        p[c] = *reinterpret_cast<const float4*>(P + q);
        m[c] = *reinterpret_cast<const float4*>(M + q);
        v[c] = *reinterpret_cast<const float4*>(V + q);
      } else {
        p[c] = m[c] = v[c] = make_float4(0.f, 0.f, 0.f, 0.f);
      }
    }
    if (h.wd != 0.f) {  // weight decay makes g' = wd p nonzero: the general element step
      AdamHyper hs = h;
      int idx = i0;
      for (int64_t s = s0; s < s1; ++s) {
        const float* e = hist + kHist * idx;
        hs.neg_step = e[0];
        hs.bc2_sqrt = e[1];
#pragma unroll
        for (int c = 0; c < KC; ++c) {
          adam_elem(p[c].x, 0.f, m[c].x, v[c].x, hs);
          adam_elem(p[c].y, 0.f, m[c].y, v[c].y, hs);
          adam_elem(p[c].z, 0.f, m[c].z, v[c].z, hs);
          adam_elem(p[c].w, 0.f, m[c].w, v[c].w, hs);
        }
        if (++idx == cap) idx = 0;
      }
    } else if (s0 < s1) {
      if (chunks_in_range(m, v, rr)) zero_steps<true>(p, m, v, hist, cap, i0, s0, s1, h);
      else zero_steps<false>(p, m, v, hist, cap, i0, s0, s1, h);
    }
#pragma unroll
    for (int c = 0; c < KC; ++c) {
      const int q = q0 + 4 * 64 * c;
      if (q >= width) continue;
      if (G) {
        AdamHyper hs = h;
        const float* e = hist + kHist * (int)(st % cap);
        hs.neg_step = e[0];
        hs.bc2_sqrt = e[1];
        const float4 g = *reinterpret_cast<const float4*>(G + q);
        adam_elem(p[c].x, g.x, m[c].x, v[c].x, hs);
        adam_elem(p[c].y, g.y, m[c].y, v[c].y, hs);
        adam_elem(p[c].z, g.z, m[c].z, v[c].z, hs);
        adam_elem(p[c].w, g.w, m[c].w, v[c].w, hs);
      }
      *reinterpret_cast<float4*>(P + q) = p[c];
      *reinterpret_cast<float4*>(M + q) = m[c];
      *reinterpret_cast<float4*>(V + q) = v[c];
    }
  }
}

// FLUSH: one wave per (tensor, row), replay through step t, no gradient.  Step: one wave per
// (tensor, id) of the step's gradient ids; the row replays through t-1, then takes step t with its
// slot's gradient row
template <bool FLUSH>
__global__ __launch_bounds__(256) void adam_lazy_rows_kernel(LazyArgs a, AdamHyper h, const int32_t* skip) {
  if (skip && *skip) return;
  const int lane = threadIdx.x & 63;
  const int total = a.row_start[a.n];
  const int waves = gridDim.x * 4;
  int t = 0;
  for (int w = blockIdx.x * 4 + (threadIdx.x >> 6); w < total; w += waves) {
    while (t + 1 < a.n && w >= a.row_start[t + 1]) ++t;
    while (t > 0 && w < a.row_start[t]) --t;
    const int64_t st = a.step[t][0];  // step mode: this step (adam_lazy_inc_kernel has advanced the counter)
    int64_t r, s0;
    int32_t slot = -1;
    if constexpr (FLUSH) {
      r = w - a.row_start[t];
      s0 = (int64_t)a.last[t][r] + 1;
    } else {
      // wave per id: the wave whose atomicMax raises last[r] to st owns the row (duplicates skip)
      r = a.ids[t][w - a.row_start[t]];
      if (r < 0 || r >= a.nrows[t]) continue;
      slot = a.rmap[t][r];
      if (slot < 0) continue;
      int32_t old = 0;
      if (lane == 0) old = atomicMax(a.last[t] + r, (int32_t)st);
      old = __shfl(old, 0, 64);
      if ((int64_t)old >= st) continue;
      s0 = (int64_t)old + 1;
    }
    const int64_t s_end = FLUSH ? st + 1 : st;  // replayed zero-gradient steps: [s0, s_end)
    if (FLUSH && s0 > st) continue;
    float* __restrict__ P = a.p[t] + (r << a.rshift[t]);
    float* __restrict__ M = a.m[t] + (r << a.rshift[t]);
    float* __restrict__ V = a.v[t] + (r << a.rshift[t]);
    const float* __restrict__ G = FLUSH ? nullptr : a.g[t] + ((int64_t)slot << a.rshift[t]);
    replay_row(P, M, V, G, 1 << a.rshift[t], lane, a.hist[t], a.cap, s0, s_end, st, h);
    if (FLUSH && lane == 0) a.last[t][r] = (int32_t)st;
  }
}

// Catch-up before a gather: the rows a step is about to read (ids, duplicates allowed) replay their
// deferred zero-gradient steps through the current step, so the forward sees dense-Adam values.
// One wave per id; the wave whose atomicMax raises last[r] does the row, duplicates skip.
constexpr int kMaxCatch = 4;
struct CatchArgs {
  float* p[kMaxCatch];
  float* m[kMaxCatch];
  float* v[kMaxCatch];
  const int64_t* step[kMaxCatch];
  int32_t* last[kMaxCatch];
  const float* hist[kMaxCatch];
  int64_t rows[kMaxCatch];
  int32_t rshift[kMaxCatch];
};

__device__ __forceinline__ void catch_up_row(float* __restrict__ P0, float* __restrict__ M0, float* __restrict__ V0,
                                             const int64_t* step, const int64_t* __restrict__ ids, int64_t i,
                                             int64_t R, int rshift, int32_t* last, const float* __restrict__ hist,
                                             int cap, const AdamHyper& h);

// blockIdx.y = table: every table of the call catches up the same ids in one launch
__global__ __launch_bounds__(256) void adam_catch_up_multi_kernel(CatchArgs a, const int64_t* __restrict__ ids,
                                                                  int64_t n, int cap, AdamHyper h) {
  const int t = blockIdx.y;
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  catch_up_row(a.p[t], a.m[t], a.v[t], a.step[t], ids, i, a.rows[t], a.rshift[t], a.last[t], a.hist[t], cap, h);
}

__global__ __launch_bounds__(256) void adam_catch_up_kernel(float* __restrict__ P0, float* __restrict__ M0,
                                                            float* __restrict__ V0, const int64_t* step,
                                                            const int64_t* __restrict__ ids, int64_t n, int64_t R,
                                                            int rshift, int32_t* last, const float* __restrict__ hist,
                                                            int cap, AdamHyper h) {
  const int64_t i = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (i >= n) return;
  catch_up_row(P0, M0, V0, step, ids, i, R, rshift, last, hist, cap, h);
}

__device__ __forceinline__ void catch_up_at(float* __restrict__ P0, float* __restrict__ M0, float* __restrict__ V0,
                                            int64_t st, int64_t r, int rshift, int32_t* last,
                                            const float* __restrict__ hist, int cap, const AdamHyper& h);

__device__ __forceinline__ void catch_up_row(float* __restrict__ P0, float* __restrict__ M0, float* __restrict__ V0,
                                             const int64_t* step, const int64_t* __restrict__ ids, int64_t i,
                                             int64_t R, int rshift, int32_t* last, const float* __restrict__ hist,
                                             int cap, const AdamHyper& h) {
  const int64_t r = ids[i];
  if (r < 0 || r >= R) return;
  catch_up_at(P0, M0, V0, step[0], r, rshift, last, hist, cap, h);
}

// Background slice of a flush: at step counter st, rows [R s / K, R (s + 1) / K) of every table
// with s = st % K replay their deferred steps through st (the rows the step's own catch-up already
// claimed are current and skip).  Issued once per step, it bounds every row's backlog by K steps,
// so the flush that a full-table read needs costs K / 2 steps per row instead of the whole run's;
// the work is the same replay the flush would do, moved to a stream that overlaps the step.
// part ``part`` of ``nparts`` of the slice (rows split evenly; nparts 1: the whole slice)
__global__ __launch_bounds__(256) void adam_catch_up_slice_kernel(CatchArgs a, int nslices, int cap, AdamHyper h,
                                                                  int part, int nparts) {
  const int t = blockIdx.y;
  const int64_t st = a.step[t][0], R = a.rows[t];
  const int64_t s = st % nslices;
  const int64_t lo0 = R * s / nslices, hi0 = R * (s + 1) / nslices;
  const int64_t lo = lo0 + (hi0 - lo0) * part / nparts, hi = lo0 + (hi0 - lo0) * (part + 1) / nparts;
  // one wave per row; a capped grid (fr_adam_slice_blocks) strides over the slice
  for (int64_t r = lo + (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < hi; r += (int64_t)gridDim.x * 4)
    catch_up_at(a.p[t], a.m[t], a.v[t], st, r, a.rshift[t], a.last[t], a.hist[t], cap, h);
}

__device__ __forceinline__ void catch_up_at(float* __restrict__ P0, float* __restrict__ M0, float* __restrict__ V0,
                                            int64_t st, int64_t r, int rshift, int32_t* last,
                                            const float* __restrict__ hist, int cap, const AdamHyper& h) {
  const int lane = threadIdx.x & 63;
  int32_t old = 0;
  if (lane == 0) old = atomicMax(last + r, (int32_t)st);
  old = __shfl(old, 0, 64);
  if ((int64_t)old >= st) return;
  replay_row(P0 + (r << rshift), M0 + (r << rshift), V0 + (r << rshift), nullptr, 1 << rshift, lane, hist, cap,
             (int64_t)old + 1, st + 1, st, h);
}
}  // namespace

static int lazy_impl(bool flush, float* const* params, const float* const* grads, float* const* exp_avg,
                     float* const* exp_avg_sq, int64_t* const* d_steps, const int64_t* numel,
                     const int32_t* const* d_rmaps, const int64_t* const* d_ids, const int64_t* n_ids,
                     const int32_t* row_dims, int32_t* const* d_last,
                     float* const* d_hist, int32_t hist_cap, int n_tensors, const double* d_lr, double lr,
                     double beta1, double beta2, double eps, double weight_decay, const int32_t* d_skip,
                     void* stream) {
  FR_REQUIRE(n_tensors >= 0 && n_tensors <= kMaxLazy, "n_tensors out of range [0, 16]");
  if (n_tensors == 0) return FR_OK;
  FR_REQUIRE(params && exp_avg && exp_avg_sq && d_steps && numel && row_dims && d_last && d_hist,
             "null host array");
  FR_REQUIRE(flush || (grads && d_rmaps), "grads and d_rmaps required");
  FR_REQUIRE(hist_cap >= 2, "hist_cap < 2");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  AdamHyper h{};
  h.lr = lr;
  h.beta1_d = beta1;
  h.beta2_d = beta2;
  h.d_lr = d_lr;
  h.w1 = (float)(1.0 - beta1);
  h.beta2 = (float)beta2;
  h.one_m_b2 = (float)(1.0 - beta2);
  h.eps = (float)eps;
  h.wd = (float)weight_decay;
  LazyArgs a{};
  a.n = n_tensors;
  a.cap = hist_cap;
  int64_t rows = 0;
  for (int t = 0; t < n_tensors; ++t) {
    const int32_t dd = row_dims[t];
    FR_REQUIRE(dd >= 4 && (dd & (dd - 1)) == 0 && numel[t] % dd == 0,
               "lazy row tensors need a power-of-two row width >= 4");
    FR_REQUIRE(params[t] && exp_avg[t] && exp_avg_sq[t] && d_steps[t] && d_last[t] && d_hist[t],
               "null tensor pointer");
    FR_REQUIRE(fr::aligned16(params[t]) && fr::aligned16(exp_avg[t]) && fr::aligned16(exp_avg_sq[t]),
               "lazy row tensors must be 16-byte aligned");
    a.p[t] = params[t];
    a.m[t] = exp_avg[t];
    a.v[t] = exp_avg_sq[t];
    a.step[t] = d_steps[t];
    a.last[t] = d_last[t];
    a.hist[t] = d_hist[t];
    a.nrows[t] = numel[t] / dd;
    a.row_start[t] = (int32_t)rows;
    if (!flush) {
      FR_REQUIRE(grads[t] && d_rmaps[t] && fr::aligned16(grads[t]), "null or misaligned gradient rows");
      FR_REQUIRE(n_ids[t] >= 0 && (n_ids[t] == 0 || d_ids[t]), "null ids");
      a.g[t] = grads[t];
      a.rmap[t] = d_rmaps[t];
      a.ids[t] = d_ids[t];
      rows += n_ids[t];
    } else {
      rows += a.nrows[t];
    }
    a.rshift[t] = 0;
    while ((1 << a.rshift[t]) < dd) ++a.rshift[t];
    FR_REQUIRE(rows < INT32_MAX, "too many rows for one launch");
  }
  a.row_start[n_tensors] = (int32_t)rows;
  const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(rows, 4), (int64_t)fr::kNumCU * 8);
  if (flush) {
    if (rows == 0) return FR_OK;
    hipLaunchKernelGGL(adam_lazy_rows_kernel<true>, dim3(blocks), dim3(256), 0, s, a, h, nullptr);
  } else {
    // the step counter advances even when no row carries a gradient (dense semantics)
    hipLaunchKernelGGL(adam_lazy_inc_kernel, dim3(1), dim3(64), 0, s, a, h, d_skip);
    FR_LAUNCH_CHECK();
    if (rows == 0) return FR_OK;
    hipLaunchKernelGGL(adam_lazy_rows_kernel<false>, dim3(blocks), dim3(256), 0, s, a, h, d_skip);
  }
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_adam_step_rows_lazy(float* const* params, const float* const* grads, float* const* exp_avg,
                                      float* const* exp_avg_sq, int64_t* const* d_steps, const int64_t* numel,
                                      const int32_t* const* d_rmaps, const int64_t* const* d_ids,
                                      const int64_t* n_ids, const int32_t* row_dims, int32_t* const* d_last,
                                      float* const* d_hist, int32_t hist_cap, int n_tensors, const double* d_lr,
                                      double lr, double beta1, double beta2, double eps, double weight_decay,
                                      const int32_t* d_skip, void* stream) {
  FR_REQUIRE(d_ids && n_ids, "d_ids and n_ids required");
  return lazy_impl(false, params, grads, exp_avg, exp_avg_sq, d_steps, numel, d_rmaps, d_ids, n_ids, row_dims,
                   d_last, d_hist,
                   hist_cap, n_tensors, d_lr, lr, beta1, beta2, eps, weight_decay, d_skip, stream);
}

extern "C" int fr_adam_flush_rows(float* const* params, float* const* exp_avg, float* const* exp_avg_sq,
                                  int64_t* const* d_steps, const int64_t* numel, const int32_t* row_dims,
                                  int32_t* const* d_last, float* const* d_hist, int32_t hist_cap, int n_tensors,
                                  double beta1, double beta2, double eps, double weight_decay, void* stream) {
  return lazy_impl(true, params, nullptr, exp_avg, exp_avg_sq, d_steps, numel, nullptr, nullptr, nullptr, row_dims,
                   d_last, d_hist,
                   hist_cap, n_tensors, nullptr, 0.0, beta1, beta2, eps, weight_decay, nullptr, stream);
}


static int adam_impl(float* const* params, const float* const* grads, float* const* exp_avg,
                     float* const* exp_avg_sq, int64_t* const* d_steps, const int64_t* numel,
                     int n_tensors, double lr, const double* d_lr, double beta1, double beta2,
                     double eps, double weight_decay, int64_t step, const int32_t* d_skip,
                     void* stream, const int32_t* const* rmaps = nullptr, const int32_t* row_dims = nullptr,
                     uint32_t* d_ticket = nullptr) {
  FR_REQUIRE(n_tensors >= 0, "n_tensors < 0");
  FR_REQUIRE(!d_steps || (d_ticket && fr::aligned16(d_ticket)),
             "device-scalar mode needs the caller's 16-byte aligned ticket words (FR_ADAM_TICKET_WORDS)");
  if (n_tensors == 0) return FR_OK;
  FR_REQUIRE(params && grads && exp_avg && exp_avg_sq && numel, "null host array");
  FR_REQUIRE(d_steps || step >= 1, "step must be >= 1 (1-based, after increment)");
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  // bias corrections in double, as the Python scalars in torch.optim.Adam
  const double bc1 = 1.0 - std::pow(beta1, (double)(d_steps ? 1 : step));
  const double bc2 = 1.0 - std::pow(beta2, (double)(d_steps ? 1 : step));
  AdamHyper h;
  h.lr = lr;
  h.beta1_d = beta1;
  h.beta2_d = beta2;
  h.d_lr = d_lr;
  // hyper-parameters arrive as doubles (Python floats) and are rounded to f32 where torch's
  // tensor ops round them: lerp weight 1-b1, mul_ b2, addcmul value 1-b2, eps, step size
  h.w1 = (float)(1.0 - beta1);
  h.beta2 = (float)beta2;
  h.one_m_b2 = (float)(1.0 - beta2);
  h.neg_step = (float)(-(lr / bc1));
  h.bc2_sqrt = (float)std::sqrt(bc2);
  h.eps = (float)eps;
  h.wd = (float)weight_decay;
  // dense tensors and row-gradient tensors go to separate launches (separate register budgets)
  for (int rows_pass = 0; rows_pass < 2; ++rows_pass) {
    int idx[kMaxTensors];
    int t = 0;
    while (t < n_tensors) {
      AdamArgs a{};
      a.n = 0;
      a.ticket = d_ticket ? reinterpret_cast<unsigned*>(d_ticket) + 16 * rows_pass : nullptr;
      int32_t blocks = 0;
      for (; t < n_tensors && a.n < kMaxTensors; ++t) {
        const bool is_rows = rmaps && rmaps[t];
        if (is_rows != (rows_pass == 1)) continue;
        FR_REQUIRE(numel[t] >= 0, "numel < 0");
        if (numel[t] == 0) continue;
        FR_REQUIRE(params[t] && grads[t] && exp_avg[t] && exp_avg_sq[t], "null tensor pointer");
        const int k = a.n++;
        idx[k] = t;
        a.p[k] = params[t];
        a.g[k] = grads[t];
        a.m[k] = exp_avg[t];
        a.v[k] = exp_avg_sq[t];
        a.step[k] = d_steps ? d_steps[t] : nullptr;
        FR_REQUIRE(!d_steps || d_steps[t], "null step counter");
        a.numel[k] = numel[t];
        a.vec4[k] = fr::aligned16(params[t]) && fr::aligned16(grads[t]) && fr::aligned16(exp_avg[t]) &&
                    fr::aligned16(exp_avg_sq[t]);
        a.rmap[k] = is_rows ? rmaps[t] : nullptr;
        a.rshift[k] = 0;
        if (is_rows) {
          const int32_t dd = row_dims[t];
          FR_REQUIRE(dd >= 4 && (dd & (dd - 1)) == 0 && numel[t] % dd == 0,
                     "row-gradient tensors need a power-of-two row width >= 4");
          FR_REQUIRE(a.vec4[k], "row-gradient tensors must be 16-byte aligned");
          while ((1 << a.rshift[k]) < dd) ++a.rshift[k];
        }
        a.blk_start[k] = blocks;
        const int64_t nb = fr::ceil_div(numel[t], kChunk);
        FR_REQUIRE(blocks + nb < INT32_MAX, "tensor too large for one launch");
        blocks += (int32_t)nb;
      }
      a.blk_start[a.n] = blocks;
      if (a.n == 0) continue;
      (void)idx;
      // device-scalar mode: the kernel's last block advances the step counters
      int64_t state_bytes = 0;
      for (int k = 0; k < a.n; ++k) state_bytes += 28 * a.numel[k];
      const bool nt = state_bytes > kTemporalBytes;
      const dim3 grid((unsigned)std::min<int32_t>(blocks, kAdamBlocks));
      if (rows_pass && nt)
        hipLaunchKernelGGL((adam_kernel<true, true>), grid, dim3(256), 0, s, a, h, d_skip);
      else if (rows_pass)
        hipLaunchKernelGGL((adam_kernel<true, false>), grid, dim3(256), 0, s, a, h, d_skip);
      else if (nt)
        hipLaunchKernelGGL((adam_kernel<false, true>), grid, dim3(256), 0, s, a, h, d_skip);
      else
        hipLaunchKernelGGL((adam_kernel<false, false>), grid, dim3(256), 0, s, a, h, d_skip);
      FR_LAUNCH_CHECK();
    }
  }
  return FR_OK;
}

extern "C" int fr_adam_step(float* const* params, const float* const* grads, float* const* exp_avg,
                            float* const* exp_avg_sq, const int64_t* numel, int n_tensors,
                            int64_t max_numel, double lr, double beta1, double beta2, double eps,
                            double weight_decay, int64_t step, const int32_t* d_skip, void* stream) {
  (void)max_numel;
  return adam_impl(params, grads, exp_avg, exp_avg_sq, nullptr, numel, n_tensors, lr, nullptr, beta1,
                   beta2, eps, weight_decay, step, d_skip, stream);
}

extern "C" int fr_adam_step_dev(float* const* params, const float* const* grads, float* const* exp_avg,
                                float* const* exp_avg_sq, int64_t* const* d_steps, const int64_t* numel,
                                int n_tensors, const double* d_lr, double lr, double beta1, double beta2,
                                double eps, double weight_decay, const int32_t* d_skip, uint32_t* d_ticket,
                                void* stream) {
  FR_REQUIRE(d_steps, "d_steps (device step counters) required");
  return adam_impl(params, grads, exp_avg, exp_avg_sq, d_steps, numel, n_tensors, lr, d_lr, beta1,
                   beta2, eps, weight_decay, 0, d_skip, stream, nullptr, nullptr, d_ticket);
}

extern "C" int fr_adam_step_rows(float* const* params, const float* const* grads, float* const* exp_avg,
                                 float* const* exp_avg_sq, int64_t* const* d_steps, const int64_t* numel,
                                 const int32_t* const* d_rmaps, const int32_t* row_dims, int n_tensors,
                                 const double* d_lr, double lr, double beta1, double beta2, double eps,
                                 double weight_decay, const int32_t* d_skip, uint32_t* d_ticket, void* stream) {
  FR_REQUIRE(d_steps && d_rmaps && row_dims, "d_steps, d_rmaps and row_dims required");
  return adam_impl(params, grads, exp_avg, exp_avg_sq, d_steps, numel, n_tensors, lr, d_lr, beta1, beta2, eps,
                   weight_decay, 0, d_skip, stream, d_rmaps, row_dims, d_ticket);
}

extern "C" int fr_adam_step_bf16(uint16_t* d_param, float* d_master, const uint16_t* d_grad, float* d_exp_avg,
                                 float* d_exp_avg_sq, int64_t* d_step, int64_t numel, const double* d_lr,
                                 double lr, double beta1, double beta2, double eps, double weight_decay,
                                 const int32_t* d_skip, void* stream) {
  FR_REQUIRE(numel >= 0 && numel % 8 == 0, "numel must be a multiple of 8");
  if (numel == 0) return FR_OK;
  FR_REQUIRE(d_param && d_master && d_grad && d_exp_avg && d_exp_avg_sq && d_step, "null pointer");
  for (const void* p : {(const void*)d_param, (const void*)d_master, (const void*)d_grad, (const void*)d_exp_avg,
                        (const void*)d_exp_avg_sq})
    FR_REQUIRE(fr::aligned16(p), "tensors must be 16-B aligned");
  AdamHyper h;
  h.lr = lr;
  h.beta1_d = beta1;
  h.beta2_d = beta2;
  h.d_lr = d_lr;
  h.w1 = (float)(1.0 - beta1);
  h.beta2 = (float)beta2;
  h.one_m_b2 = (float)(1.0 - beta2);
  h.neg_step = 0.f;
  h.bc2_sqrt = 1.f;
  h.eps = (float)eps;
  h.wd = (float)weight_decay;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(adam_bf16_step_inc_kernel, dim3(1), dim3(64), 0, s, d_step, d_skip);
  FR_LAUNCH_CHECK();
  const int64_t n8 = numel / 8;
  const unsigned blocks = (unsigned)std::min<int64_t>(fr::ceil_div(n8, 256), (int64_t)fr::kNumCU * 8);
  hipLaunchKernelGGL(adam_bf16_kernel, dim3(blocks), dim3(256), 0, s, reinterpret_cast<uint4*>(d_param), d_master,
                     reinterpret_cast<const uint4*>(d_grad), d_exp_avg, d_exp_avg_sq, n8, d_step, h, d_skip);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_adam_catch_up_rows(float* param, float* exp_avg, float* exp_avg_sq, const int64_t* d_step,
                                     const int64_t* d_ids, int64_t n, int64_t rows, int32_t row_dim, int32_t* d_last,
                                     const float* d_hist, int32_t hist_cap, double beta1, double beta2, double eps,
                                     double weight_decay, void* stream) {
  FR_REQUIRE(n >= 0 && rows >= 0, "negative size");
  if (n == 0 || rows == 0) return FR_OK;
  FR_REQUIRE(param && exp_avg && exp_avg_sq && d_step && d_ids && d_last && d_hist, "null pointer");
  FR_REQUIRE(row_dim >= 4 && (row_dim & (row_dim - 1)) == 0, "row width must be a power of two >= 4");
  FR_REQUIRE(hist_cap >= 2, "hist_cap < 2");
  FR_REQUIRE(fr::aligned16(param) && fr::aligned16(exp_avg) && fr::aligned16(exp_avg_sq), "16-byte alignment");
  FR_REQUIRE(rows < INT32_MAX, "too many rows");
  AdamHyper h{};
  h.beta1_d = beta1;
  h.beta2_d = beta2;
  h.w1 = (float)(1.0 - beta1);
  h.beta2 = (float)beta2;
  h.one_m_b2 = (float)(1.0 - beta2);
  h.eps = (float)eps;
  h.wd = (float)weight_decay;
  int rshift = 0;
  while ((1 << rshift) < row_dim) ++rshift;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(adam_catch_up_kernel, dim3((unsigned)fr::ceil_div(n, 4)), dim3(256), 0, s, param, exp_avg,
                     exp_avg_sq, d_step, d_ids, n, rows, rshift, d_last, d_hist, hist_cap, h);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

// CatchArgs + hyper-parameters of a multi-table catch-up launch (tables of one parameter group)
static int catch_args(int n_tables, float* const* params, float* const* exp_avg, float* const* exp_avg_sq,
                      const int64_t* const* d_steps, const int64_t* rows, const int32_t* row_dims,
                      int32_t* const* d_last, const float* const* d_hist, int32_t hist_cap, double beta1,
                      double beta2, double eps, double weight_decay, CatchArgs& a, AdamHyper& h) {
  FR_REQUIRE(params && exp_avg && exp_avg_sq && d_steps && rows && row_dims && d_last && d_hist, "null pointer");
  FR_REQUIRE(hist_cap >= 2, "hist_cap < 2");
  a = CatchArgs{};
  for (int t = 0; t < n_tables; ++t) {
    FR_REQUIRE(params[t] && exp_avg[t] && exp_avg_sq[t] && d_steps[t] && d_last[t] && d_hist[t], "null tensor");
    FR_REQUIRE(row_dims[t] >= 4 && (row_dims[t] & (row_dims[t] - 1)) == 0, "row width must be a power of two >= 4");
    FR_REQUIRE(fr::aligned16(params[t]) && fr::aligned16(exp_avg[t]) && fr::aligned16(exp_avg_sq[t]),
               "16-byte alignment");
    FR_REQUIRE(rows[t] >= 0 && rows[t] < INT32_MAX, "rows out of range");
    a.p[t] = params[t];
    a.m[t] = exp_avg[t];
    a.v[t] = exp_avg_sq[t];
    a.step[t] = d_steps[t];
    a.last[t] = d_last[t];
    a.hist[t] = d_hist[t];
    a.rows[t] = rows[t];
    int sh = 0;
    while ((1 << sh) < row_dims[t]) ++sh;
    a.rshift[t] = sh;
  }
  h = AdamHyper{};
  h.beta1_d = beta1;
  h.beta2_d = beta2;
  h.w1 = (float)(1.0 - beta1);
  h.beta2 = (float)beta2;
  h.one_m_b2 = (float)(1.0 - beta2);
  h.eps = (float)eps;
  h.wd = (float)weight_decay;
  return FR_OK;
}

extern "C" int fr_adam_catch_up_rows_multi(int n_tables, float* const* params, float* const* exp_avg,
                                           float* const* exp_avg_sq, const int64_t* const* d_steps,
                                           const int64_t* rows, const int32_t* row_dims, int32_t* const* d_last,
                                           const float* const* d_hist, const int64_t* d_ids, int64_t n,
                                           int32_t hist_cap, double beta1, double beta2, double eps,
                                           double weight_decay, void* stream) {
  FR_REQUIRE(n_tables >= 0 && n_tables <= kMaxCatch, "n_tables out of range [0, 4]");
  FR_REQUIRE(n >= 0, "negative size");
  if (n == 0 || n_tables == 0) return FR_OK;
  FR_REQUIRE(d_ids, "null ids");
  CatchArgs a;
  AdamHyper h;
  const int rc = catch_args(n_tables, params, exp_avg, exp_avg_sq, d_steps, rows, row_dims, d_last, d_hist, hist_cap,
                            beta1, beta2, eps, weight_decay, a, h);
  if (rc != FR_OK) return rc;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(adam_catch_up_multi_kernel, dim3((unsigned)fr::ceil_div(n, 4), (unsigned)n_tables), dim3(256), 0,
                     s, a, d_ids, n, hist_cap, h);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

// A/B: the background slice's grid capped at this many workgroups in total (0: one wave per row)
static int64_t g_slice_blocks = 0;

extern "C" int fr_adam_slice_blocks(int64_t max_blocks) {
  FR_REQUIRE(max_blocks >= 0, "max_blocks must be >= 0");
  g_slice_blocks = max_blocks;
  return FR_OK;
}

extern "C" int fr_adam_catch_up_slice_part(int n_tables, float* const* params, float* const* exp_avg,
                                           float* const* exp_avg_sq, const int64_t* const* d_steps, const int64_t* rows,
                                           const int32_t* row_dims, int32_t* const* d_last, const float* const* d_hist,
                                           int32_t n_slices, int32_t part, int32_t n_parts, int32_t hist_cap,
                                           double beta1, double beta2, double eps, double weight_decay, void* stream) {
  FR_REQUIRE(n_tables >= 0 && n_tables <= kMaxCatch, "n_tables out of range [0, 4]");
  FR_REQUIRE(n_slices >= 1, "n_slices < 1");
  FR_REQUIRE(n_parts >= 1 && part >= 0 && part < n_parts, "part out of range [0, n_parts)");
  if (n_tables == 0) return FR_OK;
  CatchArgs a;
  AdamHyper h;
  const int rc = catch_args(n_tables, params, exp_avg, exp_avg_sq, d_steps, rows, row_dims, d_last, d_hist, hist_cap,
                            beta1, beta2, eps, weight_decay, a, h);
  if (rc != FR_OK) return rc;
  int64_t most = 0;
  for (int t = 0; t < n_tables; ++t)
    most = std::max<int64_t>(most, fr::ceil_div(fr::ceil_div(rows[t], (int64_t)n_slices), (int64_t)n_parts));
  if (most == 0) return FR_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  int64_t gx = fr::ceil_div(most + 1, 4);
  if (g_slice_blocks > 0) gx = std::min<int64_t>(gx, std::max<int64_t>(1, g_slice_blocks / n_tables));
  hipLaunchKernelGGL(adam_catch_up_slice_kernel, dim3((unsigned)gx, (unsigned)n_tables),
                     dim3(256), 0, s, a, n_slices, hist_cap, h, part, n_parts);
  FR_LAUNCH_CHECK();
  return FR_OK;
}

extern "C" int fr_adam_catch_up_slice(int n_tables, float* const* params, float* const* exp_avg,
                                      float* const* exp_avg_sq, const int64_t* const* d_steps, const int64_t* rows,
                                      const int32_t* row_dims, int32_t* const* d_last, const float* const* d_hist,
                                      int32_t n_slices, int32_t hist_cap, double beta1, double beta2, double eps,
                                      double weight_decay, void* stream) {
  return fr_adam_catch_up_slice_part(n_tables, params, exp_avg, exp_avg_sq, d_steps, rows, row_dims, d_last, d_hist,
                                     n_slices, 0, 1, hist_cap, beta1, beta2, eps, weight_decay, stream);
}

// ---- self-test of the rounding shortcuts (diagnostic; tests/test_rowgrad_gpu.py) ---------------
namespace {
__device__ __forceinline__ uint32_t st_hash(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)((z ^ (z >> 31)) >> 32);
}

// reference sqrt: the correctly rounded double root rounded to fp32 (double rounding is innocuous
// for sqrt from 53 >= 2 * 24 + 2 bits)
__device__ __forceinline__ float st_ref_sqrt(float x) { return (float)__dsqrt_rn((double)x); }

// a float with random significand and exponent uniform in [e_lo, e_hi] (both inclusive, unbiased
// exponents), random sign if sgn
__device__ __forceinline__ float st_rand(uint64_t key, int e_lo, int e_hi, bool sgn) {
  const uint32_t h = st_hash(key);
  const int e = e_lo + (int)(st_hash(key ^ 0x5851F42D4C957F2Dull) % (uint32_t)(e_hi - e_lo + 1));
  const uint32_t bits = ((uint32_t)(e + 127) << 23) | (h & 0x7FFFFFu) | (sgn ? (h & 0x80000000u) : 0u);
  return __uint_as_float(bits);
}

// per element i: div_rn_inrange(a, b) vs the compiler's IEEE division over the documented range;
// sqrt_rn_inrange(x) for x in [2^-96, 2^127] and sqrt_rn(x) for x over every positive float
// (denormals included) vs the compiler's correctly rounded sqrt.  Mismatch counts -> bad[0..2].
__global__ void rounding_selftest_kernel(int64_t n, uint64_t seed, unsigned long long* bad) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t k = seed * 0x9E3779B97F4A7C15ull + (uint64_t)i * 4;
  float a = st_rand(k, -40, 39, true);
  if ((i & 255) == 0) a = 0.f;
  const float b = st_rand(k + 1, -40, 39, false);
  if (__float_as_uint(div_rn_inrange(a, b)) != __float_as_uint(__fdiv_rn(a, b))) atomicAdd(bad, 1ull);
  const float x = st_rand(k + 2, -96, 127, false);
  if (__float_as_uint(sqrt_rn_inrange(x)) != __float_as_uint(st_ref_sqrt(x))) atomicAdd(bad + 1, 1ull);
  const float y = __uint_as_float(st_hash(k + 3) & 0x7F7FFFFFu);  // any finite non-negative float
  if (__float_as_uint(sqrt_rn(y)) != __float_as_uint(st_ref_sqrt(y))) atomicAdd(bad + 2, 1ull);
}
}  // namespace

extern "C" int fr_adam_rounding_selftest(int64_t n, uint64_t seed, unsigned long long* d_bad, void* stream) {
  FR_REQUIRE(n >= 0 && d_bad, "bad arguments");
  if (n == 0) return FR_OK;
  hipLaunchKernelGGL(rounding_selftest_kernel, dim3((unsigned)fr::ceil_div(n, (int64_t)256)), dim3(256), 0,
                     reinterpret_cast<hipStream_t>(stream), n, seed, d_bad);
  FR_LAUNCH_CHECK();
  return FR_OK;
}
