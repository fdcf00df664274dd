// float_quant.hip — qtorch-style bit-level float quantisation (FP8 E5M2 / FP16 / BF16 / any
// exp,man) and the S2FP8 shift-and-squeeze round trip, for gfx950.
//
// Reference:
//   smart_compress/util/pytorch/quantization.py:187-204  float_quantize (+ check_inf, 195-199)
//   smart_compress/util/pytorch/quantization.py:138-150  _get_max_value (nearest-quantised FLT_MAX)
//   smart_compress/compress/fp8.py:27-31                 exp=5, man=2 (E5M2), stochastic
//   smart_compress/compress/s2fp8.py:27-48               log2-domain mean/max, power squeeze
//   qtorch 0.2.0 (un-vendored dependency, poetry.lock:773-781): quant_function.float_quantize ->
//     float_kernel_stochastic / float_kernel_nearest + bit_helper round_bitwise_* / clip_exponent.
//     Restated here from its published algorithm (integer arithmetic on the fp32 bit pattern).
//
// One launch of 8 B/elem for float_quantize: the reference materialises a randint_like int32
// tensor (+8 B/elem), runs the quantiser and then 3-4 more passes for check_inf; here the random
// word comes from the counter-based RNG in registers and check_inf is fused.
#include <float.h>
#include <limits.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "qtorch.h"
#include "smaq_elem.h"
#include "smaq_host.h"
#include "smq_common.h"

namespace smq {

struct FQArgs {
  const void* x;
  void* y;
  int64_t n;
  const uint32_t* rand_bits;
  const uint64_t* ctr;  // graph-safe stream position (read here, advanced by fq_bump_kernel)
  uint32_t key;
  uint64_t offset;
  int exp_bits, man_bits;
  int check_inf;
  float max_value;
  int nt_loads;  // non-temporal x loads: inputs of >= kFqNtMinMB only (see smq_float_quant)
};

// y element stores: fp32, or fp16 (precision 16: float_quantize returns .half(), RN)
template <bool HOUT>
__device__ __forceinline__ void store4_out(void* y, int64_t j, float4 o) {
  if (!HOUT) {
    store_stream(static_cast<float4*>(y) + j, o);
  } else {
    const uint32_t lo = (uint32_t)__builtin_bit_cast(uint16_t, __float2half_rn(o.x)) |
                        ((uint32_t)__builtin_bit_cast(uint16_t, __float2half_rn(o.y)) << 16);
    const uint32_t hi = (uint32_t)__builtin_bit_cast(uint16_t, __float2half_rn(o.z)) |
                        ((uint32_t)__builtin_bit_cast(uint16_t, __float2half_rn(o.w)) << 16);
    static_cast<uint2*>(y)[j] = make_uint2(lo, hi);
  }
}

template <bool HOUT>
__device__ __forceinline__ void store1_out(void* y, int64_t e, float v) {
  if (!HOUT) static_cast<float*>(y)[e] = v;
  else static_cast<__half*>(y)[e] = __float2half_rn(v);
}



// abs(y - max) <= FLT_EPSILON -> +inf (quantization.py:195-199)
__device__ __forceinline__ float check_inf_fn(float y, const FQArgs& A) {
  return (A.check_inf && fabsf(y - A.max_value) <= FLT_EPSILON) ? INFINITY : y;
}

constexpr int kFqDefaultTileV = 1;  // float4 per lane per tile (flat tiles; SMQ_FQ_TILE=1|2|4)

// TIN: element type of x (quantised as its exact fp32 value); HOUT: fp16 y (the `.half()` of
// quantization.py:201-202 fused into the store).
template <bool SR, bool RARR, bool VEC, int kFqTileV, int TIN, bool HOUT>
__global__ __launch_bounds__(kBlock) void float_quant_kernel(FQArgs A) {
  constexpr int kFqTileElems = kBlock * kFqTileV * 4;
  const int64_t n = A.n;
  const uint64_t off = A.offset + (A.ctr ? *A.ctr : 0ull);
  auto rb = [&](int64_t e) -> uint32_t {
    if (!SR) return 0u;
    return RARR ? A.rand_bits[e] : rng_u32(A.key, off + (uint64_t)e);
  };
  auto q1 = [&](float v, uint32_t r) {
    return check_inf_fn(qtorch_quant(v, r, A.exp_bits, A.man_bits, SR), A);
  };
  if (VEC) {
    const uint4* __restrict__ r4 = reinterpret_cast<const uint4*>(A.rand_bits);
    const int64_t nv = n >> 2;
    const int64_t t0 = (int64_t)blockIdx.x * (kBlock * kFqTileV) + threadIdx.x;
    float4 v[kFqTileV];
#pragma unroll
    for (int u = 0; u < kFqTileV; ++u) {
      const int64_t j = t0 + u * kBlock;
      if (j < nv) v[u] = A.nt_loads ? load4_stream<TIN>(A.x, j) : load4<TIN>(A.x, j);
    }
#pragma unroll
    for (int u = 0; u < kFqTileV; ++u) {
      const int64_t j = t0 + u * kBlock;
      if (j >= nv) continue;
      uint32_t r0, r1, r2, r3;
      if (SR && RARR) {
        const uint4 rr = r4[j];
        r0 = rr.x; r1 = rr.y; r2 = rr.z; r3 = rr.w;
      } else {
        r0 = rb(4 * j); r1 = rb(4 * j + 1); r2 = rb(4 * j + 2); r3 = rb(4 * j + 3);
      }
      float4 o;
      o.x = q1(v[u].x, r0);
      o.y = q1(v[u].y, r1);
      o.z = q1(v[u].z, r2);
      o.w = q1(v[u].w, r3);
      store4_out<HOUT>(A.y, j, o);
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x < (int)(n & 3)) {
      const int64_t e = (nv << 2) + threadIdx.x;
      store1_out<HOUT>(A.y, e, q1(load1<TIN>(A.x, e), rb(e)));
    }
  } else {
    const int64_t e0 = (int64_t)blockIdx.x * kFqTileElems + threadIdx.x;
    for (int k = 0; k < kFqTileElems / kBlock; ++k) {
      const int64_t e = e0 + (int64_t)k * kBlock;
      if (e >= n) break;
      store1_out<HOUT>(A.y, e, q1(load1<TIN>(A.x, e), rb(e)));
    }
  }
}

// Graph-safe stream: after the launch that read *ctr, advance it by the elements drawn.
__global__ void fq_bump_kernel(uint64_t* ctr, uint64_t n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *ctr += n;
}

// ---- S2FP8 ---------------------------------------------------------------------------------------
struct alignas(16) S2Partial {
  double s;  // sum of log2|x| (zeros as 0)
  float m;   // max (NaN-propagating)
  float pad;
};

__device__ __forceinline__ float nan_max(float a, float b) {
  return (b > a || b != b) ? b : a;  // torch.max propagates NaN
}

// Rounding of one S2FP8 op to its torch dtype. fp16 goes through an opaque v_cvt_f16_f32: left to
// itself the compiler fuses `fptrunc(a * b)` into v_fma_mixlo_f16(a, b, +0), which rounds the exact
// product once (torch rounds to fp32 first, then to half) and turns a -0 product into +0.
template <int T>
__device__ __forceinline__ float s2_round(float v) {
  if (T == kF16) {
    uint32_t h;
    asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(h) : "v"(v));
    return __half2float(__builtin_bit_cast(__half, (uint16_t)(h & 0xffffu)));
  }
  return round_in<T>(v);
}

template <int TIN>
__device__ __forceinline__ float s2_log(float x) {
  const float a = fabsf(x);
  return (a == 0.0f) ? a : s2_round<TIN>(log2f(a));  // torch.where(X_abs == 0.0, X_abs, torch.log2(X_abs))
}

// Graph-safe stream position: the snapshot of *ctr, advanced by n (0 without a counter). One
// thread of the call's first launch runs it; later launches read the snapshot.
__device__ __forceinline__ uint64_t take_offset(uint64_t* ctr, uint64_t n) {
  if (!ctr) return 0ull;
  const uint64_t o = *ctr;
  *ctr = o + n;
  return o;
}

// s2fp8.py:31-43 from (sum, max) of the log2 values. TIN = the input type: the reference's torch
// ops run in it (precision 16 with fp16/bf16 tensors), each op = its fp32 value rounded to TIN
// (round_in, the identity for fp32); torch rounds the mean's fp32 quotient once.
template <int TIN>
__device__ void s2fp8_derive(float mu, float m, uint32_t n_used, SmqS2fp8Stats* out) {
  // s2fp8.py:42 `15.0 / (m - mu)`: Python scalar / tensor is Tensor.__rtruediv__ =
  // reciprocal() * 15.0 — two roundings, not one division.
  const float alpha = s2_round<TIN>(s2_round<TIN>(1.0f / s2_round<TIN>(m - mu)) * 15.0f);
  const float beta = s2_round<TIN>((-alpha) * mu);                   // s2fp8.py:43
  const float bp2 = s2_round<TIN>((float)exp2((double)beta));        // 2.0 ** beta, correctly rounded
  out->mu = mu;
  out->m = m;
  out->alpha = alpha;
  out->beta = beta;
  out->beta_pow2 = bp2;
  out->inv_beta_pow2 = s2_round<TIN>(1.0f / bp2);  // beta_pow2.reciprocal_()
  out->inv_alpha = s2_round<TIN>(1.0f / alpha);    // alpha.reciprocal_()
  out->n_used = n_used;
}

template <int TIN>
__device__ void s2fp8_finalize(double s, float m, int64_t n, SmqS2fp8Stats* out) {
  const float mu = s2_round<TIN>((float)(s / (double)n));  // torch.mean(X_abs_log2)
  s2fp8_derive<TIN>(mu, m, (uint32_t)(n > 0xffffffffLL ? 0xffffffffu : (uint32_t)n), out);
}

// Statistics partials. The old shape (last-arriving workgroup reduces, one counter) paid ~12 ns of
// serialised atomic per arriving workgroup plus the tail workgroup's reduction round trip, and
// its tile-stride loop one HBM round trip per 16 KiB tile: 11.6 us at C4 for 12.6 MB. Here every
// workgroup issues all loads of a round (kS2Loads dwordx4 per lane) before consuming any, stores
// one plain partial and exits; the apply launch (after the kernel boundary, which makes the
// partials visible) reduces the <= kS2Partials partials in every workgroup, in one fixed order.
// Measured at C4 (rocprofv3, 48 rotating buffers): partials 7.7 us + apply 10.3 us, step 17.4 us
// (was 19.1); the same partials with a last-arriver derive instead: 10.8 + 7.4, step 18.4 us.
// 128 / 64 partials: 9.7 / 14.9 us (per-CU bandwidth: one workgroup per CU).
constexpr int kS2Partials = kBlock;  // one partial per lane of an apply workgroup
constexpr int kS2Loads = 16;         // dwordx4 per lane in flight per round

// Threads per partial workgroup (SMQ_S2_PTHREADS = 256 | 1024, measurement knob). One workgroup
// per CU either way (256 partials); 1024 threads put 4 waves on each SIMD instead of one, so the
// loads and the log2 chains of one wave hide behind the others'.
static inline int s2_partial_threads() {
  static const int v = [] {
    const char* e = knob_env("SMQ_S2_PTHREADS");
    const int t = e ? atoi(e) : 1024;
    return (t == 256 || t == 1024) ? t : 1024;
  }();
  return v;
}

// float4 groups per partial workgroup (whole rounds of one load per lane); depends on n only, so
// the summation order — and the statistics — are a function of n
static inline int64_t s2_groups_per_wg(int64_t ng) {
  static const int np = [] {  // measurement knob SMQ_S2_PARTIALS (<= kS2Partials)
    const char* e = knob_env("SMQ_S2_PARTIALS");
    const int v = e ? atoi(e) : kS2Partials;
    return (v >= 1 && v <= kS2Partials) ? v : kS2Partials;
  }();
  int64_t per = (ng + np - 1) / np;
  const int64_t q = s2_partial_threads();  // whole lanes
  per = (per + q - 1) / q * q;
  return per < q ? q : per;
}

template <int TIN, int PT>
__global__ __launch_bounds__(PT) void s2fp8_partial_kernel(const void* __restrict__ x, int64_t n,
                                                           int vec, int64_t per,
                                                           S2Partial* __restrict__ partials,
                                                           SmqS2fp8Stats* out,
                                                           uint64_t* rng_ctr) {
  constexpr int W = PT / kWave;
  // graph-safe random stream: one snapshot + advance per call, read by the apply launch
  if (blockIdx.x == 0 && threadIdx.x == 0) out->rng_offset = take_offset(rng_ctr, (uint64_t)n);
  __shared__ double shs[W];
  __shared__ float shm[W];
  double s = 0.0;
  float m = -INFINITY;
  if (vec) {
    // groups [g0, g1) of this workgroup; lane t takes g0 + t + k * PT
    const int64_t nv = n >> 2;
    const int64_t g0 = (int64_t)blockIdx.x * per;
    const int64_t g1 = (g0 + per < nv) ? g0 + per : nv;
    for (int64_t r0 = g0 + threadIdx.x; r0 < g1; r0 += (int64_t)kS2Loads * PT) {
      float4 v[kS2Loads];
#pragma unroll
      for (int u = 0; u < kS2Loads; ++u) {
        const int64_t j = r0 + (int64_t)u * PT;
        if (j < g1) v[u] = load4<TIN>(x, j);
      }
#pragma unroll
      for (int u = 0; u < kS2Loads; ++u) {
        const int64_t j = r0 + (int64_t)u * PT;
        if (j >= g1) continue;
        const float l0 = s2_log<TIN>(v[u].x), l1 = s2_log<TIN>(v[u].y), l2 = s2_log<TIN>(v[u].z),
                    l3 = s2_log<TIN>(v[u].w);
        s += ((double)l0 + (double)l1) + ((double)l2 + (double)l3);
        m = nan_max(nan_max(m, l0), nan_max(l1, nan_max(l2, l3)));
      }
    }
    if (blockIdx.x == gridDim.x - 1 && threadIdx.x < (int)(n & 3)) {
      const float l = s2_log<TIN>(load1<TIN>(x, (nv << 2) + threadIdx.x));
      s += (double)l;
      m = nan_max(m, l);
    }
  } else {
    const int64_t e0 = (int64_t)blockIdx.x * per * 4;
    const int64_t e1 = (e0 + per * 4 < n) ? e0 + per * 4 : n;
    for (int64_t i = e0 + threadIdx.x; i < e1; i += PT) {
      const float l = s2_log<TIN>(load1<TIN>(x, i));
      s += (double)l;
      m = nan_max(m, l);
    }
  }
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  s = wave_sum_asc(s);
  m = wave_nanmax_asc(m);
  if (lane == 0) {
    shs[wave] = s;
    shm[wave] = m;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    double S = 0.0;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < W; w += 4) {  // fixed order: groups of four waves
      S += (shs[w] + shs[w + 1]) + (shs[w + 2] + shs[w + 3]);
      M = nan_max(M, nan_max(nan_max(shm[w], shm[w + 1]), nan_max(shm[w + 2], shm[w + 3])));
    }
    S2Partial p;
    p.s = S;
    p.m = M;
    p.pad = 0.0f;
    partials[blockIdx.x] = p;
  }
}

// Every apply workgroup: reduce the P partials (lane t holds partial t) in one fixed order and
// derive alpha, beta, ... into *st (LDS). Block 0 also publishes them in the workspace header.
template <int TIN>
__device__ __forceinline__ void s2_reduce_partials(const S2Partial* __restrict__ partials, int P,
                                                   int64_t n, SmqS2fp8Stats* hdr,
                                                   SmqS2fp8Stats* st) {
  // order (shared with s2fp8_fused_kernel): lane l of one wave adds partials l, l + 64, l + 128,
  // l + 192 as (p0 + p1) + (p2 + p3), then one ascending butterfly over the 64 lanes
  static_assert(kBlock == 4 * kWave, "one partial per thread, four per lane of wave 0");
  __shared__ double shs[kBlock];
  __shared__ float shm[kBlock];
  double s = 0.0;
  float m = -INFINITY;
  if ((int)threadIdx.x < P) {
    const S2Partial p = partials[threadIdx.x];
    s = p.s;
    m = p.m;
  }
  shs[threadIdx.x] = s;
  shm[threadIdx.x] = m;
  __syncthreads();
  if (threadIdx.x < kWave) {
    const int l = threadIdx.x;
    s = (shs[l] + shs[l + 64]) + (shs[l + 128] + shs[l + 192]);
    m = nan_max(nan_max(shm[l], shm[l + 64]), nan_max(shm[l + 128], shm[l + 192]));
    s = wave_sum_asc(s);
    m = wave_nanmax_asc(m);
  }
  if (threadIdx.x == 0) {
    const double S = s;
    const float M = m;
    SmqS2fp8Stats d;
    s2fp8_finalize<TIN>(S, M, n, &d);
    *st = d;
    if (blockIdx.x == 0) {  // the header (all fields but rng_offset, owned by the partial launch)
      hdr->mu = d.mu;
      hdr->m = d.m;
      hdr->alpha = d.alpha;
      hdr->beta = d.beta;
      hdr->beta_pow2 = d.beta_pow2;
      hdr->inv_beta_pow2 = d.inv_beta_pow2;
      hdr->inv_alpha = d.inv_alpha;
      hdr->n_used = d.n_used;
    }
  }
  __syncthreads();
}

// Injected (mu, m): derive the rest exactly like the finaliser (parity tests).
template <int TIN>
__global__ void s2fp8_derive_kernel(const SmqS2fp8Stats* in, SmqS2fp8Stats* out, uint64_t* rng_ctr,
                                    uint64_t n) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    s2fp8_derive<TIN>(in->mu, in->m, in->n_used, out);
    out->rng_offset = take_offset(rng_ctr, n);
  }
}

struct S2Args {
  const void* x;
  void* y;
  int64_t n;
  const uint32_t* rand_bits;
  SmqS2fp8Stats* st;            // workspace header (derived stats, or the rng snapshot only)
  const S2Partial* partials;    // PART: the partial launch's output
  int n_partials;
  uint32_t key;
  uint64_t offset;
  int check_inf;
  float max_value;
  int out_mode;   // 0: y, 1: Y, 2: T (SMQ_S2FP8_OUT_*)
  int exact_pow;  // SMQ_S2FP8_EXACT_POW: library powf for both powers
  // XCD-aware tile order (vector path): tiles_per_chunk tiles make up partial workgroup w's chunk;
  // apply block b takes a tile of a chunk w with w % 8 == b % 8 (0: block b takes tile b)
  int tiles_per_chunk;
  int n_chunks;
};

// Apply block -> tile. Workgroups are dealt round-robin over the 8 XCDs (MI355X_MICROARCH.md
// §Workgroup dispatch: blocks b and b + 8 share an XCD; observed, speed only): the partial launch
// read chunk w on the XCD of its block w, so apply blocks b = c + 8k (one XCD) take the tiles of
// chunks c, c + 8, ... and find them in that XCD's L2 (C4: 1.6 MB of the 12.6 MB per XCD, well
// inside its 4 MiB). Any placement gives the same result; only the hit rate depends on it.
__device__ __forceinline__ int64_t s2_tile_of(int b, int tpc, int n_chunks) {
  if (tpc == 0) return b;
  const int c = b & 7, k = b >> 3;
  const int w = c + 8 * (k / tpc);
  return w < n_chunks ? (int64_t)w * tpc + (k % tpc) : -1;
}

// The fast forward power: x^p for x >= 0 (or NaN) as exp2(p * log2(x)) on the hardware v_log_f32 /
// v_exp_f32 (ocml's log2f / exp2f, ~1 ulp each), valid for finite p > 0 (the caller checks once
// per launch): 0 -> 0, inf -> inf, NaN -> NaN like powf. Relative error ~ ln2 * |p * log2 x| *
// 2^-23 (at C4 up to 92 ulp of Y), so on its own it moved 2 of 3.1M E5M2 codes to the adjacent
// code (round 2); s2_fast_uncertain finds every element where that can happen.

// Could the E5M2 code stochastic rounding gives Y_fast = exp2(alpha * lg) * 2^beta (lg = log2f|x|)
// differ from the one it gives the accurate Y = powf(|x|, alpha) * 2^beta? The code is
// (bits(v) + (r & M)) & ~M with v = Y (normal E5M2 range) or Y + 2^-14 (subnormal range),
// M = 2^21 - 1: it changes only if the two v lie on different sides of a multiple of 2^21 after
// adding the random bits. Bound on |bits(v_fast) - bits(v_accurate)| (integer bit distance, <=
// 2^24 x relative error): log2f <= 2^-22 max(|lg|, 1) absolute, the product, v_exp_f32, both
// multiplies and powf (<= 2 ulp) give relative error <= ln2 (|alpha| 2^-22 max(|lg|,1) +
// 2^-24 |alpha lg|) + 2^-21 + 2^-23, i.e. <= 3.5 |alpha| max(|lg|, 1) + 10 in bit distance; the
// test uses 4 |alpha| max(|lg|, 1) + 16. Where the random offset leaves less than that to the
// boundary the element is recomputed with powf (~2e-4 of N(0,1) elements at C4), so the fast
// path's codes — and outputs — are the accurate path's, bit for bit (tests/test_gpu_float.py
// test_s2fp8_fast_equals_exact_pow). |x| = 0 is exact on both paths.
// The margin: E >= 4 |alpha| max(|lg|, 1) + 16 for every element it is used for (lgmax: the largest
// such |lg| — one element's, or a lane's to share one margin), saturated at 2^20, where it flags all.
__device__ __forceinline__ uint32_t s2_fast_margin(float alpha, float lgmax) {
  const float e = __builtin_fmaf(4.0f * fabsf(alpha), lgmax > 1.0f ? lgmax : 1.0f, 16.0f);
  return e < 1048576.0f ? (uint32_t)e : 1048576u;  // (inf / NaN alpha: all)
}

// v: the value whose low 21 bits the rounding adds the random word rm to (Y, or Y + 2^-14 in the
// subnormal E5M2 range); uncertain iff that sum is within E of a multiple of 2^21. A NaN x (lg NaN)
// always, x = 0 (lg = -inf, Y = 0 on both paths) never.
__device__ __forceinline__ bool s2_fast_uncertain(uint32_t vb, uint32_t rm, uint32_t E, float lg) {
  const uint32_t L = (vb + rm) & 0x1fffffu;
  return ((L - E >= 0x200000u - 2u * E) && lg != -INFINITY) || lg != lg;
}

// Inverse of precision 32 by table (s2fp8.py:48: (T * 2^-beta) ** (1/alpha)). T is an E5M2 value
// (Y >= 0; a NaN Y saturates to +-57344 in the quantiser, +57344 -> +inf under check_inf), so the
// inverse power has at most 131 distinct arguments per call: each apply workgroup evaluates them
// once with the accurate library powf into LDS, and an element costs a shift and a table read
// instead of two transcendental-unit powers. Index = fp32 bits >> 21 (sign, exponent, the two
// E5M2 mantissa bits; subnormal E5M2 values are normal fp32 numbers of that form): +0 -> 0,
// 2^-16 .. 57344 -> 444 .. 571, +inf -> 1020, -57344 -> 1595. Other entries hold NaN.
constexpr int kS2LutSize = 2048;
constexpr int kS2LutArgs = 131;

__device__ __forceinline__ float s2_lut_arg(int i) {
  if (i < 128) return __builtin_bit_cast(float, (uint32_t)((111 << 2) + i) << 21);
  return i == 128 ? 0.0f : (i == 129 ? INFINITY : -57344.0f);
}

// every thread of the workgroup; ends with a barrier
__device__ __forceinline__ void s2_build_lut(float* lut, float ibp2, float ialpha) {
  for (int i = threadIdx.x; i < kS2LutSize; i += blockDim.x) lut[i] = __builtin_nanf("");
  __syncthreads();
  if (threadIdx.x < kS2LutArgs) {
    const float T = s2_lut_arg(threadIdx.x);
    lut[__builtin_bit_cast(uint32_t, T) >> 21] = powf(T * ibp2, ialpha);
  }
  __syncthreads();
}

__device__ __forceinline__ float s2_inverse_lut(float T, const float* lut) {
  if (T != T) return T;  // (unreachable: the quantiser saturates NaN)
  return lut[__builtin_bit_cast(uint32_t, T) >> 21];
}

// The forward of the hot path, branch-free: Y = exp2(alpha * log2|x|) * beta_pow2 (log2f keeps
// subnormal |x|; the raw v_exp_f32 flushes a subnormal Y, which the quantiser maps to 0 either
// way: any Y < 2^-37 rounds to 0 in its subnormal path), then qtorch's E5M2 stochastic rounding
// (qtorch_quant(Y, r, 5, 2, true) with its normal and subnormal paths both computed and one
// selected) and check_inf (+57344 -> +inf; an E5M2 value within FLT_EPSILON of 57344 is 57344).
// Returns T's bits.
template <bool FAST>
__device__ __forceinline__ float s2fp8_fwd(float xv, uint32_t r, float alpha, float bp2,
                                           int check_inf, float max_value, int out_mode);

// s2_fwd_fast from lg = log2f(|x|) (the single launch keeps it from its statistics pass); an
// element whose code the fast power's error could change (s2_fast_uncertain, margin E) takes powf.
// The callers run it only with 0 < alpha < inf (`fast`). Every element's log2|x| entered the
// statistics, so a NaN or infinite x would have made alpha NaN or 0: here x is finite, lg is not
// NaN, and Y = exp2(alpha lg) * 2^beta is +0 .. +inf or the default (positive) NaN of 0 * inf. Y
// never has its sign bit, which makes these shortcuts exact (round 3; oracle/csrc/s2_clip_check.c
// checks every such Y):
//   * qtorch's clip_exponent (exponent > 142 -> +57344) and check_inf (+57344 -> +inf) are one
//     unsigned compare, t + rm >= bits(57344): after the rounding's mask that is "exponent above
//     142, or 57344 itself", and the +inf / NaN patterns lie above it too;
//   * the subnormal path's shift is the constant +2^-14, "subnormal" is t < bits(2^-14), and both
//     paths round the same sum (t or bits(Y + 2^-14)) + rm, whose low 21 bits the uncertainty test
//     reads;
//   * a zero x (lg = -inf) needs no exclusion from that test: Y = 0 on both paths.
// Returns the code in bits 21..31 (what the inverse table is indexed by); bits 0..20 are unspecified.
__device__ __forceinline__ uint32_t s2_fwd_fast_lg(float xv, float lg, uint32_t r, float alpha,
                                                   float bp2, int check_inf, float max_value,
                                                   uint32_t E) {
  const float Y = __builtin_amdgcn_exp2f(alpha * lg) * bp2;
  const uint32_t t = __builtin_bit_cast(uint32_t, Y);
  const uint32_t vsb = __builtin_bit_cast(uint32_t, Y + 0x1p-14f);
  const bool sub = t < 0x38800000u;
  const uint32_t sum = (sub ? vsb : t) + (r & 0x1fffffu);  // round_bitwise's sum, either path
  const float qs = __builtin_bit_cast(float, sum & 0xffe00000u) - 0x1p-14f;
  const uint32_t clip = check_inf ? 0x7f800000u : 0x47600000u;
  uint32_t T = sub ? __builtin_bit_cast(uint32_t, qs) : (sum >= 0x47600000u ? clip : sum);
  if (__builtin_expect((sum & 0x1fffffu) - E >= 0x200000u - 2u * E, 0))
    T = __builtin_bit_cast(uint32_t, s2fp8_fwd<false>(xv, r, alpha, bp2, check_inf, max_value, 0));
  return T;
}

// torch.sign(x) for a FINITE x (the fast paths): +-1, and +0 for +-0. x * 2^127 * 2^127 maps every
// nonzero finite x to at least 2^105 in magnitude (the smallest subnormal is 2^-149) or to +-inf,
// the + 0 turns -0 into +0, and the median with -1 and 1 clamps: three ops instead of two compares
// and two selects.
__device__ __forceinline__ float s2_sign_finite(float x) {
  const float s = __builtin_fmaf(x * 0x1p127f, 0x1p127f, 0.0f);
  return __builtin_amdgcn_fmed3f(s, -1.0f, 1.0f);
}

__device__ __forceinline__ uint32_t s2_fwd_fast(float xv, uint32_t r, float alpha, float bp2,
                                                int check_inf, float max_value) {
  const float lg = log2f(fabsf(xv));
  return s2_fwd_fast_lg(xv, lg, r, alpha, bp2, check_inf, max_value,
                        s2_fast_margin(alpha, fabsf(lg)));
}

// T of the fast power for the generic paths (the same codes as s2_fwd_fast_lg: either equals the
// accurate path's wherever it matters)
__device__ __forceinline__ bool s2_fast_uncertain_y(float Y, uint32_t r, float alpha, float lg) {
  const uint32_t t = __builtin_bit_cast(uint32_t, Y);
  const float sh = __builtin_bit_cast(float, 0x38800000u | (t & 0x80000000u));
  const uint32_t vb = ((t & 0x7f800000u) < 0x38800000u) ? __builtin_bit_cast(uint32_t, Y + sh) : t;
  return s2_fast_uncertain(vb, r & 0x1fffffu, s2_fast_margin(alpha, fabsf(lg)), lg);
}

// Forward half of s2fp8_elem for the LUT inverse: T (after check_inf), or Y / T per out_mode.
// FAST: the hardware exp2(alpha log2|x|), with powf where the code could differ (s2_fast_uncertain;
// OUT_Y returns the fast Y itself).
template <bool FAST>
__device__ __forceinline__ float s2fp8_fwd(float xv, uint32_t r, float alpha, float bp2,
                                           int check_inf, float max_value, int out_mode) {
  const float a = fabsf(xv);
  float Y;
  if (FAST) {
    const float lg = log2f(a);
    Y = exp2f(alpha * lg) * bp2;
    if (out_mode == 1) return Y;
    if (__builtin_expect(s2_fast_uncertain_y(Y, r, alpha, lg), 0)) Y = powf(a, alpha) * bp2;
  } else {
    Y = powf(a, alpha);                                   // X_abs.pow_(alpha)
    Y = Y * bp2;                                          // .mul_(beta_pow2)
  }
  if (out_mode == 1) return Y;
  float T = qtorch_quant(Y, r, 5, 2, true);
  if (check_inf && fabsf(T - max_value) <= FLT_EPSILON) T = INFINITY;
  return T;
}

// The same at precision 16 (quantization.py:190-202: float_quantize quantises Y.float() and returns
// .half()). Forward transform in the input type TIN (fp32 keeps the fast power; fp16/bf16 use
// ocml powf before rounding to TIN, so the rounding sees an accurate power). Inverse in half:
// `truncated * beta_pow2.reciprocal_()` multiplies by the UNROUNDED TIN scalar (torch's opmath path
// for 0-dim operands), `** alpha.reciprocal_()` uses the exponent rounded to half (ialpha_h);
// each result rounds to half. E5M2 values (and inf/NaN) are exact in half, so T needs no rounding.
template <int TIN, bool FAST>
__device__ __forceinline__ float s2fp8_elem16(float xv, uint32_t r, float alpha, float bp2,
                                              float ibp2, float ialpha_h, int check_inf,
                                              float max_value) {
  const float sgn = (xv > 0.0f) ? 1.0f : ((xv < 0.0f) ? -1.0f : 0.0f);
  const float a = fabsf(xv);
  float Y;
  if (FAST && TIN == kF32) {  // fp32 data: Y is fp32, the fast power with the same check
    const float lg = log2f(a);
    Y = exp2f(alpha * lg) * bp2;
    if (__builtin_expect(s2_fast_uncertain_y(Y, r, alpha, lg), 0)) Y = powf(a, alpha) * bp2;
  } else if (TIN == kF32) {
    Y = powf(a, alpha) * bp2;
  } else {  // a power rounded to a half type: the correctly rounded float power (double pow)
    Y = s2_round<TIN>(s2_round<TIN>((float)pow((double)a, (double)alpha)) * bp2);
  }
  float T = qtorch_quant(Y, r, 5, 2, true);
  if (check_inf && fabsf(T - max_value) <= FLT_EPSILON) T = INFINITY;
  const float t1 = s2_round<kF16>(T * ibp2);
  // `** alpha.reciprocal_()` on half values: torch's result equals the correctly rounded float
  // power rounded to half; a float powf that is not correctly rounded moves whole E5M2 codes by a
  // half ulp on some draws (tests/golden f64_s2fp8_p16_powcase: 19 of 4096 elements)
  const float t2 = s2_round<kF16>((float)pow((double)t1, (double)ialpha_h));
  // `* signs` (fp16 output for fp16 inputs, fp32 otherwise). t2 is >= +0 or NaN, so the product is
  // a sign flip — written as one: `fptrunc(t2 * sgn)` is otherwise emitted as v_fma_mixlo_f16 with
  // a +0 addend, which turns -1 * +0 = -0 into +0 (measured on gfx950).
  (void)sgn;
  if (xv > 0.0f) return t2;
  if (xv < 0.0f) return __builtin_bit_cast(float, __builtin_bit_cast(uint32_t, t2) ^ 0x80000000u);
  return t2 * 0.0f;  // sign(+-0) = sign(NaN) = +0
}

// output element type: fp16 for fp16 inputs at precision 16, fp32 otherwise
template <int TIN, bool P16>
constexpr bool s2_half_out() { return P16 && TIN == kF16; }

// PART: reduce the partial launch's output first (s2_reduce_partials), else read the header that
// s2fp8_derive_kernel wrote (injected mu, m).
template <bool RARR, bool VEC, int kFqTileV, int TIN, bool P16, bool PART>
__global__ __launch_bounds__(kBlock) void s2fp8_apply_kernel(S2Args A) {
  constexpr int kFqTileElems = kBlock * kFqTileV * 4;
  constexpr bool HOUT = s2_half_out<TIN, P16>();
  __shared__ SmqS2fp8Stats sst;
  __shared__ float lut[kS2LutSize];
  const int64_t n = A.n;
  // the tile's loads go out before the statistics are reduced
  const int64_t nv = n >> 2;
  const int64_t tile = VEC ? s2_tile_of(blockIdx.x, A.tiles_per_chunk, A.n_chunks)
                           : (int64_t)blockIdx.x;
  const int64_t t0 = tile * (kBlock * kFqTileV) + threadIdx.x;
  const int64_t tiles = (nv + kBlock * kFqTileV - 1) / (kBlock * kFqTileV);
  const int64_t last_tile = tiles > 0 ? tiles - 1 : 0;  // owns the n % 4 tail
  if (VEC && (tile < 0 || (tile > last_tile && blockIdx.x != 0))) return;  // no tile
  float4 v[kFqTileV];
  if (VEC) {
#pragma unroll
    for (int u = 0; u < kFqTileV; ++u) {
      const int64_t j = t0 + u * kBlock;
      if (j < nv) v[u] = load4<TIN>(A.x, j);
    }
  }
  const SmqS2fp8Stats* st = A.st;
  if (PART) {
    s2_reduce_partials<TIN>(A.partials, A.n_partials, n, A.st, &sst);
    st = &sst;
  }
  const float alpha = st->alpha, bp2 = st->beta_pow2, ibp2 = st->inv_beta_pow2,
              ialpha = st->inv_alpha;
  const float ialpha_e = P16 ? s2_round<kF16>(ialpha) : ialpha;
  const uint64_t off = A.offset + A.st->rng_offset;
  auto rb = [&](int64_t e) -> uint32_t {
    return RARR ? A.rand_bits[e] : rng_u32(A.key, off + (uint64_t)e);
  };
  const bool fast = !A.exact_pow && alpha > 0.0f && alpha < INFINITY && ialpha > 0.0f &&
                    ialpha < INFINITY;
  if (!P16) s2_build_lut(lut, ibp2, ialpha);  // this call's inverse-power table
  auto q1 = [&](float v, uint32_t r) {
    if (P16)
      return fast ? s2fp8_elem16<TIN, true>(v, r, alpha, bp2, ibp2, ialpha_e, A.check_inf, A.max_value)
                  : s2fp8_elem16<TIN, false>(v, r, alpha, bp2, ibp2, ialpha_e, A.check_inf, A.max_value);
    const float T = fast ? s2fp8_fwd<true>(v, r, alpha, bp2, A.check_inf, A.max_value, A.out_mode)
                         : s2fp8_fwd<false>(v, r, alpha, bp2, A.check_inf, A.max_value, A.out_mode);
    if (A.out_mode) return T;
    // `* signs`: torch.sign is +1 / -1, +0 for +-0 and NaN (measured on torch 2.10 CPU)
    const float sgn = (v > 0.0f) ? 1.0f : ((v < 0.0f) ? -1.0f : 0.0f);
    return s2_inverse_lut(T, lut) * sgn;
  };
  if (VEC && !P16 && !RARR && fast && A.out_mode == 0) {
    // hot path: all forwards of the tile, then the table reads, then the stores
    uint32_t T[kFqTileV][4];
#pragma unroll
    for (int u = 0; u < kFqTileV; ++u) {
      const int64_t j = t0 + u * kBlock;
      if (j >= nv) continue;
      const uint64_t c = off + ((uint64_t)j << 2);
      uint32_t r[4];
      const uint32_t lo = (uint32_t)c;
      if (__builtin_expect(lo <= 0xfffffffcu, 1)) {  // one rotation of the high word per float4
        const uint32_t hi = (uint32_t)(c >> 32);
        const uint32_t kk = ((hi << 16) | (hi >> 16)) ^ A.key;
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = mix32((lo + (uint32_t)k) ^ kk);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) r[k] = rng_u32(A.key, c + (uint64_t)k);
      }
      T[u][0] = s2_fwd_fast(v[u].x, r[0], alpha, bp2, A.check_inf, A.max_value);
      T[u][1] = s2_fwd_fast(v[u].y, r[1], alpha, bp2, A.check_inf, A.max_value);
      T[u][2] = s2_fwd_fast(v[u].z, r[2], alpha, bp2, A.check_inf, A.max_value);
      T[u][3] = s2_fwd_fast(v[u].w, r[3], alpha, bp2, A.check_inf, A.max_value);
    }
    float t2[kFqTileV][4];
#pragma unroll
    for (int u = 0; u < kFqTileV; ++u)
#pragma unroll
      for (int k = 0; k < 4; ++k) t2[u][k] = lut[T[u][k] >> 21];
#pragma unroll
    for (int u = 0; u < kFqTileV; ++u) {
      const int64_t j = t0 + u * kBlock;
      if (j >= nv) continue;
      float4 o;
      o.x = t2[u][0] * s2_sign_finite(v[u].x);
      o.y = t2[u][1] * s2_sign_finite(v[u].y);
      o.z = t2[u][2] * s2_sign_finite(v[u].z);
      o.w = t2[u][3] * s2_sign_finite(v[u].w);
      store4_out<HOUT>(A.y, j, o);
    }
    if (tile == last_tile && threadIdx.x < (int)(n & 3)) {
      const int64_t e = (nv << 2) + threadIdx.x;
      store1_out<HOUT>(A.y, e, q1(load1<TIN>(A.x, e), rb(e)));
    }
  } else if (VEC) {
#pragma unroll
    for (int u = 0; u < kFqTileV; ++u) {
      const int64_t j = t0 + u * kBlock;
      if (j >= nv) continue;
      float4 o;
      o.x = q1(v[u].x, rb(4 * j));
      o.y = q1(v[u].y, rb(4 * j + 1));
      o.z = q1(v[u].z, rb(4 * j + 2));
      o.w = q1(v[u].w, rb(4 * j + 3));
      store4_out<HOUT>(A.y, j, o);
    }
    if (tile == last_tile && threadIdx.x < (int)(n & 3)) {
      const int64_t e = (nv << 2) + threadIdx.x;
      store1_out<HOUT>(A.y, e, q1(load1<TIN>(A.x, e), rb(e)));
    }
  } else {
    const int64_t e0 = (int64_t)blockIdx.x * kFqTileElems + threadIdx.x;
    for (int k = 0; k < kFqTileElems / kBlock; ++k) {
      const int64_t e = e0 + (int64_t)k * kBlock;
      if (e >= n) break;
      store1_out<HOUT>(A.y, e, q1(load1<TIN>(A.x, e), rb(e)));
    }
  }
}

// ---- S2FP8 in ONE launch (fp32, precision 32, tensors a resident grid holds in registers) -------
// The two-launch shape pays a kernel boundary, the apply's launch ramp and its re-read of x between
// the statistics and the transform; at C4 (12.6 MB) those are most of the call. Here workgroup b
// loads chunk b (V float4 per lane of 1024 threads) into registers ONCE, publishes the chunk's
// (sum, max) partial, waits until every chunk's partial is there, reduces them in the two-launch
// path's fixed order, derives alpha / beta and the inverse-power table, and transforms the
// registers.
//
// Hand-off: cdna_hip_programming.md Guideline 16 R2 — the data is the flag. A partial is three
// aligned 8-byte granules {epoch, 32-bit word} (low and high half of the fp64 sum, the max), each
// ONE relaxed agent-scope (sc1) store; one wave of every workgroup re-reads the granules it still
// misses with sc1 loads until every tag is this call's epoch. epoch = f(generation word, host tag),
// never 0: the generation is read by every workgroup at its start and advanced by the last
// workgroup past the wait (an arrival counter tagged with the generation, so the next call finds
// its own tag, eager or replayed; the add is issued early and looked at only at the end), so graph
// replays get fresh epochs; the host tag makes an eager call on a workspace some earlier call left
// mid-way distinct as well.
//
// No co-residency assumption: a workgroup that has waited kS2StealTicks computes the partials it
// still misses itself, from memory (every partial is a pure function of its chunk, so duplicates
// write the same bytes). So if only some workgroups are resident (another kernel holding CUs, a
// shared device) they finish the statistics, transform their own chunks and exit, and the rest
// start later, find the statistics complete and transform theirs. There is no give-up path: a
// workgroup never proceeds with a partial it has neither read nor computed (a give-up after a
// fixed time would hand a workgroup descheduled for that long incomplete statistics and corrupt
// its output silently); workgroup 0 clears hdr->reserved[0] (the former give-up flag) every call.
constexpr int kS2FT = 1024;       // threads per workgroup
constexpr int kS2FMaxV = 4;       // float4 per lane held in registers (4.2M elements)
constexpr int kS2FMaxG = 256;     // chunks (= partials; four per lane of the polling wave)
constexpr int kS2FLds = 88 * 1024;  // dynamic LDS request: one workgroup per CU
constexpr int kS2SubStride = 16;   // residue arrival words, u64 units (128 B apart)
constexpr int kS2FRep = 8;          // granule replicas: replica r is read by the blocks b % 8 == r
constexpr uint64_t kS2StealTicks = 20000;       // s_memrealtime runs at 100 MHz: 200 us

struct S2FArgs {
  const float* x;
  float* y;
  int64_t n, nv;
  int V, G;
  uint32_t key;
  uint64_t offset;
  uint64_t* ctr;  // graph-safe stream position (nullable)
  SmqS2fp8Stats* hdr;
  uint32_t* gen;               // generation word
  unsigned long long* left;    // residues whose workgroups are all past the wait (tagged)
  unsigned long long* sub;     // workgroups b % 8 == s past the wait: word s * kS2SubStride
  unsigned long long* gran;    // [kS2FRep][3][kS2FMaxG] granules: sum low word, sum high word, max
  uint32_t tag;                // host tag of the call (mixed into the epoch)
  int check_inf;
  float max_value;
  int out_mode;
  int exact_pow;
  int test_late;     // SMQ_S2FP8_TEST_LATE
  uint64_t* trace;   // measurement aid (SMQ_S2_TRACE=1 and a workspace with room): 16 words per workgroup
};

__device__ __forceinline__ void s2f_stamp(const S2FArgs& A, int i) {
  if (A.trace && threadIdx.x == 0)
    A.trace[(size_t)blockIdx.x * 16 + i] = __builtin_amdgcn_s_memrealtime();
}

// (sum, max) of log2|x| over chunk k (lane t: float4 j = k*V*kS2FT + t + u*kS2FT), the two-launch
// partial kernel's per-lane order; the last chunk adds the n % 4 tail. From the registers v, or
// (v == nullptr: a missing partial computed by another workgroup) from memory one float4 at a time.
__device__ __forceinline__ void s2f_lane_sums(const float4* v, const S2FArgs& A, int k, double& s,
                                              float& m) {
  const int64_t base = (int64_t)k * A.V * kS2FT + threadIdx.x;
  s = 0.0;
  m = -INFINITY;
#pragma unroll
  for (int u = 0; u < kS2FMaxV; ++u) {
    if (u >= A.V) break;
    const int64_t j = base + (int64_t)u * kS2FT;
    if (j >= A.nv) continue;
    const float4 xv = v ? v[u] : reinterpret_cast<const float4*>(A.x)[j];
    const float l0 = s2_log<kF32>(xv.x), l1 = s2_log<kF32>(xv.y), l2 = s2_log<kF32>(xv.z),
                l3 = s2_log<kF32>(xv.w);
    s += ((double)l0 + (double)l1) + ((double)l2 + (double)l3);
    m = nan_max(nan_max(m, l0), nan_max(l1, nan_max(l2, l3)));
  }
  if (k == A.G - 1 && threadIdx.x < (int)(A.n & 3)) {
    const float l = s2_log<kF32>(A.x[(A.nv << 2) + threadIdx.x]);
    s += (double)l;
    m = nan_max(m, l);
  }
}

// The same sums over this workgroup's registers, keeping lg = log2f(|x|) of every element for the
// forward transform (s2_log is lg with zeros as +0: the same partial bit for bit). Computing the
// logarithms once moves them off the path behind the gather.
__device__ __forceinline__ void s2f_lane_sums_keep(const float4* v, const S2FArgs& A, int k,
                                                   double& s, float& m, float (*lg)[4]) {
  const int64_t base = (int64_t)k * A.V * kS2FT + threadIdx.x;
  s = 0.0;
  m = -INFINITY;
  auto slog = [](float xv, float l) { return fabsf(xv) == 0.0f ? 0.0f : l; };
#pragma unroll
  for (int u = 0; u < kS2FMaxV; ++u) {
    if (u >= A.V) break;
    const int64_t j = base + (int64_t)u * kS2FT;
    if (j >= A.nv) continue;
    const float4 xv = v[u];
    lg[u][0] = log2f(fabsf(xv.x));
    lg[u][1] = log2f(fabsf(xv.y));
    lg[u][2] = log2f(fabsf(xv.z));
    lg[u][3] = log2f(fabsf(xv.w));
    const float l0 = slog(xv.x, lg[u][0]), l1 = slog(xv.y, lg[u][1]), l2 = slog(xv.z, lg[u][2]),
                l3 = slog(xv.w, lg[u][3]);
    s += ((double)l0 + (double)l1) + ((double)l2 + (double)l3);
    m = nan_max(nan_max(m, l0), nan_max(l1, nan_max(l2, l3)));
  }
  if (k == A.G - 1 && threadIdx.x < (int)(A.n & 3)) {
    const float l = s2_log<kF32>(A.x[(A.nv << 2) + threadIdx.x]);
    s += (double)l;
    m = nan_max(m, l);
  }
}

// The four stochastic-rounding words of elements 4j .. 4j+3 (rng_u32(key, c + q), c = off + 4j).
__device__ __forceinline__ void s2f_hash4(uint32_t key, uint64_t c, uint32_t r[4]) {
  const uint32_t lo = (uint32_t)c;
  if (__builtin_expect(lo <= 0xfffffffcu, 1)) {
    const uint32_t hi = (uint32_t)(c >> 32);
    const uint32_t kk = ((hi << 16) | (hi >> 16)) ^ key;
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = mix32((lo + (uint32_t)q) ^ kk);
  } else {
#pragma unroll
    for (int q = 0; q < 4; ++q) r[q] = rng_u32(key, c + (uint64_t)q);
  }
}

// Workgroup reduce of the lane sums in the partial kernel's order; lanes 0-23 of wave 0 store
// partial k as three granules in each of the kS2FRep replicas (one sc1 store each; nobody waits for
// them here). Barriers are LDS-only (lds_barrier) throughout the kernel: no workgroup-internal
// hand-off goes through global memory, and a __syncthreads would drain the granule stores and the
// `left` atomic on the critical path. Replicas: every workgroup polls all partials, and 256
// workgroups sweeping the same 6 KB queue on the few memory channels that hold it (first poll pass
// 2.1 us); replica b % 8 spreads the readers over 8x the channels.
__device__ void s2f_publish(double s, float m, const S2FArgs& A, int k, uint32_t epoch,
                            double* shs, float* shm, uint32_t* gw = nullptr) {
  constexpr int W = kS2FT / kWave;
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  s = wave_sum_asc(s);
  m = wave_nanmax_asc(m);
  if (lane == 0) {
    shs[wave] = s;
    shm[wave] = m;
  }
  lds_barrier();
  if (wave == 0 && lane < 3 * kS2FRep) {
    double S = 0.0;
    float M = -INFINITY;
#pragma unroll
    for (int w = 0; w < W; w += 4) {
      S += (shs[w] + shs[w + 1]) + (shs[w + 2] + shs[w + 3]);
      M = nan_max(M, nan_max(nan_max(shm[w], shm[w + 1]), nan_max(shm[w + 2], shm[w + 3])));
    }
    const uint64_t sb = __builtin_bit_cast(uint64_t, S);
    const int r = lane / 3, c = lane - 3 * r;
    const uint32_t word = c == 0 ? (uint32_t)sb
                                 : (c == 1 ? (uint32_t)(sb >> 32) : __builtin_bit_cast(uint32_t, M));
    st_sc1_u64(&A.gran[(r * 3 + c) * kS2FMaxG + k], ((unsigned long long)epoch << 32) | word);
    if (gw && lane < 3) gw[c * kS2FMaxG + k] = word;  // the gather's LDS copy (a stolen partial)
  }
}

template <int V>
__global__ __launch_bounds__(kS2FT) void s2fp8_fused_kernel(S2FArgs A) {
  __shared__ float lut[kS2LutSize];
  __shared__ double shs[kS2FT / kWave];
  __shared__ float shm[kS2FT / kWave];
  __shared__ SmqS2fp8Stats sst;
  __shared__ uint4 r0lds[kS2FMaxV][kWave];  // wave 0's rounding words, computed by waves 1..V
  __shared__ uint32_t gw[3 * kS2FMaxG];      // the gathered words: granule c of partial k at c*256+k
  __shared__ int smiss[kS2FT / kWave];
  const int b = blockIdx.x;
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  const int64_t base = (int64_t)b * A.V * kS2FT + threadIdx.x;
  const uint64_t steal_ticks = A.test_late ? 2000 : kS2StealTicks;
  s2f_stamp(A, 0);
  if (A.test_late && 2 * b >= A.G && A.G > 1) {  // test aid: start ~500 us late
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < 50000) __builtin_amdgcn_s_sleep(127);
  }
  // (then the call's generation and stream snapshot, read before this workgroup can be counted past
  // the wait)
  // this chunk into registers (nt: read once): branch-free (indices past the end re-read the last
  // float4 and are ignored), so every load is in flight before the first wait
  float4 v[kS2FMaxV];
  if (A.nv > 0) {
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int64_t j = base + (int64_t)u * kS2FT;
      v[u] = load_nt(reinterpret_cast<const float4*>(A.x) + (j < A.nv ? j : A.nv - 1));
    }
  }
  const uint32_t gen = ld_sc1_u32(A.gen);
  const uint64_t ctr_word = ld_sc1_u64(A.ctr ? A.ctr : reinterpret_cast<uint64_t*>(A.left));
  const uint64_t off0 = A.ctr ? ctr_word : 0ull;  // a select, not a branch: no wait here
  const uint32_t epoch = mix32(gen ^ mix32(A.tag)) | 1u;
  const uint64_t off = A.offset + off0;
  asm volatile("" ::"v"(off));  // materialised here: no later wait on it waits for the `left` atomic
  // the table's unreachable entries (NaN) need no statistics
  for (int i = threadIdx.x; i < kS2LutSize; i += kS2FT) lut[i] = __builtin_nanf("");
  float lg[kS2FMaxV][4];
  {
    double s;
    float m;
    s2f_lane_sums_keep(v, A, b, s, m, lg);
    s2f_stamp(A, 1);
    s2f_publish(s, m, A, b, epoch, shs, shm);
  }
  s2f_stamp(A, 2);
  // one margin for the lane's elements (s2_fast_margin): the largest |log2|x|| among them (zeros
  // and NaN aside), taken here, off the path behind the gather
  float lgmax = 1.0f;
#pragma unroll
  for (int u = 0; u < V; ++u) {
    if (base + (int64_t)u * kS2FT >= A.nv) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      lgmax = fmaxf(lgmax, lg[u][q] == -INFINITY ? 0.0f : fabsf(lg[u][q]));
  }
  // The stochastic-rounding words depend on the stream position only: waves 1..15, idle while wave
  // 0 gathers the partials, compute their own now, and waves 1..V also wave 0's slot u = wave - 1
  // (handed over in LDS behind the gather's barrier), so the transform after the statistics starts
  // without the counter hashes.
  uint32_t rw[kS2FMaxV][4];
  if (wave != 0) {
#pragma unroll
    for (int u = 0; u < kS2FMaxV; ++u)
      if (u < V) s2f_hash4(A.key, off + ((uint64_t)(base + (int64_t)u * kS2FT) << 2), rw[u]);
    if (wave <= V) {
      const int u = wave - 1;
      uint32_t r0[4];
      s2f_hash4(A.key, off + ((uint64_t)((int64_t)b * A.V * kS2FT + lane + (int64_t)u * kS2FT) << 2), r0);
      r0lds[u][lane] = make_uint4(r0[0], r0[1], r0[2], r0[3]);
    }
  }
  // every thread t < 768 gathers word t of replica b % 8 (granule c = t / 256 of partial
  // k = t % 256: each wave load reads 512 consecutive bytes) until every granule carries the epoch;
  // accepted words go to LDS (gw), then wave 0 takes its lanes' four partials from there
  const unsigned long long* rep = A.gran + (size_t)(b % kS2FRep) * 3 * kS2FMaxG;
  const int gk = threadIdx.x & (kS2FMaxG - 1);
  uint32_t miss = (threadIdx.x < 3 * kS2FMaxG && gk < A.G) ? 1u : 0u;
  int n_stolen = 0;
  bool stealing = false;
  for (;;) {
    const uint64_t t_start = __builtin_amdgcn_s_memrealtime();
    uint32_t polls = 0;
    for (;;) {
      const unsigned long long g = miss ? ld_sc1_u64(rep + threadIdx.x) : 0ull;
      if (miss && (uint32_t)(g >> 32) == epoch) {
        miss = 0u;
        gw[threadIdx.x] = (uint32_t)g;
      }
      if (polls == 0 && threadIdx.x == 0) s2f_stamp(A, 11);
      if (__all(miss == 0u) || stealing) break;
      if ((++polls & 7) != 0) {
        __builtin_amdgcn_s_sleep(2);
        continue;
      }
      if (__builtin_amdgcn_s_memrealtime() - t_start > steal_ticks) break;
      __builtin_amdgcn_s_sleep(2);
    }
    // the first missing partial after b (cyclically)
    int d = INT_MAX;
    if (miss) {
      d = gk - b;
      d += d < 0 ? A.G : 0;
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) d = min(d, __shfl_xor(d, o, kWave));
    if (lane == 0) smiss[wave] = d;
    lds_barrier();
    int m = smiss[0];
#pragma unroll
    for (int w = 1; w < kS2FT / kWave; ++w) m = min(m, smiss[w]);
    if (m == INT_MAX) break;
    // the patience ran out: the whole workgroup computes partial (m + b) % G from memory and
    // publishes it (its words also go straight to LDS, so no poll waits for them)
    const int k = m + b < A.G ? m + b : m + b - A.G;
    stealing = true;
    lds_barrier();
    double s;
    float mm;
    s2f_lane_sums(nullptr, A, k, s, mm);
    s2f_publish(s, mm, A, k, epoch, shs, shm, gw);
    ++n_stolen;
    lds_barrier();
    if (miss && gk == k) miss = 0u;
  }
  double ps[4] = {0.0, 0.0, 0.0, 0.0};
  float pm[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
  if (wave == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int k = lane + 64 * q;
      if (k < A.G) {
        ps[q] = __builtin_bit_cast(double, ((uint64_t)gw[kS2FMaxG + k] << 32) | gw[k]);
        pm[q] = __builtin_bit_cast(float, gw[2 * kS2FMaxG + k]);
      }
    }
#pragma unroll
    for (int u = 0; u < kS2FMaxV; ++u) {
      if (u < V) {
        const uint4 w = r0lds[u][lane];
        rw[u][0] = w.x;
        rw[u][1] = w.y;
        rw[u][2] = w.z;
        rw[u][3] = w.w;
      }
    }
  }
  s2f_stamp(A, 3);
  // count this workgroup past the wait now (on its residue's word); the returned word is looked at
  // only after the transform
  unsigned long long left_old = 0;
  if (threadIdx.x == 0) left_old = arrive_tagged_issue(A.sub + (b & 7) * kS2SubStride);
  // wave 0: reduce the partials in the two-launch apply's order (lane l: partials l + 64q summed
  // as (q0 + q1) + (q2 + q3), then one ascending butterfly — four butterflies before, 0.7 us) and
  // derive; then threads 0-130 tabulate the inverse powers
  if (wave == 0) {
    // s2_reduce_partials' order: per lane (p0 + p1) + (p2 + p3), then one butterfly
    const double S = wave_sum_asc((ps[0] + ps[1]) + (ps[2] + ps[3]));
    const float M = wave_nanmax_asc(nan_max(nan_max(pm[0], pm[1]), nan_max(pm[2], pm[3])));
    s2f_stamp(A, 8);
    if (lane == 0) {
      SmqS2fp8Stats d;
      s2fp8_finalize<kF32>(S, M, A.n, &d);
      sst = d;
      if (b == 0) {
        SmqS2fp8Stats* h = A.hdr;
        h->mu = d.mu;
        h->m = d.m;
        h->alpha = d.alpha;
        h->beta = d.beta;
        h->beta_pow2 = d.beta_pow2;
        h->inv_beta_pow2 = d.inv_beta_pow2;
        h->inv_alpha = d.inv_alpha;
        h->n_used = d.n_used;
        h->rng_offset = off0;
        h->reserved[0] = 0u;
      }
    }
    s2f_stamp(A, 9);
  }
  lds_barrier();
  // threads 0-130 (waves 0-2) tabulate the inverse powers; no barrier before the forward transform,
  // so the other waves' forward powers cover the powf latency (the table is read only after the
  // barrier behind the forward)
  if (threadIdx.x < kS2LutArgs) {
    const float T = s2_lut_arg(threadIdx.x);
    lut[__builtin_bit_cast(uint32_t, T) >> 21] = powf(T * sst.inv_beta_pow2, sst.inv_alpha);
  }
  s2f_stamp(A, 10);
  const float alpha = sst.alpha, bp2 = sst.beta_pow2, ialpha = sst.inv_alpha;
  const bool fast = !A.exact_pow && alpha > 0.0f && alpha < INFINITY && ialpha > 0.0f &&
                    ialpha < INFINITY;
  const bool last_chunk = b == A.G - 1;
  if (!(fast && A.out_mode == 0)) {  // (uniform over the workgroup: sst and A are)
    lds_barrier();
    s2f_stamp(A, 4);
  }
  if (fast && A.out_mode == 0) {
    const uint32_t E = s2_fast_margin(alpha, lgmax);
    uint32_t T[kS2FMaxV][4];
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int64_t j = base + (int64_t)u * kS2FT;
      if (j >= A.nv) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float xq = q == 0 ? v[u].x : (q == 1 ? v[u].y : (q == 2 ? v[u].z : v[u].w));
        T[u][q] = s2_fwd_fast_lg(xq, lg[u][q], rw[u][q], alpha, bp2, A.check_inf, A.max_value, E);
      }
    }
    lds_barrier();  // the table is complete
    s2f_stamp(A, 4);
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int64_t j = base + (int64_t)u * kS2FT;
      if (j >= A.nv) continue;
      float4 o;
      o.x = lut[T[u][0] >> 21] * s2_sign_finite(v[u].x);
      o.y = lut[T[u][1] >> 21] * s2_sign_finite(v[u].y);
      o.z = lut[T[u][2] >> 21] * s2_sign_finite(v[u].z);
      o.w = lut[T[u][3] >> 21] * s2_sign_finite(v[u].w);
      store_stream(reinterpret_cast<float4*>(A.y) + j, o);
    }
  } else {
    auto q1 = [&](float xv, uint64_t e) {
      const uint32_t r = rng_u32(A.key, off + e);
      const float T = fast ? s2fp8_fwd<true>(xv, r, alpha, bp2, A.check_inf, A.max_value, A.out_mode)
                           : s2fp8_fwd<false>(xv, r, alpha, bp2, A.check_inf, A.max_value, A.out_mode);
      if (A.out_mode) return T;
      const float sg = (xv > 0.0f) ? 1.0f : ((xv < 0.0f) ? -1.0f : 0.0f);
      return s2_inverse_lut(T, lut) * sg;
    };
#pragma unroll
    for (int u = 0; u < V; ++u) {
      const int64_t j = base + (int64_t)u * kS2FT;
      if (j >= A.nv) continue;
      const uint64_t e = (uint64_t)j << 2;
      float4 o;
      o.x = q1(v[u].x, e);
      o.y = q1(v[u].y, e + 1);
      o.z = q1(v[u].z, e + 2);
      o.w = q1(v[u].w, e + 3);
      store_stream(reinterpret_cast<float4*>(A.y) + j, o);
    }
  }
  if (last_chunk && threadIdx.x < (int)(A.n & 3)) {
    const int64_t e = (A.nv << 2) + threadIdx.x;
    const float xv = A.x[e];
    const uint32_t r = rng_u32(A.key, off + (uint64_t)e);
    const float T = fast ? s2fp8_fwd<true>(xv, r, alpha, bp2, A.check_inf, A.max_value, A.out_mode)
                         : s2fp8_fwd<false>(xv, r, alpha, bp2, A.check_inf, A.max_value, A.out_mode);
    const float sg = (xv > 0.0f) ? 1.0f : ((xv < 0.0f) ? -1.0f : 0.0f);
    A.y[e] = A.out_mode ? T : s2_inverse_lut(T, lut) * sg;
  }
  // the call's last arrival (every workgroup has read the generation, the stream position and the
  // granules before its add) advances the generation and the stream and re-arms the arrival words
  if (threadIdx.x == 0 &&
      arrive_sharded_finish(A.left, A.sub, kS2SubStride, b, A.G, gen, left_old)) {
    st_sc1_u32(A.gen, gen + 1u);
    if (A.ctr) st_sc1_u64(A.ctr, off0 + (uint64_t)A.n);
    rearm_sharded(A.left, A.sub, kS2SubStride, gen + 1u);
  }
  if (A.trace && threadIdx.x == 0) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    A.trace[(size_t)blockIdx.x * 16 + 5] = __builtin_amdgcn_s_memrealtime();
    uint32_t xcc, hwid;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    A.trace[(size_t)blockIdx.x * 16 + 6] = (uint64_t)n_stolen;
    A.trace[(size_t)blockIdx.x * 16 + 12] = (uint64_t)epoch | ((uint64_t)gen << 32);
    A.trace[(size_t)blockIdx.x * 16 + 7] = (uint64_t)xcc | ((uint64_t)hwid << 32);
  }
}

static inline bool aligned16f(const void* p) { return ((uintptr_t)p & 15u) == 0; }

static int fq_tile_v() {
  static const int v = [] {
    const char* e = knob_env("SMQ_FQ_TILE");
    const int t = e ? atoi(e) : kFqDefaultTileV;
    return (t == 1 || t == 2 || t == 4) ? t : kFqDefaultTileV;
  }();
  return v;
}

// float4 per lane per S2FP8 apply tile (SMQ_S2_TILE = 1 | 2 | 4, measurement knob): a workgroup
// pays the partial reduction and the inverse-power table once per tile
static int s2_tile_v() {
  static const int v = [] {
    const char* e = knob_env("SMQ_S2_TILE");
    const int t = e ? atoi(e) : 4;  // C4 (bench, 48 buffers): 1 / 2 / 4 -> 18.9 / 15.4 / 14.8 us
    return (t == 1 || t == 2 || t == 4) ? t : 4;
  }();
  return v;
}

static int fq_grid(int64_t n) {  // flat tiles
  const int64_t te = (int64_t)kBlock * 4 * fq_tile_v();
  int64_t g = (n + te - 1) / te;
  return (int)(g < 1 ? 1 : g);
}

template <int TV, int TIN, bool P16>
static void s2_launch(const S2Args& A, bool rarr, bool vec, bool part, int grid, hipStream_t st) {
#define SMQ_S2(R, V, P) \
  hipLaunchKernelGGL((s2fp8_apply_kernel<R, V, TV, TIN, P16, P>), dim3(grid), dim3(kBlock), 0, st, A)
  if (part) {
    if (rarr) { if (vec) SMQ_S2(true, true, true); else SMQ_S2(true, false, true); }
    else { if (vec) SMQ_S2(false, true, true); else SMQ_S2(false, false, true); }
  } else {
    if (rarr) { if (vec) SMQ_S2(true, true, false); else SMQ_S2(true, false, false); }
    else { if (vec) SMQ_S2(false, true, false); else SMQ_S2(false, false, false); }
  }
#undef SMQ_S2
}

static float host_max_value(int exp_bits, int man_bits) {
  return qtorch_quant(FLT_MAX, 0u, exp_bits, man_bits, false);
}

// workspace: header, partials, then the single-launch words (generation, top arrival word, eight
// residue arrival words: own 128-B lines) and granules
constexpr size_t kS2WsGen = (128 + sizeof(S2Partial) * (size_t)kS2Partials + 127) & ~(size_t)127;
constexpr size_t kS2WsLeft = kS2WsGen + 128;
constexpr size_t kS2WsSub = kS2WsLeft + 128;
constexpr size_t kS2WsGran = kS2WsSub + 8 * 8 * (size_t)kS2SubStride;
static size_t s2_ws_bytes() { return kS2WsGran + (size_t)kS2FRep * 3 * 8 * kS2FMaxG; }

// single-launch path (SMQ_S2_FUSED=0 keeps the two launches: measurement knob)
static bool s2_fused_enabled() {
  static const bool v = [] {
    const char* e = knob_env("SMQ_S2_FUSED");
    return e ? atoi(e) != 0 : true;
  }();
  return v;
}

}  // namespace smq

using namespace smq;

extern "C" {

float smq_float_quant_max_value(int exp_bits, int man_bits) {
  return host_max_value(exp_bits, man_bits);
}

int smq_float_quant(const void* x, int dtype_in, void* y, int dtype_out, int64_t n, int exp_bits,
                    int man_bits, int rounding, int check_inf, const uint32_t* rand_bits,
                    uint64_t seed, uint64_t offset, uint64_t* offset_counter, void* stream) {
  if (n < 0 || (n > 0 && (!x || !y))) {
    set_error("float_quant: bad tensor arguments");
    return SMQ_ERR_INVALID;
  }
  if (dtype_in != SMQ_DTYPE_F32 && dtype_in != SMQ_DTYPE_F16 && dtype_in != SMQ_DTYPE_BF16 &&
      dtype_in != SMQ_DTYPE_F64) {
    set_error("float_quant: dtype_in must be SMQ_DTYPE_F32, _F16, _BF16 or _F64 (got %d)", dtype_in);
    return SMQ_ERR_INVALID;
  }
  if (dtype_in != SMQ_DTYPE_F64 && dtype_out != SMQ_DTYPE_F32 && dtype_out != SMQ_DTYPE_F16) {
    set_error("float_quant: dtype_out must be SMQ_DTYPE_F32 or _F16 (got %d)", dtype_out);
    return SMQ_ERR_INVALID;
  }
  if (exp_bits < 2 || exp_bits > 8 || man_bits < 0 || man_bits > 22) {
    set_error("float_quant: exp_bits in [2,8] and man_bits in [0,22] required (got %d,%d)",
              exp_bits, man_bits);
    return SMQ_ERR_INVALID;
  }
  if (rounding != SMQ_ROUND_NEAREST && rounding != SMQ_ROUND_STOCHASTIC) {
    set_error("float_quant: rounding must be SMQ_ROUND_NEAREST or SMQ_ROUND_STOCHASTIC");
    return SMQ_ERR_INVALID;
  }
  if (dtype_in == SMQ_DTYPE_F64)  // fp64.hip
    return float_quant_f64(static_cast<const double*>(x), y, dtype_out, n, exp_bits, man_bits,
                           rounding, check_inf, rand_bits, seed, offset, offset_counter,
                           host_max_value(exp_bits, man_bits), (hipStream_t)stream);
  if (n == 0) return SMQ_OK;
  FQArgs A;
  A.x = x;
  A.y = y;
  A.n = n;
  A.rand_bits = rand_bits;
  A.ctr = offset_counter;
  A.key = rng_key(seed);
  A.offset = offset;
  A.exp_bits = exp_bits;
  A.man_bits = man_bits;
  A.check_inf = check_inf;
  A.max_value = host_max_value(exp_bits, man_bits);
  // non-temporal loads only for inputs beyond the Infinity Cache, the SmaQ policy (smaq.hip):
  // nt loads of cache-resident data lose its hits (C3 with 8 rotating buffers, cold: nt +2 %)
  static const int64_t nt_min = [] {
    const char* e = knob_env("SMQ_STATS_NT_MIN_MB");
    return (int64_t)(e ? atoll(e) : 512) << 20;
  }();
  A.nt_loads = (int64_t)(dtype_in == SMQ_DTYPE_F32 ? 4 : 2) * n >= nt_min ? 1 : 0;
  const bool sr = rounding == SMQ_ROUND_STOCHASTIC;
  const bool rarr = sr && rand_bits != nullptr;
  const bool hout = dtype_out == SMQ_DTYPE_F16;
  // one 4-element group per lane: 16 B of fp32 or 8 B of fp16 / bf16
  const uintptr_t xa = dtype_in == SMQ_DTYPE_F32 ? 15u : 7u, ya = hout ? 7u : 15u;
  const bool vec = ((uintptr_t)x & xa) == 0 && ((uintptr_t)y & ya) == 0 &&
                   (!rarr || aligned16f(rand_bits));
  const int grid = fq_grid(n);
  hipStream_t st = (hipStream_t)stream;
  if (dtype_in == SMQ_DTYPE_F32 && !hout) {
    const int tv = fq_tile_v();
#define SMQ_FQ(S, R, V)                                                                          \
  do {                                                                                           \
    if (tv == 1) hipLaunchKernelGGL((float_quant_kernel<S, R, V, 1, kF32, false>), dim3(grid), dim3(kBlock), 0, st, A); \
    else if (tv == 2) hipLaunchKernelGGL((float_quant_kernel<S, R, V, 2, kF32, false>), dim3(grid), dim3(kBlock), 0, st, A); \
    else hipLaunchKernelGGL((float_quant_kernel<S, R, V, 4, kF32, false>), dim3(grid), dim3(kBlock), 0, st, A); \
  } while (0)
    if (!sr) {
      if (vec) SMQ_FQ(false, false, true); else SMQ_FQ(false, false, false);
    } else if (rarr) {
      if (vec) SMQ_FQ(true, true, true); else SMQ_FQ(true, true, false);
    } else {
      if (vec) SMQ_FQ(true, false, true); else SMQ_FQ(true, false, false);
    }
#undef SMQ_FQ
  } else {
    // mixed-type variants: default tile only (the tile knob is an fp32 measurement aid)
    const int g = (int)((n + (int64_t)kBlock * 4 * kFqDefaultTileV - 1) / ((int64_t)kBlock * 4 * kFqDefaultTileV));
#define SMQ_FQ2(S, R, V, T, H) hipLaunchKernelGGL((float_quant_kernel<S, R, V, kFqDefaultTileV, T, H>), dim3(g), dim3(kBlock), 0, st, A)
#define SMQ_FQT(T, H)                                                                   \
  do {                                                                                  \
    if (!sr) { if (vec) SMQ_FQ2(false, false, true, T, H); else SMQ_FQ2(false, false, false, T, H); } \
    else if (rarr) { if (vec) SMQ_FQ2(true, true, true, T, H); else SMQ_FQ2(true, true, false, T, H); } \
    else { if (vec) SMQ_FQ2(true, false, true, T, H); else SMQ_FQ2(true, false, false, T, H); } \
  } while (0)
    if (dtype_in == SMQ_DTYPE_F32) SMQ_FQT(kF32, true);
    else if (dtype_in == SMQ_DTYPE_F16) { if (hout) SMQ_FQT(kF16, true); else SMQ_FQT(kF16, false); }
    else { if (hout) SMQ_FQT(kBF16, true); else SMQ_FQT(kBF16, false); }
#undef SMQ_FQT
#undef SMQ_FQ2
  }
  int rc = check_launch("float_quant_kernel");
  if (rc || !offset_counter) return rc;
  hipLaunchKernelGGL(fq_bump_kernel, dim3(1), dim3(64), 0, st, offset_counter, (uint64_t)n);
  return check_launch("fq_bump_kernel");
}

int smq_float_quant_f32(const float* x, float* y, int64_t n, int exp_bits, int man_bits,
                        int rounding, int check_inf, const uint32_t* rand_bits, uint64_t seed,
                        uint64_t offset, void* stream) {
  return smq_float_quant(x, SMQ_DTYPE_F32, y, SMQ_DTYPE_F32, n, exp_bits, man_bits, rounding,
                         check_inf, rand_bits, seed, offset, nullptr, stream);
}

size_t smq_s2fp8_workspace_bytes(int64_t n) {
  (void)n;
  return s2_ws_bytes();
}

int smq_s2fp8_roundtrip_ex(const void* x, int dtype, void* y, int64_t n, int precision,
                           int check_inf, const uint32_t* rand_bits, uint64_t seed,
                           uint64_t offset, uint64_t* offset_counter,
                           const SmqS2fp8Stats* stats_in, void* ws, size_t ws_bytes,
                           uint32_t flags, void* stream) {
  if (n < 1 || !x || !y) {
    set_error("s2fp8: n >= 1 and non-NULL x, y required");
    return SMQ_ERR_INVALID;
  }
  if (dtype != SMQ_DTYPE_F32 && dtype != SMQ_DTYPE_F16 && dtype != SMQ_DTYPE_BF16) {
    set_error("s2fp8: dtype must be SMQ_DTYPE_F32, _F16 or _BF16 (got %d)", dtype);
    return SMQ_ERR_INVALID;
  }
  if (precision != 16 && precision != 32) {
    set_error("s2fp8: precision must be 16 or 32 (got %d)", precision);
    return SMQ_ERR_INVALID;
  }
  if (precision == 32 && dtype != SMQ_DTYPE_F32) {
    // quantization.py:193 hands the tensor to qtorch's float_quantize as is; its kernels take fp32
    set_error("s2fp8: precision 32 quantises the tensor as is and needs fp32 input");
    return SMQ_ERR_INVALID;
  }
  if (flags & ~(SMQ_S2FP8_OUT_Y | SMQ_S2FP8_OUT_T | SMQ_S2FP8_EXACT_POW | SMQ_S2FP8_SPLIT |
                SMQ_S2FP8_TEST_LATE)) {
    set_error("s2fp8: unknown flags 0x%x", flags);
    return SMQ_ERR_INVALID;
  }
  const int out_mode = (flags & SMQ_S2FP8_OUT_Y) ? 1 : ((flags & SMQ_S2FP8_OUT_T) ? 2 : 0);
  if ((flags & SMQ_S2FP8_OUT_Y) && (flags & SMQ_S2FP8_OUT_T)) {
    set_error("s2fp8: SMQ_S2FP8_OUT_Y and SMQ_S2FP8_OUT_T are exclusive");
    return SMQ_ERR_INVALID;
  }
  if (out_mode && precision != 32) {
    set_error("s2fp8: SMQ_S2FP8_OUT_* need precision 32");
    return SMQ_ERR_INVALID;
  }
  if (!ws || ws_bytes < s2_ws_bytes()) {
    set_error("s2fp8: workspace too small: need %zu bytes", s2_ws_bytes());
    return SMQ_ERR_WORKSPACE;
  }
  hipStream_t st = (hipStream_t)stream;
  char* base = (char*)ws;
  SmqS2fp8Stats* hdr = (SmqS2fp8Stats*)base;
  S2Partial* partials = (S2Partial*)(base + 128);
  const uintptr_t align = dtype == SMQ_DTYPE_F32 ? 15u : 7u;  // one 4-element group per lane
  const bool xal = ((uintptr_t)x & align) == 0;
  const bool part = stats_in == nullptr;
  if (part && precision == 32 && !rand_bits && xal && aligned16f(y) && s2_fused_enabled() &&
      !(flags & SMQ_S2FP8_SPLIT)) {
    // one launch when a resident grid holds the tensor: <= kS2FMaxG chunks of <= kS2FMaxV float4
    // per lane (4.2M elements)
    const int64_t nv = n >> 2;
    const int64_t per_v = (int64_t)kS2FMaxG * kS2FT;
    int64_t V = (nv + per_v - 1) / per_v;
    if (V < 1) V = 1;
    if (V <= kS2FMaxV) {
      const int64_t G = nv > 0 ? (nv + V * kS2FT - 1) / (V * kS2FT) : 1;
      const ArriveTag tg = arrive_tag(ws, st);
      S2FArgs F;
      F.x = static_cast<const float*>(x);
      F.y = static_cast<float*>(y);
      F.n = n;
      F.nv = nv;
      F.V = (int)V;
      F.G = (int)G;
      F.key = rng_key(seed);
      F.offset = offset;
      F.ctr = offset_counter;
      F.hdr = hdr;
      F.gen = reinterpret_cast<uint32_t*>(base + kS2WsGen);
      F.left = reinterpret_cast<unsigned long long*>(base + kS2WsLeft);
      F.sub = reinterpret_cast<unsigned long long*>(base + kS2WsSub);
      F.gran = reinterpret_cast<unsigned long long*>(base + kS2WsGran);
      F.tag = tg.tag;
      F.check_inf = check_inf;
      F.max_value = host_max_value(5, 2);
      F.out_mode = out_mode;
      F.exact_pow = (flags & SMQ_S2FP8_EXACT_POW) ? 1 : 0;
      F.test_late = (flags & SMQ_S2FP8_TEST_LATE) ? 1 : 0;
      static const bool trace_env = [] {
        const char* e = knob_env("SMQ_S2_TRACE");
        return e && atoi(e) != 0;
      }();
      F.trace = (trace_env && ws_bytes >= s2_ws_bytes() + 128 * (size_t)kS2FMaxG)
                    ? reinterpret_cast<uint64_t*>(base + s2_ws_bytes())
                    : nullptr;
      static const hipError_t lds_attr = hipFuncSetAttribute(
          reinterpret_cast<const void*>(&s2fp8_fused_kernel<1>),
          hipFuncAttributeMaxDynamicSharedMemorySize, kS2FLds) != hipSuccess
          ? hipErrorInvalidValue
          : (hipFuncSetAttribute(reinterpret_cast<const void*>(&s2fp8_fused_kernel<2>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, kS2FLds) != hipSuccess ||
             hipFuncSetAttribute(reinterpret_cast<const void*>(&s2fp8_fused_kernel<3>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, kS2FLds) != hipSuccess ||
             hipFuncSetAttribute(reinterpret_cast<const void*>(&s2fp8_fused_kernel<4>),
                                 hipFuncAttributeMaxDynamicSharedMemorySize, kS2FLds) != hipSuccess)
                ? hipErrorInvalidValue
                : hipSuccess;
      if (lds_attr != hipSuccess) {
        set_error("s2fp8: hipFuncSetAttribute(MaxDynamicSharedMemorySize) failed: %s",
                  hipGetErrorString(lds_attr));
        return SMQ_ERR_LAUNCH;
      }
      static const int lds_bytes = [] {  // measurement knob SMQ_S2_LDS_KB (default: 1 per CU)
        const char* e = knob_env("SMQ_S2_LDS_KB");
        const int v = e ? atoi(e) * 1024 : kS2FLds;
        return (v >= 0 && v <= kS2FLds) ? v : kS2FLds;
      }();
      const dim3 grid((unsigned)G), block(kS2FT);
      if (V == 1) hipLaunchKernelGGL(s2fp8_fused_kernel<1>, grid, block, lds_bytes, st, F);
      else if (V == 2) hipLaunchKernelGGL(s2fp8_fused_kernel<2>, grid, block, lds_bytes, st, F);
      else if (V == 3) hipLaunchKernelGGL(s2fp8_fused_kernel<3>, grid, block, lds_bytes, st, F);
      else hipLaunchKernelGGL(s2fp8_fused_kernel<4>, grid, block, lds_bytes, st, F);
      return check_launch("s2fp8_fused_kernel");
    }
  }
  int n_partials = 0;
  if (!part) {
    if (dtype == SMQ_DTYPE_F32) hipLaunchKernelGGL(s2fp8_derive_kernel<kF32>, dim3(1), dim3(64), 0, st, stats_in, hdr, offset_counter, (uint64_t)n);
    else if (dtype == SMQ_DTYPE_F16) hipLaunchKernelGGL(s2fp8_derive_kernel<kF16>, dim3(1), dim3(64), 0, st, stats_in, hdr, offset_counter, (uint64_t)n);
    else hipLaunchKernelGGL(s2fp8_derive_kernel<kBF16>, dim3(1), dim3(64), 0, st, stats_in, hdr, offset_counter, (uint64_t)n);
  } else {
    const int vec = xal ? 1 : 0;
    const int64_t ng = vec ? (n >> 2) : (n + 3) / 4;
    const int64_t per = s2_groups_per_wg(ng);
    int64_t g = (ng + per - 1) / per;
    if (g < 1) g = 1;  // n < 4: the tail alone
    n_partials = (int)g;
#define SMQ_S2P(T)                                                                            \
  do {                                                                                        \
    if (s2_partial_threads() == 1024)                                                         \
      hipLaunchKernelGGL((s2fp8_partial_kernel<T, 1024>), dim3(n_partials), dim3(1024), 0, st, \
                         x, n, vec, per, partials, hdr, offset_counter);                      \
    else                                                                                      \
      hipLaunchKernelGGL((s2fp8_partial_kernel<T, kBlock>), dim3(n_partials), dim3(kBlock), 0, \
                         st, x, n, vec, per, partials, hdr, offset_counter);                  \
  } while (0)
    if (dtype == SMQ_DTYPE_F32) SMQ_S2P(kF32);
    else if (dtype == SMQ_DTYPE_F16) SMQ_S2P(kF16);
    else SMQ_S2P(kBF16);
#undef SMQ_S2P
  }
  int rc = check_launch(stats_in ? "s2fp8_derive_kernel" : "s2fp8_partial_kernel");
  if (rc) return rc;
  S2Args A;
  A.x = x;
  A.y = y;
  A.n = n;
  A.rand_bits = rand_bits;
  A.st = hdr;
  A.partials = partials;
  A.n_partials = n_partials;
  A.key = rng_key(seed);
  A.offset = offset;
  A.check_inf = check_inf;
  A.max_value = host_max_value(5, 2);
  A.out_mode = out_mode;
  A.exact_pow = (flags & SMQ_S2FP8_EXACT_POW) ? 1 : 0;
  const bool rarr = rand_bits != nullptr;
  const bool half_out = precision == 16 && dtype == SMQ_DTYPE_F16;
  const bool vec = xal && ((uintptr_t)y & (half_out ? 7u : 15u)) == 0;
  const int tv = precision == 32 ? s2_tile_v() : kFqDefaultTileV;
  int grid = (int)((n + (int64_t)kBlock * 4 * tv - 1) / ((int64_t)kBlock * 4 * tv));
  A.tiles_per_chunk = 0;
  A.n_chunks = 0;
  static const int xcd_env = [] {  // measurement knob SMQ_S2_XCD=0: tiles in index order
    const char* e = knob_env("SMQ_S2_XCD");
    return e ? atoi(e) : 1;
  }();
  if (xcd_env && part && vec && xal) {
    const int64_t per = s2_groups_per_wg(n >> 2);  // float4 groups of one partial chunk
    const int64_t tile_g = (int64_t)kBlock * tv;
    if (per % tile_g == 0 && n_partials > 1) {
      A.tiles_per_chunk = (int)(per / tile_g);
      A.n_chunks = n_partials;
      grid = 8 * ((n_partials + 7) / 8) * A.tiles_per_chunk;
    }
  }
  if (precision == 32) {
    if (tv == 1) s2_launch<1, kF32, false>(A, rarr, vec, part, grid, st);
    else if (tv == 2) s2_launch<2, kF32, false>(A, rarr, vec, part, grid, st);
    else s2_launch<4, kF32, false>(A, rarr, vec, part, grid, st);
  } else {
    // precision 16: the tile knob is not swept here
    if (dtype == SMQ_DTYPE_F32) s2_launch<kFqDefaultTileV, kF32, true>(A, rarr, vec, part, grid, st);
    else if (dtype == SMQ_DTYPE_F16) s2_launch<kFqDefaultTileV, kF16, true>(A, rarr, vec, part, grid, st);
    else s2_launch<kFqDefaultTileV, kBF16, true>(A, rarr, vec, part, grid, st);
  }
  return check_launch("s2fp8_apply_kernel");
}

int smq_s2fp8_roundtrip(const void* x, int dtype, void* y, int64_t n, int precision,
                        int check_inf, const uint32_t* rand_bits, uint64_t seed, uint64_t offset,
                        uint64_t* offset_counter, const SmqS2fp8Stats* stats_in, void* ws,
                        size_t ws_bytes, void* stream) {
  return smq_s2fp8_roundtrip_ex(x, dtype, y, n, precision, check_inf, rand_bits, seed, offset,
                                offset_counter, stats_in, ws, ws_bytes, 0u, stream);
}

int smq_s2fp8_roundtrip_f32(const float* x, float* y, int64_t n, int check_inf,
                            const uint32_t* rand_bits, uint64_t seed, uint64_t offset,
                            const SmqS2fp8Stats* stats_in, void* ws, size_t ws_bytes,
                            void* stream) {
  return smq_s2fp8_roundtrip(x, SMQ_DTYPE_F32, y, n, 32, check_inf, rand_bits, seed, offset,
                             nullptr, stats_in, ws, ws_bytes, stream);
}

}  // extern "C"
