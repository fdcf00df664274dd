// smaq_elem.h — SmaQ statistics accumulation/finalisation and the per-element transform, shared by
// the single-tensor (smaq.hip) and multi-tensor (smaq_multi.hip) kernels.
// Reference: smart_compress/compress/smart.py:100-108, 130-134, 151-182.
#pragma once

#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>
#include <math.h>

#include "smq_common.h"

namespace smq {

// ---- input element types (SMQ_DTYPE_*) ------------------------------------------------------------
// A half / bfloat16 input keeps the reference's dtype flow (verified on torch CPU with smart.py):
// statistics and the z-score `(data - mean) / std.clamp(...)` are computed in the input type
// (each op rounded to it), the bool*float scalars / ranges tensors are fp32 and promote the rest of
// the chain to fp32, so the output is fp32. One input-type op is emulated as the fp32 op followed
// by a rounding to the input type: exact, since fp32 has p' = 24 >= 2p + 2 bits for fp16 (p = 11)
// and bf16 (p = 8) (double rounding is innocuous for +, -, *, / at that margin).
enum InType { kF32 = SMQ_DTYPE_F32, kF16 = SMQ_DTYPE_F16, kBF16 = SMQ_DTYPE_BF16 };

template <int T>
__device__ __forceinline__ float round_in(float v) {
  if (T == kF16) return __half2float(__float2half_rn(v));
  if (T == kBF16) {
    // round to nearest even in hardware, ONE op: v_cvt_pk_bf16_f32 with the value as the HIGH
    // half and +0 as the low half leaves exactly the rounded fp32 bit pattern (the compiler's
    // own lowering of __float2bfloat16 adds a shift or permute back; the integer form
    // (u + 0x7fff + lsb) & 0xffff0000 with its NaN test is five). NaN stays NaN (its payload's top
    // bits kept, as torch's bf16 rounding keeps them)
    float r;
    asm("v_cvt_pk_bf16_f32 %0, 0, %1" : "=v"(r) : "v"(v));
    return r;
  }
  return v;
}

template <int T>
__device__ __forceinline__ float load1(const void* p, int64_t e) {
  if (T == kF32) return static_cast<const float*>(p)[e];
  const uint16_t h = static_cast<const uint16_t*>(p)[e];
  if (T == kF16) return __half2float(__builtin_bit_cast(__half, h));
  return __builtin_bit_cast(float, (uint32_t)h << 16);
}

// elements 4j .. 4j+3 with one 16-B (fp32) or 8-B (fp16 / bf16) load
template <int T>
__device__ __forceinline__ float4 load4(const void* p, int64_t j) {
  if (T == kF32) return static_cast<const float4*>(p)[j];
  const uint2 w = static_cast<const uint2*>(p)[j];
  float4 o;
  if (T == kF16) {
    o.x = __half2float(__builtin_bit_cast(__half, (uint16_t)(w.x & 0xffffu)));
    o.y = __half2float(__builtin_bit_cast(__half, (uint16_t)(w.x >> 16)));
    o.z = __half2float(__builtin_bit_cast(__half, (uint16_t)(w.y & 0xffffu)));
    o.w = __half2float(__builtin_bit_cast(__half, (uint16_t)(w.y >> 16)));
  } else {
    o.x = __builtin_bit_cast(float, w.x << 16);
    o.y = __builtin_bit_cast(float, w.x & 0xffff0000u);
    o.z = __builtin_bit_cast(float, w.y << 16);
    o.w = __builtin_bit_cast(float, w.y & 0xffff0000u);
  }
  return o;
}

// Streaming read of a tensor no later kernel of the call reads again (nt: bypasses L1, measured
// faster for the statistics sweep, the SmaQ apply and the float quantiser; NOT for kernels whose
// input the next launch re-reads, e.g. the S2FP8 partials -3 %, nor the multi-tensor chunks -0.8 %).
template <int T>
__device__ __forceinline__ float4 load4_stream(const void* p, int64_t j) {
  if (T == kF32) return load_nt(static_cast<const float4*>(p) + j);
  return load4<T>(p, j);
}

template <int T>
constexpr int in_bytes() { return T == kF32 ? 4 : 2; }

// ------------------------------------------------------------------------------------------------
// statistics
// ------------------------------------------------------------------------------------------------
struct StatAcc {
  double s1 = 0.0, s2 = 0.0;
  float mn = INFINITY, mx = -INFINITY;
  template <bool RANGE>
  __device__ __forceinline__ void add(float v, double shift) {
    const double d = (double)v - shift;
    s1 += d;
    s2 = fma(d, d, s2);
    if (RANGE) {
      mn = fminf(mn, v);
      mx = fmaxf(mx, v);
    }
  }
};

// Workgroup reduction of (s1, s2, mn, mx); result valid in thread 0.
template <bool RANGE>
__device__ __forceinline__ void block_reduce_stats(StatAcc& a) {
  __shared__ double sh1[kBlock / kWave], sh2[kBlock / kWave];
  __shared__ float shmn[kBlock / kWave], shmx[kBlock / kWave];
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  a.s1 = wave_sum(a.s1);
  a.s2 = wave_sum(a.s2);
  if (RANGE) {
    a.mn = wave_min(a.mn);
    a.mx = wave_max(a.mx);
  }
  if (lane == 0) {
    sh1[wave] = a.s1;
    sh2[wave] = a.s2;
    shmn[wave] = a.mn;
    shmx[wave] = a.mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    a.s1 = ((sh1[0] + sh1[1]) + (sh1[2] + sh1[3]));
    a.s2 = ((sh2[0] + sh2[1]) + (sh2[2] + sh2[3]));
    if (RANGE) {
      a.mn = fminf(fminf(shmn[0], shmn[1]), fminf(shmn[2], shmn[3]));
      a.mx = fmaxf(fmaxf(shmx[0], shmx[1]), fmaxf(shmx[2], shmx[3]));
    }
  }
  __syncthreads();
}

struct FinalizeArgs {
  float clamp_lo, clamp_hi, range_coef;  // range_coef is representable in the input type
  unsigned long long* rng_ctr = nullptr;  // graph-safe stream position (params.offset_counter)
  int64_t rng_n = 0;                      // elements the call consumes from it
  uint32_t* zero = nullptr;               // words the statistics launch clears for the next
  uint32_t zero_n = 0;                    // launch of the call (the packer's group sums)
};

// The statistics launch's first workgroup clears fin.zero (all its threads, before the sweep): the
// packer's group sums then need no launch of their own.
__device__ __forceinline__ void clear_aux(const FinalizeArgs& f) {
  if (f.zero && blockIdx.x == 0)
    for (uint32_t i = threadIdx.x; i < f.zero_n; i += blockDim.x) f.zero[i] = 0u;
}

// mean / std from shifted sums -> SmqSmaqStats (smart.py:130-134, 100-108, 151-152, 154).
// T = input type: torch reduces half tensors in fp32/fp64 and rounds the 0-dim result to half
// (through fp32, i.e. RN_T(RN32(.))), exactly what round_in<T>((float)x) does.
// Does z = RN32(RN64(dm * RN64(1/sc))) need the IEEE fallback when z is subnormal?
// dm is a multiple of 2^-149 (every fp32 / fp16 / bf16 difference is). Write sc = S * 2^e, S odd.
// The distance of dm / sc from a midpoint of the subnormal grid (2m+1) * 2^-150 is
// |dm * 2^150 - sc * (2m+1)| / (sc * 2^150). For e <= 0 the numerator is a nonzero multiple of 2^e
// (even minus odd after scaling by 2^-e), so the distance is >= 2^-174 > 2^-48 * |z| for |z| <
// 2^-126, while the double product is within 2^-52 * |z|: the fp32 rounding is the IEEE one. For
// e >= 1 (sc an even integer) exact midpoints exist, and sc >= 2^24 is excluded for margin: those
// calls keep the per-element check.
__host__ __device__ __forceinline__ uint32_t quot_check_for(float sc) {
  const float h = sc * 0.5f;
  const bool even_int = (h == truncf(h)) && h != 0.0f;  // sc = odd * 2^e with e >= 1
  return (even_int || !(fabsf(sc) < 0x1p24f)) ? 1u : 0u;
}

template <bool RANGE, int T = kF32>
__device__ __forceinline__ void finalize_stats(double s1, double s2, float mn, float mx, int64_t n,
                                               double shift, bool biased, FinalizeArgs f,
                                               SmqSmaqStats* out) {
  const double nd = (double)n;
  const double mean = shift + s1 / nd;
  float sd;
  if (RANGE) {
    const float range = round_in<T>(mx - mn);  // data.max() - data.min()
    sd = round_in<T>(range * f.range_coef);    // range_ * C
  } else {
    double var = (s2 - s1 * (s1 / nd)) / (biased ? nd : (nd - 1.0));
    if (var < 0.0) var = 0.0;
    sd = round_in<T>((float)sqrt(var));
  }
  const float std_dev = (sd == 0.0f) ? 1.0f : sd;  // smart.py:151-152
  const float lo = round_in<T>(f.clamp_lo), hi = round_in<T>(f.clamp_hi);
  float sc = std_dev < lo ? lo : std_dev;          // .clamp(*clamped_range) in the input type
  sc = sc > hi ? hi : sc;
  out->mean = round_in<T>((float)mean);
  out->std_dev = std_dev;
  out->std_clamped = sc;
  out->raw_std = sd;
  out->min_val = mn;
  out->max_val = mx;
  out->n_used = (uint32_t)(n > 0xffffffffLL ? 0xffffffffu : (uint32_t)n);
  out->n_outlier = 0ull;
  out->inv_std_clamped = 1.0 / (double)sc;  // once per call, for the element transform
  out->inv_std_clamped_f32 = (float)out->inv_std_clamped;  // half inputs: half_quot
  out->quot_check = quot_check_for(sc);
  // graph-safe random stream: snapshot the position for this call's element kernels, advance it
  unsigned long long base = 0ull;
  if (f.rng_ctr) {
    base = *f.rng_ctr;
    *f.rng_ctr = base + (unsigned long long)f.rng_n;
  }
  out->rng_offset = base;
}

// ------------------------------------------------------------------------------------------------
// element transform
// ------------------------------------------------------------------------------------------------
// The two-op fp32 quotient q / range for half inputs (quot_split_compute below).
struct QuotSplit {
  float hm, lm, ho, lo;  // main / outlier range: h = RN32(1 / r), l = RN32(1 / r - h)
  int ok;                // every reachable code checked
};

struct ElemConsts {
  float mean, sd, sc;     // mean, std (after ==0 rule), clamped std
  float thr, nthr;        // fp32(T_m), -fp32(T_m): the values of the scalars tensor (fp32)
  float cthr, cnthr;      // thresholds as compared with z: rounded to z's type
  float zh, zl;           // 0 * -T_m, 0 * T_m  (the bool*float zero terms, smart.py:159-161)
  float r_main, r_out;    // ranges
  double inv_sc;          // RN64(1 / sc): written by the statistics finaliser
  float inv_sc32;         // RN32(1 / sc): half inputs (half_quot)
  double inv_r_main, inv_r_out;  // RN64(1 / range): computed on the host
  QuotSplit qs;           // half inputs: the two-op fp32 quotient (quot_split_for), QF forms only
  uint64_t rng_off;      // the call's graph-safe stream position (SmqSmaqStats.rng_offset)
};

// Correctly rounded fp32 quotient a / b from a double reciprocal: RN32(RN64(a * RN64(1/b))).
// Why this equals IEEE a / b: for normal fp32 a, b and a normal result, an exact quotient a/b is
// never closer than 2^-49 (relative) to an fp32 rounding boundary (a midpoint needs 25 significant
// bits, a = b * M would need >= 25 bits in a), while the double evaluation is within 2^-52; the
// overflow threshold is such a midpoint too. Subnormal results lose that margin, so the caller
// re-does those with IEEE division (never taken for realistic data). Division by 0 -> +-inf / NaN
// as IEEE (1/0 = inf in double). Cost: 3 VALU (cvt, v_mul_f64, cvt) instead of ~10.
__device__ __forceinline__ float div_by_const(float a, double inv_b) {
  return (float)((double)a * inv_b);
}

// The reciprocals come precomputed (statistics record / kernel arguments): a per-workgroup fp64
// division costs ~15 dependent VALU, more than the elements of a one-vector tile.
__device__ __forceinline__ void init_consts(ElemConsts& c, const SmqSmaqStats* st, float thr,
                                            float r_main, float r_out, double inv_r_main,
                                            double inv_r_out, float cthr) {
  c.mean = st->mean;
  c.sd = st->std_dev;
  c.sc = st->std_clamped;
  c.inv_sc = st->inv_std_clamped;
  c.inv_sc32 = st->inv_std_clamped_f32;
  c.thr = thr;
  c.nthr = -thr;
  c.cthr = cthr;
  c.cnthr = -cthr;
  c.zh = 0.0f * c.nthr;
  c.zl = 0.0f * c.thr;
  c.r_main = r_main;
  c.r_out = r_out;
  c.inv_r_main = inv_r_main;
  c.inv_r_out = inv_r_out;
  c.rng_off = st->rng_offset;
}

// Host: reciprocals of the two ranges (IEEE double division, as the device would compute them).
// safe_q: with a range beyond 2^100 (absurd flags) a quotient q / range can be subnormal, where the
// reciprocal product is not exact; the element transform then takes an IEEE division.
struct RangeRecips {
  double inv_main, inv_out;
  int safe_q;
};
static inline RangeRecips range_recips(float r_main, float r_out) {
  RangeRecips R;
  R.inv_main = 1.0 / (double)r_main;
  R.inv_out = 1.0 / (double)r_out;
  const double lim = 0x1p100;
  R.safe_q = !(fabs((double)r_main) <= lim && fabs((double)r_out) <= lim);
  return R;
}

enum RoundMode { kRoundHash = 0, kRoundUniform = 1, kRoundTrunc = 2 };

// Half inputs without the BN term: the z-score is a half value (65,536 bit patterns), so the codes
// the element transform can produce form a finite set fixed by the flags — per z-score floor(d) and
// floor(d) + 1 or + 2 (stochastic rounding, whatever the draw) or trunc(d). Over that set the quotient
// q / range takes two fp32 ops,
//     RN32(q / r) == fmaf(q, h, RN32(q * l)),   h = RN32(1 / r),  l = RN32(1 / r - h),
// checked exhaustively on the host against the IEEE quotient, once per flag set (~130K codes,
// <1 ms, cached); when every code passes (ok), the half apply launch takes this form instead of
// the fp64 reciprocal product (a 64-bit select, cvt, v_mul_f64, cvt). A flag set with one failing
// code keeps the fp64 form. Sweep of 17,640 SmaQ flag sets (num_bits 3-16, thresholds on a grid):
// every stochastic-rounding set passes; under truncation q = +-inf is reachable (an overflowing
// z-score) and fails whenever l < 0 (inf - inf), so most truncating sets keep the fp64 form.
// The reachable-set argument and the check are restated in oracle/csrc/half_div_check.c (qr mode).
// (struct QuotSplit: above ElemConsts)

static inline float host_half_value(int tin, uint32_t b) {  // fp16 / bf16 bits -> fp32 (exact)
  if (tin == kBF16) return __builtin_bit_cast(float, b << 16);
  const uint32_t s = (b & 0x8000u) << 16, e = (b >> 10) & 0x1fu, m = b & 0x3ffu;
  if (e == 0x1fu) return __builtin_bit_cast(float, s | 0x7f800000u | (m << 13));
  if (e == 0) return m ? (s ? -1.0f : 1.0f) * (float)m * 0x1p-24f : __builtin_bit_cast(float, s);
  return __builtin_bit_cast(float, s | ((e + 112u) << 23) | (m << 13));
}

static inline float host_round_half(int tin, float v) {  // round_in<tin> on the host (finite v)
  const uint32_t x = __builtin_bit_cast(uint32_t, v), s = x & 0x80000000u, ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return v;
  if (tin == kBF16) return __builtin_bit_cast(float, (x + 0x7fffu + ((x >> 16) & 1u)) & 0xffff0000u);
  if (ax >= 0x477ff000u) return __builtin_bit_cast(float, s | 0x7f800000u);
  if (ax < 0x38800000u)
    return __builtin_bit_cast(float, s | __builtin_bit_cast(uint32_t, nearbyintf(__builtin_bit_cast(float, ax) * 0x1p24f) * 0x1p-24f));
  return __builtin_bit_cast(float, s | ((ax + 0x0fffu + ((ax >> 13) & 1u)) & ~0x1fffu));
}

// rm: RoundMode (kRoundTrunc or a stochastic one; the draw does not matter).
static inline QuotSplit quot_split_compute(int tin, float thr, float r_main, float r_out, int rm) {
  QuotSplit s;
  s.hm = (float)(1.0 / (double)r_main);
  s.lm = (float)(1.0 / (double)r_main - (double)s.hm);
  s.ho = (float)(1.0 / (double)r_out);
  s.lo = (float)(1.0 / (double)r_out - (double)s.ho);
  s.ok = 0;
  if (!(__builtin_isfinite(r_main) && __builtin_isfinite(r_out) && __builtin_isfinite(s.hm) &&
        __builtin_isfinite(s.ho)))
    return s;
  const float cthr = host_round_half(tin, thr), cnthr = -cthr;
  const float nthr = -thr, zh = 0.0f * nthr, zl = 0.0f * thr;
  for (uint32_t b = 0; b < 0x10000u; ++b) {
    const float z = host_half_value(tin, b);
    const bool hi = z > cthr, lo = z < cnthr, o = hi || lo;
    const float a = (hi ? nthr : zh) + (lo ? thr : zl);
    const float r = o ? r_out : r_main;
    const volatile float za = z + a;  // two roundings, as on the device
    const float d = za * r;
    float qs[3];
    int nq = 1;
    if (rm == kRoundTrunc) {
      qs[0] = truncf(d);
    } else {
      // f + rint(relu(RN(fr - u) + 0.5)) with fr = d - f in [0, 1): 0 or 1 is added, and 2 when
      // RN(fr + 0.5) ties up to 1.5 (fr = 1 - 2^-24, d < 1). d = +-inf: fr = NaN, q = NaN.
      if (__builtin_isinf(d)) continue;
      qs[0] = floorf(d);
      const volatile float f1 = qs[0] + 1.0f, f2 = qs[0] + 2.0f;
      qs[1] = f1;
      qs[2] = f2;
      nq = 3;
    }
    for (int i = 0; i < nq; ++i) {
      const float q = qs[i];
      const volatile float want = q / r;
      const volatile float ql = q * (o ? s.lo : s.lm);
      const float got = fmaf(q, o ? s.ho : s.hm, ql);
      const float w = want;
      if (!(__builtin_bit_cast(uint32_t, w) == __builtin_bit_cast(uint32_t, got) ||
            (w != w && got != got)))
        return s;
    }
  }
  s.ok = 1;
  return s;
}

// The check cached per flag set (per thread: no lock on the launch path).
static inline QuotSplit quot_split_for(int tin, float thr, float r_main, float r_out, int rm) {
  struct Key {
    int tin, rm;
    float thr, r_main, r_out;
  };
  thread_local Key key{-1, -1, 0.0f, 0.0f, 0.0f};
  thread_local QuotSplit val{};
  const bool trunc = rm == kRoundTrunc;
  if (key.tin != tin || (key.rm == kRoundTrunc) != trunc ||
      __builtin_bit_cast(uint32_t, key.thr) != __builtin_bit_cast(uint32_t, thr) ||
      __builtin_bit_cast(uint32_t, key.r_main) != __builtin_bit_cast(uint32_t, r_main) ||
      __builtin_bit_cast(uint32_t, key.r_out) != __builtin_bit_cast(uint32_t, r_out)) {
    val = quot_split_compute(tin, thr, r_main, r_out, rm);
    key = Key{tin, rm, thr, r_main, r_out};
  }
  return val;
}

// kRoundHash draws: smaq_u24 (smq_common.h) as a float (exact, < 2^24), see smaq_elem.
__device__ __forceinline__ float rng_hu(uint32_t key, uint64_t ctr) {
  return (float)smaq_u24(key, ctr);
}

// Draws for counters ctr .. ctr+3 (one float4 of elements): the same values as four rng_hu calls.
// ctr & 3 is the call's stream position mod 4 (wave-uniform): 0 (every activation-sized stream)
// takes ONE quad hash; otherwise the four counters straddle two quads.
__device__ __forceinline__ void rng_hu4(uint32_t key, uint64_t ctr, float& u0, float& u1, float& u2,
                                        float& u3) {
  const uint32_t s = (uint32_t)ctr & 3u;
  if (__builtin_expect(s == 0u, 1)) {
    const uint32_t h = quad_word(key, ctr >> 2);
    u0 = (float)(h >> 8);
    u1 = (float)((h * draw_mul(1u)) >> 8);
    u2 = (float)((h * draw_mul(2u)) >> 8);
    u3 = (float)((h * draw_mul(3u)) >> 8);
  } else {
    const uint64_t q = ctr >> 2;
    const uint32_t h0 = quad_word(key, q), h1 = quad_word(key, q + 1);
    u0 = (float)((h0 * draw_mul(s)) >> 8);
    u1 = (float)(((s + 1u < 4u ? h0 : h1) * draw_mul((s + 1u) & 3u)) >> 8);
    u2 = (float)(((s + 2u < 4u ? h0 : h1) * draw_mul((s + 2u) & 3u)) >> 8);
    u3 = (float)((h1 * draw_mul((s + 3u) & 3u)) >> 8);
  }
}

// The same draws for the float4 groups j = 0, 1, ... of a run starting at counter c0: group j's
// counters are c0 + 4j .. + 3, so its quads are (c0 >> 2) + j (and the next one when c0 & 3 != 0).
// c0 is a per-launch (or per-workgroup) value, so the offset within the quad, the quad's high word
// and its contribution to quad_word are scalar; as long as (c0 >> 2) + j + 1 does not carry into
// the high word for any group of the run (flat: checked once, on the scalar unit) a group costs a
// 32-bit add and the mix instead of a 64-bit add, the high-word rotate and a per-lane test of
// c & 3. A run that crosses a 2^32-quad boundary (one call in 2^34 stream elements) takes rng_hu4.
struct QuadRun {
  uint64_t c0;
  uint32_t key, keyx;  // keyx = key ^ rot16(high word of the quad index)
  uint32_t qlo, s;     // low word of c0 >> 2, c0 & 3
  bool flat;
};

__device__ __forceinline__ QuadRun quad_run(uint32_t key, uint64_t c0, uint64_t groups) {
  QuadRun R;
  // c0 is uniform, but read from memory (the statistics record) the compiler cannot prove it:
  // readfirstlane puts it (and everything derived) in SGPRs, so the tests below are scalar branches
  c0 = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)c0) |
       ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(c0 >> 32)) << 32);
  key = (uint32_t)__builtin_amdgcn_readfirstlane((int)key);
  const uint64_t q = c0 >> 2;
  const uint32_t hi = (uint32_t)(q >> 32);
  R.c0 = c0;
  R.key = key;
  R.keyx = key ^ ((hi << 16) | (hi >> 16));
  R.qlo = (uint32_t)q;
  R.s = (uint32_t)c0 & 3u;
  R.flat = (uint64_t)R.qlo + groups + 1u <= 0xffffffffull;
  return R;
}

__device__ __forceinline__ void rng_hu4_run(const QuadRun& R, uint32_t j, float& u0, float& u1,
                                            float& u2, float& u3) {
  if (__builtin_expect(!R.flat, 0)) {
    rng_hu4(R.key, R.c0 + ((uint64_t)j << 2), u0, u1, u2, u3);
    return;
  }
  const uint32_t q = R.qlo + j;
  const uint32_t s = R.s;
  if (__builtin_expect(s == 0u, 1)) {
    const uint32_t h = mix32x3(q ^ R.keyx);
    u0 = (float)(h >> 8);
    u1 = (float)((h * draw_mul(1u)) >> 8);
    u2 = (float)((h * draw_mul(2u)) >> 8);
    u3 = (float)((h * draw_mul(3u)) >> 8);
  } else {
    const uint32_t h0 = mix32x3(q ^ R.keyx), h1 = mix32x3((q + 1u) ^ R.keyx);
    u0 = (float)((h0 * draw_mul(s)) >> 8);
    u1 = (float)(((s + 1u < 4u ? h0 : h1) * draw_mul((s + 1u) & 3u)) >> 8);
    u2 = (float)(((s + 2u < 4u ? h0 : h1) * draw_mul((s + 2u) & 3u)) >> 8);
    u3 = (float)((h1 * draw_mul((s + 3u) & 3u)) >> 8);
  }
}

// kRoundHash: u arrives as the integer h >> 8 (a float in [0, 2^24)); fr - u is then the single
// rounding fma(h, -2^-24, fr) == RN(fr - h * 2^-24) (the product is exact), one op fewer
// (RoundMode above).

// F.relu of the stochastic-rounding term t = RN(RN(fr - u) + 0.5) (smart.py:93-98) in ONE op:
// v_maximum3_f32 (IEEE 754-2019 maximum: NaN propagates, as relu keeps it) instead of a compare
// and a select. The two differ only for t = -0 (maximum gives +0), and t is never -0: fr = d -
// floor(d) is never -0, so neither is w = RN(fr - u) (fma(u, -2^-24, fr) with u = 0 gives +0), and
// w + 0.5 cannot be -0 (a sum is -0 only when both addends are; an exact cancellation gives +0).
__device__ __forceinline__ float relu_t(float t) { return __builtin_elementwise_maximum(t, 0.0f); }

// Per-channel BatchNorm fold (smart.py:144-149 before, 174-179 after); scale = gamma[c].
struct BnTerm {
  float gamma, beta;
};

// Half-type z-score quotient RN_T(dm / sc) for fp16 / bf16 dm and sc as RN_T(RN32(dm * RN32(1/sc))):
// one fp32 multiply instead of the fp64 reciprocal product. Verified exhaustively over every pair of
// half values with a finite fp32 reciprocal (oracle/csrc/half_div_check.c: 1.7e9 fp16 and 2.0e9 bf16
// pairs, 0 mismatches) for products at or above the type's smallest normal (2^-14 fp16, 2^-126
// bf16). Below it exact midpoints of the coarse subnormal grid occur (fp16: 2,990 pairs), so those
// quotients (and zeros, which the test cannot tell apart cheaply) take the fp64 path.
template <int T>
__device__ __forceinline__ float half_quot(float dm, const ElemConsts& c) {
  const float p = dm * c.inv_sc32;
  const float lim = T == kF16 ? 0x1p-14f : 0x1p-126f;
  if (__builtin_expect(fabsf(p) < lim, 0)) {
    float z = div_by_const(dm, c.inv_sc);
    if (__builtin_amdgcn_classf(z, 0x90)) z = dm / c.sc;
    return z;
  }
  return p;
}

// Template flags: AP all_positive; SUB keep the subnormal-quotient check (quot_check_for); SQ
// divide q / range by IEEE division (RangeRecips::safe_q).

// smart.py:144-169: the integer-valued code q and the outlier sides of one element.
template <int RM, bool BN = false, int T = kF32, bool SUB = true>
__device__ __forceinline__ float smaq_quant(float v, float u, const ElemConsts& c, bool& hi,
                                            bool& lo, BnTerm bn = BnTerm{1.0f, 0.0f}) {
  constexpr int TZ = BN ? kF32 : T;  // fp32 BN parameters promote the data to fp32
  if (BN) v = (v - bn.beta) / bn.gamma;                 // (data - beta) / gamma
  const float dm = round_in<TZ>(v - c.mean);            // data - mean
  float z;                                              // / std.clamp(...)
  if (TZ != kF32) {
    z = half_quot<TZ>(dm, c);
  } else {
    z = div_by_const(dm, c.inv_sc);
    // subnormal quotient (class mask 0x90 = -/+ denormal, one v_cmp_class_f32): IEEE division.
    // (classf: the unsuffixed builtin takes a double, where a promoted float is never subnormal.)
    if (SUB && __builtin_expect(__builtin_amdgcn_classf(z, 0x90), 0)) z = dm / c.sc;
  }
  z = round_in<TZ>(z);
  hi = z > c.cthr;                                      // is_outlier_higher
  lo = z < c.cnthr;                                     // is_outlier_lower
  const bool o = hi | lo;                               // is_outlier
  const float a = (hi ? c.nthr : c.zh) + (lo ? c.thr : c.zl);  // scalars
  const float r = o ? c.r_out : c.r_main;               // ranges
  const float d = (z + a) * r;
  float q;
  if (RM == kRoundTrunc) {
    q = truncf(d);
  } else {
    const float f = floorf(d);                          // _round_stochastic, smart.py:93-98
    const float fr = d - f;
    float t = ((RM == kRoundHash) ? __builtin_fmaf(u, -0x1p-24f, fr) : (fr - u)) + 0.5f;
    t = relu_t(t);                                      // F.relu
    q = f + __builtin_rintf(t);                         // .round() = half to even
  }
  return q;
}

// smart.py:171-182: de-quantise a code q with its outlier sides.
// QF: the two-op fp32 quotient of a checked flag set (QuotSplit; half inputs without BN only).
template <bool BN = false, bool AP = false, bool SQ = false, bool QF = false>
__device__ __forceinline__ float smaq_dequant(float q, bool hi, bool lo, const ElemConsts& c,
                                              BnTerm bn = BnTerm{1.0f, 0.0f}) {
  const bool o = hi | lo;
  const float a = (hi ? c.nthr : c.zh) + (lo ? c.thr : c.zl);  // scalars
  float qr;                                             // data / ranges
  if (QF) {
    qr = __builtin_fmaf(q, o ? c.qs.ho : c.qs.hm, q * (o ? c.qs.lo : c.qs.lm));
  } else if (SQ) {
    qr = q / (o ? c.r_out : c.r_main);
  } else {
    qr = div_by_const(q, o ? c.inv_r_out : c.inv_r_main);
  }
  float out = qr - a;                                   //   - scalars
  out = (out * c.sd) + c.mean;
  if (BN) out = (out * bn.gamma) + bn.beta;             // (data * gamma) + beta
  if (AP) out = (out < 0.0f) ? 0.0f : out;              // clamp_min(0.0)
  return out;
}

// One element of smart.py:154-182 (quant then dequant, every statement one rounded fp32 op of the
// reference). T = input type (z-score rounded to it unless BN already promoted the data to fp32).
template <int RM, bool BN = false, int T = kF32, bool AP = false, bool SUB = true, bool SQ = false,
          bool QF = false>
__device__ __forceinline__ float smaq_elem(float v, float u, const ElemConsts& c,
                                           bool& is_outlier, BnTerm bn = BnTerm{1.0f, 0.0f}) {
  static_assert(!QF || (!BN && T != kF32 && !SQ), "QF: half inputs without BN");
  bool hi, lo;
  const float q = smaq_quant<RM, BN, T, SUB>(v, u, c, hi, lo, bn);
  is_outlier = hi | lo;
  return smaq_dequant<BN, AP, SQ, QF>(q, hi, lo, c, bn);
}

// smart.py:155-169 from the z-score on (smaq_quant's tail, no BN term): the code q and the sides.
template <int RM>
__device__ __forceinline__ float smaq_quant_z(float z, float u, const ElemConsts& c, bool& hi,
                                              bool& lo) {
  hi = z > c.cthr;
  lo = z < c.cnthr;
  const bool o = hi | lo;
  const float a = (hi ? c.nthr : c.zh) + (lo ? c.thr : c.zl);
  const float r = o ? c.r_out : c.r_main;
  const float d = (z + a) * r;
  if (RM == kRoundTrunc) return truncf(d);
  const float f = floorf(d);
  const float fr = d - f;
  float t = ((RM == kRoundHash) ? __builtin_fmaf(u, -0x1p-24f, fr) : (fr - u)) + 0.5f;
  t = relu_t(t);
  return f + __builtin_rintf(t);
}

// Two fp16 elements (raw bits, low half first) through smart.py:154-182: data - mean as ONE
// v_pk_add_f16 (RN16(v - mean) directly, which round_in<kF16>(v - mean) emulates through fp32) and
// both z-scores rounded to fp16 by ONE v_cvt_pk_f16_f32 (RNE, as __float2half_rn); the rest of the
// chain per element, exactly smaq_elem<RM, false, kF16, AP, SUB>.
typedef float f2v __attribute__((ext_vector_type(2)));
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
template <int RM, bool AP, bool QF = false>
__device__ __forceinline__ void smaq_elem_f16x2(uint32_t raw, float u0, float u1,
                                                const ElemConsts& c, float& o0, float& o1,
                                                bool& b0, bool& b1) {
  const _Float16 m = (_Float16)c.mean;  // exact: the mean is an fp16 value
  const h2v dh = __builtin_bit_cast(h2v, raw) - h2v{m, m};
  const float dm0 = (float)dh.x, dm1 = (float)dh.y;
  const f2v z = __builtin_convertvector(
      __builtin_convertvector(f2v{half_quot<kF16>(dm0, c), half_quot<kF16>(dm1, c)}, h2v), f2v);
  bool hi0, lo0, hi1, lo1;
  const float q0 = smaq_quant_z<RM>(z.x, u0, c, hi0, lo0);
  const float q1 = smaq_quant_z<RM>(z.y, u1, c, hi1, lo1);
  b0 = hi0 | lo0;
  b1 = hi1 | lo1;
  o0 = smaq_dequant<false, AP, false, QF>(q0, hi0, lo0, c);
  o1 = smaq_dequant<false, AP, false, QF>(q1, hi1, lo1, c);
}

// ------------------------------------------------------------------------------------------------
// Device-drawn sampled statistics (SMQ_STATS_SAMPLED_DEVICE): smart.py:86-91 with the randperm
// of line 88 replaced by Floyd's algorithm on the device, so every call — and every replay of a
// captured graph — draws a fresh index set from the call's stream position.
//
// Floyd: for i = 0 .. k-1, j = n - k + i: t = h_i mod (j + 1); pick t unless an earlier pick
// equals it, then pick j (never picked before: every earlier pick is < j). h_i is the 64-bit word
// (rng_u32(key', 2P + 2i) << 32) | rng_u32(key', 2P + 2i + 1), key' = rng_key(seed ^ kDrawSalt),
// P = offset + stream position (+ the tensor's offset in a multi-tensor call): a function of the
// call alone (smq_smaq_draw_samples and oracle/rng.py floyd_indices restate it). The candidates t
// are independent and computed in parallel; only the duplicate test is sequential: a
// register/ballot scan by one wave for k <= 64, an LDS open-addressing set walked by one lane for
// larger k.
// ------------------------------------------------------------------------------------------------
constexpr uint64_t kDrawSalt = 0xd1b54a32d192ed03ull;

__host__ __device__ __forceinline__ int64_t floyd_candidate(uint32_t key, uint64_t pos, int64_t n,
                                                            int k, int i) {
  const uint64_t c = 2ull * pos + 2ull * (uint64_t)i;
  const uint64_t h = ((uint64_t)rng_u32(key, c) << 32) | rng_u32(key, c + 1);
  return (int64_t)(h % (uint64_t)(n - k + i + 1));
}

__device__ __forceinline__ uint32_t pick_hash(int64_t t, int bits) {
  const uint32_t v = (uint32_t)t ^ (uint32_t)((uint64_t)t >> 32);
  return (v * 0x9e3779b1u) >> (32 - bits);
}

// LDS of one workgroup's draw (48 KiB at SMQ_MAX_DEVICE_SAMPLES = 4096)
struct DrawLds {
  int64_t pick[SMQ_MAX_DEVICE_SAMPLES];        // candidates, then the picks in draw order
  uint16_t table[2 * SMQ_MAX_DEVICE_SAMPLES];  // open-addressing set: pick index + 1, 0 = empty
  double shs[kBlock / kWave];
};

// Floyd's k distinct indices of draw position `pos` into L.pick (draw order), by one 256-thread
// workgroup (every thread calls it; the picks are complete after the trailing barrier).
static __device__ void draw_picks(int64_t n, int k, uint32_t key, uint64_t pos, DrawLds& L) {
  int64_t* pick = L.pick;
  uint16_t* table = L.table;
  for (int i = threadIdx.x; i < k; i += kBlock) pick[i] = floyd_candidate(key, pos, n, k, i);
  int bits = 1;
  while ((1 << bits) < 2 * k) ++bits;
  if (k > kWave)
    for (int i = threadIdx.x; i < (1 << bits); i += kBlock) table[i] = 0;
  __syncthreads();
  if (k <= kWave) {
    if (threadIdx.x < kWave) {  // lane i holds pick i; lanes < i are final at step i
      const int lane = threadIdx.x;
      int64_t p = lane < k ? pick[lane] : -1;
      for (int i = 1; i < k; ++i) {
        const int32_t lo = __builtin_amdgcn_readlane((int32_t)p, i);
        const int32_t hi = __builtin_amdgcn_readlane((int32_t)((uint64_t)p >> 32), i);
        const int64_t t = (int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo);
        const bool dup = __ballot(lane < i && p == t) != 0ull;
        if (dup && lane == i) p = n - k + i;
      }
      if (lane < k) pick[lane] = p;
    }
  } else if (threadIdx.x == 0) {
    const uint32_t mask = (1u << bits) - 1u;
    for (int i = 0; i < k; ++i) {
      int64_t t = pick[i];
      uint32_t s = pick_hash(t, bits);
      bool dup = false;
      for (uint16_t e; (e = table[s]) != 0; s = (s + 1) & mask)
        if (pick[e - 1] == t) {
          dup = true;
          break;
        }
      if (dup) {  // j = n - k + i is new: probe for its own empty slot
        t = n - k + i;
        s = pick_hash(t, bits);
        while (table[s] != 0) s = (s + 1) & mask;
      }
      pick[i] = t;
      table[s] = (uint16_t)(i + 1);
    }
  }
  __syncthreads();
}

// The k distinct indices of draw position `pos` (Floyd) and the mean / biased std (or range-std)
// of the gathered elements into *out, by one 256-thread workgroup (every thread calls it).
// idx_out (optional) receives the indices in draw order.
template <int TIN>
__device__ void draw_sample_stats(const void* x, int64_t n, int k, uint32_t key, uint64_t pos,
                                  int use_range, const FinalizeArgs& f, SmqSmaqStats* out,
                                  int64_t* idx_out, DrawLds& L) {
  const int64_t* pick = L.pick;
  draw_picks(n, k, key, pos, L);
  // gather: thread t owns samples t, t + kBlock, ... (<= 16); fp64 sums in one fixed order
  constexpr int kPer = SMQ_MAX_DEVICE_SAMPLES / kBlock;
  float v[kPer];
  double s = 0.0;
  float mn = INFINITY, mx = -INFINITY;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = threadIdx.x + u * kBlock;
    v[u] = 0.0f;
    if (i < k) {
      const int64_t e = pick[i];
      if (idx_out) idx_out[i] = e;
      v[u] = load1<TIN>(x, e);
      s += (double)v[u];
      mn = fminf(mn, v[u]);
      mx = fmaxf(mx, v[u]);
    }
  }
  const int lane = threadIdx.x & (kWave - 1), wave = threadIdx.x / kWave;
  s = wave_sum(s);
  if (lane == 0) L.shs[wave] = s;
  __syncthreads();
  const double mean = ((L.shs[0] + L.shs[1]) + (L.shs[2] + L.shs[3])) / (double)k;
  __syncthreads();
  double m2 = 0.0;
#pragma unroll
  for (int u = 0; u < kPer; ++u) {
    const int i = threadIdx.x + u * kBlock;
    if (i < k) {
      const double d = (double)v[u] - mean;
      m2 = fma(d, d, m2);
    }
  }
  StatAcc acc;
  acc.s1 = 0.0;
  acc.s2 = m2;
  acc.mn = mn;
  acc.mx = mx;
  block_reduce_stats<true>(acc);
  if (threadIdx.x == 0) {
    SmqSmaqStats st;
    // shifted sums with shift = mean: s1 = 0, s2 = the biased second moment's numerator
    if (use_range)
      finalize_stats<true, TIN>(0.0, acc.s2, acc.mn, acc.mx, k, mean, true, f, &st);
    else
      finalize_stats<false, TIN>(0.0, acc.s2, acc.mn, acc.mx, k, mean, true, f, &st);
    *out = st;
  }
}

// Workspace region and launch arguments of the multi-workgroup draw (smaq.hip).
constexpr int kDrawGridCap = 1024;

struct LargeDrawLayout {  // byte offsets from SMQ_WS_LARGE_SAMPLES_OFFSET
  int bits = 1;
  size_t pick = 0, hkey = 0, hdup = 0, h2key = 0, susp = 0, parts = 0, total = 0;
  explicit LargeDrawLayout(int64_t k) {
    while ((int64_t)1 << bits < 2 * k) ++bits;
    const size_t slots = (size_t)1 << bits;
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    pick = 0;
    hkey = up(pick + 8 * (size_t)k);
    hdup = up(hkey + 8 * slots);
    h2key = up(hdup + 4 * slots);
    susp = up(h2key + 8 * slots);
    parts = up(susp + 4 * (size_t)((k + 31) / 32));
    total = up(parts + sizeof(StatPartial) * kDrawGridCap);
  }
};

struct LargeDrawArgs {
  const void* x;
  int64_t n, k;
  uint32_t key;                   // rng_key(seed ^ kDrawSalt)
  uint64_t offset;                // params.offset
  unsigned long long* rng_ctr;    // params.offset_counter or NULL
  int bits;
  int64_t* pick;
  unsigned long long* hkey;       // candidate set (all ones = empty)
  uint32_t* hdup;                 // 1: the slot's key occurs more than once among the candidates
  unsigned long long* h2key;      // final picks of resolved suspects (all ones = empty)
  uint32_t* susp;                 // suspect bitmap, bit i % 32 of word i / 32
  StatPartial* parts;
  float clamp_lo, clamp_hi, range_coef;
  SmqSmaqStats* ws_stats;
};

}  // namespace smq
