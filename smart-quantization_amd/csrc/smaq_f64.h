// smaq_f64.h — the fp64 statistics finaliser and element transforms shared by the device kernels
// (fp64.hip) and the host path (cpu_codecs.hip): one definition, so both give the same bytes.
// Reference: smart_compress/compress/smart.py:100-108, 130-182; s2fp8.py:27-48.
#pragma once

#include <float.h>
#include <math.h>

#include "qtorch.h"
#include "smaq_elem.h"
#include "smq_common.h"

namespace smq {

// RN-even fp32 -> fp16 -> fp32 (the host twin of __half2float(__float2half_rn(v)))
__host__ __device__ __forceinline__ float rn16_f32(float v) {
#ifdef __HIP_DEVICE_COMPILE__
  return __half2float(__float2half_rn(v));
#else
  const uint32_t x = f2u(v), s = x & 0x80000000u, ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return v;                          // inf / NaN unchanged
  if (ax >= 0x477ff000u) return u2f(s | 0x7f800000u);        // rounds to inf
  if (ax < 0x38800000u) {                                    // fp16 subnormal grid 2^-24
    const float t = nearbyintf(u2f(ax) * 0x1p24f);
    return u2f(s | f2u(t * 0x1p-24f));
  }
  const uint32_t r = (ax + 0x0fffu + ((ax >> 13) & 1u)) & ~0x1fffu;
  return u2f(s | r);
#endif
}

__host__ __device__ __forceinline__ double median3_f64(double a, double b, double c) {
  return fmax(fmin(a, b), fmin(fmax(a, b), c));
}

// smart.py:100-108, 130-134, 151-154 in fp64 from shifted sums (shift, s1, s2) and extrema.
__host__ __device__ inline void finalize_f64(double s1, double s2, double mn, double mx,
                                             int64_t count, double shift, bool biased,
                                             bool range, double clamp_lo, double clamp_hi,
                                             double range_coef, SmqSmaqStatsF64* out) {
  const double nd = (double)count;
  const double mean = shift + s1 / nd;
  double sd;
  if (range) {
    sd = (mx - mn) * range_coef;  // (data.max() - data.min()) * C
  } else {
    double var = (s2 - s1 * (s1 / nd)) / (biased ? nd : (nd - 1.0));
    if (var < 0.0) var = 0.0;
    sd = sqrt(var);
  }
  const double std_dev = (sd == 0.0) ? 1.0 : sd;  // smart.py:151-152
  double sc = std_dev < clamp_lo ? clamp_lo : std_dev;
  sc = sc > clamp_hi ? clamp_hi : sc;
  out->mean = mean;
  out->std_dev = std_dev;
  out->std_clamped = sc;
  out->raw_std = sd;
  out->min_val = mn;
  out->max_val = mx;
  out->n_used = (uint32_t)(count > 0xffffffffLL ? 0xffffffffu : (uint32_t)count);
  out->reserved0 = 0u;
  out->reserved[0] = out->reserved[1] = 0ull;
}

// ---- element transform (smart.py:144-182 in fp64) -------------------------------------------------
struct ElemF64 {
  double mean, sd, sc;
  double thr, nthr;        // T_m as the Python double: compared with z
  double sthr, snthr;      // fp32(T_m), -fp32(T_m): the scalars tensor's values
  double zh, zl;           // 0 * -fp32(T_m), 0 * fp32(T_m)
  double r_main, r_out;    // fp32 ranges
};

// smart.py:144-169: the code q (an integer-valued double, or +-inf / NaN) and the outlier sides.
template <int RM, bool BN>
__host__ __device__ __forceinline__ double smaq_quant_f64(double v, double u, const ElemF64& c,
                                                          bool& hi, bool& lo, double g, double b) {
  if (BN) v = (v - b) / g;                             // (data - beta) / gamma
  const double z = (v - c.mean) / c.sc;               // (data - mean) / std.clamp(...)
  hi = z > c.thr;
  lo = z < c.nthr;
  const bool o = hi || lo;
  const double a = (hi ? c.snthr : c.zh) + (lo ? c.sthr : c.zl);  // scalars
  const double r = o ? c.r_out : c.r_main;             // ranges
  const double d = (z + a) * r;
  if (RM == kRoundTrunc) return trunc(d);
  const double f = floor(d);                           // _round_stochastic
  const double fr = d - f;
  double t = ((RM == kRoundHash) ? fma(u, -0x1p-24, fr) : (fr - u)) + 0.5;
  t = (t < 0.0) ? 0.0 : t;                             // F.relu
  return f + rint(t);                                  // .round(): half to even
}

// smart.py:171-182: de-quantise q with its sides (the packed codec's decoder shares it).
template <bool BN, bool AP>
__host__ __device__ __forceinline__ double smaq_dequant_f64(double q, bool hi, bool lo,
                                                            const ElemF64& c, double g, double b) {
  const double a = (hi ? c.snthr : c.zh) + (lo ? c.sthr : c.zl);  // scalars
  const double r = (hi || lo) ? c.r_out : c.r_main;    // ranges
  double out = (q / r) - a;
  out = (out * c.sd) + c.mean;
  if (BN) out = (out * g) + b;
  if (AP) out = (out < 0.0) ? 0.0 : out;               // clamp_min(0.0)
  return out;
}

template <int RM, bool BN, bool AP>
__host__ __device__ __forceinline__ double smaq_elem_f64(double v, double u, const ElemF64& c,
                                                         bool& outlier, double g, double b) {
  bool hi, lo;
  const double q = smaq_quant_f64<RM, BN>(v, u, c, hi, lo, g, b);
  outlier = hi || lo;
  return smaq_dequant_f64<BN, AP>(q, hi, lo, c, g, b);
}

__host__ __device__ inline ElemF64 elem_f64_consts(const SmqSmaqStatsF64& st, const SmqSmaqParams& p) {
  ElemF64 c;
  c.mean = st.mean;
  c.sd = st.std_dev;
  c.sc = st.std_clamped;
  c.thr = p.main_std_dev_threshold_f64;
  c.nthr = -c.thr;
  c.sthr = (double)p.main_std_dev_threshold;
  c.snthr = -c.sthr;
  c.zh = (double)(0.0f * -p.main_std_dev_threshold);
  c.zl = (double)(0.0f * p.main_std_dev_threshold);
  c.r_main = (double)p.range_main;
  c.r_out = (double)p.range_outlier;
  return c;
}

__host__ __device__ __forceinline__ double nan_max_f64(double a, double b) {
  return (b > a || b != b) ? b : a;
}
__host__ __device__ __forceinline__ double s2_log_f64(double v) {
  const double a = fabs(v);
  return a == 0.0 ? a : log2(a);  // torch.where(X_abs == 0, X_abs, log2(X_abs))
}

// s2fp8.py:37-43 in fp64 from (sum, max) of the log2 values
__host__ __device__ inline void s2_derive_f64(double s, double m, int64_t n, SmqS2fp8StatsF64* o) {
  const double mu = s / (double)n;
  const double alpha = (1.0 / (m - mu)) * 15.0;  // 15.0 / t = t.reciprocal() * 15.0
  const double beta = (-alpha) * mu;
  const double bp2 = pow(2.0, beta);
  o->mu = mu;
  o->m = m;
  o->alpha = alpha;
  o->beta = beta;
  o->beta_pow2 = bp2;
  o->inv_beta_pow2 = 1.0 / bp2;
  o->inv_alpha = 1.0 / alpha;
  o->n_used = (uint32_t)(n > 0xffffffffLL ? 0xffffffffu : (uint32_t)n);
  o->reserved0 = 0u;
}

// One element of s2fp8.py:45-48 for fp64 data. P16: float_quantize returns half (x.float() in,
// .half() out) and torch runs the inverse in half: the 0-dim fp64 reciprocal enters the product as
// its fp32 value (the half kernel's opmath scalar), the exponent 1/alpha is cast to half.
// out_mode 1 / 2: Y / T (precision 32).
template <bool P16>
__host__ __device__ __forceinline__ double s2_elem_f64(double xv, uint32_t r,
                                                       const SmqS2fp8StatsF64& s, int check_inf,
                                                       float max_value, int out_mode) {
  const double sgn = (xv > 0.0) ? 1.0 : ((xv < 0.0) ? -1.0 : 0.0);
  double Y = pow(fabs(xv), s.alpha);
  Y = Y * s.beta_pow2;
  if (!P16 && out_mode == 1) return Y;
  float T = qtorch_quant((float)Y, r, 5, 2, true);
  if (check_inf && fabsf(T - max_value) <= FLT_EPSILON) T = INFINITY;
  if (!P16) {
    if (out_mode == 2) return (double)T;
    return pow((double)T * s.inv_beta_pow2, s.inv_alpha) * sgn;
  }
  const float T16 = rn16_f32(T);
  const float t1 = rn16_f32(T16 * (float)s.inv_beta_pow2);
  const float e16 = rn16_f32((float)s.inv_alpha);
  // the correctly rounded float power, rounded to half: torch's half pow (powf that is not
  // correctly rounded moves whole E5M2 codes by a half ulp on some draws,
  // tests/golden/f64_s2fp8_p16_powcase)
  const float t2 = rn16_f32((float)pow((double)t1, (double)e16));
  return (double)t2 * sgn;
}

}  // namespace smq
