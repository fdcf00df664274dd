/* Test infrastructure (not product code): checks on the host that the round-3 form of the S2FP8
 * fast forward's quantiser (repo:smart-quantization_amd/csrc/float_quant.hip s2_fwd_fast_lg) gives
 * the same E5M2 code as the round-2 form it replaced, for every fp32 Y the fast path can produce
 * (+0 .. +inf, and the default NaN 0x7fc00000 of 0 * inf: alpha is finite and positive there and
 * 2^beta in [0, inf], and a NaN log2|x| takes the accurate path instead) and a set of random words
 * r, and the same low 21 bits for the uncertainty test; and that s2_sign_finite equals torch.sign
 * for every finite x. (NaN payloads from 0x7fe00001 up differ: t + r wraps into the sign bit in the round-2 form;
 * the fast path never sees them.) Both forms restate qtorch's E5M2 stochastic rounding
 * (round_bitwise, clip_exponent, the subnormal path through + 2^-14) followed by check_inf
 * (+57344 -> +inf), as oracle/qtorch_float.py does.
 *
 *   gcc -O2 -fopenmp -ffp-contract=off oracle/csrc/s2_clip_check.c -o s2_clip_check
 *   ./s2_clip_check <stride> <n_words>     (stride 1: every pattern up to +inf)
 * prints {"checked": N, "mismatches": M}.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t u_of(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

/* round 2: clip by the exponent field, sign-carrying subnormal shift, check_inf last */
static uint32_t old_form(uint32_t t, uint32_t r, int check_inf) {
  const uint32_t rm = r & 0x1fffffu;
  uint32_t qn = (t + rm) & 0xffe00000u;
  qn = ((qn >> 23) & 0xffu) > 142u ? ((t & 0x80000000u) | 0x47600000u) : qn;
  const float sh = f_of(0x38800000u | (t & 0x80000000u));
  const float vs = f_of(t) + sh;
  const float qs = f_of((u_of(vs) + rm) & 0xffe00000u) - sh;
  const int sub = (t & 0x7f800000u) < 0x38800000u;
  uint32_t T = sub ? u_of(qs) : qn;
  if (check_inf) T = (T == 0x47600000u) ? 0x7f800000u : T;
  return T;
}

/* round 3: one unsigned compare for clip + check_inf, constant shift, t < bits(2^-14), one sum
 * for both paths; the code is bits 21..31 (the low bits are unspecified) */
static uint32_t new_form(uint32_t t, uint32_t r, int check_inf) {
  const uint32_t vsb = u_of(f_of(t) + 0x1p-14f);
  const int sub = t < 0x38800000u;
  const uint32_t sum = (sub ? vsb : t) + (r & 0x1fffffu);
  const float qs = f_of(sum & 0xffe00000u) - 0x1p-14f;
  const uint32_t clip = check_inf ? 0x7f800000u : 0x47600000u;
  return sub ? u_of(qs) : (sum >= 0x47600000u ? clip : sum);
}

/* the uncertainty test's 21 low bits: (v + rm) & (2^21 - 1) with v = Y or Y + 2^-14 (round 2) */
static uint32_t old_low(uint32_t t, uint32_t r) {
  const uint32_t vsb = u_of(f_of(t) + f_of(0x38800000u | (t & 0x80000000u)));
  const uint32_t vb = ((t & 0x7f800000u) < 0x38800000u) ? vsb : t;
  return (vb + (r & 0x1fffffu)) & 0x1fffffu;
}
static uint32_t new_low(uint32_t t, uint32_t r) {
  const uint32_t vsb = u_of(f_of(t) + 0x1p-14f);
  return ((t < 0x38800000u ? vsb : t) + (r & 0x1fffffu)) & 0x1fffffu;
}

/* torch.sign and its fast-path form (float_quant.hip s2_sign_finite) for finite x */
static float sign_ref(float x) { return (x > 0.0f) ? 1.0f : ((x < 0.0f) ? -1.0f : 0.0f); }
static float sign_fast(float x) {
  const float s = fmaf(x * 0x1p127f, 0x1p127f, 0.0f);
  return fmaxf(-1.0f, fminf(s, 1.0f)); /* v_med3_f32(s, -1, 1) for a non-NaN s */
}

static uint32_t mix(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}

int main(int argc, char** argv) {
  const uint64_t stride = argc > 1 ? strtoull(argv[1], 0, 10) : 1;
  const int nw = argc > 2 ? atoi(argv[2]) : 4;
  uint64_t checked = 0, bad = 0;
  const int64_t n_t = (int64_t)(0x7f800000ull / stride) + 2;  /* + inf and the default NaN */
#pragma omp parallel for reduction(+ : checked, bad) schedule(static)
  for (int64_t i = 0; i < n_t; ++i) {
    const uint32_t t = i == n_t - 1 ? 0x7fc00000u
                       : (i == n_t - 2 ? 0x7f800000u : (uint32_t)((uint64_t)i * stride));
    for (int w = 0; w < nw; ++w) {
      /* the extreme words (0, all ones) and hashed ones */
      const uint32_t r = w == 0 ? 0u : (w == 1 ? 0xffffffffu : mix(t ^ (uint32_t)w * 0x9e3779b9u));
      for (int ci = 0; ci < 2; ++ci) {
        ++checked;
        if ((old_form(t, r, ci) >> 21) != (new_form(t, r, ci) >> 21) || old_low(t, r) != new_low(t, r))
          ++bad;
      }
    }
  }
  /* every finite x (both signs): the sign factor's bits */
#pragma omp parallel for reduction(+ : checked, bad) schedule(static)
  for (int64_t i = 0; i < (int64_t)(0x100000000ull / stride); ++i) {
    const uint32_t xb = (uint32_t)((uint64_t)i * stride);
    if ((xb & 0x7f800000u) == 0x7f800000u) continue; /* inf / NaN: not on the fast path */
    ++checked;
    if (u_of(sign_ref(f_of(xb))) != u_of(sign_fast(f_of(xb)))) ++bad;
  }
  printf("{\"checked\": %llu, \"mismatches\": %llu}\n", (unsigned long long)checked,
         (unsigned long long)bad);
  return 0;
}
