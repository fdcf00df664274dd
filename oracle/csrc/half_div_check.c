/* Exhaustive check of the fp32-reciprocal quotient for half-type z-scores (smaq_elem.h
 * half_quot): for fp16 / bf16 values dm (any bit pattern) and sc (any positive finite value),
 *     RN_T((float)(dm * r32)) == RN_T(dm / sc),   r32 = RN32(1 / sc)  (the host-rounded reciprocal),
 * where RN_T rounds to the half type. The reference value comes from the fp64 quotient (correctly
 * rounded), then RN_T: double rounding is innocuous at 53 >= 2 * 11 + 2 bits.
 * Pairs whose fp32 product lies below the type's smallest normal (|dm * r32| < 2^-14 for fp16,
 * 2^-126 for bf16) are excluded: exact midpoints of the coarse subnormal grid occur there, and the
 * kernel sends those quotients through the exact fp64 path.
 * Prints the number of mismatching (sc, dm) pairs and the first few; exit status 1 if any.
 * Compile: gcc -O2 -fopenmp -ffp-contract=off half_div_check.c -o half_div_check -lm
 * Run: ./half_div_check f16 | bf16 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }

static float h2f(uint16_t h) {
  const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
  if (e == 0x1fu) return u2f(s | 0x7f800000u | (m << 13));
  if (e == 0) return m ? (s ? -1.0f : 1.0f) * (float)m * 0x1p-24f : u2f(s);
  return u2f(s | ((e + 112u) << 23) | (m << 13));
}
/* RN-even to fp16 from double (exact handling of the whole range) */
static double rn16(double v) {
  if (v != v || isinf(v)) return v;
  const double a = fabs(v);
  if (a >= 65520.0) return copysign(INFINITY, v);
  int e;
  frexp(a, &e);                 /* a = m * 2^e, m in [0.5, 1) */
  int q = e - 11;               /* ulp exponent for 11 significant bits */
  if (q < -24) q = -24;         /* subnormal grid 2^-24 */
  const double s = ldexp(1.0, q);
  return copysign(nearbyint(a / s) * s, v);
}
static double rnbf16(double v) {
  if (v != v || isinf(v)) return v;
  const double a = fabs(v);
  int e;
  frexp(a, &e);
  int q = e - 8;
  if (q < -133) q = -133;       /* bf16 subnormal grid 2^-133 */
  const double s = ldexp(1.0, q);
  const double r = nearbyint(a / s) * s;
  if (r > 0x1.fep127) return copysign(INFINITY, v); /* beyond the bf16 maximum: inf */
  return copysign(r, v);
}
static float bf2f(uint16_t h) { return u2f((uint32_t)h << 16); }

int main(int argc, char** argv) {
  const int bf = argc > 1 && strcmp(argv[1], "bf16") == 0;
  long long bad = 0, checked = 0;
#pragma omp parallel for schedule(dynamic, 64) reduction(+ : bad, checked)
  for (int s = 1; s < 0x7c00 + (bf ? 0x7f80 - 0x7c00 : 0); ++s) {
    const float sc = bf ? bf2f((uint16_t)s) : h2f((uint16_t)s);
    if (!(sc > 0.0f) || isinf(sc)) continue;
    const float r32 = (float)(1.0 / (double)sc);
    if (isinf(r32)) continue; /* sc below 2^-128 (under the clamp's 1e-38): exact path */
    for (int d = 0; d < 0x10000; ++d) {
      const float dm = bf ? bf2f((uint16_t)d) : h2f((uint16_t)d);
      if (dm != dm || isinf(dm)) continue;
      const float p = dm * r32;
      if (p != 0.0f && fabsf(p) < (bf ? 0x1p-126f : 0x1p-14f)) continue; /* exact path */
      const double want = bf ? rnbf16((double)dm / (double)sc) : rn16((double)dm / (double)sc);
      const double got = bf ? rnbf16((double)p) : rn16((double)p);
      ++checked;
      if (!(want == got || (want != want && got != got)) || signbit(want) != signbit(got)) {
#pragma omp critical
        {
          if (bad < 8) printf("mismatch sc=%a dm=%a want=%a got=%a\n", sc, dm, want, got);
        }
        ++bad;
      }
    }
  }
  printf("%s: %lld pairs checked, %lld mismatches\n", bf ? "bf16" : "f16", checked, bad);
  return bad ? 1 : 0;
}
