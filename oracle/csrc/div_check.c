/* Exhaustive / randomised check of the division identity libsmq relies on (smaq_elem.h
 * div_by_const): for fp32 a, b with a normal (or zero) fp32 quotient,
 *     (float)((double)a * (1.0 / (double)b)) == a / b     (IEEE RN).
 * Mode "random": N random (a, b) pairs over every exponent; mode "all": every fp32 bit pattern of
 * a against the given divisors.
 * Subnormal quotients (smaq_elem.h quot_check_for): the identity also holds for them unless the
 * divisor is an even integer or >= 2^24. Mode "sub": every a with a subnormal quotient against the
 * given divisors, mismatches counted separately for divisors that need the check; mode "subrand":
 * N random divisors that do not need it, each against random dividends with subnormal quotients.
 * Compile: gcc -O2 -fopenmp -ffp-contract=off div_check.c */
#include <float.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
static uint64_t splitmix(uint64_t* s) {
  uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

/* the rule of smaq_elem.h quot_check_for */
static int quot_check_for(float sc) {
  const float h = sc * 0.5f;
  const int even_int = (h == truncf(h)) && h != 0.0f;
  return (even_int || !(fabsf(sc) < 0x1p24f)) ? 1 : 0;
}

static long check_sub(float a, float b) {
  float ref = a / b;
  if (!(fabsf(ref) < FLT_MIN && ref != 0.0f)) return -1; /* not a subnormal quotient */
  float got = (float)((double)a * (1.0 / (double)b));
  uint32_t x, y;
  memcpy(&x, &ref, 4);
  memcpy(&y, &got, 4);
  return x != y;
}

static long check(float a, float b) {
  float ref = a / b;
  float got = (float)((double)a * (1.0 / (double)b));
  if (fabsf(ref) < FLT_MIN && ref != 0.0f) return 0; /* subnormal results: IEEE fallback path */
  if (isnan(ref) && isnan(got)) return 0;
  uint32_t x, y;
  memcpy(&x, &ref, 4);
  memcpy(&y, &got, 4);
  return x != y;
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "random";
  long bad = 0, total = 0;
  if (!strcmp(mode, "random")) {
    long n = argc > 2 ? atol(argv[2]) : 100000000L;
#pragma omp parallel for reduction(+ : bad, total)
    for (long t = 0; t < n; ++t) {
      uint64_t s = (uint64_t)t * 7919u + 1;
      uint64_t r = splitmix(&s);
      float a = u2f((uint32_t)r), b = u2f((uint32_t)(r >> 32));
      if (isnan(a) || isnan(b) || b == 0.0f) continue;
      bad += check(a, b);
      total++;
    }
  } else if (!strcmp(mode, "sub")) {
    long bad_checked = 0;
    for (int k = 2; k < argc; ++k) {
      float b = strtof(argv[k], NULL);
      const int need = quot_check_for(b);
      long bk = 0, tk = 0;
#pragma omp parallel for reduction(+ : bk, tk)
      for (long u = 0; u < (1L << 32); ++u) {
        long r = check_sub(u2f((uint32_t)u), b);
        if (r < 0) continue;
        bk += r;
        tk++;
      }
      total += tk;
      if (need) bad_checked += bk; else bad += bk;
    }
    printf("{\"mode\": \"sub\", \"checked\": %ld, \"mismatches\": %ld, "
           "\"mismatches_where_checked\": %ld}\n", total, bad, bad_checked);
    return bad != 0;
  } else if (!strcmp(mode, "subrand")) {
    long n = argc > 2 ? atol(argv[2]) : 1000000L;
#pragma omp parallel for reduction(+ : bad, total)
    for (long t = 0; t < n; ++t) {
      uint64_t s = (uint64_t)t * 104729u + 7;
      uint64_t r = splitmix(&s);
      /* divisor: random significand, exponent in [-60, 23] */
      float b = ldexpf(1.0f + (float)(r & 0x7fffff) * 0x1p-23f, (int)((r >> 23) % 84) - 60);
      if (quot_check_for(b)) continue;
      for (int j = 0; j < 64; ++j) {
        uint64_t q = splitmix(&s);
        /* target quotient: random subnormal (and some just above FLT_MIN / near midpoints) */
        double zt = ldexp((double)(q & 0xffffffull) + ((q >> 24) & 1 ? 0.5 : 0.0), -149 - (int)((q >> 25) % 24));
        float a = (float)(zt * (double)b);
        if (q >> 63) a = -a;
        long c = check_sub(a, b);
        if (c < 0) continue;
        bad += c;
        total++;
      }
    }
  } else {
    for (int k = 2; k < argc; ++k) {
      float b = strtof(argv[k], NULL);
#pragma omp parallel for reduction(+ : bad, total)
      for (long u = 0; u < (1L << 32); ++u) {
        float a = u2f((uint32_t)u);
        if (isnan(a)) continue;
        bad += check(a, b);
        total++;
      }
    }
  }
  printf("{\"mode\": \"%s\", \"checked\": %ld, \"mismatches\": %ld}\n", mode, total, bad);
  return bad != 0;
}
