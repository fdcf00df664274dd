/* Exhaustive / randomised check of the division identity libsmq relies on (smaq_elem.h
 * div_by_const): for fp32 a, b with a normal (or zero) fp32 quotient,
 *     (float)((double)a * (1.0 / (double)b)) == a / b     (IEEE RN).
 * Mode "random": N random (a, b) pairs over every exponent; mode "all": every fp32 bit pattern of
 * a against the given divisors. Compile: gcc -O2 -fopenmp -ffp-contract=off div_check.c */
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
