/* Exhaustive check of the fp32-reciprocal quotient for half-type z-scores (smaq_elem.h
 * half_quot): for fp16 / bf16 values dm (any bit pattern) and sc (any positive finite value),
 *     RN_T((float)(dm * r32)) == RN_T(dm / sc),   r32 = RN32(1 / sc)  (the host-rounded reciprocal),
 * where RN_T rounds to the half type. The reference value comes from the fp64 quotient (correctly
 * rounded), then RN_T: double rounding is innocuous at 53 >= 2 * 11 + 2 bits.
 * Pairs whose fp32 product lies below the type's smallest normal (|dm * r32| < 2^-14 for fp16,
 * 2^-126 for bf16) are excluded: exact midpoints of the coarse subnormal grid occur there, and the
 * kernel sends those quotients through the exact fp64 path.
 * Prints the number of mismatching (sc, dm) pairs and the first few; exit status 1 if any.
 *
 * qr mode (test infrastructure; restates smaq_elem.h quot_split_compute for the dequant's q / range,
 * smart.py:171 `data / ranges`): with half inputs and no BN term the z-score is a half value, so
 * the codes q are known from the flags alone: per z-score (all 65,536 bit patterns) the class
 * (z > RN_T(T), z < -RN_T(T)), d = RN32(RN32(z + a) * r) and q in {floor(d) + 0, 1, 2} (stochastic
 * rounding, any draw: smart.py:93-98 adds rint(relu(fr - u + 0.5)), 2 when fr + 0.5 rounds up to
 * 1.5; d = +-inf gives NaN) or {trunc(d)}. For every such q it checks
 *     fmaf(q, h, RN32(q * l)) == RN32(q / r),   h = RN32(1 / r), l = RN32(1 / r - h),
 * the right side from the fp64 quotient (innocuous double rounding: 53 >= 2 * 24 + 2).
 *   ./half_div_check qr f16|bf16 T r_main r_out sr   one flag set: "ok h_m l_m h_o l_o"
 *   ./half_div_check qr-sweep                        a grid of SmaQ flag sets: how many pass
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

static float rn_half_f(int bf, float v) { return (float)(bf ? rnbf16((double)v) : rn16((double)v)); }

/* 1 when every reachable code passes; out = {h_m, l_m, h_o, l_o} */
static int qr_check(int bf, float T, float r_main, float r_out, int sr, float* out) {
  const float hm = (float)(1.0 / (double)r_main), lm = (float)(1.0 / (double)r_main - (double)hm);
  const float ho = (float)(1.0 / (double)r_out), lo = (float)(1.0 / (double)r_out - (double)ho);
  out[0] = hm; out[1] = lm; out[2] = ho; out[3] = lo;
  if (!isfinite(r_main) || !isfinite(r_out) || !isfinite(hm) || !isfinite(ho)) return 0;
  const float cthr = rn_half_f(bf, T), cnthr = -cthr, nthr = -T;
  const float zh = 0.0f * nthr, zl = 0.0f * T;
  for (int b = 0; b < 0x10000; ++b) {
    const float z = bf ? bf2f((uint16_t)b) : h2f((uint16_t)b);
    const int hi = z > cthr, lw = z < cnthr, o = hi || lw;
    const float a = (hi ? nthr : zh) + (lw ? T : zl);
    const float r = o ? r_out : r_main;
    const float d = (z + a) * r;
    float q[3];
    int nq = 1;
    if (sr) {  /* f + rint(relu(RN(fr - u) + 0.5)): 0, 1, or 2 when RN(fr + 0.5) ties up to 1.5 */
      if (isinf(d)) continue;  /* fr = inf - inf: q is NaN */
      q[0] = floorf(d); q[1] = q[0] + 1.0f; q[2] = q[0] + 2.0f; nq = 3;
    } else {
      q[0] = truncf(d);
    }
    for (int i = 0; i < nq; ++i) {
      const float want = (float)((double)q[i] / (double)r);
      const float got = fmaf(q[i], o ? ho : hm, q[i] * (o ? lo : lm));
      if (!(f2u(want) == f2u(got) || (want != want && got != got))) {
        if (getenv("QR_VERBOSE"))
          fprintf(stderr, "z=%a q=%a r=%a want=%a got=%a\n", z, q[i], r, want, got);
        return 0;
      }
    }
  }
  return 1;
}

static int qr_main(int argc, char** argv) {
  float out[4];
  if (strcmp(argv[1], "qr") == 0) {
    if (argc < 7) return 2;
    const int ok = qr_check(strcmp(argv[2], "bf16") == 0, strtof(argv[3], 0), strtof(argv[4], 0),
                            strtof(argv[5], 0), atoi(argv[6]), out);
    printf("%d %a %a %a %a\n", ok, out[0], out[1], out[2], out[3]);
    return 0;
  }
  /* qr-sweep: num_bits 3..16, thresholds on a grid; ranges as smart.py:75-80 computes them (fp64)
   * then rounded to fp32 (the library's float parameters) */
  static const double Tm[] = {0.5, 1.0, 1.5, 2.0, 2.5, 3.0, 4.0};
  static const double To_add[] = {0.5, 1.0, 2.0, 3.0, 5.0, 7.0};
  long sets = 0, ok = 0, sr_sets = 0, sr_ok = 0;
  for (int bf = 0; bf < 2; ++bf)
    for (int sr = 0; sr < 2; ++sr)
      for (int bm = 3; bm <= 16; ++bm)
        for (int bo = bm; bo <= 16; ++bo)
          for (unsigned i = 0; i < sizeof Tm / sizeof *Tm; ++i)
            for (unsigned j = 0; j < sizeof To_add / sizeof *To_add; ++j) {
              const double To = Tm[i] + To_add[j];
              const float rm = (float)((ldexp(1.0, bm - 2) - 1.0) / Tm[i]);
              const float ro = (float)((ldexp(1.0, bo - 2) - 1.0) / (To - Tm[i]));
              const int r = qr_check(bf, (float)Tm[i], rm, ro, sr, out);
              ++sets;
              ok += r;
              sr_sets += sr;
              sr_ok += sr && r;
              if (!r && sr && sr_sets - sr_ok <= 8)
                printf("fails: %s sr=%d bm=%d bo=%d Tm=%g To=%g\n", bf ? "bf16" : "f16", sr, bm,
                       bo, Tm[i], To);
            }
  printf("qr-sweep: %ld flag sets, %ld pass; stochastic rounding: %ld sets, %ld pass\n", sets, ok,
         sr_sets, sr_ok);
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && strncmp(argv[1], "qr", 2) == 0) return qr_main(argc, argv);
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
