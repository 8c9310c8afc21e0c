/* Host check of qdiv (distraytracer_old_amd/csrc/qdiv.h): qdiv(a, b, RN(1/b)) == a / b
   bit for bit on random and adversarial operands inside the documented ranges.
   Build: gcc -O2 -ffp-contract=off -mfma tests/qdiv_check.c -lm  (run by tests/test_qdiv.py) */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../distraytracer_old_amd/csrc/qdiv.h"

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t nx(void) {
  s ^= s << 13; s ^= s >> 7; s ^= s << 17;
  return s;
}
static double u01(void) { return (double)(nx() >> 11) * 0x1p-53; }
static double bits(uint64_t b) { double d; memcpy(&d, &b, 8); return d; }
/* a random double with exponent in [lo, hi] and random significand (or an adversarial one) */
static double rnd(int lo, int hi) {
  int e = lo + (int)(nx() % (uint64_t)(hi - lo + 1));
  uint64_t m = nx() & ((1ull << 52) - 1);
  switch (nx() % 8) {
    case 0: m = (1ull << 52) - 1; break;                  /* 1.111...1 */
    case 1: m = 0; break;                                 /* power of two */
    case 2: m = (1ull << 52) - 1 - (nx() % 16); break;    /* near all ones */
    case 3: m = nx() % 16; break;                         /* near power of two */
    default: break;
  }
  double d = bits(((uint64_t)(e + 1023) << 52) | m);
  return (nx() & 1) ? -d : d;
}

int main(int argc, char** argv) {
  long n = argc > 1 ? atol(argv[1]) : 20000000;
  long bad = 0, tried = 0;
  for (long i = 0; i < n; ++i) {
    double b, c, o;
    int k = (int)(nx() % 4);
    if (k == 0) { b = rnd(-60, 0); c = rnd(-200, 200); o = rnd(-200, 200); }
    else if (k == 1) { b = rnd(-60, 60); c = rnd(-8, 8); o = c + rnd(-60, -1) * c; }  /* cancellation */
    else if (k == 2) { b = (u01() - .5) * 2; c = (u01() - .5) * 200; o = (u01() - .5) * 200; }  /* scene-like */
    else { b = rnd(-30, 2); c = rnd(-200, 200); o = (nx() & 1) ? 0.0 : c; }  /* a == 0 */
    if (!qd_range(b) || !qc_range(c) || !qc_range(o)) continue;
    double a = c - o, y = 1.0 / b;
    double q = qdiv(a, b, y), r = a / b;
    ++tried;
    if (!(q == r) && !(q != q && r != r)) {  /* +0 == -0 allowed: no slab comparison tells them apart */
      if (bad < 10) printf("MISMATCH a=%a b=%a q=%a ref=%a\n", a, b, q, r);
      ++bad;
    }
    /* the approximate slab value (trace_device.h slab_apx): |RN(a*y) - RN(a/b)| <= 2^-51 |RN(a*y)|,
       same sign (the box tests' margins are 2^-46) */
    double t = a * y;
    if (fabs(t - r) > 0x1p-51 * fabs(t) || (t > 0) != (r > 0) || (t < 0) != (r < 0)) {
      if (bad < 10) printf("APPROX a=%a b=%a t=%a ref=%a\n", a, b, t, r);
      ++bad;
    }
  }
  printf("tried %ld mismatches %ld\n", tried, bad);
  return bad ? 1 : 0;
}
