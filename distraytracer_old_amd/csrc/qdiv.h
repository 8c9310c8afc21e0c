// Exact (correctly rounded) double division from a precomputed reciprocal; shared by the
// device slab test (trace_device.h) and its host-side exhaustive check (tests/qdiv_check.c).
#pragma once
#include <math.h>
#ifndef QD_FN
#define QD_FN static inline
#endif

// Correctly rounded a / b from y = RN(1/b) (one IEEE division per ray, not per box).
// q0 = RN(a*y) is within 1.5 ulp of a/b; one remainder step (r = a - b*q by FMA) brings
// it within 1 ulp; by Markstein's theorem (y = RN(1/b), q within 1 ulp, no underflow)
// the second step q + r*y rounds to exactly RN(a/b). The no-underflow condition is
// guaranteed by ray_inv's range checks: |b| in [2^-60, 2^60] and every coordinate
// entering a = (box - origin) is 0 or in [2^-200, 2^200], so all exact intermediates are
// multiples of 2^-476 far above the subnormal range. a == 0 gives a zero of possibly the
// other sign, which no slab comparison can tell apart.
QD_FN double qdiv(double a, double b, double y) {
  double q = a * y;
  double r = fma(-b, q, a);
  q = fma(r, y, q);
  r = fma(-b, q, a);
  return fma(r, y, q);
}
// ranges under which qdiv is exact (see above)
QD_FN int qd_range(double b) { return fabs(b) >= 0x1p-60 && fabs(b) <= 0x1p60; }
QD_FN int qc_range(double c) { return c == 0 || (fabs(c) >= 0x1p-200 && fabs(c) <= 0x1p200); }
