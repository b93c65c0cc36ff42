// Portable natural logarithm for the KL score, identical bits on host and gfx950.
//
// The reference takes glibc's log() of the determinant ratio
// (core_legacy/src/kullback_leibler.c:115).  The device libm log and glibc's
// log disagree in the last bit on some inputs, and the KL ordering that picks
// the pruned NDs is sensitive to single-ulp changes.  So the HIP
// path and the CPU oracle share this implementation: only IEEE +,-,*,/, fma and
// bit casts, evaluated in double-double (error ~2^-70 relative), then rounded
// once -- i.e. correctly rounded except in vanishingly rare cases.  glibc's log
// is itself within 0.52 ulp, so the two agree on all but ~1% of inputs, by one
// ulp (tests/test_log.py measures this).
//
// Callers define NDNET_FN (e.g. `__device__ static inline`) and NDNET_TABQ
// (e.g. `__constant__`) before including; both default to host inline.
#pragma once
#include <stdint.h>
#include <string.h>
#ifndef NDNET_FN
#define NDNET_FN static inline
#endif
#include "ndt_log_table.h"

#ifdef __HIP_DEVICE_COMPILE__
#define NDNET_FMA(a, b, c) __builtin_fma((a), (b), (c))
#else
#include <math.h>
#define NDNET_FMA(a, b, c) fma((a), (b), (c))
#endif

NDNET_FN uint64_t ndnet_dbits(double x) {
  uint64_t u;
  memcpy(&u, &x, 8);
  return u;
}
NDNET_FN double ndnet_bitsd(uint64_t u) {
  double x;
  memcpy(&x, &u, 8);
  return x;
}

// s + err == a + b exactly
NDNET_FN void ndnet_two_sum(double a, double b, double* s, double* err) {
  double t = a + b;
  double bp = t - a;
  double ap = t - bp;
  *err = (a - ap) + (b - bp);
  *s = t;
}

NDNET_FN double ndnet_log(double x) {
  uint64_t u = ndnet_dbits(x);
  if (x != x) return x;                                  // NaN propagates
  if (x == 0.0) return ndnet_bitsd(0xfff0000000000000ull);  // -inf
  if (u >> 63) return ndnet_bitsd(0xfff8000000000000ull);   // negative -> NaN (glibc: -nan)
  if (u == 0x7ff0000000000000ull) return x;             // +inf
  int e = (int)((u >> 52) & 0x7ff);
  if (e == 0) {  // subnormal: scale into the normal range
    x = x * 0x1p54;
    u = ndnet_dbits(x);
    e = (int)((u >> 52) & 0x7ff) - 54;
  }
  e -= 1023;
  uint64_t mant = u & 0x000fffffffffffffull;
  // t in [sqrt(1/2), sqrt(2)]
  if (mant > 0x6a09e667f3bcdull) {
    mant |= 0x3fe0000000000000ull;
    e += 1;
  } else {
    mant |= 0x3ff0000000000000ull;
  }
  double t = ndnet_bitsd(mant);
  int idx = (int)(t * 128.0 + 0.5);
  const double inv_c = ndnet_log_tab[idx - NDNET_LOG_TAB_LO][0];
  const double T_hi = ndnet_log_tab[idx - NDNET_LOG_TAB_LO][1];
  const double T_lo = ndnet_log_tab[idx - NDNET_LOG_TAB_LO][2];
  // r = t*inv_c - 1 exactly, as r_hi + r_lo
  double p_hi = t * inv_c;
  double p_lo = NDNET_FMA(t, inv_c, -p_hi);
  double r_hi, r_lo;
  ndnet_two_sum(p_hi - 1.0, p_lo, &r_hi, &r_lo);
  // r^2 as s_hi + s_lo
  double s_hi = r_hi * r_hi;
  double s_lo = NDNET_FMA(r_hi, r_hi, -s_hi) + 2.0 * r_hi * r_lo;
  // log1p tail from the cubic term on: r^3 (1/3 - r/4 + r^2/5 - ...)
  double q = 1.0 / 12.0;
  q = 1.0 / 11.0 - r_hi * q;
  q = 1.0 / 10.0 - r_hi * q;
  q = 1.0 / 9.0 - r_hi * q;
  q = 1.0 / 8.0 - r_hi * q;
  q = 1.0 / 7.0 - r_hi * q;
  q = 1.0 / 6.0 - r_hi * q;
  q = 1.0 / 5.0 - r_hi * q;
  q = 1.0 / 4.0 - r_hi * q;
  q = 1.0 / 3.0 - r_hi * q;
  double tail = (r_hi * s_hi) * q;
  const double fe = (double)e;
  double S, e1, e2, e3;
  ndnet_two_sum(fe * NDNET_LN2_HI, T_hi, &S, &e1);
  ndnet_two_sum(S, r_hi, &S, &e2);
  ndnet_two_sum(S, -0.5 * s_hi, &S, &e3);
  double lo = ((((((e1 + e2) + e3) + fe * NDNET_LN2_LO) + T_lo) + r_lo) - 0.5 * s_lo) + tail;
  return S + lo;
}
