/* gs_fp.h — float64 counter steps shared by the engine's kernels and the
 * tests.
 *
 * The reference bumps its float64 counters one message at a time
 * (`x += 1`: markFirstMessageDelivery / markDuplicateMessageDelivery
 * score.go:915-928, 960-963, invalid deliveries :808-810, the peer gater's
 * counters peer_gater.go:390-440).  For a fractional, decayed x,
 * (x + 1) + 1 != x + 2 in general, so n steps are n roundings — but only the
 * steps that cross a power of two can round: inside a binade [2^(e-1), 2^e)
 * with e <= 52 every integer step is exact.  gs_add_ones takes the steps of
 * one binade in one exact add and the crossing step alone, so n steps cost
 * O(number of binades crossed) instead of O(n), with the identical result.
 */
#ifndef GS_FP_H
#define GS_FP_H

#include <math.h>
#include <stdint.h>

#include "gs_rng.h" /* GS_HD */

/* x + 1 + 1 + ... (n steps, each rounded as `x += 1` is). */
GS_HD double gs_add_ones(double x, int64_t n) {
  while (n > 0) {
    if (!(x >= 1.0) || !(x < 4503599627370496.0)) { /* below 1 or at / above 2^52: one step at a time */
      x += 1.0;
      --n;
      continue;
    }
    int e;
    (void)frexp(x, &e);                /* x in [2^(e-1), 2^e) */
    const double top = ldexp(1.0, e);
    const double room = top - x;       /* exact (Sterbenz: top / 2 <= x <= top) */
    int64_t m = (int64_t)ceil(room) - 1; /* the largest m with x + m < top */
    if (m <= 0) {                      /* the next step crosses 2^e: it may round */
      x += 1.0;
      --n;
      continue;
    }
    if (m > n) m = n;
    x += (double)m;                    /* exact: x + m stays in the binade */
    n -= m;
  }
  return x;
}

/* "+1, cap" n times (stop at the first step above cap, which becomes cap):
 * the values only grow, so that is min over the uncapped result. */
GS_HD double gs_add_ones_capped(double x, int64_t n, double cap) {
  if (n <= 0) return x;
  const double y = gs_add_ones(x, n);
  return y > cap ? cap : y;
}

#endif /* GS_FP_H */
