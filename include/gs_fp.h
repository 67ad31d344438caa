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

/* floor(2^64 / q) for q >= 2 (else 0): the reciprocal gs_quantum_div uses. */
GS_HD uint64_t gs_quantum_magic(int64_t q) {
  return q >= 2 ? (uint64_t)(((unsigned __int128)1 << 64) / (uint64_t)q) : 0;
}
/* meshTime / TimeInMeshQuantum (score.go:273: Go int64 division, truncating)
 * without a 64-bit divide: the high half of mt * magic is floor(mt / q) or one
 * below it, and the remainder fixes it up.  Negative operands take the plain
 * division (meshTime is never negative). */
GS_HD int64_t gs_quantum_div(int64_t mt, int64_t q, uint64_t magic) {
  if (q == 1) return mt;
  if (magic == 0 || mt < 0) return mt / q;
#if defined(__HIP_DEVICE_COMPILE__)
  uint64_t d = __umul64hi((uint64_t)mt, magic);
#else
  uint64_t d = (uint64_t)(((unsigned __int128)(uint64_t)mt * magic) >> 64);
#endif
  uint64_t r = (uint64_t)mt - d * (uint64_t)q;
  if (r >= (uint64_t)q) { ++d; r -= (uint64_t)q; }
  if (r >= (uint64_t)q) ++d;
  return (int64_t)d;
}

#endif /* GS_FP_H */
