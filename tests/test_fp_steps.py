"""include/gs_fp.h: gs_add_ones / gs_add_ones_capped (the engine's +1-step
counter updates, one exact add per binade) equal the reference's one-step-at-
a-time `x += 1` bit for bit (CPU: compiled with g++ against a serial loop on
decayed fractional counters, binade crossings, caps, large n)."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SRC = r"""
#include <cstdio>
#include <cstring>
#include <random>
#include "gs_fp.h"
static double serial(double x, long long n) { for (long long i = 0; i < n; ++i) x += 1.0; return x; }
static double serial_cap(double x, long long n, double cap) {
  for (long long i = 0; i < n; ++i) { x += 1.0; if (x > cap) { x = cap; break; } }
  return x;
}
int main() {
  std::mt19937_64 g(7);
  std::uniform_real_distribution<double> u(0.0, 1.0);
  long long bad = 0, cases = 0;
  for (int it = 0; it < 400000; ++it) {
    double x;
    switch (it % 5) {
      case 0: x = u(g); break;                                   // [0, 1)
      case 1: x = u(g) * 300.0; break;                           // decayed counters
      case 2: x = (double)(1ll << (g() % 40)) - u(g) * 4.0; break;  // just below a power of two
      case 3: x = u(g) * 1e15; break;                            // large magnitudes
      default: { double d = u(g) * 50.0; for (int k = 0; k < (int)(g() % 30); ++k) d *= 0.9; x = d; }
    }
    if (x < 0) x = 0;
    const long long n = (long long)(g() % (it % 7 == 0 ? 5000 : 300));
    const double cap = u(g) * 400.0;
    const double a = serial(x, n), b = gs_add_ones(x, n);
    const double c = serial_cap(x, n, cap), e = gs_add_ones_capped(x, n, cap);
    if (std::memcmp(&a, &b, 8) || std::memcmp(&c, &e, 8)) ++bad;
    ++cases;
  }
  std::printf("%lld %lld\n", cases, bad);
  return 0;
}
"""


def test_add_ones_equals_serial_steps(tmp_path):
    src = tmp_path / "fp.cpp"
    src.write_text(SRC)
    exe = tmp_path / "fp"
    try:
        subprocess.run(["g++", "-O2", "-ffp-contract=off", "-I", os.path.join(REPO, "include"), str(src), "-o",
                        str(exe)], check=True, capture_output=True, timeout=120)
    except FileNotFoundError:
        pytest.skip("g++ not available")
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=300).stdout.split()
    cases, bad = int(out[0]), int(out[1])
    assert cases == 400000 and bad == 0


QSRC = r"""
#include <cstdio>
#include <random>
#include "gs_fp.h"
int main() {
  std::mt19937_64 g(11);
  long long bad = 0, cases = 0;
  const long long qs[] = {1, 2, 3, 7, 1000, 1000000000LL, 1000000007LL, 60000000000LL, (1LL << 40) + 3,
                          (1LL << 62) + 1, 9223372036854775807LL};
  for (long long q : qs)
    for (int it = 0; it < 200000; ++it) {
      long long mt;
      switch (it % 4) {
        case 0: mt = (long long)(g() >> 1); break;                 // any int64 >= 0
        case 1: mt = (long long)(g() % 100000000000000ULL); break; // hours of ns
        case 2: mt = (long long)(g() % 1000) * q + (long long)(g() % 3) - 1; break;  // around multiples
        default: mt = (long long)(g() % 4096); break;
      }
      if (mt < 0) mt = 0;
      const long long want = mt / q, got = gs_quantum_div(mt, q, gs_quantum_magic(q));
      bad += want != got;
      ++cases;
    }
  std::printf("%lld %lld\n", cases, bad);
  return 0;
}
"""


def test_quantum_div_equals_integer_division(tmp_path):
    """gs_quantum_div (the engine's meshTime / TimeInMeshQuantum, score.go:273)
    equals Go's int64 division on 2.2M cases: quanta from 1 to 2^63 - 1,
    times anywhere in [0, 2^63) and right around the multiples of q."""
    src = tmp_path / "q.cpp"
    src.write_text(QSRC)
    exe = tmp_path / "q"
    subprocess.run(["g++", "-O2", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True,
                   capture_output=True, timeout=120)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True, timeout=300).stdout.split()
    assert int(out[0]) == 11 * 200000 and int(out[1]) == 0
