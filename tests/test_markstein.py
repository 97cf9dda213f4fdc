"""The what-if class path's BalancedAllocation fractions (k_whatif_cls1,
csrc/engine.hip) divide without a division per pair: with y = RN(1/b) computed
once per node, q = RN(a*y), r = a - b*q (exact, one FMA) and RN(q + r*y) is the
correctly rounded a/b (Markstein's correction) — Go's float64 division
(balanced_allocation.go: requested / allocatable).  This checks the identity on
the CPU (C, libm fma) over the domain the host admits to that kernel (cpu /
memory below 2^45, requests below 2^46), at random and at the edges."""
import os
import subprocess
import tempfile

import pytest

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
static uint64_t s = 0x9E3779B97F4A7C15ull;
static inline uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static long bad = 0;
static void check(int64_t a, int64_t b) {
  const double A = (double)a, B = (double)b, y = 1.0 / B, q = A * y;
  const double m = fma(fma(-B, q, A), y, q);
  if (m != A / B) { if (bad < 4) printf("a=%lld b=%lld\n", (long long)a, (long long)b); ++bad; }
}
int main(int argc, char** argv) {
  const long n = atol(argv[1]);
  for (int64_t b = 1; b < 2000; ++b)
    for (int64_t a = 0; a <= 2 * b; ++a) check(a, b);
  for (int e = 0; e < 46; ++e) {
    const int64_t b = (int64_t)1 << e;
    check(b - 1, b); check(b, b); check(b + 1, b); check(1, b); check(((int64_t)1 << 46) - 1, b);
    if (b > 1) { check(b, b - 1); check(b - 2, b - 1); }
  }
  for (long i = 0; i < n; ++i) {
    const int bb = 1 + (int)(xr() % 45), ba = 1 + (int)(xr() % 46);
    const int64_t b = (int64_t)(xr() & (((uint64_t)1 << bb) - 1)) + 1;
    int64_t a = (int64_t)(xr() & (((uint64_t)1 << ba) - 1));
    if (i & 1) a = b - (int64_t)(xr() % (uint64_t)b);
    check(a, b);
  }
  printf("bad %ld\n", bad);
  return bad != 0;
}
"""


def test_markstein_division_is_correctly_rounded():
    with tempfile.TemporaryDirectory() as d:
        src, exe = os.path.join(d, "m.c"), os.path.join(d, "m")
        open(src, "w").write(SRC)
        try:
            subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", exe, src, "-lm"])
        except (OSError, subprocess.CalledProcessError):
            pytest.skip("no C compiler")
        out = subprocess.run([exe, "20000000"], capture_output=True, text=True, timeout=300)
        assert out.returncode == 0, out.stdout
        assert out.stdout.strip().endswith("bad 0"), out.stdout
