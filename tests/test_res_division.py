"""The resource flows' constant divisions (resources.hip div_const): x / c for
c = sqrt(2) (a diagonal flow, cResourceCount.cc FlowMatter's / dist) and c = 3
(the gravity terms) computed as y = RN(x r), e = fma(-c, y, x),
RN(fma(e, r, y)) with r = RN(1 / c) -- Markstein's correction -- must equal
the IEEE quotient the oracle computes, bit for bit, including signed zeros.
A C restatement of the device sequence (C fma is correctly rounded) against
C division over random quotients of resource-like and arbitrary magnitudes."""
import subprocess

SRC = r"""
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
static uint64_t s = 88172645463325252ull;
static uint64_t xr(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double divc(double x, double c, double r) {
  double ax = fabs(x);
  if (ax == 0.0) return x * r;
  if (!(ax >= 0x1p-900 && ax <= 0x1p+900)) return x / c;
  double y = x * r;
  double e = fma(-c, y, x);
  return fma(e, r, y);
}
int main(void) {
  const double cs[2] = {1.4142135623730951, 3.0};
  long bad = 0, n = 0;
  for (int k = 0; k < 2; k++) {
    const double c = cs[k], r = 1.0 / c;
    const double edge[6] = {0.0, -0.0, 0x1p-900, -0x1p-901, 0x1p+900, 1e-310};
    for (int i = 0; i < 6; i++) {
      double q1 = edge[i] / c, q2 = divc(edge[i], c, r);
      n++; if (memcmp(&q1, &q2, 8)) bad++;
    }
    for (long i = 0; i < 20000000L; i++) {
      uint64_t b = xr();
      double x;
      if (i & 1) {
        b = (b & 0x800FFFFFFFFFFFFFull) | ((uint64_t)(1023 - 60 + (xr() % 120)) << 52);
        memcpy(&x, &b, 8);
      } else {
        x = ((double)(b >> 11) * 0x1p-53) * ldexp(1.0, (int)(xr() % 80) - 40);
      }
      double q1 = x / c, q2 = divc(x, c, r);
      n++;
      if (memcmp(&q1, &q2, 8)) bad++;
    }
  }
  printf("%ld %ld\n", n, bad);
  return bad != 0;
}
"""


def test_constant_division_is_correctly_rounded(tmp_path):
    src = tmp_path / "divc.c"
    src.write_text(SRC)
    exe = tmp_path / "divc"
    subprocess.check_call(["gcc", "-O2", "-ffp-contract=off", "-o", str(exe), str(src), "-lm"])
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    n, bad = map(int, out.stdout.split())
    assert n > 4e7 and bad == 0, out.stdout
