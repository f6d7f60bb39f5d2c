/* Host restatement of the device back substitution's division (tpl_kernels.hip div_rn /
 * k_ftk_inv): q0 = RN(a y), q = RN(q0 + RN(a - b q0) y) with y = RN(1 / b) — Markstein's
 * correction — must give the IEEE quotient's bits whenever a, b and q lie in
 * [2^-900, 2^901) in magnitude (exp_in_range), and +-0 = RN(a y) for a = +-0. Checks N
 * random pairs over wide exponents, near-exact quotients and quotients at binade
 * boundaries; prints "OK (0 failures)". Test infrastructure (tests/test_native.py). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 88172645463325252ULL;
static uint64_t nx(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double mk(int emin, int emax) {
  uint64_t bits = ((uint64_t)(emin + (int)(nx() % (uint64_t)(emax - emin + 1)) + 1023) << 52) |
                  (nx() & 0xFFFFFFFFFFFFFULL);
  if (nx() & 1) bits |= 1ULL << 63;
  double d;
  memcpy(&d, &bits, 8);
  return d;
}
static double nudge(double v, int k) {
  uint64_t u;
  memcpy(&u, &v, 8);
  u += (uint64_t)(int64_t)k;
  memcpy(&v, &u, 8);
  return v;
}
static int in_range(double v) {  /* the device's exp_in_range */
  uint64_t u;
  memcpy(&u, &v, 8);
  const unsigned e = (unsigned)(u >> 52) & 0x7FFu;
  return e - (1023u - 900u) <= 1800u;
}
int main(int argc, char** argv) {
  const long N = argc > 1 ? atol(argv[1]) : 20000000;
  long fails = 0, checked = 0;
  for (long i = 0; i < N; ++i) {
    double a, b;
    switch (i % 5) {
      case 0: a = mk(-60, 60); b = mk(-60, 60); break;
      case 1: a = mk(-900, 900); b = mk(-900, 900); break;
      case 2: b = mk(-30, 30); a = nudge(mk(-30, 30) * b, (int)(nx() % 5) - 2); break;
      case 3: b = mk(-30, 30); a = nudge(ldexp(1.0, (int)(nx() % 60) - 30) * b, (int)(nx() % 9) - 4); break;
      default: b = mk(-30, 30); a = (nx() & 1) ? 0.0 : -0.0; break;
    }
    const double y = 1.0 / b;
    const double q0 = a * y;
    const double q = a == 0.0 ? q0 : fma(fma(-b, q0, a), y, q0);
    if (!(in_range(b) && (a == 0.0 || (in_range(a) && in_range(q))))) continue;  /* IEEE path */
    ++checked;
    const double ref = a / b;
    if (memcmp(&q, &ref, 8) != 0) {
      if (fails < 5) printf("a=%a b=%a q=%a ref=%a\n", a, b, q, ref);
      ++fails;
    }
  }
  printf("checked %ld of %ld\n", checked, N);
  if (fails) { printf("FAILED (%ld failures)\n", fails); return 1; }
  printf("OK (0 failures)\n");
  return 0;
}
