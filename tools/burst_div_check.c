/* Exhaustive check (host, gcc -O2 -ffp-contract=off ... -lm): for every uint16 u,
 * fma(fma(-q, 358.4, u), inv, q) with q = u * inv, inv = 1/358.4, equals u / 358.4
 * (the comb burst level, comb-ntsc.cxx:560; csrc/comb.hip burst_level). */
#include <stdio.h>
#include <math.h>
int main(void) {
  const double d = 358.4, inv = 1.0 / 358.4;
  int bad = 0;
  for (int u = 0; u < 65536; u++) {
    volatile double x = (double)u;
    double ref = x / d;
    double q = x * inv;
    double r = fma(-q, d, x);
    double q2 = fma(r, inv, q);
    if (q2 != ref) { if (bad < 5) printf("u=%d ref=%.17g q2=%.17g\n", u, ref, q2); bad++; }
  }
  printf("bad %d of 65536\n", bad);
  return 0;
}
