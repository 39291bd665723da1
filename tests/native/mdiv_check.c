/* Host check of ts_ops.hip's mdiv (test infrastructure): RN(x / n) for integer n from
 * r = RN(1 / n) by q0 = RN(x r), rem = fma(-q0, n, x), q = fma(rem, r, q0), against the IEEE
 * quotient, bit for bit.  n = 1 .. NMAX; x: random doubles over many binades (random 53-bit
 * significands), x near multiples of n (k n +- few ulps: the cases where q0 lands 1-1.5 ulp
 * off), and integers.  Exit status = number of mismatches (0 = pass).
 *   gcc -O2 -ffp-contract=off -o mdiv_check mdiv_check.c -lm && ./mdiv_check [NMAX] [PER_N] */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static uint64_t ubits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

static double mdiv(double x, double n, double r) {
  const double q0 = x * r;
  const uint32_t e = (uint32_t)(ubits(q0) >> 52) & 0x7ffu;
  if (e - 64u > 1958u - 64u) return x / n;
  const double rem = fma(-q0, n, x);
  return fma(rem, r, q0);
}

int main(int argc, char** argv) {
  const int nmax = argc > 1 ? atoi(argv[1]) : 4096;
  const int per = argc > 2 ? atoi(argv[2]) : 20000;
  long bad = 0, tot = 0;
  for (int n = 1; n <= nmax; ++n) {
    const double nd = (double)n, r = 1.0 / nd;
    for (int i = 0; i < per; ++i) {
      double x;
      const int kind = i % 5;
      if (kind == 0) {                          /* random significand and exponent in +-2^60 */
        const uint64_t e = 1023 - 60 + rnd() % 121;
        x = bits((rnd() & 0x800fffffffffffffull) | (e << 52));
      } else if (kind == 1) {                   /* k n +- a few ulps */
        const double k = (double)(rnd() % (1ull << 40)) * (rnd() % 2 ? 1.0 : 1e-9);
        x = k * nd;
        const int64_t off = (int64_t)(rnd() % 9) - 4;
        x = bits(ubits(x) + off);
      } else if (kind == 2) {                   /* integers and halves */
        x = (double)(int64_t)(rnd() % (1ull << 52)) * (rnd() % 2 ? 0.5 : 1.0) * (rnd() % 2 ? -1.0 : 1.0);
      } else if (kind == 3) {                   /* O(1) data with ties to a decimal */
        x = ((double)(rnd() % 2000001) - 1000000.0) / 1000.0;
      } else {                                  /* zeros, infinities, NaN, tiny and huge */
        static const double sp[] = {0.0, -0.0, INFINITY, -INFINITY, NAN, 0x1p-1000, -0x1p-1060, 0x1p-960,
                                    0x1p+1000, -0x1p+1023, 0x1.fffffffffffffp+1023, 4.9e-324};
        x = sp[rnd() % 12] * (rnd() % 2 ? 1.0 : 3.0);
      }
      const double a = mdiv(x, nd, r), b = x / nd;
      ++tot;
      if (ubits(a) != ubits(b) && !(a != a && b != b)) {
        if (bad < 10) fprintf(stderr, "mismatch n=%d x=%.17g: %.17g vs %.17g\n", n, x, a, b);
        ++bad;
      }
    }
  }
  printf("mdiv_check: %ld cases, %ld mismatches\n", tot, bad);
  return bad ? 1 : 0;
}
