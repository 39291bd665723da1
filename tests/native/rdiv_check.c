/* Host check of fmx_common.hpp's rdiv (test infrastructure): RN(x / b) for a general
 * divisor b from r = RN(1 / b) -- q0 = RN(x r), rem = fma(-q0, b, x), q = fma(rem, r, q0)
 * (Markstein's correction: y within 1/2 ulp of 1/b and q0 within 1 ulp of x/b give the
 * correctly rounded quotient) -- against the IEEE quotient, bit for bit, with rdiv's range
 * guards (b outside [2^-800, 2^800], x below 2^-895, q0 outside [2^-959, 2^936], zeros and
 * non-finite values take the IEEE divide).  Divisors: random significands over many
 * binades, z-score-like standard deviations, integers; numerators: random, near multiples
 * of b (q0 off by ~1 ulp), O(1) data with decimal ties, specials.  Exit status 0 = pass.
 *   gcc -O2 -ffp-contract=off -o rdiv_check rdiv_check.c -lm && ./rdiv_check [NB] [PER_B] */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static uint64_t s = 0x2545F4914F6CDD1Dull;
static uint64_t rnd(void) { s ^= s << 13; s ^= s >> 7; s ^= s << 17; return s; }
static double bits(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static uint64_t ubits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }

static int rdiv_ok(double b) {
  const uint32_t e = (uint32_t)(ubits(b) >> 52) & 0x7ffu;
  return e - (1023u - 800u) <= 1600u;
}
static double rdiv(double x, double b, double r, int b_ok) {
  const double q0 = x * r;
  const uint32_t eq = (uint32_t)(ubits(q0) >> 52) & 0x7ffu, ex = (uint32_t)(ubits(x) >> 52) & 0x7ffu;
  if (!b_ok || eq - 64u > 1958u - 64u || ex < 128u) return x / b;
  const double rem = fma(-q0, b, x);
  return fma(rem, r, q0);
}

int main(int argc, char** argv) {
  const int nb = argc > 1 ? atoi(argv[1]) : 20000;
  const int per = argc > 2 ? atoi(argv[2]) : 4000;
  long bad = 0, tot = 0;
  for (int j = 0; j < nb; ++j) {
    double b;
    const int bk = j % 4;
    if (bk == 0) {                              /* random significand, exponent in +-60 */
      const uint64_t e = 1023 - 60 + rnd() % 121;
      b = bits((rnd() & 0x000fffffffffffffull) | (e << 52));
    } else if (bk == 1) {                       /* standard deviations of O(1) data */
      b = 0.5 + (double)(rnd() >> 11) * 0x1p-53 * 1.5;
    } else if (bk == 2) {                       /* integers */
      b = (double)(1 + rnd() % 100000);
    } else {                                    /* wide binades, incl. the guard edges */
      const uint64_t e = 1 + rnd() % 2046;
      b = bits((rnd() & 0x800fffffffffffffull) | (e << 52));
    }
    const double r = 1.0 / b;
    const int ok = rdiv_ok(b);
    for (int i = 0; i < per; ++i) {
      double x;
      const int kind = i % 5;
      if (kind == 0) {
        const uint64_t e = 1023 - 60 + rnd() % 121;
        x = bits((rnd() & 0x800fffffffffffffull) | (e << 52));
      } else if (kind == 1) {                   /* k b +- a few ulps */
        const double k = (double)(rnd() % (1ull << 40)) * (rnd() % 2 ? 1.0 : 1e-9);
        x = bits(ubits(k * b) + (int64_t)(rnd() % 9) - 4);
      } else if (kind == 2) {                   /* x - mean of O(1) data */
        x = ((double)(rnd() % 2000001) - 1000000.0) / 1000.0 - 0.0123456789;
      } else if (kind == 3) {                   /* any binade */
        const uint64_t e = rnd() % 2047;
        x = bits((rnd() & 0x800fffffffffffffull) | (e << 52));
      } else {
        static const double sp[] = {0.0, -0.0, INFINITY, -INFINITY, NAN, 0x1p-1000, -0x1p-1060, 0x1p-960,
                                    0x1p+1000, -0x1p+1023, 0x1.fffffffffffffp+1023, 4.9e-324};
        x = sp[rnd() % 12] * (rnd() % 2 ? 1.0 : 3.0);
      }
      const double a = rdiv(x, b, r, ok), c = x / b;
      ++tot;
      if (ubits(a) != ubits(c) && !(a != a && c != c)) {
        if (bad < 10) fprintf(stderr, "mismatch b=%a x=%a: %a vs %a\n", b, x, a, c);
        ++bad;
      }
    }
  }
  printf("rdiv_check: %ld cases, %ld mismatches\n", tot, bad);
  return bad ? 1 : 0;
}
