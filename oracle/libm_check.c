/*
 * libm_check.c -- TEST INFRASTRUCTURE ONLY.  Pins the glibc sin / cos / pow(x, 2) restatements of
 * oracle_math.h against this host's libm, which is what the
 * reference's math.sin / math.cos / `x**2` call (tests/test_glibc_sincos.py).
 */
#include <math.h>
#include <stdint.h>
#include "oracle_math.h"

/* separate calls through pointers: the compiler must not fuse sin(x), cos(x) into sincos(),
   which glibc implements with different roundings (CPython calls sin and cos separately) */
static double (*volatile libm_sin)(double) = sin;
static double (*volatile libm_cos)(double) = cos;
static double (*volatile libm_pow)(double, double) = pow;

/* n uniform arguments in [lo, hi) (xorshift64, seed); counts of mismatches */
void orc_libm_check(int64_t n, double lo, double hi, uint64_t seed, int64_t *bad_sin, int64_t *bad_cos,
                    int64_t *bad_sq)
{
    uint64_t s = seed | 1u;
    int64_t bs = 0, bc = 0, bq = 0;
    for (int64_t i = 0; i < n; ++i) {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        const double x = lo + (hi - lo) * ((double)(s >> 11) * 0x1p-53);
        bs += libm_sin(x) != orc_glibc_sin(x);
        bc += libm_cos(x) != orc_glibc_cos(x);
        bq += libm_pow(x, 2.0) != orc_glibc_pow2(x);
    }
    *bad_sin = bs;
    *bad_cos = bc;
    *bad_sq = bq;
}
