/*
 * cdiv_check.c -- TEST INFRASTRUCTURE ONLY.  Evidence for the step kernels' division by a
 * constant (csrc/futbol_v1_impl.hpp `cdiv`): q0 = RN(x * rc), r = fma(-q0, c, x) (exact),
 * q = copysign(fma(r, rc, q0), x), rc = RN(1 / c), compared bit for bit with the IEEE quotient RN(x / c)
 * that the reference (CPython float division) computes.  The GPU's v_fma_f64 / v_mul_f64 are
 * the same correctly rounded IEEE operations as C's fma() and *, so agreement here is
 * agreement there.  Samples: random doubles over a wide exponent range, plus x chosen so that
 * x / c lies within a few ulps of a rounding midpoint (the cases a reciprocal-based division
 * gets wrong first).
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

static uint64_t sm64(uint64_t *s)
{
    uint64_t z = (*s += 0x9e3779b97f4a7c15ull);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}

static double cdiv(double x, double c, double rc)
{
    const double q0 = x * rc;
    const double r = fma(-q0, c, x);
    return copysign(fma(r, rc, q0), x);
}

static int same(double a, double b)
{
    uint64_t ua, ub;
    memcpy(&ua, &a, 8);
    memcpy(&ub, &b, 8);
    return ua == ub;
}

/* number of mismatches over n random + n near-midpoint samples; exponents of x in
 * [-emax, emax] around 1 (the kernels divide positions, velocities, impulses and dot products) */
long long orc_cdiv_check(double c, long long n, uint64_t seed, int emax)
{
    const double rc = 1.0 / c;
    long long bad = 0;
    uint64_t s = seed;
    /* signed zeros: the quotient keeps x's sign */
    if (!same(cdiv(0.0, c, rc), 0.0 / c)) ++bad;
    if (!same(cdiv(-0.0, c, rc), -0.0 / c)) ++bad;
    for (long long k = 0; k < n; ++k) {
        /* random sign, exponent, mantissa */
        uint64_t u = sm64(&s);
        int ex = (int)(sm64(&s) % (uint64_t)(2 * emax + 1)) - emax;
        double m = 1.0 + (double)(u >> 12) * 0x1p-52;
        double x = ldexp((u & 1) ? -m : m, ex);
        if (!same(cdiv(x, c, rc), x / c)) ++bad;
        /* near a midpoint: q on the grid, x = RN(c * (q + half ulp of q + t ulps)), t small */
        uint64_t v = sm64(&s);
        double q = ldexp(1.0 + (double)(v >> 12) * 0x1p-52, ex);
        double ulp = nextafter(q, INFINITY) - q;
        int t = (int)(sm64(&s) % 9) - 4;
        double xm = c * (q + 0.5 * ulp + (double)t * ldexp(ulp, -52));
        if (!same(cdiv(xm, c, rc), xm / c)) ++bad;
        if (!same(cdiv(-xm, c, rc), -xm / c)) ++bad;
    }
    return bad;
}

/* control for the checker: the uncorrected reciprocal product x * RN(1/c), which is NOT always
 * the correctly rounded quotient -- the sampler must find its failures */
long long orc_mul_check(double c, long long n, uint64_t seed, int emax)
{
    const double rc = 1.0 / c;
    long long bad = 0;
    uint64_t s = seed;
    for (long long k = 0; k < n; ++k) {
        uint64_t u = sm64(&s);
        int ex = (int)(sm64(&s) % (uint64_t)(2 * emax + 1)) - emax;
        double m = 1.0 + (double)(u >> 12) * 0x1p-52;
        double x = ldexp((u & 1) ? -m : m, ex);
        if (!same(x * rc, x / c)) ++bad;
    }
    return bad;
}
