/*
 * oracle_math.h -- TEST INFRASTRUCTURE ONLY.
 *
 * The oracle is built twice (oracle/Makefile):
 *
 *  liboracle.so           (default)  "faithful": every `x**2` of the reference is
 *                         libm pow(x, 2.0) and sin/cos/log are libm, exactly like
 *                         CPython/numpy on this glibc.  Pinned bit-for-bit against
 *                         the reference's own outputs (tests/golden/).
 *
 *  liboracle_portable.so  (-DORACLE_PORTABLE) squares with `*` and uses the
 *                         portable +,-,*,/-only log/sin/cos below, i.e. the
 *                         arithmetic the HIP kernels use (glibc's pow is not
 *                         correctly rounded: pow(x,2) != x*x for ~0.08% of
 *                         doubles, and it cannot be reproduced on the GPU).  The
 *                         kernels are compared against this build bit-for-bit;
 *                         this build is compared against the faithful one with a
 *                         tolerance (tests/test_oracle_modes.py).
 *
 * The portable functions are an independent restatement of the kernel's
 * (gym-futbol_amd/csrc/futbol_math.hpp); both compile with -ffp-contract=off.
 */
#ifndef ORACLE_MATH_H
#define ORACLE_MATH_H
#include <math.h>
#include <stdint.h>
#include <string.h>

#ifdef ORACLE_PORTABLE

static inline double orc_pm_log(double x)
{
    /* x > 0, finite.  x = m * 2^e, m in [sqrt(1/2), sqrt(2)) */
    uint64_t bits;
    memcpy(&bits, &x, 8);
    int e = (int)((bits >> 52) & 0x7ff) - 1023;
    bits = (bits & 0x000fffffffffffffULL) | 0x3ff0000000000000ULL;
    double m;
    memcpy(&m, &bits, 8);
    if (m > 1.4142135623730951) { m = m * 0.5; e = e + 1; }
    double s = (m - 1.0) / (m + 1.0);
    double s2 = s * s;
    /* 2*atanh(s) = 2s(1 + s^2/3 + s^4/5 + ...), |s| <= 0.1716 */
    double p = 1.0 / 25.0;
    p = p * s2 + 1.0 / 23.0;
    p = p * s2 + 1.0 / 21.0;
    p = p * s2 + 1.0 / 19.0;
    p = p * s2 + 1.0 / 17.0;
    p = p * s2 + 1.0 / 15.0;
    p = p * s2 + 1.0 / 13.0;
    p = p * s2 + 1.0 / 11.0;
    p = p * s2 + 1.0 / 9.0;
    p = p * s2 + 1.0 / 7.0;
    p = p * s2 + 1.0 / 5.0;
    p = p * s2 + 1.0 / 3.0;
    double lm = 2.0 * s + 2.0 * s * (s2 * p);
    const double ln2_hi = 6.93147180369123816490e-01, ln2_lo = 1.90821492927058770002e-10;
    double de = (double)e;
    return (de * ln2_hi + lm) + de * ln2_lo;
}

/* sin and cos of a finite |a| < 1e5 */
static inline void orc_pm_sincos(double a, double *sn, double *cs)
{
    const double inv_pio2 = 6.36619772367581382433e-01;
    const double p1 = 1.57079632673412561417e+00, p2 = 6.07710050630396597660e-11,
                 p3 = 2.02226624879595063154e-21;
    double kq = floor(a * inv_pio2 + 0.5);
    double r = ((a - kq * p1) - kq * p2) - kq * p3;
    double r2 = r * r;
    /* Taylor to r^17 / r^18 on |r| <= pi/4 */
    double s = -1.0 / 355687428096000.0;          /* -1/17! */
    s = s * r2 + 1.0 / 1307674368000.0;            /* 1/15! */
    s = s * r2 - 1.0 / 6227020800.0;               /* -1/13! */
    s = s * r2 + 1.0 / 39916800.0;                 /* 1/11! */
    s = s * r2 - 1.0 / 362880.0;                   /* -1/9! */
    s = s * r2 + 1.0 / 5040.0;                     /* 1/7! */
    s = s * r2 - 1.0 / 120.0;                      /* -1/5! */
    s = s * r2 + 1.0 / 6.0;                        /* 1/3! */
    double sr = r - r * (r2 * s);
    double c = 1.0 / 6402373705728000.0;           /* 1/18! */
    c = c * r2 - 1.0 / 20922789888000.0;           /* -1/16! */
    c = c * r2 + 1.0 / 87178291200.0;              /* 1/14! */
    c = c * r2 - 1.0 / 479001600.0;                /* -1/12! */
    c = c * r2 + 1.0 / 3628800.0;                  /* 1/10! */
    c = c * r2 - 1.0 / 40320.0;                    /* -1/8! */
    c = c * r2 + 1.0 / 720.0;                      /* 1/6! */
    c = c * r2 - 1.0 / 24.0;                       /* -1/4! */
    c = c * r2 + 0.5;                              /* 1/2! */
    double cr = 1.0 - r2 * c;
    long q = (long)kq;
    int qm = (int)(q & 3);
    if (qm == 0) { *sn = sr; *cs = cr; }
    else if (qm == 1) { *sn = cr; *cs = -sr; }
    else if (qm == 2) { *sn = -sr; *cs = -cr; }
    else { *sn = -cr; *cs = sr; }
}

#define ORC_SQ(x) ((x) * (x))
static inline double ORC_LOG(double x) { return orc_pm_log(x); }
static inline double ORC_SIN(double x) { double s, c; orc_pm_sincos(x, &s, &c); return s; }
static inline double ORC_COS(double x) { double s, c; orc_pm_sincos(x, &s, &c); return c; }

#else

#define ORC_SQ(x) pow((x), 2.0)
#define ORC_LOG(x) log(x)
#define ORC_SIN(x) sin(x)
#define ORC_COS(x) cos(x)

#endif
#endif
