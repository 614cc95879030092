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
 *                         correctly rounded double-double sin/cos below, i.e. the
 *                         arithmetic the HIP kernels use (glibc's pow is not
 *                         correctly rounded: pow(x,2) != x*x for ~0.08% of
 *                         doubles, and neither are its sin/cos; neither can be
 *                         reproduced on the GPU).  The
 *                         kernels are compared against this build bit-for-bit;
 *                         this build is compared against the faithful one with a
 *                         tolerance (tests/test_oracle_modes.py).
 *
 * The tape's normal draw uses the +,-,*,/-only orc_pm_log / orc_pm_sincos in BOTH
 * builds (and in tests/rng_tape.py): it is part of the tape contract.
 *
 * The portable functions are an independent restatement of the kernel's
 * (gym-futbol_amd/csrc/futbol_math.hpp); both compile with -ffp-contract=off.
 */
#ifndef ORACLE_MATH_H
#define ORACLE_MATH_H
#include <math.h>
#include <stdint.h>
#include <string.h>

/* ---- tape functions: the normal draw of the RNG tape is
 * DEFINED with these +,-,*,/-only functions in every implementation (Python tape,
 * both oracle builds, HIP), so a tape draw is the same double everywhere. */

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

/* ---- correctly rounded sin/cos (double-double, error < 2^-100 relative on
 * |a| < 1e5) for the reference's own math.sin/math.cos (screw_vec,
 * envs/futbol_env.py:107-108).  glibc 2.35's sin/cos are NOT correctly rounded
 * (measured: 0.2% / 0.1% of angles in the shot range differ by 1 ulp from the
 * exact value); correctly rounded is the platform-independent target. */
typedef struct { double h, l; } orc_dd;
static inline orc_dd orc_two_sum(double a, double b) { double s = a + b, bb = s - a; orc_dd r = { s, (a - (s - bb)) + (b - bb) }; return r; }
static inline orc_dd orc_fast2(double a, double b) { double s = a + b; orc_dd r = { s, b - (s - a) }; return r; }
static inline orc_dd orc_dd_mul(orc_dd x, orc_dd y)
{
    double p = x.h * y.h, e = fma(x.h, y.h, -p);
    e = e + (x.h * y.l + x.l * y.h);
    return orc_fast2(p, e);
}
static inline orc_dd orc_dd_add(orc_dd x, orc_dd y)
{
    orc_dd s = orc_two_sum(x.h, y.h);
    return orc_fast2(s.h, s.l + (x.l + y.l));
}

/* sin tail: sum_{n=11..29 odd} (-1)^((n-1)/2) r^(n-11) / n!  (Horner, highest first) */
static const double ORC_CR_STAIL[10] = { 0x1.259f98b4358adp-103, -0x1.d1ab1c2dccea3p-94, 0x1.3f3ccdd165fa9p-84, -0x1.761b41316381ap-75, 0x1.71b8ef6dcf572p-66, -0x1.2f49b46814157p-57, 0x1.952c77030ad4ap-49, -0x1.ae7f3e733b81fp-41, 0x1.6124613a86d09p-33, -0x1.ae64567f544e4p-26 };
static const double ORC_CR_CTAIL[9] = { 0x1.0a18a2635085dp-98, -0x1.88e85fc6a4e5ap-89, 0x1.f2cf01972f578p-80, -0x1.0ce396db7f853p-70, 0x1.e542ba4020225p-62, -0x1.6827863b97d97p-53, 0x1.ae7f3e733b81fp-45, -0x1.93974a8c07c9dp-37, 0x1.1eed8eff8d898p-29 };
static const double ORC_CR_SHEAD[4][2] = { { 0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73 }, { -0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73 }, { 0x1.1111111111111p-7, 0x1.1111111111111p-63 }, { -0x1.5555555555555p-3, -0x1.5555555555555p-57 } };
static const double ORC_CR_CHEAD[5][2] = { { -0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76 }, { 0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76 }, { -0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65 }, { 0x1.5555555555555p-5, 0x1.5555555555555p-59 }, { -0x1.0000000000000p-1, 0x0.0p+0 } };

static inline void orc_cr_sincos(double a, double *sn, double *cs)
{
    /* pi/2 = P1 + P2 + P3 + P4 (P1, P2 with <= 32 significant bits: k*P1, k*P2 exact) */
    const double kq = floor(a * 6.36619772367581382433e-01 + 0.5);
    orc_dd r = orc_two_sum(a, -(kq * 1.57079632673412561417e+00));
    orc_dd t2 = { -(kq * 6.07710050630396597660e-11), 0.0 };
    r = orc_dd_add(r, t2);
    const double t = kq * 2.02226624879595063154e-21;
    orc_dd t3 = { -t, -(fma(kq, 2.02226624879595063154e-21, -t) + kq * 1.0085854035872483e-37) };
    r = orc_dd_add(r, t3);
    const orc_dd r2 = orc_dd_mul(r, r);
    /* tails (n >= 11 / n >= 12) in double, heads in double-double */
    double ps = ORC_CR_STAIL[0], pc = ORC_CR_CTAIL[0];
    for (int i = 1; i < 10; ++i) ps = ps * r2.h + ORC_CR_STAIL[i];
    for (int i = 1; i < 9; ++i) pc = pc * r2.h + ORC_CR_CTAIL[i];
    orc_dd s = { ps, 0.0 }, c = { pc, 0.0 };
    for (int i = 0; i < 4; ++i) { orc_dd k = { ORC_CR_SHEAD[i][0], ORC_CR_SHEAD[i][1] }; s = orc_dd_add(orc_dd_mul(s, r2), k); }
    for (int i = 0; i < 5; ++i) { orc_dd k = { ORC_CR_CHEAD[i][0], ORC_CR_CHEAD[i][1] }; c = orc_dd_add(orc_dd_mul(c, r2), k); }
    s = orc_dd_add(r, orc_dd_mul(r, orc_dd_mul(s, r2)));   /* r + r^3 (-1/6 + ...) */
    orc_dd one = { 1.0, 0.0 };
    c = orc_dd_add(one, orc_dd_mul(c, r2));                 /* 1 + r^2 (-1/2 + ...) */
    const int q = (int)((long long)kq & 3);
    if (q == 0) { *sn = s.h; *cs = c.h; }
    else if (q == 1) { *sn = c.h; *cs = -s.h; }
    else if (q == 2) { *sn = -s.h; *cs = -c.h; }
    else { *sn = -c.h; *cs = s.h; }
}

#ifdef ORACLE_PORTABLE
#define ORC_SQ(x) ((x) * (x))
static inline double ORC_SIN(double x) { double s, c; orc_cr_sincos(x, &s, &c); return s; }
static inline double ORC_COS(double x) { double s, c; orc_cr_sincos(x, &s, &c); return c; }
#else
#define ORC_SQ(x) pow((x), 2.0)
#define ORC_SIN(x) sin(x)
#define ORC_COS(x) cos(x)
#endif

/* the tape's normal draw -- identical in both builds */
static inline double orc_tape_z(double u1, double u2)
{
    double s, c;
    orc_pm_sincos(6.283185307179586 * u2, &s, &c);
    return sqrt(-2.0 * orc_pm_log(1.0 - u1)) * c;
}
#endif
