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
 *  liboracle_portable.so  (-DORACLE_PORTABLE) the arithmetic the HIP kernels use,
 *                         written without calls into the host libm: glibc's
 *                         pow(x, 2.0) and sin / cos restated operation for
 *                         operation (orc_glibc_pow2 / orc_glibc_sin / _cos below:
 *                         glibc's pow is not correctly rounded -- pow(x,2) != x*x
 *                         for ~0.08% of doubles -- and neither are its sin/cos) for
 *                         every v0 square and sin/cos and for the envs_v1 squares
 *                         that feed the state; only the envs_v1 reward's squares
 *                         are x*x (ORC_SQ_V1).  The kernels are compared against
 *                         this build bit-for-bit; this build against the faithful
 *                         one in tests/test_oracle_modes.py (observations
 *                         bit-identical; reward bits differ by <= 2.3e-13).
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

/* ---- glibc 2.35 sin / cos, restated (the reference's math.sin / math.cos in screw_vec,
 * envs/futbol_env.py:109-110, run glibc's; CPython calls libm directly).  The IBM Accurate
 * Mathematical Library algorithm of sysdeps/ieee754/dbl-64/s_sin.c (do_sin, do_cos, TAYLOR_SIN,
 * reduce_sincos, do_sincos) as compiled into the variant glibc selects on x86-64 hosts with FMA and
 * AVX2 (__sin_fma / __cos_fma, the one this image's CPUs run): every a*b+c the compiler fused is
 * an fma() here, in the same association.  Table: glibc's __sincostab (futbol_sincostab.h,
 * scripts/gen_sincostab.py).  Valid for |x| < 105414350 (the __branred range is never reached by
 * screw_vec's angles, |x| < 4.5); pinned against the host libm by tests/test_glibc_sincos.py. */
#include "../gym-futbol_amd/csrc/futbol_sincostab.h"
static const double ORC_SINCOSTAB[440] = { FUTBOL_SINCOSTAB_ROWS };
#define ORC_G_BIG 0x1.8p45
#define ORC_G_SN3 (-0x1.5555555555515p-3)
#define ORC_G_SN5 0x1.11110e829872fp-7
#define ORC_G_CS2 0x1.0p-1
#define ORC_G_CS4 (-0x1.5555555555535p-5)
#define ORC_G_CS6 0x1.6c16bedd9e239p-10
#define ORC_G_S1 (-0x1.5555555555555p-3)
#define ORC_G_S2 0x1.1111111110ecep-7
#define ORC_G_S3 (-0x1.a01a019db08b8p-13)
#define ORC_G_S4 0x1.71de27b9a7ed9p-19
#define ORC_G_S5 (-0x1.addffc2fcdf59p-26)
#define ORC_G_HP0 0x1.921fb54442d18p0
#define ORC_G_HP1 0x1.1a62633145c07p-54
#define ORC_G_HPINV 0x1.45f306dc9c883p-1
#define ORC_G_TOINT 0x1.8p52
#define ORC_G_MP1 0x1.921fb58p0
#define ORC_G_MP2 (-0x1.dde973cp-27)
#define ORC_G_PP3 (-0x1.cb3b398p-55)
#define ORC_G_PP4 (-0x1.d747f23e32ed7p-83)

static inline int orc_g_index(double u)
{
    uint64_t b;
    memcpy(&b, &u, 8);
    return (int)((uint32_t)b << 2);
}
static inline uint32_t orc_g_hi(double x)
{
    uint64_t b;
    memcpy(&b, &x, 8);
    return (uint32_t)(b >> 32) & 0x7fffffffu;
}
/* do_sin (x, dx), TAYLOR_SIN below |x| = 0.126 */
static inline double orc_g_do_sin(double x, double dx)
{
    if (fabs(x) < 0.126) {
        const double xx = x * x;
        double p = fma(xx, ORC_G_S5, ORC_G_S4);
        p = fma(xx, p, ORC_G_S3);
        p = fma(xx, p, ORC_G_S2);
        p = fma(xx, p, ORC_G_S1);
        return x + fma(xx, fma(p, x, -(0.5 * dx)), dx);
    }
    if (x <= 0) dx = -dx;
    const double ax = fabs(x);
    const double u = ax + ORC_G_BIG;
    const double xr = ax - (u - ORC_G_BIG);
    const int k = orc_g_index(u);
    const double *T = ORC_SINCOSTAB + k;
    const double xx = xr * xr;
    const double s = xr + fma(xr * xx, fma(xx, ORC_G_SN5, ORC_G_SN3), dx);
    const double c = fma(xr, dx, xx * fma(xx, fma(xx, ORC_G_CS6, ORC_G_CS4), ORC_G_CS2));
    const double cor = fma(s, T[2], fma(-c, T[0], fma(s, T[3], T[1])));
    return copysign(T[0] + cor, x);
}
/* do_cos (x, dx) */
static inline double orc_g_do_cos(double x, double dx)
{
    if (x < 0) dx = -dx;
    const double ax = fabs(x);
    const double u = ax + ORC_G_BIG;
    const double xr = (ax - (u - ORC_G_BIG)) + dx;
    const int k = orc_g_index(u);
    const double *T = ORC_SINCOSTAB + k;
    const double xx = xr * xr;
    const double s = fma(xr * xx, fma(xx, ORC_G_SN5, ORC_G_SN3), xr);
    const double c = xx * fma(xx, fma(xx, ORC_G_CS6, ORC_G_CS4), ORC_G_CS2);
    const double cor = fma(-s, T[0], fma(-c, T[2], fma(-s, T[1], T[3])));
    return T[2] + cor;
}
/* reduce_sincos: x = n pi/2 + a + da */
static inline int orc_g_reduce(double x, double *a, double *da)
{
    const double t = fma(x, ORC_G_HPINV, ORC_G_TOINT);
    const double xn = t - ORC_G_TOINT;
    uint64_t tb;
    memcpy(&tb, &t, 8);
    double y = fma(-xn, ORC_G_MP1, x);
    y = fma(-xn, ORC_G_MP2, y);
    const double t2 = fma(-xn, ORC_G_PP3, y);
    const double db = fma(-xn, ORC_G_PP3, y - t2);
    const double b = fma(-xn, ORC_G_PP4, t2);
    *da = db + fma(-xn, ORC_G_PP4, t2 - b);
    *a = b;
    return (int)(tb & 3);
}
static inline double orc_g_do_sincos(double a, double da, int n)
{
    const double r = (n & 1) ? orc_g_do_cos(a, da) : orc_g_do_sin(a, da);
    return (n & 2) ? -r : r;
}
static inline double orc_glibc_sin(double x)
{
    const uint32_t k = orc_g_hi(x);
    if (k < 0x3e500000u) return x;
    if (k < 0x3feb6000u) return orc_g_do_sin(x, 0.0);
    if (k < 0x400368fdu) return copysign(orc_g_do_cos(ORC_G_HP0 - fabs(x), ORC_G_HP1), x);
    if (k < 0x419921fbu) {
        double a, da;
        const int n = orc_g_reduce(x, &a, &da);
        return orc_g_do_sincos(a, da, n);
    }
    double s, c;  /* outside screw_vec's range: correctly rounded instead of __branred */
    orc_cr_sincos(x, &s, &c);
    return s;
}
static inline double orc_glibc_cos(double x)
{
    const uint32_t k = orc_g_hi(x);
    if (k < 0x3e400000u) return 1.0;
    if (k < 0x3feb6000u) return orc_g_do_cos(x, 0.0);
    if (k < 0x400368fdu) {
        const double y = ORC_G_HP0 - fabs(x);
        const double a = y + ORC_G_HP1;
        const double da = (y - a) + ORC_G_HP1;
        return orc_g_do_sin(a, da);
    }
    if (k < 0x419921fbu) {
        double a, da;
        const int n = orc_g_reduce(x, &a, &da);
        return orc_g_do_sincos(a, da, n + 1);
    }
    double s, c;
    orc_cr_sincos(x, &s, &c);
    return c;
}

/* ---- glibc 2.35 pow(x, 2.0), restated: the reference's `x**2` (CPython float and numpy float64
 * powers call libm pow).  glibc's pow is exp(y log x) in double-double (ARM optimized-routines
 * algorithm, sysdeps/ieee754/dbl-64/e_pow.c; the __pow_fma build with its fused multiply-adds as
 * fma() here), NOT x*x: the two differ on ~0.08% of arguments.  Main path only (x normal and
 * x^2 within [2^-738, 2^738]; elsewhere x*x -- squares of the envs' coordinates never leave it).
 * Tables: futbol_powtab.h (scripts/gen_powtab.py). */
#include "../gym-futbol_amd/csrc/futbol_powtab.h"
static const double ORC_POW_LOG[128 * 3] = { FUTBOL_POW_LOG_ROWS };
static const uint64_t ORC_POW_EXP[256] = { FUTBOL_POW_EXP_ROWS };
static inline double orc_asd(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }
static inline uint64_t orc_asu(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
static inline double orc_glibc_pow2(double x)
{
    const double Y = 2.0;
    uint64_t ix = orc_asu(x) & 0x7fffffffffffffffULL;   /* y even: pow(-x, 2) = pow(x, 2) */
    const uint32_t topx = (uint32_t)(ix >> 52);
    if (topx == 0 || topx >= 0x7ff || topx < 0x3ff - 369 || topx > 0x3ff + 369) return x * x;
    /* log_inline */
    const uint64_t tmp = ix - 0x3fe6955500000000ULL;
    const int i = (int)((tmp >> 45) & 127);
    const int64_t k = (int64_t)tmp >> 52;
    const double z = orc_asd(ix - (tmp & 0xfff0000000000000ULL));
    const double kd = (double)k;
    const double invc = ORC_POW_LOG[3 * i], logc = ORC_POW_LOG[3 * i + 1], logctail = ORC_POW_LOG[3 * i + 2];
    const double r = fma(z, invc, -1.0);
    const double t1 = fma(kd, 0x1.62e42fefa3800p-1, logc);
    const double t2 = t1 + r;
    const double lo1 = fma(kd, 0x1.ef35793c76730p-45, logctail);
    const double lo2 = (t1 - t2) + r;
    const double ar = r * -0x1.0p-1;
    const double ar2 = r * ar, ar3 = r * ar2;
    const double hi = t2 + ar2;
    const double lo3 = fma(ar, r, -ar2);
    const double lo4 = (t2 - hi) + ar2;
    const double q = fma(ar2, fma(ar2, fma(r, 0x1.0002b8b263fc3p+0, -0x1.2495b9b4845e9p+0),
                                  fma(r, -0x1.555555529a47ap-1, 0x1.999999959554ep-1)),
                         fma(r, 0x1.0000000000006p-1, -0x1.5555555555560p-1));
    const double lo = fma(ar3, q, ((lo1 + lo2) + lo3) + lo4);
    const double ly = hi + lo;
    const double ltail = (hi - ly) + lo;
    /* y * log x */
    const double ehi = Y * ly;
    const double elo = fma(Y, ltail, fma(ly, Y, -ehi));
    /* exp_inline (sign_bias 0) */
    const uint32_t abstop = (uint32_t)(orc_asu(ehi) >> 52) & 0x7ff;
    if (abstop < 0x3c9) return 1.0 + ehi;                      /* |ehi| < 2^-54 */
    if (abstop >= 0x408) return x * x;                         /* outside the squares' range */
    double kx = fma(ehi, 0x1.71547652b82fep+7, 0x1.8p52);
    const uint64_t ki = orc_asu(kx);
    kx = kx - 0x1.8p52;
    double rr = fma(kx, -0x1.62e42fefa0000p-8, ehi);
    rr = fma(kx, -0x1.cf79abc9e3b3ap-47, rr);
    rr = elo + rr;
    const int idx = 2 * (int)(ki & 127);
    const uint64_t top = ki << 45;
    const double tail = orc_asd(ORC_POW_EXP[idx]);
    const double scale = orc_asd(ORC_POW_EXP[idx + 1] + top);
    const double r2 = rr * rr;
    const double t = fma(r2 * r2, fma(rr, 0x1.1111167a4d017p-7, 0x1.55555cf172b91p-5),
                         fma(fma(rr, 0x1.555555555543cp-3, 0x1.ffffffffffdbdp-2), r2, tail + rr));
    return fma(t, scale, scale);
}

#ifdef ORACLE_PORTABLE
/* the kernels' arithmetic: the glibc pow(x, 2.0) and sin / cos restatements above for v0 (the
 * reference-pinned path) and for envs_v1's squares that feed the state (_process_action's get_vec,
 * pymunk's Vec2d.length in limit_velocity: futbol_v1_oracle.c SQS); the envs_v1 reward's squares
 * (get_vec, _ball_to_team_distance_arr) stay x*x in the kernels -- a deliberate, measured
 * difference from Python's pow in the reward's last bits only */
#define ORC_SQ(x) orc_glibc_pow2(x)
#define ORC_SQ_V1(x) ((x) * (x))
#define ORC_SIN(x) orc_glibc_sin(x)
#define ORC_COS(x) orc_glibc_cos(x)
#else
#define ORC_SQ(x) pow((x), 2.0)
#define ORC_SQ_V1(x) pow((x), 2.0)
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
