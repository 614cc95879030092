// futbol_math.hpp -- reproducible elementary functions for the env kernels.
//
// The kernels are compiled with -ffp-contract=off and use only correctly
// rounded IEEE operations (+ - * / sqrt), so every result is a pure function
// of the inputs, identical on gfx950 and on a CPU.  log/sin/cos (only needed
// by v0's noisy shot, envs/futbol_env.py:101-116, and by Box-Muller) are
// therefore written here with + - * / only, instead of calling ocml, whose
// last-bit behaviour differs from glibc's.  Accuracy: a few ulp.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

namespace futbol {

__host__ __device__ inline double pm_log(double x)
{
    // x = m * 2^e with m in [sqrt(1/2), sqrt(2)); log m = 2 atanh((m-1)/(m+1))
    uint64_t bits;
    memcpy(&bits, &x, 8);
    int e = (int)((bits >> 52) & 0x7ff) - 1023;
    bits = (bits & 0x000fffffffffffffull) | 0x3ff0000000000000ull;
    double m;
    memcpy(&m, &bits, 8);
    if (m > 1.4142135623730951) {
        m = m * 0.5;
        e = e + 1;
    }
    const double s = (m - 1.0) / (m + 1.0);
    const double s2 = s * s;
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
    const double lm = 2.0 * s + 2.0 * s * (s2 * p);
    const double de = (double)e;
    return (de * 6.93147180369123816490e-01 + lm) + de * 1.90821492927058770002e-10;
}

__host__ __device__ inline void pm_sincos(double a, double* sn, double* cs)
{
    // Cody-Waite reduction by pi/2 (three-part constant), Taylor on |r| <= pi/4
    const double kq = floor(a * 6.36619772367581382433e-01 + 0.5);
    const double r = ((a - kq * 1.57079632673412561417e+00) - kq * 6.07710050630396597660e-11) -
                     kq * 2.02226624879595063154e-21;
    const double r2 = r * r;
    double s = -1.0 / 355687428096000.0;
    s = s * r2 + 1.0 / 1307674368000.0;
    s = s * r2 - 1.0 / 6227020800.0;
    s = s * r2 + 1.0 / 39916800.0;
    s = s * r2 - 1.0 / 362880.0;
    s = s * r2 + 1.0 / 5040.0;
    s = s * r2 - 1.0 / 120.0;
    s = s * r2 + 1.0 / 6.0;
    const double sr = r - r * (r2 * s);
    double c = 1.0 / 6402373705728000.0;
    c = c * r2 - 1.0 / 20922789888000.0;
    c = c * r2 + 1.0 / 87178291200.0;
    c = c * r2 - 1.0 / 479001600.0;
    c = c * r2 + 1.0 / 3628800.0;
    c = c * r2 - 1.0 / 40320.0;
    c = c * r2 + 1.0 / 720.0;
    c = c * r2 - 1.0 / 24.0;
    c = c * r2 + 0.5;
    const double cr = 1.0 - r2 * c;
    const int q = (int)((long long)kq & 3);
    if (q == 0) { *sn = sr; *cs = cr; }
    else if (q == 1) { *sn = cr; *cs = -sr; }
    else if (q == 2) { *sn = -sr; *cs = -cr; }
    else { *sn = -cr; *cs = sr; }
}

__host__ __device__ inline double pm_sin(double a)
{
    double s, c;
    pm_sincos(a, &s, &c);
    return s;
}
__host__ __device__ inline double pm_cos(double a)
{
    double s, c;
    pm_sincos(a, &s, &c);
    return c;
}

// ---- correctly rounded sin/cos ---------------------------------------------
struct dd_t {
    double h, l;
};
__host__ __device__ inline dd_t dd_two_sum(double a, double b)
{
    const double s = a + b, bb = s - a;
    return {s, (a - (s - bb)) + (b - bb)};
}
__host__ __device__ inline dd_t dd_fast2(double a, double b)
{
    const double s = a + b;
    return {s, b - (s - a)};
}
__host__ __device__ inline dd_t dd_mul(dd_t x, dd_t y)
{
    const double p = x.h * y.h;
    double e = fma(x.h, y.h, -p);
    e = e + (x.h * y.l + x.l * y.h);
    return dd_fast2(p, e);
}
__host__ __device__ inline dd_t dd_add(dd_t x, dd_t y)
{
    const dd_t s = dd_two_sum(x.h, y.h);
    return dd_fast2(s.h, s.l + (x.l + y.l));
}

// sin tail: sum_{n=11..29 odd} (-1)^((n-1)/2) r^(n-11) / n!  (Horner, highest first); cos tail n=12..28
static constexpr double CR_STAIL[10] = { 0x1.259f98b4358adp-103, -0x1.d1ab1c2dccea3p-94, 0x1.3f3ccdd165fa9p-84, -0x1.761b41316381ap-75, 0x1.71b8ef6dcf572p-66, -0x1.2f49b46814157p-57, 0x1.952c77030ad4ap-49, -0x1.ae7f3e733b81fp-41, 0x1.6124613a86d09p-33, -0x1.ae64567f544e4p-26 };
static constexpr double CR_CTAIL[9] = { 0x1.0a18a2635085dp-98, -0x1.88e85fc6a4e5ap-89, 0x1.f2cf01972f578p-80, -0x1.0ce396db7f853p-70, 0x1.e542ba4020225p-62, -0x1.6827863b97d97p-53, 0x1.ae7f3e733b81fp-45, -0x1.93974a8c07c9dp-37, 0x1.1eed8eff8d898p-29 };
static constexpr double CR_SHEAD[4][2] = { { 0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73 }, { -0x1.a01a01a01a01ap-13, -0x1.a01a01a01a01ap-73 }, { 0x1.1111111111111p-7, 0x1.1111111111111p-63 }, { -0x1.5555555555555p-3, -0x1.5555555555555p-57 } };
static constexpr double CR_CHEAD[5][2] = { { -0x1.27e4fb7789f5cp-22, -0x1.cbbc05b4fa99ap-76 }, { 0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76 }, { -0x1.6c16c16c16c17p-10, 0x1.f49f49f49f49fp-65 }, { 0x1.5555555555555p-5, 0x1.5555555555555p-59 }, { -0x1.0000000000000p-1, 0x0.0p+0 } };

__host__ __device__ inline void cr_sincos(double a, double* sn, double* cs)
{
    // pi/2 = P1 + P2 + P3 + P4; P1, P2 have <= 32 significant bits so k*P1, k*P2 are exact
    const double kq = floor(a * 6.36619772367581382433e-01 + 0.5);
    dd_t r = dd_two_sum(a, -(kq * 1.57079632673412561417e+00));
    r = dd_add(r, {-(kq * 6.07710050630396597660e-11), 0.0});
    const double t = kq * 2.02226624879595063154e-21;
    r = dd_add(r, {-t, -(fma(kq, 2.02226624879595063154e-21, -t) + kq * 1.0085854035872483e-37)});
    const dd_t r2 = dd_mul(r, r);
    double ps = CR_STAIL[0], pc = CR_CTAIL[0];
#pragma unroll
    for (int i = 1; i < 10; ++i) ps = ps * r2.h + CR_STAIL[i];
#pragma unroll
    for (int i = 1; i < 9; ++i) pc = pc * r2.h + CR_CTAIL[i];
    dd_t s = {ps, 0.0}, c = {pc, 0.0};
#pragma unroll
    for (int i = 0; i < 4; ++i) s = dd_add(dd_mul(s, r2), {CR_SHEAD[i][0], CR_SHEAD[i][1]});
#pragma unroll
    for (int i = 0; i < 5; ++i) c = dd_add(dd_mul(c, r2), {CR_CHEAD[i][0], CR_CHEAD[i][1]});
    s = dd_add(r, dd_mul(r, dd_mul(s, r2)));
    c = dd_add({1.0, 0.0}, dd_mul(c, r2));
    const int q = (int)((long long)kq & 3);
    if (q == 0) { *sn = s.h; *cs = c.h; }
    else if (q == 1) { *sn = c.h; *cs = -s.h; }
    else if (q == 2) { *sn = -s.h; *cs = -c.h; }
    else { *sn = -c.h; *cs = s.h; }
}

}  // namespace futbol
