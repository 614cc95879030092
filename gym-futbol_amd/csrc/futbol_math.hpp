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

}  // namespace futbol
