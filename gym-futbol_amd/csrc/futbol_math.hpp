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
#include "futbol_sincostab.h"
#include "futbol_powtab.h"

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

// ---- glibc 2.35 sin / cos ---------------------------------------------------
// The reference's screw_vec (envs/futbol_env.py:101-116) rotates a shot by math.sin / math.cos,
// i.e. glibc's: on x86-64 hosts with FMA + AVX2 (the reference's goldens were produced on one)
// glibc runs the __sin_fma / __cos_fma build of the IBM Accurate Mathematical Library's
// sysdeps/ieee754/dbl-64/s_sin.c.  Restated here operation for operation -- do_sin with
// TAYLOR_SIN below 0.126, do_cos, reduce_sincos, do_sincos, and every multiply-add the compiler
// fused in that build as an fma -- with glibc's table (futbol_sincostab.h), so the kernel's shot
// directions are bit-identical to the reference's (oracle/oracle_math.h holds the checker's own
// restatement, tests/test_glibc_sincos.py pins it against the host libm).  |x| < 105414350 only
// (screw_vec's angles are below 4.5 in magnitude); beyond, the correctly rounded cr_sincos.
// (16-byte aligned: the v0 step kernel copies it into LDS in 16-byte LDS-DMA pieces, futbol_v0.hip)
alignas(16) static constexpr double kSinCosTab[440] = {FUTBOL_SINCOSTAB_ROWS};

namespace glibc_sincos {
constexpr double BIG = 0x1.8p45, SN3 = -0x1.5555555555515p-3, SN5 = 0x1.11110e829872fp-7;
constexpr double CS2 = 0x1.0p-1, CS4 = -0x1.5555555555535p-5, CS6 = 0x1.6c16bedd9e239p-10;
constexpr double S1 = -0x1.5555555555555p-3, S2 = 0x1.1111111110ecep-7, S3 = -0x1.a01a019db08b8p-13,
                 S4 = 0x1.71de27b9a7ed9p-19, S5 = -0x1.addffc2fcdf59p-26;
constexpr double HP0 = 0x1.921fb54442d18p0, HP1 = 0x1.1a62633145c07p-54;
constexpr double HPINV = 0x1.45f306dc9c883p-1, TOINT = 0x1.8p52;
constexpr double MP1 = 0x1.921fb58p0, MP2 = -0x1.dde973cp-27, PP3 = -0x1.cb3b398p-55, PP4 = -0x1.d747f23e32ed7p-83;

__host__ __device__ inline uint32_t hi_word(double x)
{
    uint64_t b;
    memcpy(&b, &x, 8);
    return (uint32_t)(b >> 32) & 0x7fffffffu;
}
// the table row of |x| (u = |x| + BIG rounds |x| to a multiple of 1/128); rows 0..109
// (tab: kSinCosTab or a copy of it, e.g. staged in LDS by a kernel)
__host__ __device__ inline const double* row(double u, const double* tab)
{
    uint64_t b;
    memcpy(&b, &u, 8);
    uint32_t i = (uint32_t)b;
    i = i < 110u ? i : 109u;  // |x| < 0.8555 keeps i <= 109; the clamp only bounds the address
    return tab + 4 * i;
}
__host__ __device__ inline double do_sin(double x, double dx, const double* tab)
{
    if (fabs(x) < 0.126) {  // TAYLOR_SIN
        const double xx = x * x;
        double p = fma(xx, S5, S4);
        p = fma(xx, p, S3);
        p = fma(xx, p, S2);
        p = fma(xx, p, S1);
        return x + fma(xx, fma(p, x, -(0.5 * dx)), dx);
    }
    const double d = x <= 0 ? -dx : dx;
    const double ax = fabs(x), u = ax + BIG, xr = ax - (u - BIG);
    const double* T = row(u, tab);
    const double xx = xr * xr;
    const double sv = xr + fma(xr * xx, fma(xx, SN5, SN3), d);
    const double cv = fma(xr, d, xx * fma(xx, fma(xx, CS6, CS4), CS2));
    const double cor = fma(sv, T[2], fma(-cv, T[0], fma(sv, T[3], T[1])));
    return copysign(T[0] + cor, x);
}
__host__ __device__ inline double do_cos(double x, double dx, const double* tab)
{
    const double d = x < 0 ? -dx : dx;
    const double ax = fabs(x), u = ax + BIG, xr = (ax - (u - BIG)) + d;
    const double* T = row(u, tab);
    const double xx = xr * xr;
    const double sv = fma(xr * xx, fma(xx, SN5, SN3), xr);
    const double cv = xx * fma(xx, fma(xx, CS6, CS4), CS2);
    const double cor = fma(-sv, T[0], fma(-cv, T[2], fma(-sv, T[1], T[3])));
    return T[2] + cor;
}
__host__ __device__ inline int reduce(double x, double& a, double& da)
{
    const double t = fma(x, HPINV, TOINT);
    const double xn = t - TOINT;
    uint64_t tb;
    memcpy(&tb, &t, 8);
    double y = fma(-xn, MP1, x);
    y = fma(-xn, MP2, y);
    const double t2 = fma(-xn, PP3, y);
    const double db = fma(-xn, PP3, y - t2);
    const double b = fma(-xn, PP4, t2);
    da = db + fma(-xn, PP4, t2 - b);
    a = b;
    return (int)(tb & 3u);
}
__host__ __device__ inline double do_sincos(double a, double da, int n, const double* tab)
{
    const double r = (n & 1) ? do_cos(a, da, tab) : do_sin(a, da, tab);
    return (n & 2) ? -r : r;
}
}  // namespace glibc_sincos

__host__ __device__ inline double glibc_sin(double x, const double* tab = kSinCosTab)
{
    using namespace glibc_sincos;
    const uint32_t k = hi_word(x);
    if (k < 0x3e500000u) return x;
    if (k < 0x3feb6000u) return do_sin(x, 0.0, tab);
    if (k < 0x400368fdu) return copysign(do_cos(HP0 - fabs(x), HP1, tab), x);
    if (k < 0x419921fbu) {
        double a, da;
        const int n = reduce(x, a, da);
        return do_sincos(a, da, n, tab);
    }
    double sn, cs;
    cr_sincos(x, &sn, &cs);
    return sn;
}
__host__ __device__ inline double glibc_cos(double x, const double* tab = kSinCosTab)
{
    using namespace glibc_sincos;
    const uint32_t k = hi_word(x);
    if (k < 0x3e400000u) return 1.0;
    if (k < 0x3feb6000u) return do_cos(x, 0.0, tab);
    if (k < 0x400368fdu) {
        const double y = HP0 - fabs(x);
        const double a = y + HP1;
        return do_sin(a, (y - a) + HP1, tab);
    }
    if (k < 0x419921fbu) {
        double a, da;
        const int n = reduce(x, a, da);
        return do_sincos(a, da, n + 1, tab);
    }
    double sn, cs;
    cr_sincos(x, &sn, &cs);
    return cs;
}

// ---- glibc 2.35 pow(x, 2.0) -----------------------------------------------
// The reference's `x**2` (get_vec, _step_by_observation, _ball_to_team_distance_arr, pymunk's
// Vec2d.length in limit_velocity) is libm pow(x, 2.0): CPython floats and numpy float64 scalars
// call it.  glibc's pow (ARM optimized-routines algorithm, the __pow_fma build) computes
// exp(2 log x) in double-double with 128-entry tables and rounds once at the end; before that
// rounding it is within 1.11 / 128 + poly error (< 0.009) ulp of x^2, so its result is the
// correctly rounded x*x unless x^2 lies within that distance of a rounding midpoint (~2% of
// arguments; the results then differ on ~0.08%).  glibc_pow2: x*x, and the restated glibc
// computation only where |x^2 - midpoint| < 2^-6 ulp (exact test: lo = fma(x, x, -x*x) is the
// exact rounding error of x*x).  Main path only: x normal with x^2 in [2^-738, 2^738], x*x
// elsewhere (never reached by squared coordinate differences).  Tables: futbol_powtab.h.
alignas(16) static constexpr double kPowLog[128 * 3] = {FUTBOL_POW_LOG_ROWS};
alignas(16) static constexpr uint64_t kPowExp[256] = {FUTBOL_POW_EXP_ROWS};
constexpr int kPowTabBytes = (int)(sizeof(kPowLog) + sizeof(kPowExp));  // 5 KB

__host__ __device__ inline double bits_to_f64(uint64_t u)
{
    double d;
    memcpy(&d, &u, 8);
    return d;
}
__host__ __device__ inline uint64_t f64_to_bits(double d)
{
    uint64_t u;
    memcpy(&u, &d, 8);
    return u;
}

// glibc's pow(x, 2.0) computed in full (log_inline, y * log, exp_inline), |x| normal.  The tables
// may be a copy (a kernel stages them in LDS: the two dependent lookups are most of the latency).
// Inlined at every site (~30 in the v0 step kernel, 80 KB of code): a non-inlined copy (850 bytes,
// 22 VGPRs) measured 1% slower
__host__ __device__ __forceinline__ double glibc_pow2_full(double x, const double* kPowLog = futbol::kPowLog,
                                                          const uint64_t* kPowExp = futbol::kPowExp)
{
    const uint64_t ix = f64_to_bits(x) & 0x7fffffffffffffffull;  // y even: pow(-x, 2) = pow(x, 2)
    const uint32_t topx = (uint32_t)(ix >> 52);
    if (topx < 0x3ff - 369 || topx > 0x3ff + 369) return x * x;
    const uint64_t tmp = ix - 0x3fe6955500000000ull;
    const int i = (int)((tmp >> 45) & 127u);
    const double kd = (double)((int64_t)tmp >> 52);
    const double z = bits_to_f64(ix - (tmp & 0xfff0000000000000ull));
    const double invc = kPowLog[3 * i], logc = kPowLog[3 * i + 1], logctail = kPowLog[3 * i + 2];
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
    const double ly = hi + lo, ltail = (hi - ly) + lo;
    const double ehi = 2.0 * ly;
    const double elo = fma(2.0, ltail, fma(ly, 2.0, -ehi));
    const uint32_t abstop = (uint32_t)(f64_to_bits(ehi) >> 52) & 0x7ffu;
    if (abstop < 0x3c9u) return 1.0 + ehi;
    if (abstop >= 0x408u) return x * x;
    double kx = fma(ehi, 0x1.71547652b82fep+7, 0x1.8p52);
    const uint64_t ki = f64_to_bits(kx);
    kx = kx - 0x1.8p52;
    double rr = fma(kx, -0x1.62e42fefa0000p-8, ehi);
    rr = fma(kx, -0x1.cf79abc9e3b3ap-47, rr);
    rr = elo + rr;
    const int idx = 2 * (int)(ki & 127u);
    const double tail = bits_to_f64(kPowExp[idx]);
    const double scale = bits_to_f64(kPowExp[idx + 1] + (ki << 45));
    const double r2 = rr * rr;
    const double t = fma(r2 * r2, fma(rr, 0x1.1111167a4d017p-7, 0x1.55555cf172b91p-5),
                         fma(fma(rr, 0x1.555555555543cp-3, 0x1.ffffffffffdbdp-2), r2, tail + rr));
    return fma(t, scale, scale);
}

// x*x is glibc's pow(x, 2.0) unless x^2 lies within 2^-6 ulp of a rounding midpoint (glibc's
// pre-rounding error is below 0.0097 ulp: 1e8 samples, and 1.11 / 128 ulp + poly error by its own
// bound); h = x*x, l = fma(x, x, -h) its exact rounding error
__host__ __device__ __forceinline__ bool pow2_near_midpoint(double h, double l)
{
    // ulp(h) / 2 * (1 - 2^-5) = 2^(E - 53) * (1 - 2^-5) for h = m 2^E, m in [1, 2): frexp's exponent is
    // E + 1 (v_frexp_exp_i32_f64 + v_ldexp_f64 on the GPU: 2 instructions instead of the exponent-field
    // arithmetic, compare and select).  h = 0 (x = 0, common: aligned bodies): e = 0, near > 0 = |l|, not
    // near.  Tiny, infinite or NaN h may be reported near or not -- glibc's full path returns x*x for
    // them (glibc_pow2_full's topx test), so the square is x*x either way
    int e;
    (void)__builtin_frexp(h, &e);
    const double near = __builtin_ldexp(1.0 - 0x1.0p-5, e - 54);
    return !(__builtin_fabs(l) < near);
}

// glibc pow(x, 2.0)
__host__ __device__ __forceinline__ double glibc_pow2(double x)
{
    const double h = x * x;
    if (__builtin_expect(pow2_near_midpoint(h, fma(x, x, -h)), 0)) return glibc_pow2_full(x);
    return h;
}

// glibc pow(x, 2.0) + glibc pow(y, 2.0) (get_vec's `vec[0]**2 + vec[1]**2`).  In a wave64 some lane
// nearly always needs the slow path at a given call site (~3% per square), so the slow rounds of
// glibc_pow2_batch (below) are each site's real cost; batch independent squares where possible
template <int M>
__host__ __device__ __forceinline__ void glibc_pow2_batch(const double (&x)[M], double (&h)[M], const double* logt,
                                                         const uint64_t* expt);
__host__ __device__ __forceinline__ double glibc_sq2(double x, double y, const double* logt = kPowLog,
                                                    const uint64_t* expt = kPowExp)
{
    const double xs[2] = {x, y};
    double h[2];
    glibc_pow2_batch<2>(xs, h, logt, expt);
    return h[0] + h[1];
}

// h[i] = glibc pow(x[i], 2.0) for M independent squares: x*x everywhere, then the exact glibc
// computation for the near-midpoint ones, one per lane per round (each lane takes its lowest
// pending square), so a wave runs max-over-lanes(pending) rounds -- nearly always one -- instead
// of one slow branch per square.  Compile-time indices only (registers, no scratch).
template <int M>
__host__ __device__ __forceinline__ void glibc_pow2_batch(const double (&x)[M], double (&h)[M], const double* logt,
                                                         const uint64_t* expt)
{
    static_assert(M <= 32, "pending mask");
    uint32_t pend = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        h[i] = x[i] * x[i];
        pend |= pow2_near_midpoint(h[i], fma(x[i], x[i], -h[i])) ? 1u << i : 0u;
    }
#ifdef FUTBOL_DIAG_PLAIN_SQ  // diagnostic builds only (cost of the exact squares): x*x, NOT glibc's
    pend = 0u;
#endif
    while (__builtin_expect(pend != 0u, 0)) {
        const uint32_t bit = pend & (0u - pend);
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) v = bit == (1u << i) ? x[i] : v;
        const double f = glibc_pow2_full(v, logt, expt);
#pragma unroll
        for (int i = 0; i < M; ++i) h[i] = bit == (1u << i) ? f : h[i];
        pend &= pend - 1u;
    }
}

// Copy the pow tables (kPowLog, then kPowExp: 5 KB) into `lds` with the wave's active lanes (16 bytes
// per lane and access: the active lanes stride over the 320 chunks, so a partial wave -- the lanes past
// B of the last block have returned, a restart phase runs on some lanes only -- copies all of them);
// returns the LDS copies' addresses.  `lds` is 16-byte aligned and not in use; one-wave blocks.
__device__ __forceinline__ void stage_pow_tables(void* lds, const double*& logt, const uint64_t*& expt)
{
    const uint4* sl = reinterpret_cast<const uint4*>(kPowLog);
    const uint4* se = reinterpret_cast<const uint4*>(kPowExp);
    uint4* d = reinterpret_cast<uint4*>(lds);
    constexpr int NL = (int)sizeof(kPowLog) / 16, NE = (int)sizeof(kPowExp) / 16;  // 192, 128
    const uint64_t live = __ballot(1);
    const int A = __popcll(live);
    const int w = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
    // the LDS held double2 rows until now: keep these stores after every earlier access to it (type-based
    // alias analysis would otherwise be free to move them up, see glibc_pow2_need_lds)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (A == 64) {  // the common case: five independent loads per lane
        const uint4 a0 = sl[w], a1 = sl[w + 64], a2 = sl[w + 128], b0 = se[w], b1 = se[w + 64];
        d[w] = a0;
        d[w + 64] = a1;
        d[w + 128] = a2;
        d[NL + w] = b0;
        d[NL + w + 64] = b1;
    } else {
        for (int i = w; i < NL + NE; i += A) d[i] = i < NL ? sl[i] : se[i - NL];
    }
    static_assert(NL == 192 && NE == 128, "5 uint4 per lane");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    logt = reinterpret_cast<const double*>(lds);
    expt = reinterpret_cast<const uint64_t*>(d + NL);
}

// glibc_pow2_need (below) with the tables staged in LDS (stage_pow_tables into `lds`) when some lane
// of the wave needs glibc's path: two LDS lookups per slow round instead of two global ones.  (Loading
// the tables' chunks with the step's state instead, so that staging waits for no memory at the use,
// measured 2v2 +2.8% (22.51 -> 23.15 us, 20 more live VGPRs), 5v5 neutral; copied by LDS-DMA at the
// step's start instead -- the v0 kernel's form: 2v2 -0.4%, 5v5 +0.4%; neither adopted, round 5.)
template <int M>
__device__ __forceinline__ void glibc_pow2_need_lds(const double (&x)[M], double (&h)[M], uint64_t need, void* lds);

// h[i] = glibc pow(x[i], 2.0) for the squares whose bit i of `need` is set, x*x for the others
// (squares whose value cannot matter for this lane: the caller's superset of the used ones).  Like
// glibc_pow2_batch, the near-midpoint squares are recomputed one per lane per round, so a wave runs
// max-over-lanes(pending) rounds; up to 64 squares.
template <int M>
__host__ __device__ __forceinline__ void glibc_pow2_need(const double (&x)[M], double (&h)[M], uint64_t need,
                                                        const double* logt = kPowLog, const uint64_t* expt = kPowExp);
// glibc_pow2_full as a real call (global-memory tables): the envs_v1 instances at the register limit inline
// it at every player and body (~40 copies for 10v10), and the compiler hoists the copies' polynomial
// constants out of them -- materialised once, then spilled to scratch for the whole step
__host__ __device__ __attribute__((noinline)) inline double glibc_pow2_full_call(double x)
{
    return glibc_pow2_full(x);
}
template <int M, bool CALL>
__host__ __device__ __forceinline__ void glibc_pow2_need_t(const double (&x)[M], double (&h)[M], uint64_t need)
{
    static_assert(M <= 64, "pending mask");
    uint64_t pend = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        h[i] = x[i] * x[i];
        pend |= (uint64_t)pow2_near_midpoint(h[i], fma(x[i], x[i], -h[i])) << i;
    }
    pend &= need;
#ifdef FUTBOL_DIAG_PLAIN_SQ  // diagnostic builds only (cost of the exact squares): x*x, NOT glibc's
    pend = 0u;
#endif
    while (__builtin_expect(pend != 0u, 0)) {
        const uint64_t bit = pend & (0ull - pend);
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) v = bit == (1ull << i) ? x[i] : v;
        const double f = CALL ? glibc_pow2_full_call(v) : glibc_pow2_full(v);
#pragma unroll
        for (int i = 0; i < M; ++i) h[i] = bit == (1ull << i) ? f : h[i];
        pend &= pend - 1u;
    }
}
template <int M>
__host__ __device__ __forceinline__ void glibc_pow2_need(const double (&x)[M], double (&h)[M], uint64_t need,
                                                        const double* logt, const uint64_t* expt)
{
    static_assert(M <= 64, "pending mask");
    uint64_t pend = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        h[i] = x[i] * x[i];
        pend |= (uint64_t)pow2_near_midpoint(h[i], fma(x[i], x[i], -h[i])) << i;
    }
    pend &= need;
#ifdef FUTBOL_DIAG_PLAIN_SQ  // diagnostic builds only (cost of the exact squares): x*x, NOT glibc's
    pend = 0u;
#endif
    while (__builtin_expect(pend != 0u, 0)) {
        const uint64_t bit = pend & (0ull - pend);
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < M; ++i) v = bit == (1ull << i) ? x[i] : v;
        const double f = glibc_pow2_full(v, logt, expt);
#pragma unroll
        for (int i = 0; i < M; ++i) h[i] = bit == (1ull << i) ? f : h[i];
        pend &= pend - 1u;
    }
}

template <int M>
__device__ __forceinline__ void glibc_pow2_need_lds(const double (&x)[M], double (&h)[M], uint64_t need, void* lds)
{
    static_assert(M <= 64, "pending mask");
    uint64_t pend = 0;
#pragma unroll
    for (int i = 0; i < M; ++i) {
        h[i] = x[i] * x[i];
        pend |= (uint64_t)pow2_near_midpoint(h[i], fma(x[i], x[i], -h[i])) << i;
    }
    pend &= need;
#ifdef FUTBOL_DIAG_PLAIN_SQ  // diagnostic builds only (cost of the exact squares): x*x, NOT glibc's
    pend = 0u;
#endif
    if (__builtin_expect(__ballot(pend != 0u) != 0ull, 0)) {  // wave-uniform
        const double* logt;
        const uint64_t* expt;
#ifdef FUTBOL_DIAG_POW_GLOBAL  // diagnostic builds only: the tables read from global memory
        (void)lds;
        logt = kPowLog;
        expt = kPowExp;
#else
        stage_pow_tables(lds, logt, expt);
#endif
        while (pend != 0u) {
            const uint64_t bit = pend & (0ull - pend);
            double v = 0.0;
#pragma unroll
            for (int i = 0; i < M; ++i) v = bit == (1ull << i) ? x[i] : v;
            const double f = glibc_pow2_full(v, logt, expt);
#pragma unroll
            for (int i = 0; i < M; ++i) h[i] = bit == (1ull << i) ? f : h[i];
            pend &= pend - 1u;
        }
        // The caller reuses this LDS with other types next (the solver rows are double2): the barrier
        // keeps those stores after the last u64 / double table reads whatever type-based alias analysis
        // concludes (a precaution: it was not the cause of the N = 6 divergence)
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

}  // namespace futbol
