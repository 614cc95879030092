// futbol_v1_impl.hpp -- envs_v1 `Futbol` step as one HIP kernel for gfx950.
//
// Reference: gym_futbol/envs_v1/futbol_env.py (step :427-483), team.py,
// ball.py, player.py, and the Chipmunk2D 7.0.x cpSpaceStep that pymunk 5.6
// runs under them.  One env per lane; the lane keeps
// its env's bodies in registers (fp64, like cpFloat), reads/writes the SoA
// state once per step (coalesced), draws the opponent's actions and every
// other random choice from a counter-based Philox stream, and implements
// DummyVecEnv's auto-reset in the same launch.
//
// Contacts: the narrowphase runs over all Nb*12 circle-segment and
// Nb(Nb-1)/2 circle-circle pairs in the canonical order, with
// exact broadphase rejections (cpBBIntersects, plus an "interior" test that
// provably rejects all 12 segments at once).  Contact records go to LDS
// (K slots per lane, lane-contiguous: conflict-free) and beyond K to a global
// spill area, so there is no capacity limit.  During the sequential-impulse
// solve the bodies' v / v_bias live in LDS too (per-lane dynamic indexing).
// The persistent arbiter cache is a compact per-env list of (pair, age, jnAcc).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "futbol_rng.hpp"
#include "futbol_state.hpp"
#include "futbol_kernels.hpp"
#include "futbol_util.hpp"

namespace futbol {

// ---- reference constants, envs_v1/futbol_env.py:19-50, player.py:7, ball.py:7
constexpr double kPlayerR = 1.5, kBallR = 1.0, kSegR = 1.0;
constexpr double kPlayerMinv = 1.0 / 20.0, kBallMinv = 1.0 / 10.0;
constexpr double kPlayerVmax = 10.0, kBallVmax = 25.0;
constexpr double kE = 0.2;  // elasticity of players and ball; segments 0

template <int N>
struct V1Shape {
    static constexpr int Nb = 2 * N + 1;
    static constexpr int BALL = 2 * N;
    static constexpr int P = v1_npairs(N);
    // LDS slots per lane for contact records: 4 blocks (waves) per CU fit 160 KB
    static constexpr int K = N <= 2 ? 7 : (N <= 5 ? 4 : 2);
};

__device__ __forceinline__ double radius_of(int k, int ball) { return k == ball ? kBallR : kPlayerR; }
__device__ __forceinline__ double minv_of(int k, int ball) { return k == ball ? kBallMinv : kPlayerMinv; }

// contact record fields
enum { F_NX = 0, F_NY, F_NMASS, F_BIAS, F_BOUNCE, F_JN, F_JB, F_NFIELDS };

template <int N>
struct Scratch {
    using S = V1Shape<N>;
    double rec[S::K][F_NFIELDS][64];
    int info[S::K][64];
    double vel[S::Nb][4][64];  // vx, vy, bx, by during the solve
};

template <int N>
struct Lane {
    using S = V1Shape<N>;
    Scratch<N>* sh;
    double* spill;
    uint16_t* ckey;
    double* cjn;
    int lane, env, B;

    __device__ __forceinline__ double rget(int s, int f) const
    {
        if (s < S::K) return sh->rec[s][f][lane];
        return spill[((size_t)(s - S::K) * 8 + f) * B + env];
    }
    __device__ __forceinline__ void rset(int s, int f, double v) const
    {
        if (s < S::K) sh->rec[s][f][lane] = v;
        else spill[((size_t)(s - S::K) * 8 + f) * B + env] = v;
    }
    __device__ __forceinline__ int iget(int s) const
    {
        if (s < S::K) return sh->info[s][lane];
        return (int)__double_as_longlong(spill[((size_t)(s - S::K) * 8 + 7) * B + env]);
    }
    __device__ __forceinline__ void iset(int s, int v) const
    {
        if (s < S::K) sh->info[s][lane] = v;
        else spill[((size_t)(s - S::K) * 8 + 7) * B + env] = __longlong_as_double((long long)v);
    }
    __device__ __forceinline__ double& vel(int body, int c) const { return sh->vel[body][c][lane]; }
};

// info word: a (5 bits) | bcode (6 bits: body id, or 32 + segment) << 5 | pair << 11 | normal << 20
__device__ __forceinline__ int pack_info(int a, int bcode, int pair, bool normal)
{
    return a | (bcode << 5) | (pair << 11) | ((normal ? 1 : 0) << 20);
}

template <int N>
struct Env {
    using S = V1Shape<N>;
    double px[S::Nb], py[S::Nb], vx[S::Nb], vy[S::Nb], bx[S::Nb], by[S::Nb];
    Meta meta;
};

// ---------------------------------------------------------------------------
// narrowphase (cpCollision.c CircleToCircle / CircleToSegment), exact op order
__device__ __forceinline__ bool cc_test(double ax, double ay, double ra, double bx_, double by_, double rb,
                                        double& nx, double& ny, double& p1x, double& p1y, double& p2x,
                                        double& p2y)
{
    const double mind = ra + rb;
    const double dx = bx_ - ax, dy = by_ - ay;
    const double d2 = dx * dx + dy * dy;
    if (!(d2 < mind * mind)) return false;
    const double d = sqrt(d2);
    if (d != 0.0) {
        const double inv = 1.0 / d;
        nx = dx * inv;
        ny = dy * inv;
    } else {
        nx = 1.0;
        ny = 0.0;
    }
    p1x = ax + nx * ra;
    p1y = ay + ny * ra;
    p2x = bx_ + nx * (-rb);
    p2y = by_ + ny * (-rb);
    return true;
}

__device__ __forceinline__ bool cc_hit(double ax, double ay, double ra, double bx_, double by_, double rb)
{
    const double mind = ra + rb;
    const double dx = bx_ - ax, dy = by_ - ay;
    return dx * dx + dy * dy < mind * mind;
}

__device__ __forceinline__ bool cs_test(double cx, double cy, double rc, double sax, double say, double sbx,
                                        double sby, double& nx, double& ny, double& p1x, double& p1y,
                                        double& p2x, double& p2y)
{
    const double sdx = sbx - sax, sdy = sby - say;
    double t = (sdx * (cx - sax) + sdy * (cy - say)) / (sdx * sdx + sdy * sdy);
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
    const double qx = sax + sdx * t, qy = say + sdy * t;
    const double mind = rc + kSegR;
    const double dx = qx - cx, dy = qy - cy;
    const double d2 = dx * dx + dy * dy;
    if (!(d2 < mind * mind)) return false;
    const double d = sqrt(d2);
    if (d != 0.0) {
        const double inv = 1.0 / d;
        nx = dx * inv;
        ny = dy * inv;
    } else {
        const double inv = 1.0 / sqrt(sdx * sdx + sdy * sdy);
        nx = -sdy * inv;
        ny = sdx * inv;
    }
    p1x = cx + nx * rc;
    p1y = cy + ny * rc;
    p2x = qx + nx * (-kSegR);
    p2y = qy + ny * (-kSegR);
    return true;
}

__device__ __forceinline__ bool cs_hit(double cx, double cy, double rc, double sax, double say, double sbx,
                                       double sby)
{
    const double sdx = sbx - sax, sdy = sby - say;
    double t = (sdx * (cx - sax) + sdy * (cy - say)) / (sdx * sdx + sdy * sdy);
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
    const double qx = sax + sdx * t, qy = say + sdy * t;
    const double mind = rc + kSegR;
    const double dx = qx - cx, dy = qy - cy;
    return dx * dx + dy * dy < mind * mind;
}

// ball within reach of no wall/goal segment: provably rejects all 12 segment tests
// (every segment lies on x<=0, x>=W, y<=0 or y>=H; the test needs distance < rc+1)
__device__ __forceinline__ bool far_from_segments(double x, double y, double reach, double W, double H)
{
    return x > reach && x < W - reach && y > reach && y < H - reach;
}

// ---------------------------------------------------------------------------
// preStep of one new contact (cpArbiterPreStep), written to contact slot n.
// Called with the bodies' values already loaded (no per-lane array indexing).
template <int N>
__device__ __forceinline__ void record_contact(const Lane<N>& L, int n, int info, double biasCoef, double dt,
                                               double slop, double nx, double ny, double p1x, double p1y,
                                               double p2x, double p2y, double apx, double apy, double avx,
                                               double avy, double ma, double bpx, double bpy, double bvx_,
                                               double bvy_, double mb, double ee)
{
    const double r1x = p1x - apx, r1y = p1y - apy;
    const double r2x = p2x - bpx, r2y = p2y - bpy;
    const double nMass = 1.0 / (ma + mb);
    const double bdx = bpx - apx, bdy = bpy - apy;
    const double dist = ((r2x - r1x) + bdx) * nx + ((r2y - r1y) + bdy) * ny;
    double m = dist + slop;
    m = (0.0 < m) ? 0.0 : m;
    const double bias = -biasCoef * m / dt;
    const double bounce = ((bvx_ - avx) * nx + (bvy_ - avy) * ny) * ee;
    L.rset(n, F_NX, nx);
    L.rset(n, F_NY, ny);
    L.rset(n, F_NMASS, nMass);
    L.rset(n, F_BIAS, bias);
    L.rset(n, F_BOUNCE, bounce);
    L.rset(n, F_JN, 0.0);
    L.rset(n, F_JB, 0.0);
    L.iset(n, info);
}

// cpSpaceStep(dt) for one env.  dtc: 1 -> 1e-4, 2 -> 0.1
template <int N>
__device__ __forceinline__ void space_step(const V1Params* __restrict__ P, const Lane<N>& L, Env<N>& e, int dtc)
{
    using S = V1Shape<N>;
    const double dt = dtc == 2 ? P->dtv[2] : P->dtv[1];
    const uint32_t pc = e.meta.dtcode();
    const double prev_dt = pc == 2 ? P->dtv[2] : (pc == 1 ? P->dtv[1] : 0.0);
    const double biasCoef = dtc == 2 ? P->biasc[2] : P->biasc[1];
    const double damping = dtc == 2 ? P->damp[2] : P->damp[1];
    const double slop = P->slop, W = P->W, H = P->H;
    e.meta.set_dtcode(dtc);
    const int B = L.B, env = L.env;
    const uint32_t ncache = e.meta.ncache();

    // cpBodyUpdatePosition
    sfor<S::Nb>([&](auto K) {
        constexpr int k = K;
        e.px[k] = e.px[k] + (e.vx[k] + e.bx[k]) * dt;
        e.py[k] = e.py[k] + (e.vy[k] + e.by[k]) * dt;
        e.bx[k] = 0.0;
        e.by[k] = 0.0;
    });

    // collide in canonical order, preStep folded in (it needs pre-damping v)
    int n = 0;
    sfor<S::Nb>([&](auto I) {
        constexpr int i = I;
        constexpr double ri = i == S::BALL ? kBallR : kPlayerR;
        constexpr double mi = i == S::BALL ? kBallMinv : kPlayerMinv;
        const double cl = e.px[i] - ri, cb = e.py[i] - ri, cr = e.px[i] + ri, ct = e.py[i] + ri;
        // every segment's cpBB lies within 1 of the field border: exact reject of all 12
        const bool interior = cl > 1.0 && cr < W - 1.0 && cb > 1.0 && ct < H - 1.0;
        if (!interior) {
            for (int s = 0; s < kNSeg; ++s) {  // wave-uniform s: scalar loads of the geometry
                if (!(cl <= P->sr[s] && P->sl[s] <= cr && cb <= P->st[s] && P->sb[s] <= ct)) continue;
                double nx, ny, p1x, p1y, p2x, p2y;
                if (cs_test(e.px[i], e.py[i], ri, P->sax[s], P->say[s], P->sbx[s], P->sby[s], nx, ny, p1x, p1y,
                            p2x, p2y)) {
                    record_contact<N>(L, n, pack_info(i, 32 + s, i * kNSeg + s, false), biasCoef, dt, slop, nx,
                                      ny, p1x, p1y, p2x, p2y, e.px[i], e.py[i], e.vx[i], e.vy[i], mi, 0.0, 0.0,
                                      0.0, 0.0, 0.0, kE * 0.0);
                    ++n;
                }
            }
        }
        sfor<i + 1, S::Nb>([&](auto J) {
            constexpr int j = J;
            constexpr double rj = j == S::BALL ? kBallR : kPlayerR;
            constexpr double mj = j == S::BALL ? kBallMinv : kPlayerMinv;
            if (!(cl <= e.px[j] + rj && e.px[j] - rj <= cr && cb <= e.py[j] + rj && e.py[j] - rj <= ct)) return;
            double nx, ny, p1x, p1y, p2x, p2y;
            if (cc_test(e.px[i], e.py[i], ri, e.px[j], e.py[j], rj, nx, ny, p1x, p1y, p2x, p2y)) {
                constexpr int pair = S::Nb * kNSeg + i * S::Nb - i * (i + 1) / 2 + (j - i - 1);
                record_contact<N>(L, n, pack_info(i, j, pair, false), biasCoef, dt, slop, nx, ny, p1x, p1y, p2x,
                                  p2y, e.px[i], e.py[i], e.vx[i], e.vy[i], mi, e.px[j], e.py[j], e.vx[j],
                                  e.vy[j], mj, kE * kE);
                ++n;
            }
        });
    });

    // arbiter cache lookup (cpArbiterUpdate copies the old contact's jnAcc;
    // an arbiter touched by the previous step is NORMAL -> warm started)
    for (int s = 0; s < n; ++s) {
        const int info = L.iget(s);
        const int pair = (info >> 11) & 511;
        for (uint32_t c = 0; c < ncache; ++c) {
            const uint32_t key = L.ckey[(size_t)c * B + env];
            if ((int)(key & 0x3ffu) == pair) {
                L.rset(s, F_JN, L.cjn[(size_t)c * B + env]);
                if ((key >> 12) == 0) L.iset(s, info | (1 << 20));
                break;
            }
        }
    }

    // cpBodyUpdateVelocity + the reference's limit_velocity callback
    sfor<S::Nb>([&](auto K) {
        constexpr int k = K;
        e.vx[k] = e.vx[k] * damping + 0.0 * dt;
        e.vy[k] = e.vy[k] * damping + 0.0 * dt;
        const double l = sqrt(e.vx[k] * e.vx[k] + e.vy[k] * e.vy[k]);
        constexpr double vmax = k == S::BALL ? kBallVmax : kPlayerVmax;
        if (l > vmax) {
            const double sc = vmax / l;
            e.vx[k] = e.vx[k] * sc;
            e.vy[k] = e.vy[k] * sc;
        }
    });

    if (n > 0) {
        sfor<S::Nb>([&](auto K) {
            constexpr int k = K;
            L.vel(k, 0) = e.vx[k];
            L.vel(k, 1) = e.vy[k];
            L.vel(k, 2) = 0.0;
            L.vel(k, 3) = 0.0;
        });
        // cpArbiterApplyCachedImpulse
        const double dt_coef = (prev_dt == 0.0) ? 0.0 : dt / prev_dt;
        for (int s = 0; s < n; ++s) {
            const int info = L.iget(s);
            if (!((info >> 20) & 1)) continue;
            const int a = info & 31, bcode = (info >> 5) & 63;
            const double nx = L.rget(s, F_NX), ny = L.rget(s, F_NY), jn = L.rget(s, F_JN);
            const double jx = (nx * jn) * dt_coef, jy = (ny * jn) * dt_coef;
            const double ma = minv_of(a, S::BALL);
            L.vel(a, 0) = L.vel(a, 0) + (-jx) * ma;
            L.vel(a, 1) = L.vel(a, 1) + (-jy) * ma;
            if (bcode < 32) {
                const double mb = minv_of(bcode, S::BALL);
                L.vel(bcode, 0) = L.vel(bcode, 0) + jx * mb;
                L.vel(bcode, 1) = L.vel(bcode, 1) + jy * mb;
            }
        }
        // cpArbiterApplyImpulse x 10 (frictionless: u = 0)
        for (int it = 0; it < 10; ++it) {
            for (int s = 0; s < n; ++s) {
                const int info = L.iget(s);
                const int a = info & 31, bcode = (info >> 5) & 63;
                const bool dyn = bcode < 32;
                const int bb = dyn ? bcode : a;  // any valid slot; masked by dyn below
                const double nx = L.rget(s, F_NX), ny = L.rget(s, F_NY);
                const double nMass = L.rget(s, F_NMASS);
                const double avx = L.vel(a, 0), avy = L.vel(a, 1), abx = L.vel(a, 2), aby = L.vel(a, 3);
                const double bvx_ = dyn ? L.vel(bb, 0) : 0.0, bvy_ = dyn ? L.vel(bb, 1) : 0.0;
                const double bbx_ = dyn ? L.vel(bb, 2) : 0.0, bby_ = dyn ? L.vel(bb, 3) : 0.0;
                const double vbn = (bbx_ - abx) * nx + (bby_ - aby) * ny;
                const double vrn = (bvx_ - avx) * nx + (bvy_ - avy) * ny;
                const double jbn = (L.rget(s, F_BIAS) - vbn) * nMass;
                const double jbOld = L.rget(s, F_JB);
                const double tb = jbOld + jbn;
                const double jb = tb > 0.0 ? tb : 0.0;
                const double jnv = -(L.rget(s, F_BOUNCE) + vrn) * nMass;
                const double jnOld = L.rget(s, F_JN);
                const double tn = jnOld + jnv;
                const double jnAcc = tn > 0.0 ? tn : 0.0;
                L.rset(s, F_JB, jb);
                L.rset(s, F_JN, jnAcc);
                const double db = jb - jbOld, dj = jnAcc - jnOld;
                const double jbx = nx * db, jby = ny * db, jx = nx * dj, jy = ny * dj;
                const double ma = minv_of(a, S::BALL);
                L.vel(a, 2) = abx + (-jbx) * ma;
                L.vel(a, 3) = aby + (-jby) * ma;
                L.vel(a, 0) = avx + (-jx) * ma;
                L.vel(a, 1) = avy + (-jy) * ma;
                if (dyn) {
                    const double mb = minv_of(bb, S::BALL);
                    L.vel(bb, 2) = bbx_ + jbx * mb;
                    L.vel(bb, 3) = bby_ + jby * mb;
                    L.vel(bb, 0) = bvx_ + jx * mb;
                    L.vel(bb, 1) = bvy_ + jy * mb;
                }
            }
        }
        sfor<S::Nb>([&](auto K) {
            constexpr int k = K;
            e.vx[k] = L.vel(k, 0);
            e.vy[k] = L.vel(k, 1);
            e.bx[k] = L.vel(k, 2);
            e.by[k] = L.vel(k, 3);
        });
    }

    // cpSpaceArbiterSetFilter + store jnAcc: survivors (untouched, age+1 < 3) then this step's contacts
    uint32_t w = 0;
    for (uint32_t c = 0; c < ncache; ++c) {
        const uint32_t key = L.ckey[(size_t)c * B + env];
        const int pair = (int)(key & 0x3ffu);
        const uint32_t age = key >> 12;
        bool touched = false;
        for (int s = 0; s < n; ++s) touched |= ((L.iget(s) >> 11) & 511) == pair;
        if (!touched && age + 1 < 3) {
            if (w != c) L.cjn[(size_t)w * B + env] = L.cjn[(size_t)c * B + env];
            L.ckey[(size_t)w * B + env] = (uint16_t)(pair | ((age + 1) << 12));
            ++w;
        }
    }
    for (int s = 0; s < n; ++s) {
        L.ckey[(size_t)w * B + env] = (uint16_t)((L.iget(s) >> 11) & 511);
        L.cjn[(size_t)w * B + env] = L.rget(s, F_JN);
        ++w;
    }
    e.meta.set_ncache(w);
}

// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void position_to_initial(const V1Params* __restrict__ P, Env<N>& e)
{
    sfor<V1Shape<N>::Nb>([&](auto K) {
        constexpr int k = K;
        e.px[k] = P->fx[k];
        e.py[k] = P->fy[k];
        e.vx[k] = 0.0;
        e.vy[k] = 0.0;
    });
}

// _get_observation (envs_v1/futbol_env.py:154-180): [ball, A0.., B0..] x [x, y, vx, vy]
template <int N, typename OT>
__device__ __forceinline__ void write_obs(const Env<N>& e, OT* o)
{
    using S = V1Shape<N>;
    o[0] = (OT)((e.px[S::BALL] - 52.5) / 52.5);
    o[1] = (OT)((e.py[S::BALL] - 34.0) / 34.0);
    o[2] = (OT)((e.vx[S::BALL] - 0.0) / 25.0);
    o[3] = (OT)((e.vy[S::BALL] - 0.0) / 25.0);
    sfor<2 * N>([&](auto K) {
        constexpr int k = K;
        o[4 + 4 * k + 0] = (OT)((e.px[k] - 52.5) / 55.5);
        o[4 + 4 * k + 1] = (OT)((e.py[k] - 34.0) / 34.0);
        o[4 + 4 * k + 2] = (OT)((e.vx[k] - 0.0) / 10.0);
        o[4 + 4 * k + 3] = (OT)((e.vy[k] - 0.0) / 10.0);
    });
}

template <int N>
__device__ __forceinline__ void load_env(const V1Ptrs& st, int env, int B, Env<N>& e)
{
    sfor<V1Shape<N>::Nb>([&](auto K) {
        constexpr int k = K;
        const size_t o = (size_t)k * B + env;
        e.px[k] = st.px[o];
        e.py[k] = st.py[o];
        e.vx[k] = st.vx[o];
        e.vy[k] = st.vy[o];
        e.bx[k] = st.bx[o];
        e.by[k] = st.by[o];
    });
    e.meta.w = st.meta[env];
}

template <int N>
__device__ __forceinline__ void store_env(const V1Ptrs& st, int env, int B, const Env<N>& e)
{
    sfor<V1Shape<N>::Nb>([&](auto K) {
        constexpr int k = K;
        const size_t o = (size_t)k * B + env;
        st.px[o] = e.px[k];
        st.py[o] = e.py[k];
        st.vx[o] = e.vx[k];
        st.vy[o] = e.vy[k];
        st.bx[o] = e.bx[k];
        st.by[o] = e.by[k];
    });
    st.meta[env] = e.meta.w;
}

// Futbol.reset (envs_v1/futbol_env.py:146-150): owner draw, formation, space.step(1e-4)
template <int N>
__device__ __forceinline__ void do_reset(const V1Params* __restrict__ P, const Lane<N>& L, Env<N>& e)
{
    const uint32_t ev = e.meta.event();
    e.meta.set_event(ev + 1);
    Stream rs(P->seed, P->env_base + (uint32_t)L.env, ev, 0);
    e.meta.set_owner((uint32_t)rs.choice(2));
    e.meta.set_steps(0);
    position_to_initial<N>(P, e);
    space_step<N>(P, L, e, 1);
}

// Team.get_pass_target_teammate (team.py:136-180) for player `me` of team `side`:
// returns the teammate's position.
template <int N, int side, int me>
__device__ __forceinline__ void pass_target(const Env<N>& e, Stream& rs, int ar, double& tx, double& ty)
{
    constexpr int base = side * N;
    if constexpr (N == 1) {
        tx = e.px[base];
        ty = e.py[base];
        return;
    } else {
        int t = rs.choice(N - 1);  // random.choices over teammates != self
        t = t >= me ? t + 1 : t;
        if (ar != 0) {
            const double x0 = e.px[base + me], y0 = e.py[base + me];
            auto dir_ok = [&](double mx, double my) {
                return (ar == 1 && my > 0) || (ar == 2 && mx > 0) || (ar == 3 && my < 0) || (ar == 4 && mx < 0);
            };
            int cnt = 0;
            sfor<N>([&](auto Q) {
                constexpr int q = Q;
                cnt += dir_ok(e.px[base + q] - x0, e.py[base + q] - y0) ? 1 : 0;
            });
            if (cnt > 0) {
                int pick = rs.choice(cnt);
                sfor<N>([&](auto Q) {
                    constexpr int q = Q;
                    if (dir_ok(e.px[base + q] - x0, e.py[base + q] - y0)) {
                        if (pick == 0) t = q;
                        --pick;
                    }
                });
            }
        }
        tx = 0.0;
        ty = 0.0;
        sfor<N>([&](auto Q) {
            constexpr int q = Q;
            if (q == t) {
                tx = e.px[base + q];
                ty = e.py[base + q];
            }
        });
    }
}

// ---------------------------------------------------------------------------
// Futbol.step (envs_v1/futbol_env.py:427-483) + DummyVecEnv auto-reset
template <int N, typename OT>
__global__ void __launch_bounds__(64) v1_step_kernel(const V1Params* __restrict__ P, V1Ptrs st,
                                                     const uint8_t* __restrict__ actions, OT* __restrict__ obs,
                                                     OT* __restrict__ reward, uint8_t* __restrict__ done_out,
                                                     OT* __restrict__ term_obs)
{
    using S = V1Shape<N>;
    constexpr int BL = S::BALL;
    __shared__ Scratch<N> sh;
    const int env = blockIdx.x * 64 + threadIdx.x;
    const int B = P->B;
    if (env >= B) return;
    const Lane<N> L{&sh, st.spill, st.ckey, st.cjn, (int)threadIdx.x, env, B};
    Env<N> e;
    load_env<N>(st, env, B, e);
    const double W = P->W, H = P->H;

    const uint32_t ev = e.meta.event();
    e.meta.set_event(ev + 1);
    Stream rs(P->seed, P->env_base + (uint32_t)env, ev, 0);

    // actions: left team from HBM, right team = action_space.sample() (:306-307, :429)
    int arrow[2 * N], key[2 * N];
    int bad = 0;
    sfor<2 * N>([&](auto I) {
        constexpr int i = I;
        int a = actions[(size_t)env * (2 * N) + i];
        bad += a > 4;
        a = a > 4 ? 4 : a;
        if constexpr (i & 1) key[i >> 1] = a; else arrow[i >> 1] = a;
    });
    sfor<2 * N>([&](auto I) {
        constexpr int i = I;
        const int a = rs.choice(5);
        if constexpr (i & 1) key[N + (i >> 1)] = a; else arrow[N + (i >> 1)] = a;
    });
    if (bad) atomicAdd(st.invalid, (unsigned long long)bad);

    // _ball_to_team_distance_arr(team_A), ball_init (:433-435)
    double d0[N];
    sfor<N>([&](auto I) {
        constexpr int i = I;
        const double dx = e.px[i] - e.px[BL], dy = e.py[i] - e.py[BL];
        d0[i] = sqrt(dx * dx + dy * dy);
    });
    const double bix = e.px[BL], biy = e.py[BL];

    // positions do not change during the action loop: one contact test per player
    bool touch[2 * N];
    sfor<2 * N>([&](auto K) {
        constexpr int k = K;
        touch[k] = cc_hit(e.px[BL], e.py[BL], kBallR, e.px[k], e.py[k], kPlayerR);
    });

    // _process_action per player, then owner update (:309-422, :447-453)
    uint32_t owner = e.meta.owner();
    sfor<2 * N>([&](auto K) {
        constexpr int k = K;
        constexpr int side = k < N ? 0 : 1;
        const int ar = arrow[k], ky = key[k];
        const int fx = ar == 2 ? 1 : (ar == 4 ? -1 : 0);
        const int fy = ar == 1 ? 1 : (ar == 3 ? -1 : 0);
        if (ky <= 1) {  // noop / dash: impulse 20 / 40, then _ball_move_with_player
            const int f = ky == 0 ? 20 : 40;
            e.vx[k] = e.vx[k] + (double)(f * fx) * kPlayerMinv;
            e.vy[k] = e.vy[k] + (double)(f * fy) * kPlayerMinv;
            if (touch[k]) {
                e.vx[BL] = e.vx[k];
                e.vy[BL] = e.vy[k];
            }
        } else if (ky == 2) {  // shoot
            if (touch[k]) {
                const double gx = side == 0 ? W : 0.0, gy = H / 2;
                const double dx = gx - e.px[BL], dy = gy - e.py[BL];
                const double mag = sqrt(dx * dx + dy * dy);
                const double fbx = 120.0 * dx / mag, fby = 120.0 * dy / mag;
                e.vx[BL] = e.vx[BL] / 2;
                e.vy[BL] = e.vy[BL] / 2;
                owner = side;
                e.vx[BL] = e.vx[BL] + fbx * kBallMinv;
                e.vy[BL] = e.vy[BL] + fby * kBallMinv;
            }
        } else if (ky == 3) {  // press: only without ball and without arrow
            if (!touch[k] && ar == 0) {
                const double dx = e.px[BL] - e.px[k], dy = e.py[BL] - e.py[k];
                const double mag = sqrt(dx * dx + dy * dy);
                e.vx[k] = e.vx[k] + (40.0 * dx / mag) * kPlayerMinv;
                e.vy[k] = e.vy[k] + (40.0 * dy / mag) * kPlayerMinv;
            }
        } else {  // pass
            if (touch[k]) {
                double tx, ty;
                pass_target<N, side, k - side * N>(e, rs, ar, tx, ty);
                const double dx = tx - e.px[BL], dy = ty - e.py[BL];
                const double mag = sqrt(dx * dx + dy * dy);
                const double fbx = 100.0 * dx / mag, fby = 100.0 * dy / mag;
                e.vx[BL] = e.vx[BL] / 10;
                e.vy[BL] = e.vy[BL] / 10;
                owner = side;
                e.vx[BL] = e.vx[BL] + fbx * kBallMinv;
                e.vy[BL] = e.vy[BL] + fby * kBallMinv;
            }
        }
        if (touch[k]) owner = side;
    });

    // check_and_fix_out_bounds (:247-287), before physics
    bool out = false;
    if (!far_from_segments(e.px[BL], e.py[BL], 2.0, W, H)) {
        int w = -1;
        for (int s = 0; s < 6; ++s)
            if (w < 0 && cs_hit(e.px[BL], e.py[BL], kBallR, P->sax[s], P->say[s], P->sbx[s], P->sby[s])) w = s;
        if (w >= 0) {
            out = true;
            const double bx0 = e.px[BL], by0 = e.py[BL];
            double dbx = 0, dby = 0, dpx = 0, dpy = 0;
            if (w <= 1) { dbx = 3.5; dpx = 1; }
            else if (w == 3 || w == 4) { dbx = -3.5; dpx = -1; }
            else if (w == 2) { dby = -3.5; dpy = -1; }
            else { dby = 3.5; dpy = 1; }
            e.px[BL] = bx0 + dbx;
            e.py[BL] = by0 + dby;
            e.vx[BL] = 0.0;
            e.vy[BL] = 0.0;
            int pick;
            if (owner == 1) { pick = rs.choice(N); owner = 0; }
            else { pick = N + rs.choice(N); owner = 1; }
            sfor<2 * N>([&](auto Q) {
                constexpr int q = Q;
                if (q == pick) {
                    e.px[q] = bx0 + dpx;
                    e.py[q] = by0 + dpy;
                    e.vx[q] = 0.0;
                    e.vy[q] = 0.0;
                }
            });
        }
    }
    e.meta.set_owner(owner);

    // Up to three cpSpaceSteps per call, through ONE inlined call site:
    //   phase 0: space.step(TIME_STEP) of this step            (:459)
    //   phase 1: _position_to_initial after a goal, step(1e-4) (:474, :129-144)
    //   phase 2: DummyVecEnv auto-reset -> reset(), step(1e-4) (:146-150)
    double r = 0.0, ret = 0.0;
    bool goal = false, done = false;
    for (int ph = 0; ph < 3; ++ph) {
        if (ph == 1 && !goal) continue;
        if (ph == 2 && !(done && P->auto_reset)) continue;
        if (ph == 1) position_to_initial<N>(P, e);
        if (ph == 2) {
            if (term_obs) write_obs<N, OT>(e, term_obs + (size_t)env * (4 * S::Nb));
            st.stat_ret[env] = st.stat_ret[env] + ret;
            st.stat_cnt[env] = st.stat_cnt[env] + 1;
            ret = 0.0;
            const uint32_t ev2 = e.meta.event();
            e.meta.set_event(ev2 + 1);
            rs = Stream(P->seed, P->env_base + (uint32_t)env, ev2, 0);
            e.meta.set_owner((uint32_t)rs.choice(2));
            e.meta.set_steps(0);
            position_to_initial<N>(P, e);
        }
        space_step<N>(P, L, e, ph == 0 ? 2 : 1);
        if (ph == 0) {
            if (!out) {  // get_team_reward + get_ball_reward (:493-515)
                double mx = 0.0;
                sfor<N>([&](auto I) {
                    constexpr int i = I;
                    const double dx = e.px[i] - e.px[BL], dy = e.py[i] - e.py[BL];
                    const double diff = d0[i] - sqrt(dx * dx + dy * dy);
                    if constexpr (N == 5) {
                        if constexpr (i == 3) mx = diff;
                        if constexpr (i == 4) mx = diff > mx ? diff : mx;
                    } else {
                        if (i == 0 || diff > mx) mx = diff;
                    }
                });
                r = r + mx * 10;
                const double gx = W, gy = H / 2;
                const double ax_ = e.px[BL] - gx, ay_ = e.py[BL] - gy;
                const double ix_ = bix - gx, iy_ = biy - gy;
                r = r + (sqrt(ix_ * ix_ + iy_ * iy_) - sqrt(ax_ * ax_ + ay_ * ay_)) * 10;
            }
            // ball_contact_goal (:291-296); a goal restarts from formation, the episode goes on
            if (!far_from_segments(e.px[BL], e.py[BL], 2.0, W, H)) {
                for (int s = 6; s < 12; ++s)
                    goal = goal || cs_hit(e.px[BL], e.py[BL], kBallR, P->sax[s], P->say[s], P->sbx[s], P->sby[s]);
            }
            if (goal) r = r + (e.px[BL] > W - 2 ? 1000.0 : -1000.0);
            // current_time += 0.1; done = current_time > total_time
            uint32_t steps = e.meta.steps() + 1;
            steps = steps > (uint32_t)kMaxSteps ? (uint32_t)kMaxSteps : steps;  // saturate (no auto-reset)
            e.meta.set_steps(steps);
            done = (int)steps >= P->K_done;
            ret = st.ep_ret[env] + r;
            if (done && !P->auto_reset) {
                if ((int)steps == P->K_done) {
                    st.stat_ret[env] = st.stat_ret[env] + ret;
                    st.stat_cnt[env] = st.stat_cnt[env] + 1;
                }
                ret = 0.0;
            }
        } else if (ph == 1) {
            e.meta.set_owner((uint32_t)rs.choice(2));  // random.choice(["left","right"]) (:475)
        }
    }
    write_obs<N, OT>(e, obs + (size_t)env * (4 * S::Nb));
    st.ep_ret[env] = ret;
    reward[env] = (OT)r;
    done_out[env] = done ? 1 : 0;
    store_env<N>(st, env, B, e);
    if (env == 0) *st.act_step += 1;  // stream-ordered after this step's fill_actions
}

// futbol_create (init=1: Futbol.__init__, which ends in reset()) / futbol_reset (masked)
template <int N, typename OT>
__global__ void __launch_bounds__(64) v1_reset_kernel(const V1Params* __restrict__ P, V1Ptrs st,
                                                      const uint8_t* __restrict__ mask, OT* __restrict__ obs,
                                                      int init)
{
    using S = V1Shape<N>;
    __shared__ Scratch<N> sh;
    const int env = blockIdx.x * 64 + threadIdx.x;
    const int B = P->B;
    if (env >= B) return;
    if (mask && !mask[env]) return;
    const Lane<N> L{&sh, st.spill, st.ckey, st.cjn, (int)threadIdx.x, env, B};
    Env<N> e;
    if (init) {
        sfor<S::Nb>([&](auto K) {
            constexpr int k = K;
            e.px[k] = P->fx[k];
            e.py[k] = P->fy[k];
            e.vx[k] = e.vy[k] = e.bx[k] = e.by[k] = 0.0;
        });
        e.meta.w = 0;
        st.stat_ret[env] = 0.0;
        st.stat_cnt[env] = 0;
    } else {
        load_env<N>(st, env, B, e);
    }
    st.ep_ret[env] = 0.0;
    do_reset<N>(P, L, e);
    if (obs) write_obs<N, OT>(e, obs + (size_t)env * (4 * S::Nb));
    store_env<N>(st, env, B, e);
}

}  // namespace futbol
