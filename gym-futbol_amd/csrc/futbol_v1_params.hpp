// futbol_v1_params.hpp -- the envs_v1 per-context constants (V1Params), built by one
// constexpr function used both by the C ABI at futbol_create (any width/height) and,
// at compile time, for the registered ids' default field (105 x 68): the step kernel
// is instantiated twice, and the default-field instance sees every geometry and
// physics constant as an immediate.  The host picks that instance only when the
// runtime-built parameters are bit-identical to the compile-time ones.
#pragma once
#include <stdint.h>
#include "futbol_kernels.hpp"

namespace futbol {

// Team._create_pos_array (team.py:52-112): formation of player k of `side`
constexpr void v1_formation(int N, double W, double H, int side, int k, double& x, double& y)
{
    if (N <= 3) {
        x = side == 0 ? W * 0.25 : W * 0.75;
        y = (H / (double)(N + 1)) * (double)(k + 1);
    } else if (N <= 6) {
        if (k < 3) {
            x = side == 0 ? (W * 1) / 6 : (W * 5) / 6;
            y = (H / 4.0) * (double)(k + 1);
        } else {
            x = side == 0 ? (W * 2) / 6 : (W * 4) / 6;
            y = (H / (double)(N - 3 + 1)) * (double)(k - 3 + 1);
        }
    } else {
        if (k < 4) {
            x = side == 0 ? (W * 1) / 8 : (W * 7) / 8;
            y = (H / 5.0) * (double)(k + 1);
        } else if (k < 7) {
            x = side == 0 ? (W * 2) / 8 : (W * 6) / 8;
            y = (H / 4.0) * (double)(k - 4 + 1);
        } else {
            x = side == 0 ? (W * 3) / 8 : (W * 5) / 8;
            y = (H / (double)(N - 7 + 1)) * (double)(k - 7 + 1);
        }
    }
}

// Values that need libm / a search, computed by the caller:
//   damp[i] = pow(0.95, dt_i), biasc[i] = 1 - pow(pow((double)0.9f, 60), dt_i), i = 1 (1e-4), 2 (0.1)
//   clamp2_* = largest s with RN(sqrt(s)) <= vmax
struct V1Pow {
    double damp1, damp2, biasc1, biasc2, clamp2_player, clamp2_ball;
};

// glibc 2.35 values of the above (checked against the runtime computation at futbol_create)
constexpr V1Pow kV1PowGlibc = {0x1.ffff53e38235p-1, 0x1.fd6168eb56e59p-1, 0x1.4b54b3d2fa4p-11,
                               0x1.dfcdf3e02c8a4p-2, 0x1.9000000000001p+6, 0x1.388p+9};

// Geometry and physics constants; the runtime fields (seed, env_base, B, K_done,
// auto_reset) are left 0 and filled by the caller.
constexpr V1Params v1_params_geometry(int N, double W, double H, const V1Pow& pw)
{
    V1Params p{};
    const double G = 20.0;  // GOAL_SIZE (envs_v1/futbol_env.py:21)
    p.W = W;
    p.H = H;
    const double lo = H / 2 - G / 2, hi = H / 2 + G / 2;
    // _setup_walls (envs_v1/futbol_env.py:182-234): 6 walls then 6 goal-box segments
    const double seg[12][4] = {{0, 0, 0, lo},          {0, hi, 0, H},        {0, H, W, H},
                               {W, 0, W, lo},          {W, hi, W, H},        {0, 0, W, 0},
                               {-2, lo, -2, hi},       {-2, lo, 0, lo},      {-2, hi, 0, hi},
                               {W + 2, lo, W + 2, hi}, {W, lo, W + 2, lo},   {W, hi, W + 2, hi}};
    for (int s = 0; s < 12; ++s) {
        p.sax[s] = seg[s][0];
        p.say[s] = seg[s][1];
        p.sbx[s] = seg[s][2];
        p.sby[s] = seg[s][3];
        // cpSegmentShapeCacheData: bb = (min - r, ..., max + r), r = 1
        const double l = seg[s][0] < seg[s][2] ? seg[s][0] : seg[s][2];
        const double r = seg[s][0] < seg[s][2] ? seg[s][2] : seg[s][0];
        const double b = seg[s][1] < seg[s][3] ? seg[s][1] : seg[s][3];
        const double t = seg[s][1] < seg[s][3] ? seg[s][3] : seg[s][1];
        p.sl[s] = l - 1.0;
        p.sb[s] = b - 1.0;
        p.sr[s] = r + 1.0;
        p.st[s] = t + 1.0;
        const double sdx = seg[s][2] - seg[s][0], sdy = seg[s][3] - seg[s][1];
        p.L2[s] = sdx * sdx + sdy * sdy;
        p.rL2[s] = 1.0 / p.L2[s];
    }
    // distinct BB bounds, segment by segment as used by the kernel's candidate test
    BBT& T = p.bbt;
    T.r1 = p.sr[0]; T.rW1 = p.sr[2]; T.rm1 = p.sr[6]; T.rW3 = p.sr[9];
    T.lm1 = p.sl[0]; T.lW1 = p.sl[3]; T.lm3 = p.sl[6]; T.lWp1 = p.sl[9];
    T.tlo = p.st[0]; T.tH = p.st[1]; T.t1 = p.st[5]; T.thi = p.st[6];
    T.bm1 = p.sb[0]; T.bhi = p.sb[1]; T.bH = p.sb[2]; T.blo = p.sb[6];
    for (int side = 0; side < 2; ++side)
        for (int k = 0; k < N; ++k) v1_formation(N, W, H, side, k, p.fx[side * N + k], p.fy[side * N + k]);
    p.fx[2 * N] = W * 0.5;  // Ball(width*0.5, height*0.5) (envs_v1/futbol_env.py:122,135)
    p.fy[2 * N] = H * 0.5;
    // cpSpace defaults (Chipmunk 7 cpSpaceInit): collisionSlop 0.1f; damping 0.95
    // (envs_v1/futbol_env.py:99); dt 0.1 (TIME_STEP) and 1e-4 (_position_to_initial)
    p.dtv[0] = 0.0;
    p.dtv[1] = 0.0001;
    p.dtv[2] = 0.1;
    p.damp[1] = pw.damp1;
    p.damp[2] = pw.damp2;
    p.biasc[1] = pw.biasc1;
    p.biasc[2] = pw.biasc2;
    p.rdt[1] = 1.0 / p.dtv[1];
    p.rdt[2] = 1.0 / p.dtv[2];
    p.slop = (double)0.1f;
    p.clamp2_player = pw.clamp2_player;
    p.clamp2_ball = pw.clamp2_ball;
    // The reset micro-step (space.step(1e-4) right after _position_to_initial) moves body k from
    // its formation point by v_bias_k * 1e-4 and nothing else (v = 0).  clear = a lower bound of
    // every surface gap at formation -- body pairs and body-segment pairs, from per-axis distances
    // (Euclidean >= each axis's) -- so a step in which every |v_bias| component stays below
    // clear / 4 / 1e-4 moves each body by less than clear / 2 (sqrt(2) / 4 < 1 / 2) and provably
    // collides nothing.  0 (fast path off) when the formation itself is crowded.
    const int Nb = 2 * N + 1;
    double clear = 1e300;
    for (int i = 0; i < Nb; ++i) {
        const double ri = i == 2 * N ? 1.0 : 1.5;  // Ball / Player radius
        for (int j = i + 1; j < Nb; ++j) {
            const double rj = j == 2 * N ? 1.0 : 1.5;
            const double ax = p.fx[i] < p.fx[j] ? p.fx[j] - p.fx[i] : p.fx[i] - p.fx[j];
            const double ay = p.fy[i] < p.fy[j] ? p.fy[j] - p.fy[i] : p.fy[i] - p.fy[j];
            const double g = (ax > ay ? ax : ay) - (ri + rj);
            clear = g < clear ? g : clear;
        }
        for (int s = 0; s < 12; ++s) {
            const double l = p.sl[s] + 1.0, r = p.sr[s] - 1.0, b = p.sb[s] + 1.0, t = p.st[s] - 1.0;
            const double ax = p.fx[i] < l ? l - p.fx[i] : (p.fx[i] > r ? p.fx[i] - r : 0.0);
            const double ay = p.fy[i] < b ? b - p.fy[i] : (p.fy[i] > t ? p.fy[i] - t : 0.0);
            const double g = (ax > ay ? ax : ay) - (ri + 1.0);  // segment radius 1
            clear = g < clear ? g : clear;
        }
    }
    p.form_vb = clear > 1.0 ? clear * 0.25 * 1e4 : 0.0;
    return p;
}

template <int N>
struct V1Default {
    static constexpr double W = 105.0, H = 68.0;  // WIDTH, HEIGHT (envs_v1/futbol_env.py:19-20)
};

template <int N>
constexpr V1Params v1_default_geometry()
{
    return v1_params_geometry(N, V1Default<N>::W, V1Default<N>::H, kV1PowGlibc);
}

}  // namespace futbol
