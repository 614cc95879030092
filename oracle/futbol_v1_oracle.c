/*
 * futbol_v1_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never shipped).
 *
 * A literal, scalar, fp64 restatement of one envs_v1 `Futbol` env
 * (gym_futbol/envs_v1/futbol_env.py, team.py, ball.py, player.py) together with
 * the part of Chipmunk2D 7.0.x's cpSpaceStep that pymunk 5.6.0 runs for it.
 *
 * PARITY VS PYMUNK: UNPINNED.  pymunk/Chipmunk are absent from this machine and
 * cannot be installed.  The Chipmunk steps below are restated
 * from Chipmunk 7.0.x's published sources (cpSpaceStep.c, cpArbiter.c,
 * cpCollision.c, cpBody.c, cpShape.c) as summarised in SURVEY.md Appendix A.5,
 * with its deliberate simplifications:
 *   - angular DOFs dropped (A.6): the only torques come from contact lever arms
 *     that are collinear with the normal up to rounding (~1e-16 of the impulse);
 *   - canonical arbiter order (D.1): every circle-segment pair (body i ascending,
 *     segments 0..11), then every circle pair (i, j>i) row-major.  Chipmunk's
 *     BBTree order is not reproducible.
 * Pinned instead by the hand-derived KATs in tests/test_oracle_v1.py.
 *
 * This file is deliberately written as "one env, plain structs, dense arbiter
 * table indexed by pair id, absolute stamps and arbiter states", i.e. the way
 * Chipmunk keeps it -- unlike the HIP kernel (SoA over envs, compact age-coded
 * contact cache), so the parity tests compare two independent codings.
 */
#include <math.h>
#include <string.h>
#include <stdint.h>
#include "futbol_oracle.h"
#include "oracle_math.h"
#include "oracle_rng.h"

/* ---- module constants, envs_v1/futbol_env.py:19-50 ---- */
#define GOAL_SIZE 20.0
#define TIME_STEP 0.1
#define BALL_MAX_VELOCITY 25.0
#define PLAYER_MAX_VELOCITY 10.0
#define BALL_WEIGHT 10.0
#define PLAYER_WEIGHT 20
#define PLAYER_FORCE_LIMIT 40
#define BALL_FORCE_LIMIT 120
#define PLAYER_RADIUS 1.5 /* player.py:7 */
#define BALL_RADIUS 1.0   /* ball.py:7 */
#define SEG_RADIUS 1.0    /* futbol_env.py:187.. (last ctor arg) */

/* Python's float `x**2`: libm pow in the faithful build (see oracle_math.h) */

/* Diagnostic (tests/sq_divergence.py): the faithful build squares with x*x at the call sites set in
   this mask instead of pow -- bit 0 get_vec in _process_action (state), bit 1 limit_velocity's
   Vec2d.length (state), bit 2 the reward's get_vec / _ball_to_team_distance_arr (reward only) --
   to find which site's difference reaches a discrete outcome.  0 (default): every site faithful. */
#ifdef ORACLE_PORTABLE
/* the kernels: glibc's pow(x, 2) restated at the two sites that feed the state (bits 0, 1), x*x at
   the reward's (bit 2: the reward never feeds back into the state, and its squares' last-bit
   differences stay below 1e-11) */
static double SQS(double x, int bit) { return bit == 2 ? x * x : ORC_SQ(x); }
#else
static double SQ(double x) { return ORC_SQ_V1(x); }
static int orc_sq_xx_mask = 0;
static double SQS(double x, int bit) { return (orc_sq_xx_mask >> bit) & 1 ? x * x : SQ(x); }
#endif
void orc_v1_set_sq_mask(int mask)
{
#ifndef ORACLE_PORTABLE
    orc_sq_xx_mask = mask;
#else
    (void)mask;
#endif
}

/* get_vec, envs_v1/futbol_env.py:56-59: vector from o to t and its magnitude */
static double get_vec_site(double tx, double ty, double ox, double oy, double *vx, double *vy, int bit)
{
    *vx = tx - ox;
    *vy = ty - oy;
    return sqrt(SQS(*vx, bit) + SQS(*vy, bit));
}
#define get_vec(tx, ty, ox, oy, vx, vy) get_vec_site(tx, ty, ox, oy, vx, vy, 0)

static void seg_endpoints(const OrcV1 *e, int s, double *ax, double *ay, double *bx, double *by)
{
    /* _setup_walls, envs_v1/futbol_env.py:182-234 */
    const double W = e->width, H = e->height;
    const double lo = H / 2 - GOAL_SIZE / 2, hi = H / 2 + GOAL_SIZE / 2;
    switch (s) {
    case 0: *ax = 0; *ay = 0; *bx = 0; *by = lo; break;
    case 1: *ax = 0; *ay = hi; *bx = 0; *by = H; break;
    case 2: *ax = 0; *ay = H; *bx = W; *by = H; break;
    case 3: *ax = W; *ay = 0; *bx = W; *by = lo; break;
    case 4: *ax = W; *ay = hi; *bx = W; *by = H; break;
    case 5: *ax = 0; *ay = 0; *bx = W; *by = 0; break;
    case 6: *ax = -2; *ay = lo; *bx = -2; *by = hi; break;
    case 7: *ax = -2; *ay = lo; *bx = 0; *by = lo; break;
    case 8: *ax = -2; *ay = hi; *bx = 0; *by = hi; break;
    case 9: *ax = W + 2; *ay = lo; *bx = W + 2; *by = hi; break;
    case 10: *ax = W; *ay = lo; *bx = W + 2; *by = lo; break;
    default: *ax = W; *ay = hi; *bx = W + 2; *by = hi; break;
    }
}

static double body_radius(const OrcV1 *e, int k) { return k == 2 * e->N ? BALL_RADIUS : PLAYER_RADIUS; }
static double body_minv(const OrcV1 *e, int k) { return k == 2 * e->N ? 1.0 / BALL_WEIGHT : 1.0 / (double)PLAYER_WEIGHT; }
static double body_vmax(const OrcV1 *e, int k) { return k == 2 * e->N ? BALL_MAX_VELOCITY : PLAYER_MAX_VELOCITY; }
static double body_e(const OrcV1 *e, int k) { (void)e; (void)k; return 0.2; } /* team.py:12,30; futbol_env.py:125 */

/* ---- Chipmunk narrowphase (cpCollision.c CircleToCircle / CircleToSegment) ---- */
static int circle_circle(double ax, double ay, double ra, double bx, double by, double rb,
                         double *nx, double *ny, double *p1x, double *p1y, double *p2x, double *p2y)
{
    double mindist = ra + rb;
    double dx = bx - ax, dy = by - ay;
    double distsq = dx * dx + dy * dy;
    if (!(distsq < mindist * mindist)) return 0;
    double dist = sqrt(distsq);
    if (dist != 0.0) { double inv = 1.0 / dist; *nx = dx * inv; *ny = dy * inv; }
    else { *nx = 1.0; *ny = 0.0; }
    *p1x = ax + *nx * ra; *p1y = ay + *ny * ra;
    *p2x = bx + *nx * (-rb); *p2y = by + *ny * (-rb);
    return 1;
}

static int circle_segment(double cx, double cy, double rc, double sax, double say, double sbx, double sby,
                          double rs, double *nx, double *ny, double *p1x, double *p1y, double *p2x, double *p2y)
{
    double sdx = sbx - sax, sdy = sby - say;
    double t = (sdx * (cx - sax) + sdy * (cy - say)) / (sdx * sdx + sdy * sdy);
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t); /* cpfclamp01 */
    double qx = sax + sdx * t, qy = say + sdy * t;
    double mindist = rc + rs;
    double dx = qx - cx, dy = qy - cy;
    double distsq = dx * dx + dy * dy;
    if (!(distsq < mindist * mindist)) return 0;
    double dist = sqrt(distsq);
    if (dist != 0.0) { double inv = 1.0 / dist; *nx = dx * inv; *ny = dy * inv; }
    else {
        /* segment->tn: normalized perp of (b-a) */
        double len = sqrt(sdx * sdx + sdy * sdy);
        double inv = 1.0 / len;
        *nx = -sdy * inv; *ny = sdx * inv;
    }
    *p1x = cx + *nx * rc; *p1y = cy + *ny * rc;
    *p2x = qx + *nx * (-rs); *p2y = qy + *ny * (-rs);
    return 1;
}

/* cpShapesCollide(ball, player).points != []  (ball.py:39-40) */
static int ball_touches(const OrcV1 *e, int k)
{
    double nx, ny, a, b, c, d;
    int ball = 2 * e->N;
    return circle_circle(e->px[ball], e->py[ball], BALL_RADIUS, e->px[k], e->py[k], PLAYER_RADIUS,
                         &nx, &ny, &a, &b, &c, &d);
}

static int ball_touches_seg(const OrcV1 *e, int s)
{
    double ax, ay, bx, by, nx, ny, a, b, c, d;
    int ball = 2 * e->N;
    seg_endpoints(e, s, &ax, &ay, &bx, &by);
    return circle_segment(e->px[ball], e->py[ball], BALL_RADIUS, ax, ay, bx, by, SEG_RADIUS,
                          &nx, &ny, &a, &b, &c, &d);
}

/* cpBodyApplyImpulseAtLocalPoint at (0,0): v += j * m_inv (ball.py:33-35, player.py:34-36) */
static void apply_impulse(OrcV1 *e, int k, double jx, double jy)
{
    double m = body_minv(e, k);
    e->vx[k] = e->vx[k] + jx * m;
    e->vy[k] = e->vy[k] + jy * m;
}

/* ---------------- cpSpaceStep (Chipmunk 7.0.x cpSpaceStep.c) ---------------- */
typedef struct {
    int a, b; /* body ids; b < 0: static segment (-1 - s) */
    int pair;
    double nx, ny, r1x, r1y, r2x, r2y;
    double nMass, bias, jBias, bounce, jnAcc, e;
} OrcContact;

static double bvx(const OrcV1 *e, int k) { return k < 0 ? 0.0 : e->vx[k]; }
static double bvy(const OrcV1 *e, int k) { return k < 0 ? 0.0 : e->vy[k]; }
static double bbx(const OrcV1 *e, int k) { return k < 0 ? 0.0 : e->bx[k]; }
static double bby(const OrcV1 *e, int k) { return k < 0 ? 0.0 : e->by[k]; }
static double bpx(const OrcV1 *e, int k) { return k < 0 ? 0.0 : e->px[k]; }
static double bpy(const OrcV1 *e, int k) { return k < 0 ? 0.0 : e->py[k]; }
static double bminv(const OrcV1 *e, int k) { return k < 0 ? 0.0 : body_minv(e, k); }


/* apply_impulses(a, b, r1, r2, j): a gets -j*m_inv_a, b gets +j*m_inv_b */
static void apply_impulses(OrcV1 *e, int a, int b, double jx, double jy)
{
    double ma = bminv(e, a), mb = bminv(e, b);
    if (a >= 0) { e->vx[a] = e->vx[a] + (-jx) * ma; e->vy[a] = e->vy[a] + (-jy) * ma; }
    if (b >= 0) { e->vx[b] = e->vx[b] + jx * mb; e->vy[b] = e->vy[b] + jy * mb; }
}
static void apply_bias_impulses(OrcV1 *e, int a, int b, double jx, double jy)
{
    double ma = bminv(e, a), mb = bminv(e, b);
    if (a >= 0) { e->bx[a] = e->bx[a] + (-jx) * ma; e->by[a] = e->by[a] + (-jy) * ma; }
    if (b >= 0) { e->bx[b] = e->bx[b] + jx * mb; e->by[b] = e->by[b] + jy * mb; }
}

static int bb_intersects(double al, double ab, double ar, double at, double bl, double bb, double br, double bt)
{
    return al <= br && bl <= ar && ab <= bt && bb <= at; /* cpBBIntersects */
}

static void collide_pair(OrcV1 *e, OrcContact *list, int *n, int a, int b, int pair,
                         double nx, double ny, double p1x, double p1y, double p2x, double p2y)
{
    /* cpSpaceCollideShapes + cpArbiterUpdate (cpSpaceStep.c / cpArbiter.c) */
    OrcContact *c = &list[(*n)++];
    c->a = a; c->b = b; c->pair = pair;
    c->nx = nx; c->ny = ny;
    c->r1x = p1x - bpx(e, a); c->r1y = p1y - bpy(e, a);
    c->r2x = p2x - bpx(e, b); c->r2y = p2y - bpy(e, b);
    if (!e->arb_exists[pair]) {
        /* cpArbiterInit: fresh arbiter, no old contacts -> jnAcc = 0 */
        e->arb_exists[pair] = 1;
        e->arb_state[pair] = ORC_ST_FIRST;
        e->arb_inlist[pair] = 0;
        e->arb_jn[pair] = 0.0;
        c->jnAcc = 0.0;
    } else {
        c->jnAcc = e->arb_jn[pair]; /* contact hash 0 matches: copy persistent jnAcc */
    }
    c->e = (b < 0) ? body_e(e, a) * 0.0 : body_e(e, a) * body_e(e, b);
    if (e->arb_state[pair] == ORC_ST_CACHED) e->arb_state[pair] = ORC_ST_FIRST;
    e->arb_stamp[pair] = e->stamp;
}

void orc_v1_space_step(OrcV1 *e, double dt)
{
    const int Nb = e->Nb;
    OrcContact list[ORC_MAXP];
    int n = 0;

    e->stamp++;
    double prev_dt = e->curr_dt;
    e->curr_dt = dt;
    for (int p = 0; p < e->P; ++p)
        if (e->arb_exists[p] && e->arb_inlist[p]) { e->arb_state[p] = ORC_ST_NORMAL; e->arb_inlist[p] = 0; }

    /* integrate positions: cpBodyUpdatePosition */
    for (int k = 0; k < Nb; ++k) {
        e->px[k] = e->px[k] + (e->vx[k] + e->bx[k]) * dt;
        e->py[k] = e->py[k] + (e->vy[k] + e->by[k]) * dt;
        e->bx[k] = 0.0; e->by[k] = 0.0;
    }

    /* collide, canonical order: all circle-segment pairs (body i ascending, segment
     * ascending), then all circle-circle pairs (i < j, row-major) */
    for (int i = 0; i < Nb; ++i) {
        double ri = body_radius(e, i);
        double cl = e->px[i] - ri, cb = e->py[i] - ri, cr = e->px[i] + ri, ct = e->py[i] + ri;
        for (int s = 0; s < ORC_NSEG; ++s) {
            double ax, ay, bx, by;
            seg_endpoints(e, s, &ax, &ay, &bx, &by);
            double l = ax < bx ? ax : bx, r = ax < bx ? bx : ax;
            double bo = ay < by ? ay : by, t = ay < by ? by : ay;
            if (!bb_intersects(cl, cb, cr, ct, l - SEG_RADIUS, bo - SEG_RADIUS, r + SEG_RADIUS, t + SEG_RADIUS)) continue;
            double nx, ny, p1x, p1y, p2x, p2y;
            if (circle_segment(e->px[i], e->py[i], ri, ax, ay, bx, by, SEG_RADIUS, &nx, &ny, &p1x, &p1y, &p2x, &p2y))
                collide_pair(e, list, &n, i, -1 - s, i * ORC_NSEG + s, nx, ny, p1x, p1y, p2x, p2y);
        }
    }
    for (int i = 0; i < Nb; ++i) {
        double ri = body_radius(e, i);
        double cl = e->px[i] - ri, cb = e->py[i] - ri, cr = e->px[i] + ri, ct = e->py[i] + ri;
        for (int j = i + 1; j < Nb; ++j) {
            double rj = body_radius(e, j);
            if (!bb_intersects(cl, cb, cr, ct, e->px[j] - rj, e->py[j] - rj, e->px[j] + rj, e->py[j] + rj)) continue;
            double nx, ny, p1x, p1y, p2x, p2y;
            if (circle_circle(e->px[i], e->py[i], ri, e->px[j], e->py[j], rj, &nx, &ny, &p1x, &p1y, &p2x, &p2y)) {
                /* pair index of (i,j), i<j, in row-major upper triangle */
                int idx = i * Nb - i * (i + 1) / 2 + (j - i - 1);
                collide_pair(e, list, &n, i, j, Nb * ORC_NSEG + idx, nx, ny, p1x, p1y, p2x, p2y);
            }
        }
    }

    /* cpSpaceArbiterSetFilter over the cached arbiters */
    for (int p = 0; p < e->P; ++p) {
        if (!e->arb_exists[p]) continue;
        uint32_t ticks = e->stamp - e->arb_stamp[p];
        if (ticks >= 1 && e->arb_state[p] != ORC_ST_CACHED) e->arb_state[p] = ORC_ST_CACHED;
        if (ticks >= 3) { e->arb_exists[p] = 0; e->arb_inlist[p] = 0; }
    }

    /* cpArbiterPreStep */
    const double slop = (double)0.1f;                              /* collisionSlop = 0.1f */
    const double collisionBias = pow((double)(1.0f - 0.1f), 60.0); /* cpfpow(1.0f - 0.1f, 60.0f) */
    const double biasCoef = 1.0 - pow(collisionBias, dt);
    for (int c = 0; c < n; ++c) {
        OrcContact *k = &list[c];
        double bdx = bpx(e, k->b) - bpx(e, k->a), bdy = bpy(e, k->b) - bpy(e, k->a);
        k->nMass = 1.0 / (bminv(e, k->a) + bminv(e, k->b));
        double dist = ((k->r2x - k->r1x) + bdx) * k->nx + ((k->r2y - k->r1y) + bdy) * k->ny;
        double m = dist + slop;
        m = (0.0 < m) ? 0.0 : m; /* cpfmin(0.0f, dist + slop) */
        k->bias = -biasCoef * m / dt;
        k->jBias = 0.0;
        double rvx = bvx(e, k->b) - bvx(e, k->a), rvy = bvy(e, k->b) - bvy(e, k->a);
        k->bounce = (rvx * k->nx + rvy * k->ny) * k->e;
    }

    /* integrate velocities: cpBodyUpdateVelocity then limit_velocity (ball.py:49-56, player.py:45-52) */
    const double damping = pow(0.95, dt);
    for (int k = 0; k < Nb; ++k) {
        e->vx[k] = e->vx[k] * damping + 0.0 * dt;
        e->vy[k] = e->vy[k] * damping + 0.0 * dt;
        double l = sqrt(SQS(e->vx[k], 1) + SQS(e->vy[k], 1)); /* Vec2d.length */
        double vmax = body_vmax(e, k);
        if (l > vmax) {
            double scale = vmax / l;
            e->vx[k] = e->vx[k] * scale;
            e->vy[k] = e->vy[k] * scale;
        }
    }

    /* cpArbiterApplyCachedImpulse */
    const double dt_coef = (prev_dt == 0.0) ? 0.0 : dt / prev_dt;
    for (int c = 0; c < n; ++c) {
        OrcContact *k = &list[c];
        if (e->arb_state[k->pair] == ORC_ST_FIRST) continue;
        double jx = (k->nx * k->jnAcc) * dt_coef, jy = (k->ny * k->jnAcc) * dt_coef;
        apply_impulses(e, k->a, k->b, jx, jy);
    }

    /* cpArbiterApplyImpulse x iterations (10) */
    for (int it = 0; it < 10; ++it) {
        for (int c = 0; c < n; ++c) {
            OrcContact *k = &list[c];
            double vbn = (bbx(e, k->b) - bbx(e, k->a)) * k->nx + (bby(e, k->b) - bby(e, k->a)) * k->ny;
            double vrn = (bvx(e, k->b) - bvx(e, k->a)) * k->nx + (bvy(e, k->b) - bvy(e, k->a)) * k->ny;
            double jbn = (k->bias - vbn) * k->nMass;
            double jbnOld = k->jBias;
            double t = jbnOld + jbn;
            k->jBias = t > 0.0 ? t : 0.0;
            double jn = -(k->bounce + vrn) * k->nMass;
            double jnOld = k->jnAcc;
            double u = jnOld + jn;
            k->jnAcc = u > 0.0 ? u : 0.0;
            double db = k->jBias - jbnOld;
            apply_bias_impulses(e, k->a, k->b, k->nx * db, k->ny * db);
            double dj = k->jnAcc - jnOld;
            apply_impulses(e, k->a, k->b, k->nx * dj, k->ny * dj);
        }
    }

    for (int c = 0; c < n; ++c) {
        e->arb_jn[list[c].pair] = list[c].jnAcc;
        e->arb_inlist[list[c].pair] = 1;
    }
}

/* ---------------- game logic ---------------- */
int orc_v1_obs_dim(int N) { return 4 * (2 * N + 1); }

void orc_v1_observe(const OrcV1 *e, double *obs)
{
    /* _get_observation, futbol_env.py:154-180; BALL/PLAYER_{avg,range}_arr, :39-50 */
    int ball = 2 * e->N;
    obs[0] = (e->px[ball] - 52.5) / 52.5;
    obs[1] = (e->py[ball] - 34.0) / 34.0;
    obs[2] = (e->vx[ball] - 0.0) / 25.0;
    obs[3] = (e->vy[ball] - 0.0) / 25.0;
    for (int k = 0; k < 2 * e->N; ++k) {
        obs[4 + 4 * k + 0] = (e->px[k] - 52.5) / 55.5;
        obs[4 + 4 * k + 1] = (e->py[k] - 34.0) / 34.0;
        obs[4 + 4 * k + 2] = (e->vx[k] - 0.0) / 10.0;
        obs[4 + 4 * k + 3] = (e->vy[k] - 0.0) / 10.0;
    }
}

/* Team._create_pos_array, team.py:52-112 (k = index inside the team) */
static void formation(const OrcV1 *e, int side, int k, double *x, double *y)
{
    const int N = e->N;
    const double W = e->width, H = e->height;
    if (N <= 3) {
        *x = side == 0 ? W * 0.25 : W * 0.75;
        *y = (H / (double)(N + 1)) * (double)(k + 1);
    } else if (N <= 6) {
        if (k < 3) { *x = side == 0 ? (W * 1) / 6 : (W * 5) / 6; *y = (H / 4.0) * (double)(k + 1); }
        else { *x = side == 0 ? (W * 2) / 6 : (W * 4) / 6; *y = (H / (double)(N - 3 + 1)) * (double)(k - 3 + 1); }
    } else {
        if (k < 4) { *x = side == 0 ? (W * 1) / 8 : (W * 7) / 8; *y = (H / 5.0) * (double)(k + 1); }
        else if (k < 7) { *x = side == 0 ? (W * 2) / 8 : (W * 6) / 8; *y = (H / 4.0) * (double)(k - 4 + 1); }
        else { *x = side == 0 ? (W * 3) / 8 : (W * 5) / 8; *y = (H / (double)(N - 7 + 1)) * (double)(k - 7 + 1); }
    }
}

/* _position_to_initial, futbol_env.py:129-144 */
static void position_to_initial(OrcV1 *e)
{
    for (int side = 0; side < 2; ++side)
        for (int k = 0; k < e->N; ++k) {
            int b = side * e->N + k;
            formation(e, side, k, &e->px[b], &e->py[b]);
            e->vx[b] = 0.0; e->vy[b] = 0.0;
        }
    int ball = 2 * e->N;
    e->px[ball] = e->width * 0.5; e->py[ball] = e->height * 0.5;
    e->vx[ball] = 0.0; e->vy[ball] = 0.0;
    orc_v1_space_step(e, 0.0001);
}

void orc_v1_init(OrcV1 *e, int N, double width, double height, double total_time, uint64_t seed, uint32_t env_id)
{
    memset(e, 0, sizeof(*e));
    e->N = N; e->Nb = 2 * N + 1;
    e->P = e->Nb * ORC_NSEG + e->Nb * (e->Nb - 1) / 2;
    e->width = width; e->height = height; e->total_time = total_time;
    e->seed = seed; e->env_id = env_id;
    /* bodies are created at formation / centre (team.py:24-31, futbol_env.py:122-125);
       cpSpace: stamp 0, curr_dt 0 */
    for (int side = 0; side < 2; ++side)
        for (int k = 0; k < N; ++k) formation(e, side, k, &e->px[side * N + k], &e->py[side * N + k]);
    e->px[2 * N] = width * 0.5; e->py[2 * N] = height * 0.5;
    orc_v1_reset(e, 0); /* Futbol.__init__ ends with self.reset(), futbol_env.py:127 */
}

/* Futbol.reset, futbol_env.py:146-150 */
void orc_v1_reset(OrcV1 *e, double *obs)
{
    OracleRng g = { e->seed, e->env_id, e->event++, 0, 0 };
    e->current_time = 0.0;
    e->owner = oracle_choice(&g, 2); /* random.choice(["left","right"]) */
    position_to_initial(e);
    if (obs) orc_v1_observe(e, obs);
}

/* Team.get_pass_target_teammate, team.py:136-180; returns body index */
static int pass_target(OrcV1 *e, OracleRng *g, int side, int k, int arrow)
{
    const int N = e->N;
    const int base = side * N;
    if (N == 1) return base + k;
    int cand[ORC_MAXN], nc = 0;
    for (int i = 0; i < N; ++i) if (i != k) cand[nc++] = i;
    int target = cand[oracle_choice(g, nc)];
    if (arrow != 0) {
        double pxk = e->px[base + k], pyk = e->py[base + k];
        nc = 0;
        for (int i = 0; i < N; ++i) {
            double mx = e->px[base + i] - pxk, my = e->py[base + i] - pyk;
            int ok = (arrow == 1 && my > 0) || (arrow == 2 && mx > 0) || (arrow == 3 && my < 0) || (arrow == 4 && mx < 0);
            if (ok) cand[nc++] = i;
        }
        if (nc > 0) target = cand[oracle_choice(g, nc)];
    }
    return base + target;
}

/* Futbol._process_action, futbol_env.py:309-422 */
static void process_action(OrcV1 *e, OracleRng *g, int k, int arrow, int key)
{
    const int ball = 2 * e->N;
    const int side = k < e->N ? 0 : 1;
    int fx = 0, fy = 0;
    switch (arrow) {
    case 1: fy = 1; break;
    case 2: fx = 1; break;
    case 3: fy = -1; break;
    case 4: fx = -1; break;
    default: break;
    }
    if (key == 0 || key == 1) {
        int f = key == 0 ? PLAYER_WEIGHT : PLAYER_FORCE_LIMIT;
        apply_impulse(e, k, (double)(f * fx), (double)(f * fy));
        if (ball_touches(e, k)) { e->vx[ball] = e->vx[k]; e->vy[ball] = e->vy[k]; } /* _ball_move_with_player */
    } else if (key == 2) {
        if (ball_touches(e, k)) {
            double gx = side == 0 ? e->width : 0.0, gy = e->height / 2;
            double dx, dy, mag = get_vec(gx, gy, e->px[ball], e->py[ball], &dx, &dy);
            double fbx = BALL_FORCE_LIMIT * dx / mag, fby = BALL_FORCE_LIMIT * dy / mag;
            e->vx[ball] = e->vx[ball] / 2; e->vy[ball] = e->vy[ball] / 2;
            e->owner = side;
            apply_impulse(e, ball, fbx, fby);
        }
    } else if (key == 3) {
        if (ball_touches(e, k)) {
        } else if (arrow == 0) {
            double dx, dy, mag = get_vec(e->px[ball], e->py[ball], e->px[k], e->py[k], &dx, &dy);
            apply_impulse(e, k, PLAYER_FORCE_LIMIT * dx / mag, PLAYER_FORCE_LIMIT * dy / mag);
        }
    } else if (key == 4) {
        if (ball_touches(e, k)) {
            int t = pass_target(e, g, side, k - side * e->N, arrow);
            double dx, dy, mag = get_vec(e->px[t], e->py[t], e->px[ball], e->py[ball], &dx, &dy);
            double fbx = (BALL_FORCE_LIMIT - 20) * dx / mag, fby = (BALL_FORCE_LIMIT - 20) * dy / mag;
            e->vx[ball] = e->vx[ball] / 10; e->vy[ball] = e->vy[ball] / 10;
            e->owner = side;
            apply_impulse(e, ball, fbx, fby);
        }
    }
}

/* check_and_fix_out_bounds, futbol_env.py:247-287 */
static int check_and_fix_out_bounds(OrcV1 *e, OracleRng *g)
{
    const int ball = 2 * e->N;
    int w = -1;
    for (int s = 0; s < 6; ++s) if (ball_touches_seg(e, s)) { w = s; break; }
    e->last_out_wall = w;
    e->last_out_pick = -1;
    if (w < 0) return 0;
    double bx = e->px[ball], by = e->py[ball];
    double dbx = 0, dby = 0, dpx = 0, dpy = 0;
    if (w == 1 || w == 0) { dbx = 3.5; dpx = 1; }
    else if (w == 3 || w == 4) { dbx = -3.5; dpx = -1; }
    else if (w == 2) { dby = -3.5; dpy = -1; }
    else { dby = 3.5; dpy = 1; }
    e->px[ball] = bx + dbx; e->py[ball] = by + dby;
    e->vx[ball] = 0.0; e->vy[ball] = 0.0;
    int pick;
    if (e->owner == 1) { pick = oracle_choice(g, e->N); e->owner = 0; }
    else { pick = e->N + oracle_choice(g, e->N); e->owner = 1; }
    e->px[pick] = bx + dpx; e->py[pick] = by + dpy;
    e->vx[pick] = 0.0; e->vy[pick] = 0.0;
    e->last_out_pick = pick;
    return 1;
}

/* _ball_to_team_distance_arr (team A), futbol_env.py:485-491 */
static void team_a_dist(const OrcV1 *e, double *d)
{
    const int ball = 2 * e->N;
    for (int i = 0; i < e->N; ++i)
        d[i] = sqrt(SQS(e->px[i] - e->px[ball], 2) + SQS(e->py[i] - e->py[ball], 2));
}

/* Futbol.step, futbol_env.py:427-483 */
int orc_v1_step(OrcV1 *e, const int32_t *left, double *obs, double *reward)
{
    const int N = e->N, ball = 2 * N;
    OracleRng g = { e->seed, e->env_id, e->event++, 0, 0 };
    int right[2 * ORC_MAXN];
    /* action_space.sample() (futbol_env.py:306-307, :429): 2N uniform integers in [0, 5), four per
       Philox block (RNG contract: DESIGN.md section 3) */
    oracle_words_choice(&g, 2 * N, 5, right);

    double d0[ORC_MAXN];
    team_a_dist(e, d0);
    double bix = e->px[ball], biy = e->py[ball];
    double r = 0.0;

    for (int k = 0; k < 2 * N; ++k) {
        const int32_t *a = k < N ? &left[2 * k] : &right[2 * (k - N)];
        process_action(e, &g, k, a[0], a[1]);
        if (ball_touches(e, k)) e->owner = k < N ? 0 : 1;
    }
    int out = check_and_fix_out_bounds(e, &g);
    orc_v1_space_step(e, TIME_STEP);
    double o[4 * ORC_MAXB];
    orc_v1_observe(e, o);

    if (!out) {
        double d1[ORC_MAXN], diff[ORC_MAXN];
        team_a_dist(e, d1);
        for (int i = 0; i < N; ++i) diff[i] = d0[i] - d1[i];
        double mx;
        if (N == 5) mx = diff[3] > diff[4] ? diff[3] : diff[4];   /* np.max([d[3], d[4]]) */
        else { mx = diff[0]; for (int i = 1; i < N; ++i) if (diff[i] > mx) mx = diff[i]; }
        r = r + mx * 10;
        double gx = e->width, gy = e->height / 2, t0, t1;
        double ma = get_vec_site(e->px[ball], e->py[ball], gx, gy, &t0, &t1, 2);
        double mi = get_vec_site(bix, biy, gx, gy, &t0, &t1, 2);
        r = r + (mi - ma) * 10;
    }
    int goal = 0;
    for (int s = 6; s < 12 && !goal; ++s) goal = ball_touches_seg(e, s);
    if (goal) {
        double bx = e->px[ball];
        r = r + (bx > e->width - 2 ? 1000.0 : -1000.0);
        position_to_initial(e);
        orc_v1_observe(e, o);
        e->owner = oracle_choice(&g, 2);
    }
    e->n_out += (uint32_t)out;
    e->n_goal += (uint32_t)goal;
    e->current_time = e->current_time + TIME_STEP;
    int done = e->current_time > e->total_time;
    if (obs) memcpy(obs, o, sizeof(double) * 4 * e->Nb);
    if (reward) *reward = r;
    return done;
}

void orc_v1_vec_step(OrcV1 *envs, int B, const int32_t *actions, double *obs, double *reward,
                     uint8_t *done, double *terminal_obs, int nthreads)
{
    if (B <= 0) return;
    const int N = envs[0].N, od = orc_v1_obs_dim(N);
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
    for (int i = 0; i < B; ++i) {
        OrcV1 *e = &envs[i];
        double r;
        int d = orc_v1_step(e, actions + (size_t)i * 2 * N, obs + (size_t)i * od, &r);
        reward[i] = r;
        done[i] = (uint8_t)d;
        if (d) {
            if (terminal_obs) memcpy(terminal_obs + (size_t)i * od, obs + (size_t)i * od, sizeof(double) * od);
            orc_v1_reset(e, obs + (size_t)i * od);
        }
    }
}

/* one env stepped nsteps times in a C loop (no per-step Python), left-team actions
   from the synthetic Philox stream (tag 1, key act_seed, counter (j/4, step, env id)), DummyVecEnv
   auto-reset on done.  Returns the number of finished episodes; *ret_sum = sum of their returns
   (so the work cannot be optimised away and the run is checkable). */
int orc_v1_run(OrcV1 *e, int nsteps, uint64_t act_seed, double *ret_sum)
{
    double obs[4 * ORC_MAXB], ret = 0.0, tot = 0.0;
    int32_t left[2 * ORC_MAXN];
    int episodes = 0;
    for (int t = 0; t < nsteps; ++t) {
        OracleRng g = { act_seed, e->env_id, (uint32_t)t, 0, 1 };
        oracle_words_choice(&g, 2 * e->N, 5, left);
        double r;
        const int d = orc_v1_step(e, left, obs, &r);
        ret += r;
        if (d) {
            tot += ret;
            ret = 0.0;
            ++episodes;
            orc_v1_reset(e, obs);
        }
    }
    *ret_sum = tot;
    return episodes;
}

/* bench.py cpu_baseline: B envs, each stepped nsteps times by orc_v1_run's loop, envs split over
   nthreads OpenMP threads (every thread steps its own contiguous block of envs through all nsteps:
   no per-step fork/join and no Python per step, the fastest schedule of independent envs on a
   host).  Returns the finished episodes; *ret_sum = the sum of their returns. */
long long orc_v1_vec_run(OrcV1 *envs, int B, int nsteps, uint64_t act_seed, int nthreads, double *ret_sum)
{
    long long eps = 0;
    double tot = 0.0;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : eps, tot)
    for (int i = 0; i < B; ++i) {
        double r = 0.0;
        eps += orc_v1_run(&envs[i], nsteps, act_seed, &r);
        tot += r;
    }
    *ret_sum = tot;
    return eps;
}

void orc_philox(const uint32_t *ctr, const uint32_t *key, uint32_t *out) { oracle_philox4x32_10(ctr, key, out); }

void orc_draw_u01(uint64_t seed, uint32_t env_id, uint32_t event, uint32_t j, uint32_t tag, double *u, double *z)
{
    OracleRng g = { seed, env_id, event, j, tag };
    OracleRng h = g;
    *u = oracle_uniform01(&g);
    *z = oracle_normal(&h, 0.0, 1.0);
}

int orc_sizeof_v1(void) { return (int)sizeof(OrcV1); }
int orc_sizeof_v0(void) { return (int)sizeof(OrcV0); }
