// futbol_v0.hip -- v0 `FutbolEnv` step (gym_futbol/envs/futbol_env.py) as one
// HIP kernel for gfx950, including the hard-coded opponent team
// (`_opp_team_set_vector_observation`, :864-983) and `Easy_Agent.get_action_type`
// (envs/easy_agent.py:53-98).  One env per lane, the 5 obs rows (25 fp64) in
// registers; agent indices are template constants so no per-lane array is ever
// indexed dynamically.  Randomness: the Philox tape of futbol_rng.hpp, drawn in
// the reference's program order.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "futbol_kernels.hpp"
#include "futbol_rng.hpp"
#include "futbol_state.hpp"
#include "futbol_util.hpp"

namespace futbol {
namespace v0 {

// module constants, envs/futbol_env.py:18-58
constexpr double FIELD_LEN = 105.0, FIELD_WID = 68.0;
constexpr double GOAL_UPPER = FIELD_WID / 2 + 10.0 / 2, GOAL_LOWER = FIELD_WID / 2 - 10.0 / 2;
constexpr double STEP_SIZE = 0.1;
constexpr int SHOOT_SPEED = 20;
enum { AI_1 = 0, AI_2 = 1, OPP_1 = 2, OPP_2 = 3, NOONE = 4 };  // ballowner.py
enum { RUN = 0, INTERCEPT = 1, SHOOT = 2, ASSIST = 3 };          // action.py
constexpr int BALL = 4;
constexpr int MATE[4] = {1, 0, 3, 2};
constexpr int kViewsLive = 6, kRowValid = 7;

struct Env {
    double r[5][5];
    double vw[8];  // frozen Easy_Agent views (x, y) x 4, loaded with the state
    uint32_t owner, last_owner;
    bool views_live;
    bool pending_done;
    // a shot whose direction is still to be computed (resolve_shot): at most one agent holds the
    // ball when it shoots, so the transcendental part runs once per step, not once per agent
    bool shot;
    uint32_t shot_pos;  // the draw index of the shot's normal (screw_vec), drawn by resolve_shot
    double shot_cs, shot_sn, shot_mag, shot_acc;
};

// glibc pow(x, 2.0)'s tables (futbol_powtab.h), staged in LDS by every step launch: the near-midpoint
// squares (glibc_sq2) look them up twice in dependent succession, and some lane of a wave needs that
// at nearly every get_vec
alignas(16) __shared__ double s_pow_log[128 * 3];
alignas(16) __shared__ uint64_t s_pow_exp[256];
// and glibc's sin / cos table (resolve_shot: some lane of nearly every wave shoots)
alignas(16) __shared__ double s_sincos[440];

// The tables are copied by LDS-DMA (global_load_lds_dwordx4: 16 bytes per lane and instruction, no
// registers), issued before the step's state loads and waited for with them (pow_tables_ready): one
// memory round trip per step.  Round 4 copied them with plain loads, ds_writes and a barrier first --
// a round trip of its own ahead of the state's: C3 21.98 -> 20.01 us (round 5, profiles/r05/ab/).
__device__ __forceinline__ void stage_pow_tables()
{
    typedef __attribute__((address_space(3))) void lds_void;
    const int lane = (int)threadIdx.x;  // (a one-wave block: every lane is active here)
    const uint4* pl = reinterpret_cast<const uint4*>(kPowLog);
    const uint4* pe = reinterpret_cast<const uint4*>(kPowExp);
    const uint4* ps = reinterpret_cast<const uint4*>(kSinCosTab);
    char* dl = reinterpret_cast<char*>(s_pow_log);
    char* de = reinterpret_cast<char*>(s_pow_exp);
    char* ds = reinterpret_cast<char*>(s_sincos);
    static_assert(sizeof(s_pow_log) == 3 * 1024 && sizeof(s_pow_exp) == 2 * 1024 && sizeof(s_sincos) == 3 * 1024 + 448,
                  "DMA pieces");
    static_assert(__alignof__(kSinCosTab) >= 16 && __alignof__(kPowLog) >= 16 && __alignof__(kPowExp) >= 16,
                  "16-byte LDS-DMA pieces need 16-byte aligned sources");
#pragma unroll
    for (int j = 0; j < 3; ++j) __builtin_amdgcn_global_load_lds(pl + 64 * j + lane, (lds_void*)(dl + 1024 * j), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 2; ++j) __builtin_amdgcn_global_load_lds(pe + 64 * j + lane, (lds_void*)(de + 1024 * j), 16, 0, 0);
#pragma unroll
    for (int j = 0; j < 3; ++j) __builtin_amdgcn_global_load_lds(ps + 64 * j + lane, (lds_void*)(ds + 1024 * j), 16, 0, 0);
    if (lane < 28) __builtin_amdgcn_global_load_lds(ps + 192 + lane, (lds_void*)(ds + 3072), 16, 0, 0);
}
// before the first table read: the DMA has landed (vmcnt(0): the state's loads, issued after it, are
// waited for at this point anyway)
__device__ __forceinline__ void pow_tables_ready()
{
    __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// get_vec (:62-65): vector from o to t and its magnitude; `vec[0]**2` is numpy's float64 power,
// i.e. libm pow(x, 2.0) (glibc_sq2, futbol_math.hpp)
__device__ __forceinline__ double get_vec(double tx, double ty, double ox, double oy, double& vx, double& vy)
{
    vx = tx - ox;
    vy = ty - oy;
    return sqrt(glibc_sq2(vx, vy, s_pow_log, s_pow_exp));
}
// get_vec whose magnitude the reference discards (`vec, _ = get_vec(...)`, :348-350, :434-436,
// :941-947): pow(x, 2.0) has no side effect, so only the vector is computed
__device__ __forceinline__ void vec_only(double tx, double ty, double ox, double oy, double& vx, double& vy)
{
    vx = tx - ox;
    vy = ty - oy;
}
// two independent get_vec magnitudes, their four squares in one glibc_pow2_batch
__device__ __forceinline__ void get_mag2(double t1x, double t1y, double o1x, double o1y, double t2x, double t2y,
                                         double o2x, double o2y, double& m1, double& m2)
{
    const double d[4] = {t1x - o1x, t1y - o1y, t2x - o2x, t2y - o2y};
    double q[4];
    glibc_pow2_batch<4>(d, q, s_pow_log, s_pow_exp);
    m1 = sqrt(q[0] + q[1]);
    m2 = sqrt(q[2] + q[3]);
}

__device__ __forceinline__ double intercept_chance(double d) /* :122-129, d1 = 1, d2 = 2 */
{
    if (d < 1.0) return 0.9;
    if (d >= 1.0 && d <= 2.0) {
        const double k = 0.9 / (1.0 - 2.0);
        return k * (d - 2.0);
    }
    return 0.0;
}

struct Ctx {
    const V0Params* P;
    double2* view;
    int env, B;
    Stream* rs;
};

// defence_near (:280-289) with the agent's (possibly stale) Easy_Agent view
template <int a>
__device__ __forceinline__ int defence_near(const Ctx& c, const Env& e)
{
    double vx, vy;
    const bool live = a < 2 ? e.views_live : (!c.P->random_opp || e.views_live);
    if (live) {
        vx = e.r[a][0];
        vy = e.r[a][1];
    } else {
        vx = e.vw[2 * a];
        vy = e.vw[2 * a + 1];
    }
    constexpr int o = a < 2 ? 2 : 0;
    double d1, d2;
    get_mag2(e.r[o][0], e.r[o][1], vx, vy, e.r[o + 1][0], e.r[o + 1][1], vx, vy, d1, d2);
    if (d1 <= 2 && d2 <= 2) return 2;  // bigger_than (:76-82)
    if (d1 > 2 && d2 > 2) return 0;
    return 1;
}

// _set_vector_observation (:300-530)
// pre_mag >= 0: |ball - agent| of the step's initial state (the step's first batch of squares), valid
// while the ball is where it was then (the agents' positions do not change before the physics): the
// non-holder's get_vec then reuses it instead of squaring again -- the same squares of the same
// differences, so the same magnitude, and one slow glibc round less per agent in most waves
template <int a>
__device__ __forceinline__ void set_vector_observation(const Ctx& c, Env& e, bool has_ball, int action,
                                                       bool set_target, double tgx, double tgy,
                                                       double pre_mag = -1.0, double pbx = 0.0, double pby = 0.0,
                                                       double mate_pre = -1.0)
{
    constexpr bool right = a >= 2;
    const V0Params* P = c.P;
    double* ag = e.r[a];
    double* ball = e.r[BALL];
    // every path draws target_y first and then at most three more (shoot): the first two blocks
    // are computed here, where the wave is converged, and each exclusive branch takes its draws by
    // position -- one Philox per draw position instead of one per draw site.  The third (shoot's
    // normal) is computed by resolve_shot, once per step; the fourth (shoot's randint(0, 9)) only
    // advances the counter: its value is never used
    Philox4 blk[2];
    c.rs->lookahead(blk);
    uint32_t used = 1;
    const double target_y = (double)Stream::randint_of(blk[0], P->ty_lo, P->ty_hi);
    if (has_ball) {
        if (action == INTERCEPT) {
            ag[2] = 0; ag[3] = 0; ag[4] = 0;
            ball[2] = 0; ball[3] = 0; ball[4] = 0;
            e.shot = false;
        } else if (action == RUN) {
            ag[4] = P->player_speed;
            if (set_target) {
                ag[2] = tgx;
                ag[3] = tgy;
            } else {
                double vx, vy;
                vec_only(right ? 0.0 : P->length, target_y, ag[0], ag[1], vx, vy);
                ag[2] = vx;
                ag[3] = vy;
            }
            used = 2;
            if (Stream::uniform01_of(blk[1]) < 0.05) e.owner = NOONE;
            else {
#pragma unroll
                for (int f = 0; f < 5; ++f) ball[f] = ag[f];
                e.shot = false;
            }
        } else if (action == SHOOT) {
            const int acc = 10 + defence_near<a>(c, e) * 20;
            ball[4] = Stream::randint_of(blk[1], P->shoot_lo, P->shoot_hi) * 1.0;
            double vx, vy;
            const double mag = get_vec(right ? 0.0 : P->length, target_y, ball[0], ball[1], vx, vy);
            // screw_vec (:101-116): one normal draw, then randint(0, 9) for the index; the
            // rotation (Box-Muller, sin/cos) is applied by resolve_shot before the ball moves
            e.shot_pos = c.rs->j + 2u;
            e.shot_acc = (double)acc;
            e.shot_cs = vx * 1.0 / mag;
            e.shot_sn = vy * 1.0 / mag;
            e.shot_mag = mag;
            e.shot = true;
            used = 4;  // + randint(0, 9) (screw_vec's index): drawn, value unused
            e.last_owner = e.owner;
            e.owner = NOONE;
            ag[2] = 0; ag[3] = 0; ag[4] = 0;
        } else {  // ASSIST
            const double* mate = e.r[MATE[a]];
            double vx, vy;
            double mag;
            // |mate - ball| = |ball - mate| of the first batch while the ball has not moved
            // (mate - ball = -(ball - mate) exactly, and pow(-x, 2) = pow(x, 2))
            if (mate_pre >= 0.0 && ball[0] == pbx && ball[1] == pby) {
                vec_only(mate[0], mate[1], ball[0], ball[1], vx, vy);
                mag = mate_pre;
            } else {
                mag = get_vec(mate[0], mate[1], ball[0], ball[1], vx, vy);
            }
            double cps = mag / STEP_SIZE;
            if (cps > SHOOT_SPEED) cps = SHOOT_SPEED;
            ball[4] = Stream::uniform_of(blk[1], cps - 1, cps + 1);
            used = 2;
            ball[2] = vx;
            ball[3] = vy;
            e.shot = false;
            e.last_owner = e.owner;
            e.owner = NOONE;
            ag[2] = 0; ag[3] = 0; ag[4] = 0;
        }
    } else {
        double btax, btay, gtax, gtay;
        double btam;
        if (pre_mag >= 0.0 && ball[0] == pbx && ball[1] == pby) {
            vec_only(ball[0], ball[1], ag[0], ag[1], btax, btay);
            btam = pre_mag;
        } else {
            btam = get_vec(ball[0], ball[1], ag[0], ag[1], btax, btay);
        }
        vec_only(right ? 0.0 : P->length, P->width / 2, ag[0], ag[1], gtax, gtay);
        if (action == INTERCEPT) {
            const bool success = Stream::uniform01_of(blk[1]) < intercept_chance(btam);
            used = 2;
            if (success || (e.owner == NOONE && btam < 2 + 2)) {
                ball[2] = ag[2]; ball[3] = ag[3]; ball[4] = ag[4];
                ball[0] = ag[0]; ball[1] = ag[1];
                e.shot = false;
                e.last_owner = e.owner;
                e.owner = a;
            }
        } else if (action == RUN) {
            ag[4] = P->player_speed;
            if (set_target) { ag[2] = tgx; ag[3] = tgy; }
            else if (e.owner != (uint32_t)a) { ag[2] = btax; ag[3] = btay; }
            else { ag[2] = gtax; ag[3] = gtay; }
        } else {
            ag[2] = 0; ag[3] = 0; ag[4] = 0;
        }
    }
    c.rs->skip(used);
}

// Easy_Agent.get_action_type (easy_agent.py:53-98), shoot_range = 20 (futbol_env.py:196-201).
// ub: the block of the stream's current draw, computed once for both opponents by opp_team (at
// most one of them holds the ball, so at most one draws, and at that position)
// btam, mtam: |ball - agent| and |mate - agent|, computed with the step's first batch of squares
template <int a>
__device__ __forceinline__ int get_action_type(const Ctx& c, const Env& e, bool has_ball, bool team_has_ball,
                                               const Philox4& ub, double btam, double mtam)
{
    constexpr bool right = a >= 2;
    const double* ag = e.r[a];
    const double* mate = e.r[MATE[a]];
    const double shoot_x = right ? 0.0 + 20 : c.P->length - 20;
    if (has_ball) {
        if ((right && ag[0] <= shoot_x) || (!right && ag[0] >= shoot_x)) return SHOOT;
        if (mate[0] < ag[0] || mate[1] < ag[1] - 7 || mate[1] > ag[1] + 7) {  // random() drawn only then
            c.rs->skip(1);
            if (Stream::uniform01_of(ub) > 0.8 && mtam > 12) return ASSIST;
        }
        return RUN;
    }
    if (btam <= 1 && !team_has_ball) return INTERCEPT;
    return RUN;
}

// _step_by_observation (:560-571); DECELERATION = 0
__device__ __forceinline__ void step_by_observation_mag(double* o, double mag)
{
    const double tx = o[2], ty = o[3];
    if (mag != 0) {
        o[0] = o[0] + o[4] * (tx * STEP_SIZE / mag);
        o[1] = o[1] + o[4] * (ty * STEP_SIZE / mag);
    }
}
__device__ __forceinline__ void step_by_observation(double* o)
{
    const double tx = o[2], ty = o[3];
    const double mag = sqrt(glibc_sq2(tx, ty, s_pow_log, s_pow_exp));
    if (mag != 0) {
        o[0] = o[0] + o[4] * (tx * STEP_SIZE / mag);
        o[1] = o[1] + o[4] * (ty * STEP_SIZE / mag);
    }
}

// the deferred part of a shot (:362-381, screw_vec :101-116): nothing between the shot and
// the ball's _step_by_observation reads the ball's direction -- later agents either leave it or
// overwrite it (which cancels the pending shot), and the opponents' ball anticipation only runs
// when neither opponent's action was SHOOT
__device__ __forceinline__ void resolve_shot(Env& e, const Stream& rs)
{
    if (!e.shot) return;
    const double nd = Stream::normal_of(rs.block(e.shot_pos), 0.0, e.shot_acc);
    const double ang = (nd / 180) * 3.141592653589793;
    // math.sin / math.cos of the reference: glibc's (futbol_math.hpp glibc_sin / glibc_cos)
    const double ss = glibc_sin(ang, s_sincos), sc = glibc_cos(ang, s_sincos);
    const double cs = e.shot_cs, sn = e.shot_sn;
    const double tc = (cs * sc) - (sn * ss), ts = (sn * sc) + (cs * ss);
    e.r[BALL][2] = tc * e.shot_mag;
    e.r[BALL][3] = ts * e.shot_mag;
    e.shot = false;
}

// _opp_team_set_vector_observation (:864-983); m3 = |ball - opp_1|, |ball - opp_2|, |opp_2 - opp_1|
// (= |opp_1 - opp_2|: pow(-x, 2) = pow(x, 2)) of the state at the top of the step
__device__ __forceinline__ void opp_team(const Ctx& c, Env& e, const double (&m3)[3], double bx0, double by0,
                                         double bvx0, double bvy0, double bvmag0)
{
    const V0Params* P = c.P;
    const bool o1has = e.owner == OPP_1, o2has = e.owner == OPP_2;
    const bool team = o1has || o2has;
    const Philox4 ub = c.rs->block(c.rs->j);
    int a1 = get_action_type<OPP_1>(c, e, o1has, team, ub, m3[0], m3[2]);
    int a2 = get_action_type<OPP_2>(c, e, o2has, team, ub, m3[1], m3[2]);
    const int opp1_action = a1, opp2_action = a2;  // the Action enums keep the pre-override values (D.13)
    bool s1 = false, s2 = false;
    double t1x = 0, t1y = 0, t2x = 0, t2y = 0;
    double* o1 = e.r[OPP_1];
    double* o2 = e.r[OPP_2];
    if (o1has && opp1_action == RUN) {
        if (o1[1] > P->width * 0.2) { s1 = true; t1x = -1; t1y = -1; }
        if (opp2_action == RUN && o2[0] > P->length * 0.1)
            if (o2[1] < P->width * 0.8) { s2 = true; t2x = -1; t2y = 1; }
    }
    if (o2has && opp2_action == RUN) {
        if (o2[1] < P->width * 0.8) { s2 = true; t2x = -1; t2y = 1; }
        if (opp1_action == RUN && o1[0] > P->length * 0.1)
            if (o1[1] > P->width * 0.2) { s1 = true; t1x = -1; t1y = -1; }
    }
    if (e.owner == AI_1 || e.owner == AI_2) {
        if (e.r[BALL][0] < P->length * 0.6) {
            const double dpx = P->length * 0.75, dpy = P->width * 0.5;
            if (o1[0] > o2[0]) { a1 = RUN; s1 = true; vec_only(dpx, dpy, o1[0], o1[1], t1x, t1y); }
            else { a2 = RUN; s2 = true; vec_only(dpx, dpy, o2[0], o2[1], t2x, t2y); }
        }
    }
    set_vector_observation<OPP_1>(c, e, o1has, a1, s1, t1x, t1y, m3[0], bx0, by0, m3[1]);
    set_vector_observation<OPP_2>(c, e, o2has, a2, s2, t2x, t2y, m3[1], bx0, by0, m3[0]);
    if (e.owner == NOONE && opp1_action == RUN && opp2_action == RUN) {
        // anticipate the ball (:962-982)
        double nb[5];
#pragma unroll
        for (int f = 0; f < 5; ++f) nb[f] = e.r[BALL][f];
        // (no opponent touched the ball: its velocity is the step's initial one, whose magnitude the
        // first batch of squares computed)
        if (nb[2] == bvx0 && nb[3] == bvy0) step_by_observation_mag(nb, bvmag0);
        else step_by_observation(nb);
        const double v1x = nb[0] - o1[0], v1y = nb[1] - o1[1], v2x = nb[0] - o2[0], v2y = nb[1] - o2[1];
        double m1, m2;
        get_mag2(nb[0], nb[1], o1[0], o1[1], nb[0], nb[1], o2[0], o2[1], m1, m2);
        // selects rather than if / else-if: the branchy form lets the compiler sink the three
        // stores behind a select of row pointers, which demotes those rows to scratch
        const bool u1 = m1 < STEP_SIZE * P->player_speed, u2 = !u1 && m2 < STEP_SIZE * P->player_speed;
        const double s1 = m1 / STEP_SIZE, s2 = m2 / STEP_SIZE;
        o1[2] = u1 ? v1x : o1[2]; o1[3] = u1 ? v1y : o1[3]; o1[4] = u1 ? s1 : o1[4];
        o2[2] = u2 ? v2x : o2[2]; o2[3] = u2 ? v2y : o2[3]; o2[4] = u2 ? s2 : o2[4];
    }
}

__device__ __forceinline__ bool obj_out(const double* o) /* out, :574-577 */
{
    return (o[0] < 0 || o[0] > FIELD_LEN) || (o[1] < 0 || o[1] > FIELD_WID);
}

__device__ __forceinline__ bool score(const Env& e) /* :580-583 */
{
    const double* b = e.r[BALL];
    const bool ai_in = b[0] <= 0 && (b[1] > GOAL_LOWER && b[1] < GOAL_UPPER);
    const bool opp_in = b[0] >= FIELD_LEN && (b[1] > GOAL_LOWER && b[1] < GOAL_UPPER);
    return ai_in || opp_in;
}

// _get_reward (:752-861); ob/oa1/oa2/oown: copies taken at the top of step(); b2a1 / b2a2 =
// |ob - oa1| / |ob - oa2|, computed with the step's first batch of squares
__device__ __forceinline__ double get_reward(const V0Params* P, const Env& e, const double* ob, const double* oa1,
                                             const double* oa2, const double* oown, int act1, int act2,
                                             double b2a1, double b2a2)
{
    const double running_r = (act1 == RUN || act2 == RUN) ? 10 * 0.2 : 0;
    const double player_adv_r = ((oown[0] == 10 && act2 == RUN) || (oown[1] == 10 && act1 == RUN)) ? 10 * 0.2 : 0;
    double bad1, bad2;
    if (oown[0] == 0) {
        if (act1 == ASSIST || act1 == SHOOT) bad1 = 2 * -0.5;
        else if (b2a1 > 2 && act1 == INTERCEPT) bad1 = 1 * -0.5;
        else bad1 = 0;
    } else bad1 = act1 == INTERCEPT ? 2 * -0.5 : 0;
    if (oown[1] == 0) {
        if (act2 == ASSIST || act2 == SHOOT) bad2 = 2 * -0.5;
        else if (b2a2 > 2 && act1 == INTERCEPT) bad2 = 1 * -0.5;  // the reference tests action1 (D.9)
        else bad2 = 0;
    } else bad2 = act2 == INTERCEPT ? 2 * -0.5 : 0;
    const double bad = bad1 + bad2;
    const double oof = (obj_out(e.r[AI_1]) || obj_out(e.r[AI_2])) ? -0.6 : 0;
    double get_ball;
    if ((e.owner == AI_1 || e.owner == AI_2) && (oown[0] == 0 && oown[1] == 0)) {
        if (ob[2] > ob[3] && ob[2] > 0 && ob[0] > oa1[0] && ob[0] > oa2[0] && oown[4] == 10) get_ball = -50 * 0.3;
        else get_ball = 60 * 0.3;
    } else if ((e.owner == AI_1 && oown[0] == 10) || (e.owner == AI_2 && oown[1] == 10)) {
        get_ball = 30 * 0.3;
    } else get_ball = 0;
    const bool sc = score(e);
    const double s = (sc && e.r[BALL][0] >= FIELD_LEN) ? 1000 : 0;
    const double gs = (sc && e.r[BALL][0] <= 0) ? -1000 : 0;
    if (P->only_reward_goal) return s + gs;
    return get_ball + s + gs + oof + bad + player_adv_r + running_r;
}

__device__ __forceinline__ void formation(Env& e)
{
    constexpr double init[5][2] = {{FIELD_LEN / 2 - 9, FIELD_WID / 2 + 5}, {FIELD_LEN / 2 - 9, FIELD_WID / 2 - 5},
                                   {FIELD_LEN / 2 + 9, FIELD_WID / 2 + 5}, {FIELD_LEN / 2 + 9, FIELD_WID / 2 - 5},
                                   {FIELD_LEN / 2, FIELD_WID / 2}};
#pragma unroll
    for (int r = 0; r < 5; ++r) {
        e.r[r][0] = init[r][0];
        e.r[r][1] = init[r][1];
        e.r[r][2] = 0;
        e.r[r][3] = 0;
        e.r[r][4] = 0;
    }
    e.owner = NOONE;
    e.last_owner = NOONE;
}

// self.obs re-bound (reset() / goal): Easy_Agent views still point at the old array
__device__ __forceinline__ void rebind(const Ctx& c, Env& e)
{
    if (e.views_live) {
        e.views_live = false;
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            e.vw[2 * a] = e.r[a][0];
            e.vw[2 * a + 1] = e.r[a][1];
            c.view[(size_t)a * c.B + c.env] = make_double2(e.r[a][0], e.r[a][1]);
        }
    }
}

template <typename OT>
__device__ __forceinline__ void write_obs(const Env& e, bool row_valid, OT* o)
{
#pragma unroll
    for (int r = 0; r < 5; ++r)
#pragma unroll
        for (int f = 0; f < 5; ++f) o[r * 5 + f] = (OT)e.r[r][f];
    const int idx = e.owner <= 3 ? (int)e.owner : 4;  // ball_owner_array_update (:720-736)
#pragma unroll
    for (int f = 0; f < 5; ++f) o[25 + f] = (OT)((row_valid && f == idx) ? 10 : 0);
}

__device__ __forceinline__ void load(const V0Ptrs& st, int env, int B, Env& e, Meta& m)
{
    // the 25 row entries as 13 pairs (16-byte loads: half the memory instructions)
#pragma unroll
    for (int q = 0; q < 13; ++q) {
        const double2 v = st.row[(size_t)q * B + env];
        e.r[(2 * q) / 5][(2 * q) % 5] = v.x;
        if (2 * q + 1 < 25) e.r[(2 * q + 1) / 5][(2 * q + 1) % 5] = v.y;
    }
    // the views with the rows, in the same batch of loads: read on every step once the views are
    // frozen (after the first goal or reset), and then the only other HBM reads of the step
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const double2 v = st.view[(size_t)a * B + env];
        e.vw[2 * a] = v.x;
        e.vw[2 * a + 1] = v.y;
    }
    m.w = st.meta[env];
    e.owner = m.owner();
    e.last_owner = m.last_owner();
    e.views_live = m.bit(kViewsLive);
    e.pending_done = false;
    e.shot = false;
}

__device__ __forceinline__ void store(const V0Ptrs& st, int env, int B, const Env& e, Meta& m, bool row_valid)
{
#pragma unroll
    for (int q = 0; q < 13; ++q) {
        const double y = 2 * q + 1 < 25 ? e.r[(2 * q + 1) / 5][(2 * q + 1) % 5] : 0.0;
        st.row[(size_t)q * B + env] = make_double2(e.r[(2 * q) / 5][(2 * q) % 5], y);
    }
    m.set_owner(e.owner);
    m.set_last_owner(e.last_owner);
    m.set_bit(kViewsLive, e.views_live);
    m.set_bit(kRowValid, row_valid);
    st.meta[env] = m.w;
}

}  // namespace v0

using namespace v0;

// FutbolEnv.step (:628-717) + DummyVecEnv auto-reset
template <typename OT>
__device__ __forceinline__ void v0_step_body(const V0Params* __restrict__ P, const V0Ptrs& st,
                                             const uint8_t* __restrict__ actions, OT* __restrict__ obs,
                                             OT* __restrict__ reward, uint8_t* __restrict__ done_out,
                                             OT* __restrict__ term_obs)
{
    const int env = blockIdx.x * 64 + threadIdx.x;
    const int B = P->B;
    if (env >= B) return;
    Env e;
    Meta m;
    load(st, env, B, e, m);
    const double ep_ret0 = st.ep_ret[env];
    const bool row_valid_before = m.bit(kRowValid);
    const uint32_t ev = m.event();
    m.set_event(ev + 1);
    Stream rs(P->seed, P->env_base + (uint32_t)env, ev, 0);
    const Ctx c{P, st.view, env, B, &rs};

    int a0, a1, bad = 0;
    if (P->action_as_int) {
        int a = actions[env];
        bad = a > 15;
        a = a > 15 ? 15 : a;
        a0 = a / 4;
        a1 = a % 4;
    } else {
        a0 = actions[(size_t)env * 2];
        a1 = actions[(size_t)env * 2 + 1];
        bad = (a0 > 3) + (a1 > 3);
        a0 = a0 > 3 ? 3 : a0;
        a1 = a1 > 3 ? 3 : a1;
    }
    pow_tables_ready();  // (the tables' DMA was issued before the state loads; every later read is after here)

    double ob[5], oa1[5], oa2[5], oown[5];
    const int oidx = e.owner <= 3 ? (int)e.owner : 4;
#pragma unroll
    for (int f = 0; f < 5; ++f) {
        ob[f] = e.r[BALL][f];
        oa1[f] = e.r[AI_1][f];
        oa2[f] = e.r[AI_2][f];
        oown[f] = (row_valid_before && f == oidx) ? 10 : 0;
    }

    // the magnitudes of the step's initial state, their squares in one batch: _get_reward's ball to
    // ai_1 / ai_2 (of the copies o_b, o_ai_1, o_ai_2) and the opponents' get_action_type (hard-coded
    // opponent: ball to opp_1 / opp_2, opp_1 to opp_2)
    double b2a1, b2a2, m3[3], bvmag0 = 0.0;
    {
        const double* o1 = e.r[OPP_1];
        const double* o2 = e.r[OPP_2];
        const double d[12] = {ob[0] - oa1[0], ob[1] - oa1[1], ob[0] - oa2[0], ob[1] - oa2[1],
                              ob[0] - o1[0], ob[1] - o1[1], ob[0] - o2[0], ob[1] - o2[1], o2[0] - o1[0], o2[1] - o1[1],
                              ob[2], ob[3]};
        double q[12];
        if (P->random_opp) {
            glibc_pow2_batch<4>(*reinterpret_cast<const double(*)[4]>(d), *reinterpret_cast<double(*)[4]>(q),
                                s_pow_log, s_pow_exp);
        } else {
            glibc_pow2_batch<12>(d, q, s_pow_log, s_pow_exp);
            bvmag0 = sqrt(q[10] + q[11]);
            m3[0] = sqrt(q[4] + q[5]);
            m3[1] = sqrt(q[6] + q[7]);
            m3[2] = sqrt(q[8] + q[9]);
        }
        b2a1 = sqrt(q[0] + q[1]);
        b2a2 = sqrt(q[2] + q[3]);
    }
    if (P->random_opp) {
        const int t = rs.randint(0, 15);
        set_vector_observation<OPP_1>(c, e, e.owner == OPP_1, t / 4, false, 0, 0);
        set_vector_observation<OPP_2>(c, e, e.owner == OPP_2, t % 4, false, 0, 0);
    } else {
        opp_team(c, e, m3, ob[0], ob[1], ob[2], ob[3], bvmag0);
    }
    set_vector_observation<AI_1>(c, e, e.owner == AI_1, a0, false, 0, 0, b2a1, ob[0], ob[1], b2a2);
    set_vector_observation<AI_2>(c, e, e.owner == AI_2, a1, false, 0, 0, b2a2, ob[0], ob[1], b2a1);
    resolve_shot(e, rs);
    {   // _step_vector_observations + the ball's _step_by_observation: the five magnitudes are
        // independent, so their squares go through one glibc_pow2_batch
        double d[10], sq[10];
#pragma unroll
        for (int r = 0; r < 5; ++r) {
            d[2 * r] = e.r[r][2];
            d[2 * r + 1] = e.r[r][3];
        }
        glibc_pow2_batch<10>(d, sq, s_pow_log, s_pow_exp);
#pragma unroll
        for (int r = 0; r < 5; ++r) step_by_observation_mag(e.r[r], sqrt(sq[2 * r] + sq[2 * r + 1]));
    }

    const double rw = get_reward(P, e, ob, oa1, oa2, oown, a0, a1, b2a1, b2a2);
    bool done = false;
    if (score(e)) {
        const int who = e.r[BALL][0] <= 0 ? 1 : 0;
        st.score[(size_t)who * B + env] = st.score[(size_t)who * B + env] + 1;
        if (P->one_goal_end) done = true;
        rebind(c, e);
        formation(e);
    }
    {  // out_of_field (:621-625) + fix (:587-604)
        double* b = e.r[BALL];
        const bool x_out = b[0] < 0 || b[0] > P->length;
        const bool y_out = b[1] < 0 || b[1] > P->width;
        const double gd = P->width / 2 - P->goal_size / 2, gu = P->width / 2 + P->goal_size / 2;
        const bool y_score = b[1] > gd - 2 && b[1] < gu + 2;
        if ((x_out && !y_score) || y_out) {
            const uint32_t nw = (e.last_owner == OPP_1 || e.last_owner == OPP_2) ? AI_1 : OPP_1;
            b[0] = b[0] < 0 ? 0.0 : (b[0] > FIELD_LEN ? FIELD_LEN : b[0]);
            b[1] = b[1] < 0 ? 0.0 : (b[1] > FIELD_WID ? FIELD_WID : b[1]);
            e.owner = nw;
            b[2] = 0; b[3] = 0; b[4] = 0;
            if (nw == AI_1) {
#pragma unroll
                for (int f = 0; f < 5; ++f) e.r[AI_1][f] = b[f];
            } else {
#pragma unroll
                for (int f = 0; f < 5; ++f) e.r[OPP_1][f] = b[f];
            }
            if (P->one_goal_end) done = true;
        }
    }
    const uint32_t steps = m.steps();
    if ((int)steps + 1 >= P->K_done) done = true;  // time >= game_time, checked before time += 0.1
    m.set_steps(steps + 1 > (uint32_t)kMaxSteps ? (uint32_t)kMaxSteps : steps + 1);

    double ret = ep_ret0 + rw;
    bool row_valid = true;
    if (done && !P->auto_reset) {
        st.stat_ret[env] = st.stat_ret[env] + ret;
        st.stat_cnt[env] = st.stat_cnt[env] + 1;
        ret = 0.0;
    }
    if (done && P->auto_reset) {
        if (term_obs) write_obs<OT>(e, true, term_obs + (size_t)env * 30);
        st.stat_ret[env] = st.stat_ret[env] + ret;
        st.stat_cnt[env] = st.stat_cnt[env] + 1;
        ret = 0.0;
        // reset() (:205-245): new event (no draws), rebind, formation, time/scores 0
        m.set_event(m.event() + 1);
        rebind(c, e);
        formation(e);
        m.set_steps(0);
        st.score[env] = 0;
        st.score[(size_t)B + env] = 0;
        row_valid = false;
    }
    write_obs<OT>(e, row_valid, obs + (size_t)env * 30);
    st.ep_ret[env] = ret;
    reward[env] = (OT)rw;
    done_out[env] = done ? 1 : 0;
    store(st, env, B, e, m, row_valid);
    // the clamped-action count at the very end, where no value is live across the atomic's divergent
    // `if` (see futbol_v1_impl.hpp: a copy the register allocator placed at the join of that `if`
    // before its exec restore miscompiled the large envs_v1 instances)
    if (bad) atomicAdd(st.invalid, (unsigned long long)bad);
}

// ROLL (nsteps > 1): open-loop rollout (futbol_rollout), step k on the k-th [B][...] slice of every
// buffer; the single-step instance has no loop around the body
template <typename OT, bool ROLL>
__global__ void __launch_bounds__(64) v0_step_kernel(const V0Params* __restrict__ P, V0Ptrs st,
                                                     const uint8_t* __restrict__ actions, OT* __restrict__ obs,
                                                     OT* __restrict__ reward, uint8_t* __restrict__ done_out,
                                                     OT* __restrict__ term_obs, int nsteps)
{
    stage_pow_tables();
    if constexpr (!ROLL) {
        v0_step_body<OT>(P, st, actions, obs, reward, done_out, term_obs);
        return;
    }
    const size_t B = (size_t)P->B, adim = P->action_as_int ? 1 : 2;
#pragma unroll 1
    for (int k = 0; k < nsteps; ++k)
        v0_step_body<OT>(P, st, actions + (size_t)k * B * adim, obs + (size_t)k * B * 30, reward + (size_t)k * B,
                         done_out + (size_t)k * B, term_obs ? term_obs + (size_t)k * B * 30 : nullptr);
}

template <typename OT>
__global__ void __launch_bounds__(64) v0_reset_kernel(const V0Params* __restrict__ P, V0Ptrs st,
                                                      const uint8_t* __restrict__ mask, OT* __restrict__ obs,
                                                      int init)
{
    const int env = blockIdx.x * 64 + threadIdx.x;
    const int B = P->B;
    if (env >= B) return;
    if (mask && !mask[env]) return;
    Env e;
    Meta m;
    Stream rs(P->seed, P->env_base + (uint32_t)env, 0, 0);
    const Ctx c{P, st.view, env, B, &rs};
    if (init) {
        // __init__: self.obs = self.reset() (event 0, no draws); agents hold live views into it
        formation(e);
        m.w = 0;
        m.set_event(1);
        e.views_live = true;
        st.stat_ret[env] = 0.0;
        st.stat_cnt[env] = 0;
    } else {
        load(st, env, B, e, m);
        m.set_event(m.event() + 1);
        rebind(c, e);
        formation(e);
    }
    m.set_steps(0);
    st.score[env] = 0;
    st.score[(size_t)B + env] = 0;
    st.ep_ret[env] = 0.0;
    if (obs) write_obs<OT>(e, false, obs + (size_t)env * 30);
    store(st, env, B, e, m, false);
}

int launch_v0(const V0Params* P, int B, const V0Ptrs& st, int out64, int what, const uint8_t* actions,
              const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, int nsteps,
              hipStream_t stream)
{
    const dim3 grid((B + 63) / 64), block(64);
    if (what == 0) {
        if (out64) {
            if (nsteps > 1)
                launch_kernel(v0_step_kernel<double, true>, grid, block, stream, P, st, actions, (double*)obs,
                              (double*)reward, done, (double*)term, nsteps);
            else
                launch_kernel(v0_step_kernel<double, false>, grid, block, stream, P, st, actions, (double*)obs,
                              (double*)reward, done, (double*)term, 1);
        } else {
            if (nsteps > 1)
                launch_kernel(v0_step_kernel<float, true>, grid, block, stream, P, st, actions, (float*)obs,
                              (float*)reward, done, (float*)term, nsteps);
            else
                launch_kernel(v0_step_kernel<float, false>, grid, block, stream, P, st, actions, (float*)obs,
                              (float*)reward, done, (float*)term, 1);
        }
    } else {
        if (out64)
            hipLaunchKernelGGL((v0_reset_kernel<double>), grid, block, 0, stream, P, st, mask, (double*)obs, init);
        else
            hipLaunchKernelGGL((v0_reset_kernel<float>), grid, block, 0, stream, P, st, mask, (float*)obs, init);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace futbol
