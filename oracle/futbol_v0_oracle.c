/*
 * futbol_v0_oracle.c -- TEST INFRASTRUCTURE ONLY (the checker, never shipped).
 *
 * Literal scalar fp64 restatement of one v0 `FutbolEnv`
 * (gym_futbol/envs/futbol_env.py) with its hard-coded opponent
 * (`_opp_team_set_vector_observation`, :864-983) and `Easy_Agent`
 * (gym_futbol/envs/easy_agent.py:53-98).  Every stochastic call of the
 * reference (`random.random/randint/uniform`, `np.random.normal`) is replaced
 * by the RNG tape of oracle_rng.h in program order; the golden generator
 * (tests/golden/gen_v0_golden.py) feeds the very same tape to the real
 * reference, which pins this file bit-for-bit (faithful build).
 *
 * Row layout of obs (futbol_env.py:225): 0 ai_1, 1 ai_2, 2 opp_1, 3 opp_2,
 * 4 ball, 5 owner array; row = [x, y, target_dx, target_dy, speed].
 */
#include <math.h>
#include <string.h>
#include <stdint.h>
#include "futbol_oracle.h"
#include "oracle_math.h"
#include "oracle_rng.h"

/* module constants, envs/futbol_env.py:18-58 */
#define FIELD_LEN 105.0
#define FIELD_WID 68.0
#define GOAL_UPPER (FIELD_WID / 2 + 10.0 / 2)
#define GOAL_LOWER (FIELD_WID / 2 - 10.0 / 2)
#define SHOOT_SPEED 20
#define STEP_SIZE 0.1
#define GOAL_REWARD 1000
#define PLAYER_ADV_REWARD_BASE 0.2
#define OUT_OF_FIELD_PENALTY (-0.6)
#define BAD_ACTION_PENALTY (-0.5)
#define BALL_CONTROL 0.3
#define NORMAL_MISS 10
#define UNDER_DEFENCE_MISS 20
#define MAX_INTERCEPT_PROB 0.9
#define MAX_INTERCEPT_DIST 2
#define MIN_INTERCEPT_DIST 1
#define DECELERATION 0

enum { AI_1 = 0, AI_2 = 1, OPP_1 = 2, OPP_2 = 3, NOONE = 4 };   /* ballowner.py */
enum { RUN = 0, INTERCEPT = 1, SHOOT = 2, ASSIST = 3 };          /* action.py */
#define BALL 4
#define OWNROW 5

/* get_vec, futbol_env.py:62-65 (and easy_agent.py:10-13) */
static double get_vec(double tx, double ty, double ox, double oy, double *vx, double *vy)
{
    *vx = tx - ox;
    *vy = ty - oy;
    return sqrt(ORC_SQ(*vx) + ORC_SQ(*vy));
}

static int bigger_than(double x1, double x2, double v) /* :76-82 */
{
    if (x1 <= v && x2 <= v) return 2;
    if (x1 > v && x2 > v) return 0;
    return 1;
}

static double intercept_chance(double d, double d1, double d2) /* :122-129 */
{
    if (d < d1) return MAX_INTERCEPT_PROB;
    if (d >= d1 && d <= d2) {
        double k = MAX_INTERCEPT_PROB / (d1 - d2);
        return k * (d - d2);
    }
    return 0.0;
}

static double lock_in(double val, double mx) { return val < 0 ? 0.0 : (val > mx ? mx : val); } /* :68-74 */

/* screw_vec, :101-116 -- np.random.normal(0, acc, 10) is ONE tape draw
   (all 10 entries equal), random.randint(0, 9) still consumes one draw */
static void screw_vec(OracleRng *g, double vx, double vy, double mag, double acc, double *ox, double *oy)
{
    double nd = oracle_normal(g, 0.0, acc);
    double c = vx * 1.0 / mag;
    double s = vy * 1.0 / mag;
    (void)oracle_randint(g, 0, 9);
    double ang = (nd / 180) * 3.141592653589793;
    double ss = ORC_SIN(ang), sc = ORC_COS(ang);
    double tc = (c * sc) - (s * ss);
    double ts = (s * sc) + (c * ss);
    *ox = tc * mag;
    *oy = ts * mag;
}

/* the Easy_Agent objects: name, agent_index, mate_index, team */
static const int AG_MATE[4] = { 1, 0, 3, 2 };
static int ag_right(int a) { return a >= 2; }

static void formation(OrcV0 *e)
{
    static const double init[5][2] = {
        { FIELD_LEN / 2 - 9, FIELD_WID / 2 + 5 }, { FIELD_LEN / 2 - 9, FIELD_WID / 2 - 5 },
        { FIELD_LEN / 2 + 9, FIELD_WID / 2 + 5 }, { FIELD_LEN / 2 + 9, FIELD_WID / 2 - 5 },
        { FIELD_LEN / 2, FIELD_WID / 2 } };
    memset(e->obs, 0, sizeof(e->obs));
    for (int r = 0; r < 5; ++r) { e->obs[r][0] = init[r][0]; e->obs[r][1] = init[r][1]; }
    e->ball_owner = NOONE;
    e->last_ball_owner = NOONE;
}

/* self.obs is re-bound to a new array (reset / goal): the AI agents' (and, with
   random_opp, the opp agents') agent_observation views freeze */
static void rebind(OrcV0 *e)
{
    if (e->views_live) {
        e->views_live = 0;
        for (int a = 0; a < 2; ++a) { e->ai_view[a][0] = e->obs[a][0]; e->ai_view[a][1] = e->obs[a][1]; }
        e->opp_view_frozen[0][0] = e->obs[2][0]; e->opp_view_frozen[0][1] = e->obs[2][1];
        e->opp_view_frozen[1][0] = e->obs[3][0]; e->opp_view_frozen[1][1] = e->obs[3][1];
    }
}

static void agent_view(const OrcV0 *e, int a, double *x, double *y)
{
    if (a < 2) {
        if (e->views_live) { *x = e->obs[a][0]; *y = e->obs[a][1]; }
        else { *x = e->ai_view[a][0]; *y = e->ai_view[a][1]; }
    } else {
        /* random_opp=False: get_action_type refreshes the view every step */
        if (!e->random_opp || e->views_live) { *x = e->obs[a][0]; *y = e->obs[a][1]; }
        else { *x = e->opp_view_frozen[a - 2][0]; *y = e->opp_view_frozen[a - 2][1]; }
    }
}

/* defence_near, :280-289 */
static int defence_near(const OrcV0 *e, int a)
{
    double vx, vy, t0, t1;
    agent_view(e, a, &vx, &vy);
    int o = a < 2 ? 2 : 0; /* left team measures opps, right team measures ais */
    double d1 = get_vec(e->obs[o][0], e->obs[o][1], vx, vy, &t0, &t1);
    double d2 = get_vec(e->obs[o + 1][0], e->obs[o + 1][1], vx, vy, &t0, &t1);
    return bigger_than(d1, d2, 2);
}

/* _set_vector_observation, :300-530 */
static void set_vector_observation(OrcV0 *e, OracleRng *g, int a, int has_ball, int action,
                                   int set_target, double tgx, double tgy)
{
    double *ag = e->obs[a];
    double *ball = e->obs[BALL];
    int ty = oracle_randint(g, (int)(e->width / 2 - e->goal_size / 2 + 3), (int)(e->width / 2 + e->goal_size / 2 - 3));
    double target_y = (double)ty;
    if (has_ball) {
        if (action == INTERCEPT) {
            ag[2] = 0; ag[3] = 0; ag[4] = 0;
            ball[2] = 0; ball[3] = 0; ball[4] = 0;
        } else if (action == RUN) {
            ag[4] = e->player_speed;
            if (set_target) { ag[2] = tgx; ag[3] = tgy; }
            else {
                double gx = ag_right(a) ? 0.0 : e->length, vx, vy;
                get_vec(gx, target_y, ag[0], ag[1], &vx, &vy);
                ag[2] = vx; ag[3] = vy;
            }
            if (oracle_uniform01(g) < 0.05) e->ball_owner = NOONE;
            else memcpy(ball, ag, sizeof(double) * 5);
        } else if (action == SHOOT) {
            int acc = NORMAL_MISS + defence_near(e, a) * UNDER_DEFENCE_MISS;
            ball[4] = oracle_randint(g, (int)e->shoot_speed - 16, (int)e->shoot_speed) * 1.0;
            double gx = ag_right(a) ? 0.0 : e->length, vx, vy;
            double mag = get_vec(gx, target_y, ball[0], ball[1], &vx, &vy);
            double ox, oy;
            screw_vec(g, vx, vy, mag, (double)acc, &ox, &oy);
            ball[2] = ox; ball[3] = oy;
            e->last_ball_owner = e->ball_owner;
            e->ball_owner = NOONE;
            ag[2] = 0; ag[3] = 0; ag[4] = 0;
        } else { /* ASSIST */
            const double *mate = e->obs[AG_MATE[a]];
            double vx, vy;
            double mag = get_vec(mate[0], mate[1], ball[0], ball[1], &vx, &vy);
            double cps = mag / STEP_SIZE;
            if (cps > SHOOT_SPEED) cps = SHOOT_SPEED;
            ball[4] = oracle_uniform(g, cps - 1, cps + 1);
            ball[2] = vx; ball[3] = vy;
            e->last_ball_owner = e->ball_owner;
            e->ball_owner = NOONE;
            ag[2] = 0; ag[3] = 0; ag[4] = 0;
        }
    } else {
        double btax, btay, gtax, gtay;
        double btam = get_vec(ball[0], ball[1], ag[0], ag[1], &btax, &btay);
        get_vec(ag_right(a) ? 0.0 : e->length, e->width / 2, ag[0], ag[1], &gtax, &gtay);
        if (action == INTERCEPT) {
            int success = oracle_uniform01(g) < intercept_chance(btam, MIN_INTERCEPT_DIST, MAX_INTERCEPT_DIST);
            if (success || (e->ball_owner == NOONE && btam < MAX_INTERCEPT_DIST + 2)) {
                ball[2] = ag[2]; ball[3] = ag[3]; ball[4] = ag[4];
                ball[0] = ag[0]; ball[1] = ag[1];
                e->last_ball_owner = e->ball_owner;
                e->ball_owner = a;
            }
        } else if (action == RUN) {
            ag[4] = e->player_speed;
            if (set_target) { ag[2] = tgx; ag[3] = tgy; }
            else if (e->ball_owner != a) { ag[2] = btax; ag[3] = btay; }
            else { ag[2] = gtax; ag[3] = gtay; }
        } else {
            ag[2] = 0; ag[3] = 0; ag[4] = 0;
        }
    }
}

/* Easy_Agent.get_action_type, easy_agent.py:53-98 */
static int get_action_type(OrcV0 *e, OracleRng *g, int a, int has_ball, int team_has_ball)
{
    const double *ag = e->obs[a], *mate = e->obs[AG_MATE[a]], *ball = e->obs[BALL];
    double t0, t1;
    double btam = get_vec(ball[0], ball[1], ag[0], ag[1], &t0, &t1);
    double mtam = get_vec(mate[0], mate[1], ag[0], ag[1], &t0, &t1);
    double shoot_x = ag_right(a) ? 0.0 + 20 : e->length - 20; /* shoot_range = 20 (:196-201) */
    if (has_ball) {
        if ((ag_right(a) && ag[0] <= shoot_x) || (!ag_right(a) && ag[0] >= shoot_x)) return SHOOT;
        if ((mate[0] < ag[0] || mate[1] < ag[1] - 7 || mate[1] > ag[1] + 7) && oracle_uniform01(g) > 0.8 && mtam > 12)
            return ASSIST;
        return RUN;
    }
    if (btam <= 1 && !team_has_ball) return INTERCEPT;
    return RUN;
}

/* _agent_set_vector_observation(agent, action_set=True, ...), :536-555 */
static void agent_set_vector_observation(OrcV0 *e, OracleRng *g, int a, int action)
{
    int has = e->ball_owner == a;
    set_vector_observation(e, g, a, has, action, 0, 0.0, 0.0);
}

/* _step_by_observation, :560-571 */
static void step_by_observation(OrcV0 *e, double *o, int is_ball)
{
    double tx = o[2], ty = o[3];
    double mag = sqrt(ORC_SQ(tx) + ORC_SQ(ty));
    if (mag != 0) {
        o[0] = o[0] + o[4] * (tx * STEP_SIZE / mag);
        o[1] = o[1] + o[4] * (ty * STEP_SIZE / mag);
    }
    if (is_ball && e->ball_owner == NOONE) o[4] = o[4] - DECELERATION * STEP_SIZE;
}

/* _opp_team_set_vector_observation, :864-983 */
static void opp_team_set_vector_observation(OrcV0 *e, OracleRng *g)
{
    int o1has = e->ball_owner == OPP_1, o2has = e->ball_owner == OPP_2;
    int team = o1has || o2has;
    int a1 = get_action_type(e, g, OPP_1, o1has, team);
    int a2 = get_action_type(e, g, OPP_2, o2has, team);
    const int opp1_action = a1, opp2_action = a2; /* Action(...) enums, D.13 */
    int s1 = 0, s2 = 0;
    double t1x = 0, t1y = 0, t2x = 0, t2y = 0;
    double *o1 = e->obs[OPP_1], *o2 = e->obs[OPP_2];
    if (o1has && opp1_action == RUN) {
        if (o1[1] > e->width * 0.2) { s1 = 1; t1x = -1; t1y = -1; }
        if (opp2_action == RUN && o2[0] > e->length * 0.1)
            if (o2[1] < e->width * 0.8) { s2 = 1; t2x = -1; t2y = 1; }
    }
    if (o2has && opp2_action == RUN) {
        if (o2[1] < e->width * 0.8) { s2 = 1; t2x = -1; t2y = 1; }
        if (opp1_action == RUN && o1[0] > e->length * 0.1)
            if (o1[1] > e->width * 0.2) { s1 = 1; t1x = -1; t1y = -1; }
    }
    if (e->ball_owner == AI_1 || e->ball_owner == AI_2) {
        if (e->obs[BALL][0] < e->length * 0.6) {
            double dpx = e->length * 0.75, dpy = e->width * 0.5;
            if (o1[0] > o2[0]) { a1 = RUN; s1 = 1; get_vec(dpx, dpy, o1[0], o1[1], &t1x, &t1y); }
            else { a2 = RUN; s2 = 1; get_vec(dpx, dpy, o2[0], o2[1], &t2x, &t2y); }
        }
    }
    set_vector_observation(e, g, OPP_1, o1has, a1, s1, t1x, t1y);
    set_vector_observation(e, g, OPP_2, o2has, a2, s2, t2x, t2y);
    if (e->ball_owner == NOONE && opp1_action == RUN && opp2_action == RUN) {
        double nb[5];
        memcpy(nb, e->obs[BALL], sizeof(nb));
        step_by_observation(e, nb, 0);
        double v1x, v1y, v2x, v2y;
        double m1 = get_vec(nb[0], nb[1], o1[0], o1[1], &v1x, &v1y);
        double m2 = get_vec(nb[0], nb[1], o2[0], o2[1], &v2x, &v2y);
        if (m1 < STEP_SIZE * e->player_speed) { o1[2] = v1x; o1[3] = v1y; o1[4] = m1 / STEP_SIZE; }
        else if (m2 < STEP_SIZE * e->player_speed) { o2[2] = v2x; o2[3] = v2y; o2[4] = m2 / STEP_SIZE; }
    }
}

static int obj_out(const double *o) /* out, :574-577 */
{
    return (o[0] < 0 || o[0] > FIELD_LEN) || (o[1] < 0 || o[1] > FIELD_WID);
}

static int score(const OrcV0 *e) /* :580-583 */
{
    const double *b = e->obs[BALL];
    int ai_in = b[0] <= 0 && (b[1] > GOAL_LOWER && b[1] < GOAL_UPPER);
    int opp_in = b[0] >= FIELD_LEN && (b[1] > GOAL_LOWER && b[1] < GOAL_UPPER);
    return ai_in || opp_in;
}

/* _get_reward, :752-861 (o_* are the copies taken at the top of step) */
static double get_reward(const OrcV0 *e, const double *ob, const double *oa1, const double *oa2,
                         const double *oown, int act1, int act2)
{
    double t0, t1;
    double b2a1 = get_vec(ob[0], ob[1], oa1[0], oa1[1], &t0, &t1);
    double b2a2 = get_vec(ob[0], ob[1], oa2[0], oa2[1], &t0, &t1);
    double running_r = (act1 == RUN || act2 == RUN) ? 10 * PLAYER_ADV_REWARD_BASE : 0;
    double player_adv_r = ((oown[0] == 10 && act2 == RUN) || (oown[1] == 10 && act1 == RUN)) ? 10 * PLAYER_ADV_REWARD_BASE : 0;
    double bad1, bad2;
    if (oown[0] == 0) {
        if (act1 == ASSIST || act1 == SHOOT) bad1 = 2 * BAD_ACTION_PENALTY;
        else if (b2a1 > 2 && act1 == INTERCEPT) bad1 = 1 * BAD_ACTION_PENALTY;
        else bad1 = 0;
    } else bad1 = act1 == INTERCEPT ? 2 * BAD_ACTION_PENALTY : 0;
    if (oown[1] == 0) {
        if (act2 == ASSIST || act2 == SHOOT) bad2 = 2 * BAD_ACTION_PENALTY;
        else if (b2a2 > 2 && act1 == INTERCEPT) bad2 = 1 * BAD_ACTION_PENALTY; /* reference bug kept (D.9) */
        else bad2 = 0;
    } else bad2 = act2 == INTERCEPT ? 2 * BAD_ACTION_PENALTY : 0;
    double bad = bad1 + bad2;
    double oof = (obj_out(e->obs[AI_1]) || obj_out(e->obs[AI_2])) ? OUT_OF_FIELD_PENALTY : 0;
    double get_ball;
    if ((e->ball_owner == AI_1 || e->ball_owner == AI_2) && (oown[0] == 0 && oown[1] == 0)) {
        if (ob[2] > ob[3] && ob[2] > 0 && ob[0] > oa1[0] && ob[0] > oa2[0] && oown[4] == 10) get_ball = -50 * BALL_CONTROL;
        else get_ball = 60 * BALL_CONTROL;
    } else if ((e->ball_owner == AI_1 && oown[0] == 10) || (e->ball_owner == AI_2 && oown[1] == 10)) {
        get_ball = 30 * BALL_CONTROL;
    } else get_ball = 0;
    double sc = (score(e) && e->obs[BALL][0] >= FIELD_LEN) ? GOAL_REWARD : 0;
    double gs = (score(e) && e->obs[BALL][0] <= 0) ? -GOAL_REWARD : 0;
    if (e->only_reward_goal) return sc + gs;
    return get_ball + sc + gs + oof + bad + player_adv_r + running_r;
}

static void owner_array_update(OrcV0 *e) /* :720-736 */
{
    int idx = e->ball_owner <= OPP_2 ? e->ball_owner : BALL;
    for (int i = 0; i < 5; ++i) e->obs[OWNROW][i] = i == idx ? 10 : 0;
}

static void out_fix(OrcV0 *e) /* out_of_field :621-625 + fix :587-604 */
{
    double *b = e->obs[BALL];
    int x_out = b[0] < 0 || b[0] > e->length;
    int y_out = b[1] < 0 || b[1] > e->width;
    double gd = e->width / 2 - e->goal_size / 2, gu = e->width / 2 + e->goal_size / 2;
    int y_score = b[1] > gd - 2 && b[1] < gu + 2;
    if (!((x_out && !y_score) || y_out)) return;
    int player = e->last_ball_owner;
    int nw = (player == OPP_1 || player == OPP_2) ? AI_1 : OPP_1;
    b[0] = lock_in(b[0], FIELD_LEN);
    b[1] = lock_in(b[1], FIELD_WID);
    e->ball_owner = nw;
    b[2] = 0; b[3] = 0; b[4] = 0;
    memcpy(e->obs[nw == AI_1 ? AI_1 : OPP_1], b, sizeof(double) * 5);
    e->pending_done |= e->one_goal_end;
}

void orc_v0_init(OrcV0 *e, double length, double width, double goal_size, double game_time,
                 double player_speed, double shoot_speed, int one_goal_end, int only_reward_goal,
                 int random_opp, uint64_t seed, uint32_t env_id)
{
    memset(e, 0, sizeof(*e));
    e->length = length; e->width = width; e->goal_size = goal_size; e->game_time = game_time;
    e->player_speed = player_speed; e->shoot_speed = shoot_speed;
    e->one_goal_end = one_goal_end; e->only_reward_goal = only_reward_goal; e->random_opp = random_opp;
    e->seed = seed; e->env_id = env_id;
    /* __init__: self.obs = self.reset(); agents hold views into that array */
    formation(e);
    e->time = 0; e->ai_score = 0; e->opp_score = 0;
    e->views_live = 1;
    e->event = 1; /* the constructor's reset() is event 0 (it draws nothing) */
}

void orc_v0_reset(OrcV0 *e, double *obs) /* :205-245 */
{
    e->event++;
    rebind(e);
    formation(e);
    e->time = 0; e->ai_score = 0; e->opp_score = 0;
    if (obs) memcpy(obs, e->obs, sizeof(e->obs));
}

/* FutbolEnv.step, :628-717; a0/a1 = (a // 4, a % 4) */
int orc_v0_step(OrcV0 *e, int32_t a0, int32_t a1, double *obs, double *reward)
{
    OracleRng g = { e->seed, e->env_id, e->event++, 0, 0 };
    double ob[5], oa1[5], oa2[5], oown[5];
    memcpy(ob, e->obs[BALL], sizeof(ob));
    memcpy(oa1, e->obs[AI_1], sizeof(oa1));
    memcpy(oa2, e->obs[AI_2], sizeof(oa2));
    memcpy(oown, e->obs[OWNROW], sizeof(oown));
    e->pending_done = 0;

    if (e->random_opp) {
        int t = oracle_randint(&g, 0, 15);
        agent_set_vector_observation(e, &g, OPP_1, t / 4);
        agent_set_vector_observation(e, &g, OPP_2, t % 4);
    } else {
        opp_team_set_vector_observation(e, &g);
    }
    agent_set_vector_observation(e, &g, AI_1, a0);
    agent_set_vector_observation(e, &g, AI_2, a1);
    for (int r = 0; r < 4; ++r) step_by_observation(e, e->obs[r], 0);
    step_by_observation(e, e->obs[BALL], 1);

    double r = get_reward(e, ob, oa1, oa2, oown, a0, a1);
    int done = 0;
    if (score(e)) {
        if (e->obs[BALL][0] <= 0) e->opp_score += 1; else e->ai_score += 1;
        if (e->one_goal_end) done = 1;
        rebind(e);
        formation(e);
    }
    out_fix(e);
    if (e->pending_done) done = 1;
    owner_array_update(e);
    if (e->time >= e->game_time) done = 1;
    e->time = e->time + STEP_SIZE;
    if (obs) memcpy(obs, e->obs, sizeof(e->obs));
    if (reward) *reward = r;
    return done;
}

/* bench.py cpu_baseline (C3): B envs, each stepped nsteps times with synthetic Philox actions
   (tag 1, one word per step: a in [0, 16) -> (a / 4, a % 4)), auto-reset, envs split over nthreads
   OpenMP threads that each step their own block through all nsteps.  Returns the finished
   episodes; *ret_sum = the sum of every step's reward. */
long long orc_v0_vec_run(OrcV0 *envs, int B, int nsteps, uint64_t act_seed, int nthreads, double *ret_sum)
{
    long long eps = 0;
    double tot = 0.0;
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1) reduction(+ : eps, tot)
    for (int i = 0; i < B; ++i) {
        OrcV0 *e = &envs[i];
        double obs[30], r;
        for (int t = 0; t < nsteps; ++t) {
            OracleRng g = { act_seed, e->env_id, (uint32_t)t, 0, 1 };
            int32_t a;
            oracle_words_choice(&g, 1, 16, &a);
            const int d = orc_v0_step(e, a / 4, a % 4, obs, &r);
            tot += r;
            if (d) {
                ++eps;
                orc_v0_reset(e, obs);
            }
        }
    }
    *ret_sum = tot;
    return eps;
}

void orc_v0_vec_step(OrcV0 *envs, int B, const int32_t *actions, double *obs, double *reward,
                     uint8_t *done, double *terminal_obs, int nthreads)
{
#pragma omp parallel for schedule(static) num_threads(nthreads > 0 ? nthreads : 1)
    for (int i = 0; i < B; ++i) {
        OrcV0 *e = &envs[i];
        double r;
        int a = actions[i];
        int d = orc_v0_step(e, a / 4, a % 4, obs + (size_t)i * 30, &r);
        reward[i] = r;
        done[i] = (uint8_t)d;
        if (d) {
            if (terminal_obs) memcpy(terminal_obs + (size_t)i * 30, obs + (size_t)i * 30, sizeof(double) * 30);
            orc_v0_reset(e, obs + (size_t)i * 30);
        }
    }
}
