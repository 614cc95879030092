/*
 * futbol_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's per-env step, used as the checker for the
 * HIP kernels (tests/, __graft_entry__.smoke(), bench.py cpu_baseline leg).
 * The product (gym-futbol_amd/) never includes, links or loads this.
 *
 *  v1: gym_futbol/envs_v1/{futbol_env,team,ball,player}.py + the subset of
 *      Chipmunk2D 7.0.x (bundled in pymunk 5.6.0) that path calls.
 *      PARITY VS REAL PYMUNK IS UNPINNED (pymunk is not installable here, see
 *      SURVEY.md 8c); pinned instead by hand-derived KATs (tests/test_oracle_v1.py).
 *  v0: gym_futbol/envs/{futbol_env,easy_agent}.py -- pinned against golden
 *      vectors produced by the real reference (tests/golden/gen_v0_golden.py).
 *
 * Python's float `x**2` calls libm pow(); the oracle does the same at every
 * place the reference writes `**2` (ORACLE_SQ) so that it is bit-identical to
 * the reference on the same libm.  Chipmunk's own C code squares with `*`.
 */
#ifndef FUTBOL_ORACLE_H
#define FUTBOL_ORACLE_H
#include <stdint.h>

#define ORC_MAXN 10
#define ORC_MAXB (2 * ORC_MAXN + 1)
#define ORC_NSEG 12
#define ORC_MAXP (ORC_MAXB * ORC_NSEG + ORC_MAXB * (ORC_MAXB - 1) / 2)

/* Chipmunk arbiter states (cpArbiter.h) */
enum { ORC_ST_FIRST = 0, ORC_ST_NORMAL = 1, ORC_ST_CACHED = 2 };

typedef struct {
    /* --- configuration (Futbol.__init__ kwargs, envs_v1/futbol_env.py:63-65) --- */
    int32_t N, Nb, P;
    double width, height, total_time;
    uint64_t seed;
    uint32_t env_id;
    /* --- bodies: A0..A(N-1), B0..B(N-1), ball (insertion order, futbol_env.py:105-125) --- */
    double px[ORC_MAXB], py[ORC_MAXB];
    double vx[ORC_MAXB], vy[ORC_MAXB];
    double bx[ORC_MAXB], by[ORC_MAXB];          /* cpBody.v_bias */
    /* --- game state --- */
    double current_time;                        /* futbol_env.py:147,478 */
    int32_t owner;                              /* ball_owner_side: 0 left, 1 right */
    uint32_t event;                             /* next RNG event index */
    /* --- cpSpace state --- */
    uint32_t stamp;
    double curr_dt;
    /* arbiter hash set, dense by pair id */
    int32_t arb_exists[ORC_MAXP];
    uint32_t arb_stamp[ORC_MAXP];
    int32_t arb_state[ORC_MAXP];
    int32_t arb_inlist[ORC_MAXP];               /* in last cpSpaceStep's arbiter list */
    double arb_jn[ORC_MAXP];                    /* jnAcc of its (single) contact */
    uint32_t n_out, n_goal;                     /* diagnostics: out-of-bounds fixes, goals so far */
    int32_t last_out_wall, last_out_pick;       /* diagnostics: the last step's out-of-bounds wall (-1: none) and
                                                   restarted player (tests/test_gpu_v1_parity.py covers every leaf) */
} OrcV1;

/* v0 (gym_futbol/envs/futbol_env.py) */
typedef struct {
    /* config: FutbolEnv.__init__ kwargs, envs/futbol_env.py:134-138 */
    double length, width, goal_size, game_time, player_speed, shoot_speed;
    int32_t one_goal_end, only_reward_goal, random_opp;
    uint64_t seed;
    uint32_t env_id;
    /* obs rows ai_1, ai_2, opp_1, opp_2, ball, owner-array (futbol_env.py:225) */
    double obs[6][5];
    int32_t ball_owner, last_ball_owner;        /* BallOwner enum 0..4 */
    double time;
    int32_t ai_score, opp_score;
    /* Easy_Agent.agent_observation views of the AI agents (stale after the
       first rebind of self.obs) */
    int32_t views_live;
    double ai_view[2][2];                       /* frozen AI agent views */
    double opp_view_frozen[2][2];               /* frozen opp views (random_opp=True) */
    int32_t pending_done;
    uint32_t event;
} OrcV0;

#ifdef __cplusplus
extern "C" {
#endif
int  orc_v1_obs_dim(int N);
void orc_v1_init(OrcV1 *e, int N, double width, double height, double total_time, uint64_t seed, uint32_t env_id);
void orc_v1_reset(OrcV1 *e, double *obs);
int  orc_v1_step(OrcV1 *e, const int32_t *left_actions, double *obs, double *reward);
void orc_v1_observe(const OrcV1 *e, double *obs);
void orc_v1_space_step(OrcV1 *e, double dt);
/* batched VecEnv semantics (auto-reset, terminal obs); OpenMP over envs */
void orc_v1_vec_step(OrcV1 *envs, int B, const int32_t *actions, double *obs, double *reward,
                     uint8_t *done, double *terminal_obs, int nthreads);

/* C1: one env, nsteps steps in a C loop, synthetic Philox (tag 1) left actions, auto-reset */
int  orc_v1_run(OrcV1 *e, int nsteps, uint64_t act_seed, double *ret_sum);
/* cpu_baseline: B envs x nsteps of orc_v1_run's loop, envs split over nthreads OpenMP threads */
long long orc_v1_vec_run(OrcV1 *envs, int B, int nsteps, uint64_t act_seed, int nthreads, double *ret_sum);
long long orc_v0_vec_run(OrcV0 *envs, int B, int nsteps, uint64_t act_seed, int nthreads, double *ret_sum);

void orc_v0_init(OrcV0 *e, double length, double width, double goal_size, double game_time,
                 double player_speed, double shoot_speed, int one_goal_end, int only_reward_goal,
                 int random_opp, uint64_t seed, uint32_t env_id);
void orc_v0_reset(OrcV0 *e, double *obs);
int  orc_v0_step(OrcV0 *e, int32_t a0, int32_t a1, double *obs, double *reward);
void orc_v0_vec_step(OrcV0 *envs, int B, const int32_t *actions, double *obs, double *reward,
                     uint8_t *done, double *terminal_obs, int nthreads);

/* diagnostic: faithful-build squares as x*x at the sites of this mask (futbol_v1_oracle.c) */
void orc_v1_set_sq_mask(int mask);

/* RNG contract probes (tests) */
void orc_philox(const uint32_t *ctr, const uint32_t *key, uint32_t *out);
void orc_draw_u01(uint64_t seed, uint32_t env_id, uint32_t event, uint32_t j, uint32_t tag, double *u, double *z);
int  orc_sizeof_v1(void);
int  orc_sizeof_v0(void);
#ifdef __cplusplus
}
#endif
#endif
