/*
 * futbol.h -- C ABI of the MI355X-native vectorised gym-futbol envs.
 *
 * One context = B independent envs of one kind, resident in the HBM of one
 * GPU, stepped in lockstep by hand-written HIP kernels (gfx950).  The caller
 * owns every per-step buffer (actions, obs, reward, done, terminal_obs): they
 * are DEVICE pointers on the context's GPU and every call is asynchronous on
 * the caller's hipStream_t (passed as void*).  No allocation, no host sync
 * inside futbol_reset / futbol_step (they are hipGraph-capturable).
 *
 * Reference interfaces replaced (Python; /root/reference):
 *   futbol_create   <- gym.make('Futbol2v2-v1'|'Futbol5v5-v1'|'Futbol-v1'|'Futbol-v0')
 *                      gym_futbol/__init__.py:3-28 ->
 *                      envs_v1/futbol_env.py:63-127 Futbol.__init__ (incl. its reset())
 *                      envs/futbol_env.py:134-201   FutbolEnv.__init__
 *   futbol_reset    <- envs_v1/futbol_env.py:146-150 Futbol.reset
 *                      envs/futbol_env.py:205-245   FutbolEnv.reset
 *   futbol_step     <- envs_v1/futbol_env.py:427-483 Futbol.step (opponent =
 *                      random_action(), :306-307, drawn in-kernel)
 *                      envs/futbol_env.py:628-717   FutbolEnv.step (hard-coded or
 *                      random opponent, :864-983 / :639-645, in-kernel)
 *                      + stable-baselines DummyVecEnv auto-reset semantics
 *                      (terminal obs, reset on done) for B envs at once.
 *   futbol_fill_actions <- envs_v1/futbol_env.py:306-307 random_action() for the
 *                      LEFT team (the notebook's random-rollout driver,
 *                      colab_notebook.ipynb:280), used as the synthetic policy.
 *   futbol_episode_stats <- stable-baselines Monitor episode return/length
 *                      (colab_notebook.ipynb:820), reduced on device.
 *
 * Errors: every function returns FUTBOL_OK (0) or a negative code;
 * futbol_last_error(ctx) (or futbol_last_error(NULL) for create) gives text.
 * Out-of-range actions are rejected at the boundary in the reference too
 * (envs_v1/futbol_env.py:326-327 prints then raises); the kernel clamps them
 * into range and counts them, see futbol_invalid_actions().
 */
#ifndef FUTBOL_H
#define FUTBOL_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FUTBOL_ABI_VERSION 1

enum { FUTBOL_ENV_V0 = 0, FUTBOL_ENV_V1 = 1 };
enum { FUTBOL_F32 = 0, FUTBOL_F64 = 1 };
enum {
    FUTBOL_OK = 0,
    FUTBOL_EINVAL = -1,
    FUTBOL_EHIP = -2,
    FUTBOL_ENOMEM = -3,
    FUTBOL_EUNSUPPORTED = -4
};

typedef struct FutbolConfig {
    int32_t abi_version;       /* FUTBOL_ABI_VERSION */
    int32_t env_kind;          /* FUTBOL_ENV_V1 (envs_v1.Futbol) / FUTBOL_ENV_V0 (envs.FutbolEnv) */
    int32_t out_dtype;         /* FUTBOL_F32 / FUTBOL_F64 for obs, reward, terminal_obs */
    int32_t number_of_player;  /* v1 kwarg, 1..10 (envs_v1/futbol_env.py:65) */
    double width, height, total_time; /* v1 kwargs (envs_v1/futbol_env.py:63-64) */
    /* v0 kwargs (envs/futbol_env.py:134-138) */
    double length0, width0, goal_size0, game_time0, player_speed0, shoot_speed0;
    int32_t one_goal_end0, action_as_int0, only_reward_goal0, random_opp0;
    /* 1: DummyVecEnv semantics (reset on done, terminal_obs).  0: the reference's
       single-env semantics (no reset; done stays true while stepping on). */
    int32_t auto_reset;
} FutbolConfig;

typedef struct FutbolCtx FutbolCtx;

/* Fill *cfg with the reference's defaults for the registered ids:
   kind V1 + number_of_player 2/5/10 = Futbol2v2-v1 / Futbol5v5-v1 / Futbol-v1,
   kind V0 = Futbol-v0 (random_opp=True, as registered). */
int futbol_config_default(int32_t env_kind, int32_t number_of_player, FutbolConfig* cfg);

/* Create B envs on `device`; env i has global id env_id_base + i (RNG key).
   Runs each env's constructor (which in the reference already calls reset()).
   FUTBOL_EINVAL if env_id_base + B exceeds 32 bits, or if B * 16 or B * obs_dim does not fit 32 bits
   (the kernels' per-env offsets; no GPU memory holds that many envs anyway). */
int futbol_create(const FutbolConfig* cfg, int32_t device, uint64_t seed, uint64_t env_id_base,
                  int32_t num_envs, FutbolCtx** out);
/* Releases every resource of ctx (NULL: no-op) whatever fails; returns FUTBOL_EHIP if a HIP call
   failed, with its text in futbol_last_error(NULL) (the context is gone). */
int futbol_destroy(FutbolCtx* ctx);
const char* futbol_last_error(const FutbolCtx* ctx);

/* obs_dim: floats per env (v1 4*(2N+1), v0 30); action_dim: u8 per env
   (v1 2N, v0 1 if action_as_int else 2). */
int futbol_dims(const FutbolCtx* ctx, int32_t* obs_dim, int32_t* action_dim, int32_t* num_envs);

/* reset() the envs whose mask byte is non-zero (mask == NULL: all) and write
   their obs (rows of the other envs are left untouched). */
int futbol_reset(FutbolCtx* ctx, const uint8_t* mask, void* obs, void* stream);

/* step() all envs.  actions: [B][action_dim] u8.  Writes obs [B][obs_dim],
   reward [B], done [B] (u8); for done envs the episode's final obs goes to
   terminal_obs [B][obs_dim] (may be NULL) and obs holds the reset obs. */
int futbol_step(FutbolCtx* ctx, const uint8_t* actions, void* obs, void* reward, uint8_t* done,
                void* terminal_obs, void* stream);

/* Open-loop rollout: nsteps consecutive futbol_step calls in ONE launch, for callers whose actions
   do not depend on the observations (a recorded or synthetic action sequence, a random policy).
   actions [nsteps][B][action_dim]; obs [nsteps][B][obs_dim]; reward [nsteps][B]; done [nsteps][B];
   terminal_obs [nsteps][B][obs_dim] or NULL -- slice k holds exactly what the k-th futbol_step call
   would have returned (bit-identical; tested).  The envs' blocks do not wait for each other
   between steps.  Not a reference interface: a batch-synchronous VecEnv steps with futbol_step. */
int futbol_rollout(FutbolCtx* ctx, const uint8_t* actions, int32_t nsteps, void* obs, void* reward, uint8_t* done,
                   void* terminal_obs, void* stream);

/* Synthetic policy: actions[i] = iid uniform actions of env (env_id_base+i) at
   `step`: action j = (w * nvals) >> 32, w = word j % 4 of the Philox4x32-10 block
   (counter {j / 4, step, env id, 1}, key = seed).  step == UINT64_MAX: the
   step is the number of earlier UINT64_MAX calls on this context (0, 1, 2, ...),
   counted on the device, so a captured hipGraph draws fresh actions per replay.
   The counter is independent of futbol_step: a fill may run on another stream
   concurrently with a step (double-buffered actions). */
int futbol_fill_actions(FutbolCtx* ctx, uint64_t seed, uint64_t step, uint8_t* actions, void* stream);

/* The fills of `nsteps` consecutive steps in one launch: actions [nsteps][B][action_dim],
   slice t = futbol_fill_actions(ctx, seed, step + t, ...).  step == UINT64_MAX: step is
   the total nsteps of the earlier UINT64_MAX calls of this function on the context (a
   device counter of its own, advanced in stream order).  For benchmark loops: the synthetic policy does not depend on
   observations, so a graph of K steps can draw all K steps' actions up front. */
int futbol_fill_actions_steps(FutbolCtx* ctx, uint64_t seed, uint64_t step, int32_t nsteps, uint8_t* actions,
                              void* stream);

/* Episode statistics since the last clear: out3 (device, f64[3]) =
   {sum of finished-episode returns, finished episodes, env-steps}. */
int futbol_episode_stats(FutbolCtx* ctx, double* out3, int32_t clear, void* stream);

/* Number of out-of-range actions clamped so far (device u64 counter copied to *out; syncs the stream). */
int futbol_invalid_actions(FutbolCtx* ctx, uint64_t* out, void* stream);

/* Raw SoA state, for checkpoint/restore and parity tests.  The layout is
   described field by field: name, byte offset, element type code
   (0 f64, 1 u64, 2 u32, 3 u16, 4 u8), element count.  Vectors are stored as
   consecutive pairs (v1 "pxy" / "vxy" / "bxy": [Nb][B][2]; v0 "row2": the 25
   row entries as [13][B][2], "view2": [4][B][2]); the Python get_state /
   set_state present them as the reference-shaped px, py, ..., row, view
   arrays (csrc/futbol_state.hpp). */
int futbol_state_bytes(const FutbolCtx* ctx, size_t* bytes);
int futbol_state_field(const FutbolCtx* ctx, int32_t index, const char** name, size_t* offset,
                       int32_t* type_code, int64_t* count);
int futbol_get_state(FutbolCtx* ctx, void* dst, int32_t dst_is_host, void* stream);
int futbol_set_state(FutbolCtx* ctx, const void* src, int32_t src_is_host, void* stream);

/* Kernel-side time base: number of steps after which an episode is done
   (the reference accumulates current_time += 0.1 in fp64). */
int futbol_episode_limit(const FutbolCtx* ctx, int32_t* steps);

/* Diagnostic builds only (compiled with -DFUTBOL_STAMPS; FUTBOL_EUNSUPPORTED otherwise):
   per-64-env-block sums of s_memtime cycles spent in each step phase, [blocks][16] u64. */
int futbol_debug_stamps(FutbolCtx* ctx, uint64_t* host_out, int64_t n, int32_t clear);

/* Kernel timing (measurement, not part of the reference interface).  mode 1: start
 * timing the following futbol_step launches (up to 8192) with HIP events stamped by
 * the dispatch itself (hipExtLaunchKernelGGL: kernel begin/end on the launch stream);
 * mode 0: stop, wait for the last timed launch and return the summed kernel time and
 * the number of timed launches.  Not usable inside hipGraph capture. */
int futbol_kernel_timing(FutbolCtx* ctx, int32_t mode, double* total_ms, int64_t* count);

/* HBM copy ceiling (measurement, not part of the reference interface): copies `bytes`
 * (a multiple of 16) from device buffer src to dst with a plain 16-byte-per-lane copy kernel
 * on `stream`.  bench.py times it to report the achievable stream-copy bandwidth next to
 * the 8 TB/s spec (Roofline). */
int futbol_stream_copy(const void* src, void* dst, uint64_t bytes, void* stream);

/* envs_v1 solver layout of the team size's compiled step kernel (host-only query, no GPU; for
 * the parity tests, which must exercise every record path the build ships, and for diagnostics):
 * out[0] LDS contact-record slots per env, [1] spill records held in registers through the solve,
 * [2] arbiter-cache entries preloaded with the state, [3] cache entries per batched read past
 * those, [4] arbiters per env (segment + pair), [5] one set of solver rows, [6] per-component
 * split solve, [7] batched exact squares.  Writes min(n, 8) values (zeros past 8). */
int futbol_solver_layout(int32_t number_of_player, int32_t* out, int32_t n);

#ifdef __cplusplus
}
#endif
#endif
