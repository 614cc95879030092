// futbol_capi.hip -- the C ABI of include/futbol.h: context lifetime, the HBM
// state allocation, constants derived from the reference's constructor
// kwargs, and stream-ordered launches.  No host<->device sync on the
// step/reset path (graph-capturable); no torch types.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <string>
#include <vector>
#include "../../include/futbol.h"
#include "futbol_kernels.hpp"
#include "futbol_v1_params.hpp"
#include "futbol_rng.hpp"

using namespace futbol;

namespace {

struct Field {
    const char* name;
    size_t offset;
    int32_t type;  // 0 f64, 1 u64, 2 u32, 3 u16, 4 u8
    int64_t count;
};

size_t type_size(int t) { return t == 0 || t == 1 ? 8 : (t == 2 ? 4 : (t == 3 ? 2 : 1)); }

thread_local std::string g_create_error;

}  // namespace

struct FutbolCtx {
    FutbolConfig cfg;
    int device = 0;
    uint64_t seed = 0, env_base = 0;
    int B = 0, N = 0, obs_dim = 0, act_dim = 0, K_done = 0;
    int epw = 64;     // envs per one-wave block of the v1 kernels
    int v1_def = 0;   // the default-field (compile-time geometry) kernel applies
    void* d_params = nullptr;
    char* d_state = nullptr;
    size_t state_bytes = 0;
    std::vector<Field> fields;
    double* d_spill = nullptr;
    unsigned long long* d_invalid = nullptr;  // [0] invalid-action count, [1] / [2] counters of the counter-driven fills (blocks)
    V1Ptrs v1{};
    V0Ptrs v0{};
    double steps_since_clear = 0.0;
    unsigned long long* d_stamps = nullptr;  // diagnostic builds (FUTBOL_STAMPS) only
    // futbol_kernel_timing: one (start, stop) event pair per timed step launch
    std::vector<hipEvent_t> t_ev;
    int64_t t_count = 0;
    bool timing = false;
    std::string err;
};

#define FB_CHECK_HIP(ctx, expr)                                                                         \
    do {                                                                                                \
        hipError_t _e = (expr);                                                                         \
        if (_e != hipSuccess) {                                                                         \
            (ctx)->err = std::string(#expr) + ": " + hipGetErrorString(_e);                             \
            return FUTBOL_EHIP;                                                                         \
        }                                                                                               \
    } while (0)

static int fail(FutbolCtx* ctx, int code, const std::string& msg)
{
    if (ctx) ctx->err = msg;
    else g_create_error = msg;
    return code;
}

extern "C" int futbol_config_default(int32_t env_kind, int32_t number_of_player, FutbolConfig* c)
{
    if (!c) return FUTBOL_EINVAL;
    memset(c, 0, sizeof(*c));
    c->abi_version = FUTBOL_ABI_VERSION;
    c->env_kind = env_kind;
    c->out_dtype = FUTBOL_F32;
    // envs_v1/futbol_env.py:19-28,63-65
    c->number_of_player = number_of_player > 0 ? number_of_player : 5;
    c->width = 105;
    c->height = 68;
    c->total_time = 30;
    // envs/futbol_env.py:18-58,134-138
    c->length0 = 105;
    c->width0 = 68;
    c->goal_size0 = 10;
    c->game_time0 = 40;
    c->player_speed0 = 12;
    c->shoot_speed0 = 20;
    c->one_goal_end0 = 0;
    c->action_as_int0 = 1;
    c->only_reward_goal0 = 0;
    c->random_opp0 = 1;
    c->auto_reset = 1;
    return (env_kind == FUTBOL_ENV_V0 || env_kind == FUTBOL_ENV_V1) ? FUTBOL_OK : FUTBOL_EINVAL;
}

// Team._create_pos_array (team.py:52-112), player k of a team
// largest double s with RN(sqrt(s)) <= vmax: `sqrt(s) > vmax` <=> `s > T` (sqrt is correctly
// rounded, hence monotone), which lets the kernel skip the sqrt of limit_velocity when no clamp happens
static double clamp_threshold(double vmax)
{
    double s = vmax * vmax;
    while (sqrt(s) > vmax) s = nextafter(s, 0.0);
    while (sqrt(nextafter(s, INFINITY)) <= vmax) s = nextafter(s, INFINITY);
    return s;
}

// the kernel's 16-bound candidate test must equal cpBBIntersects against every segment bb
static bool bbt_consistent(const V1Params* p)
{
    const BBT& T = p->bbt;
    const double L[12] = {T.lm1, T.lm1, T.lm1, T.lW1, T.lW1, T.lm1, T.lm3, T.lm3, T.lm3, T.lWp1, T.lW1, T.lW1};
    const double Bo[12] = {T.bm1, T.bhi, T.bH, T.bm1, T.bhi, T.bm1, T.blo, T.blo, T.bhi, T.blo, T.blo, T.bhi};
    const double R[12] = {T.r1, T.r1, T.rW1, T.rW1, T.rW1, T.rW1, T.rm1, T.r1, T.r1, T.rW3, T.rW3, T.rW3};
    const double Tt[12] = {T.tlo, T.tH, T.tH, T.tlo, T.tH, T.t1, T.thi, T.tlo, T.thi, T.thi, T.tlo, T.thi};
    for (int s = 0; s < 12; ++s)
        if (L[s] != p->sl[s] || Bo[s] != p->sb[s] || R[s] != p->sr[s] || Tt[s] != p->st[s]) return false;
    return true;
}

static int fill_v1_params(const FutbolConfig* c, uint64_t seed, uint64_t env_base, int B, int K_done, V1Params* p)
{
    // cpSpace defaults (Chipmunk 7 cpSpaceInit): collisionBias cpfpow(1.0f - 0.1f, 60.0f);
    // damping 0.95 (envs_v1/futbol_env.py:99) over dt 1e-4 and 0.1
    const double cbias = pow((double)(1.0f - 0.1f), 60.0);
    V1Pow pw{};
    pw.damp1 = pow(0.95, 0.0001);
    pw.damp2 = pow(0.95, 0.1);
    pw.biasc1 = 1.0 - pow(cbias, 0.0001);
    pw.biasc2 = 1.0 - pow(cbias, 0.1);
    pw.clamp2_player = clamp_threshold(10.0);  // PLAYER_MAX_VELOCITY
    pw.clamp2_ball = clamp_threshold(25.0);    // BALL_MAX_VELOCITY
    *p = v1_params_geometry(c->number_of_player, c->width, c->height, pw);
    p->seed = seed;
    p->env_base = (uint32_t)env_base;
    p->B = B;
    p->K_done = K_done;
    p->auto_reset = c->auto_reset;
    return bbt_consistent(p) ? 0 : -1;
}

// steps until `current_time += 0.1` (fp64, from 0) makes `current_time > total` (v1, :478-481)
static int v1_episode_steps(double total)
{
    double t = 0.0;
    for (int k = 1; k <= kMaxSteps; ++k) {
        t += 0.1;
        if (t > total) return k;
    }
    return -1;
}

// v0 checks `time >= game_time` BEFORE `time += 0.1` (envs/futbol_env.py:712-716)
static int v0_episode_steps(double game_time)
{
    double t = 0.0;
    for (int k = 1; k <= kMaxSteps; ++k) {
        if (t >= game_time) return k;
        t += 0.1;
    }
    return -1;
}

static void fill_v0_params(const FutbolConfig* c, uint64_t seed, uint64_t env_base, int B, int K_done, V0Params* p)
{
    memset(p, 0, sizeof(*p));
    p->length = c->length0;
    p->width = c->width0;
    p->goal_size = c->goal_size0;
    p->player_speed = c->player_speed0;
    p->shoot_speed = c->shoot_speed0;
    // random.randint(goal_down + 3, goal_up - 3) (envs/futbol_env.py:305-306)
    p->ty_lo = (int)(c->width0 / 2 - c->goal_size0 / 2 + 3);
    p->ty_hi = (int)(c->width0 / 2 + c->goal_size0 / 2 - 3);
    // random.randint(shoot_speed - 16, shoot_speed) (:367)
    p->shoot_lo = (int)c->shoot_speed0 - 16;
    p->shoot_hi = (int)c->shoot_speed0;
    p->one_goal_end = c->one_goal_end0;
    p->only_reward_goal = c->only_reward_goal0;
    p->random_opp = c->random_opp0;
    p->action_as_int = c->action_as_int0;
    p->seed = seed;
    p->env_base = (uint32_t)env_base;
    p->B = B;
    p->K_done = K_done;
    p->auto_reset = c->auto_reset;
}

static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

extern "C" int futbol_create(const FutbolConfig* cfg, int32_t device, uint64_t seed, uint64_t env_id_base,
                             int32_t num_envs, FutbolCtx** out)
{
    if (!cfg || !out) return fail(nullptr, FUTBOL_EINVAL, "null argument");
    *out = nullptr;
    if (cfg->abi_version != FUTBOL_ABI_VERSION) return fail(nullptr, FUTBOL_EINVAL, "ABI version mismatch");
    if (num_envs <= 0) return fail(nullptr, FUTBOL_EINVAL, "num_envs must be > 0");
    if (env_id_base + (uint64_t)num_envs > 0xffffffffull)
        return fail(nullptr, FUTBOL_EINVAL, "global env ids must fit in 32 bits");
    if (cfg->out_dtype != FUTBOL_F32 && cfg->out_dtype != FUTBOL_F64) return fail(nullptr, FUTBOL_EINVAL, "out_dtype");
    if (cfg->env_kind == FUTBOL_ENV_V1 && !v1_supported(cfg->number_of_player))
        return fail(nullptr, FUTBOL_EUNSUPPORTED, "number_of_player must be 1..10 (team.py:52-112)");
    if (cfg->env_kind != FUTBOL_ENV_V1 && cfg->env_kind != FUTBOL_ENV_V0)
        return fail(nullptr, FUTBOL_EINVAL, "env_kind");
    if (cfg->env_kind == FUTBOL_ENV_V1) {
        // the N >= 6 step instances address per-env data as a wave-uniform row base plus a 32-bit lane
        // offset (kScalarBase, futbol_v1_impl.hpp): env * 16 bytes (a double2 row element) and the
        // observation element offset env * 4 Nb must fit 32 bits.  Unreachable in practice (10v10 needs
        // ~51 M envs, whose spill area alone exceeds the HBM) -- checked for every N all the same
        const uint64_t nb = 2u * (uint64_t)cfg->number_of_player + 1u;
        if ((uint64_t)num_envs * 16u >= (1ull << 32) || (uint64_t)num_envs * 4u * nb >= (1ull << 32))
            return fail(nullptr, FUTBOL_EINVAL, "num_envs too large for the kernels' 32-bit per-env offsets");
    }

    FutbolCtx* ctx = new FutbolCtx();
    ctx->cfg = *cfg;
    ctx->device = device;
    ctx->seed = seed;
    ctx->env_base = env_id_base;
    ctx->B = num_envs;
    const int B = num_envs;
    hipError_t he = hipSetDevice(device);
    if (he != hipSuccess) {
        delete ctx;
        return fail(nullptr, FUTBOL_EHIP, std::string("hipSetDevice: ") + hipGetErrorString(he));
    }

    size_t off = 0;
    auto add = [&](const char* name, int type, int64_t count) {
        ctx->fields.push_back({name, off, type, count});
        off = align_up(off + type_size(type) * (size_t)count);
    };
    if (cfg->env_kind == FUTBOL_ENV_V1) {
        const int N = cfg->number_of_player, Nb = 2 * N + 1, P = v1_npairs(N);
        ctx->N = N;
        ctx->obs_dim = 4 * Nb;
        ctx->act_dim = 2 * N;
        ctx->K_done = v1_episode_steps(cfg->total_time);
        if (ctx->K_done < 0) {
            delete ctx;
            return fail(nullptr, FUTBOL_EUNSUPPORTED, "total_time too long for the 14-bit step counter");
        }
        for (const char* f : {"pxy", "vxy", "bxy"}) add(f, 0, (int64_t)2 * Nb * B);  // [Nb][B][2]
        add("meta", 1, B);
        add("ep_ret", 0, B);
        add("ckey", 3, (int64_t)P * B);
        add("cjn", 0, (int64_t)P * B);
        add("stat_ret", 0, B);
        add("stat_cnt", 2, B);
    } else {
        ctx->N = 2;
        ctx->obs_dim = 30;
        ctx->act_dim = cfg->action_as_int0 ? 1 : 2;
        ctx->K_done = v0_episode_steps(cfg->game_time0);
        if (ctx->K_done < 0) {
            delete ctx;
            return fail(nullptr, FUTBOL_EUNSUPPORTED, "game_time too long for the 14-bit step counter");
        }
        add("row2", 0, (int64_t)13 * 2 * B);  // [13][B][2] (futbol_state.hpp)
        add("view2", 0, (int64_t)4 * 2 * B);  // [4][B][2]
        add("meta", 1, B);
        add("ep_ret", 0, B);
        add("score", 2, (int64_t)2 * B);
        add("stat_ret", 0, B);
        add("stat_cnt", 2, B);
    }
    ctx->state_bytes = off;
    auto bail = [&](hipError_t e, const char* what) {
        std::string m = std::string(what) + ": " + hipGetErrorString(e);
        futbol_destroy(ctx);
        return fail(nullptr, FUTBOL_ENOMEM, m);
    };
    if ((he = hipMalloc((void**)&ctx->d_state, ctx->state_bytes)) != hipSuccess) return bail(he, "hipMalloc(state)");
    if ((he = hipMemset(ctx->d_state, 0, ctx->state_bytes)) != hipSuccess) return bail(he, "hipMemset(state)");
    if ((he = hipMalloc((void**)&ctx->d_invalid, 3 * sizeof(unsigned long long))) != hipSuccess)
        return bail(he, "hipMalloc(counters)");
    if ((he = hipMemset(ctx->d_invalid, 0, 3 * sizeof(unsigned long long))) != hipSuccess)
        return bail(he, "hipMemset");

    auto fptr = [&](const char* name) -> char* {
        for (auto& f : ctx->fields)
            if (!strcmp(f.name, name)) return ctx->d_state + f.offset;
        return nullptr;
    };
    if (cfg->env_kind == FUTBOL_ENV_V1) {
        const int N = ctx->N;
        const size_t slots = v1_spill_slots(N);
        if ((he = hipMalloc((void**)&ctx->d_spill, slots * 8 * sizeof(double) * (size_t)B)) != hipSuccess)
            return bail(he, "hipMalloc(spill)");
        V1Params hp;
        if (fill_v1_params(cfg, seed, env_id_base, B, ctx->K_done, &hp)) {
            futbol_destroy(ctx);
            return fail(nullptr, FUTBOL_EINVAL, "segment bounding boxes inconsistent (width/height)");
        }
        // FUTBOL_GENERIC=1 forces the runtime-geometry kernel (tests compare both instances)
        const char* gen = getenv("FUTBOL_GENERIC");
        ctx->v1_def = (gen && atoi(gen)) ? 0 : (v1_is_default_geometry(N, hp) ? 1 : 0);
        if ((he = hipMalloc(&ctx->d_params, sizeof(V1Params))) != hipSuccess) return bail(he, "hipMalloc(params)");
        if ((he = hipMemcpy(ctx->d_params, &hp, sizeof(hp), hipMemcpyHostToDevice)) != hipSuccess)
            return bail(he, "hipMemcpy(params)");
        V1Ptrs& s = ctx->v1;
        s.pxy = (double2*)fptr("pxy");
        s.vxy = (double2*)fptr("vxy");
        s.bxy = (double2*)fptr("bxy");
        s.meta = (uint64_t*)fptr("meta");
        s.ep_ret = (double*)fptr("ep_ret");
        s.ckey = (uint16_t*)fptr("ckey");
        s.cjn = (double*)fptr("cjn");
        s.stat_ret = (double*)fptr("stat_ret");
        s.stat_cnt = (uint32_t*)fptr("stat_cnt");
        s.spill = ctx->d_spill;
        s.invalid = ctx->d_invalid;
        s.stamps = nullptr;
#ifdef FUTBOL_STAMPS
        if ((he = hipMalloc((void**)&ctx->d_stamps, (size_t)((B + 63) / 64 + 1) * kStampStride * 8)) != hipSuccess)
            return bail(he, "hipMalloc(stamps)");
        if ((he = hipMemset(ctx->d_stamps, 0, (size_t)((B + 63) / 64) * kStampStride * 8)) != hipSuccess)
            return bail(he, "hipMemset(stamps)");
        s.stamps = ctx->d_stamps;
#endif
#ifdef FUTBOL_CRUMBS
        if ((he = hipHostMalloc((void**)&ctx->d_stamps, (size_t)((B + 63) / 64 + 1) * kStampStride * 8,
                                hipHostMallocMapped | hipHostMallocCoherent)) != hipSuccess)
            return bail(he, "hipHostMalloc(crumbs)");
        memset(ctx->d_stamps, 0, (size_t)((B + 63) / 64 + 1) * kStampStride * 8);
        s.stamps = ctx->d_stamps;
#endif
        int rc = launch_v1(N, ctx->epw, ctx->v1_def, (const V1Params*)ctx->d_params, B, s, 0, 1, nullptr, nullptr, nullptr,
                           nullptr, nullptr, nullptr, 1, 1, 0);
        if (rc) return bail(hipGetLastError(), "launch(init)");
    } else {
        V0Params hp;
        fill_v0_params(cfg, seed, env_id_base, B, ctx->K_done, &hp);
        if ((he = hipMalloc(&ctx->d_params, sizeof(V0Params))) != hipSuccess) return bail(he, "hipMalloc(params)");
        if ((he = hipMemcpy(ctx->d_params, &hp, sizeof(hp), hipMemcpyHostToDevice)) != hipSuccess)
            return bail(he, "hipMemcpy(params)");
        V0Ptrs& s = ctx->v0;
        s.row = (double2*)fptr("row2");
        s.view = (double2*)fptr("view2");
        s.meta = (uint64_t*)fptr("meta");
        s.ep_ret = (double*)fptr("ep_ret");
        s.score = (uint32_t*)fptr("score");
        s.stat_ret = (double*)fptr("stat_ret");
        s.stat_cnt = (uint32_t*)fptr("stat_cnt");
        s.invalid = ctx->d_invalid;
        int rc = launch_v0((const V0Params*)ctx->d_params, B, s, 0, 1, nullptr, nullptr, nullptr, nullptr, nullptr,
                           nullptr, 1, 1, 0);
        if (rc) return bail(hipGetLastError(), "launch(init)");
    }
    if ((he = hipDeviceSynchronize()) != hipSuccess) return bail(he, "init kernel");
    *out = ctx;
    return FUTBOL_OK;
}

extern "C" int futbol_destroy(FutbolCtx* ctx)
{
    if (!ctx) return FUTBOL_OK;
    // every resource is released whatever fails; the first failure is reported (the context is gone
    // afterwards, so its text goes to the global error string)
    hipError_t first = hipSuccess;
    auto keep = [&](hipError_t e) {
        if (first == hipSuccess && e != hipSuccess) first = e;
    };
    keep(hipSetDevice(ctx->device));
    if (ctx->d_state) keep(hipFree(ctx->d_state));
    if (ctx->d_spill) keep(hipFree(ctx->d_spill));
    if (ctx->d_params) keep(hipFree(ctx->d_params));
    if (ctx->d_invalid) keep(hipFree(ctx->d_invalid));
#ifdef FUTBOL_CRUMBS
    if (ctx->d_stamps) keep(hipHostFree(ctx->d_stamps));
#else
    if (ctx->d_stamps) keep(hipFree(ctx->d_stamps));
#endif
    for (auto e : ctx->t_ev)
        if (e) keep(hipEventDestroy(e));
    delete ctx;
    if (first != hipSuccess) {
        g_create_error = std::string("futbol_destroy: ") + hipGetErrorString(first);
        return FUTBOL_EHIP;
    }
    return FUTBOL_OK;
}

extern "C" const char* futbol_last_error(const FutbolCtx* ctx)
{
    return ctx ? ctx->err.c_str() : g_create_error.c_str();
}

extern "C" int futbol_dims(const FutbolCtx* ctx, int32_t* obs_dim, int32_t* action_dim, int32_t* num_envs)
{
    if (!ctx) return FUTBOL_EINVAL;
    if (obs_dim) *obs_dim = ctx->obs_dim;
    if (action_dim) *action_dim = ctx->act_dim;
    if (num_envs) *num_envs = ctx->B;
    return FUTBOL_OK;
}

extern "C" int futbol_episode_limit(const FutbolCtx* ctx, int32_t* steps)
{
    if (!ctx || !steps) return FUTBOL_EINVAL;
    *steps = ctx->K_done;
    return FUTBOL_OK;
}

namespace futbol {
thread_local LaunchEvents g_launch_events;
}

static constexpr int64_t kTimingCap = 8192;

extern "C" int futbol_kernel_timing(FutbolCtx* ctx, int32_t mode, double* total_ms, int64_t* count)
{
    if (!ctx || (mode != 0 && mode != 1)) return FUTBOL_EINVAL;
    FB_CHECK_HIP(ctx, hipSetDevice(ctx->device));
    if (mode == 1) {
        if (ctx->t_ev.empty()) {
            ctx->t_ev.resize(2 * kTimingCap, nullptr);
            for (auto& e : ctx->t_ev) FB_CHECK_HIP(ctx, hipEventCreate(&e));
        }
        ctx->t_count = 0;
        ctx->timing = true;
        return FUTBOL_OK;
    }
    ctx->timing = false;
    double tot = 0.0;
    for (int64_t i = 0; i < ctx->t_count; ++i) {
        float ms = 0.f;
        FB_CHECK_HIP(ctx, hipEventSynchronize(ctx->t_ev[2 * i + 1]));
        FB_CHECK_HIP(ctx, hipEventElapsedTime(&ms, ctx->t_ev[2 * i], ctx->t_ev[2 * i + 1]));
        tot += ms;
    }
    if (total_ms) *total_ms = tot;
    if (count) *count = ctx->t_count;
    return FUTBOL_OK;
}

static int launch(FutbolCtx* ctx, int what, const uint8_t* actions, const uint8_t* mask, void* obs, void* reward,
                  uint8_t* done, void* term, void* stream, int nsteps = 1)
{
    FB_CHECK_HIP(ctx, hipSetDevice(ctx->device));
    const int out64 = ctx->cfg.out_dtype == FUTBOL_F64;
    const bool timed = what == 0 && ctx->timing && ctx->t_count < kTimingCap;
    if (timed) {
        g_launch_events.start = ctx->t_ev[2 * ctx->t_count];
        g_launch_events.stop = ctx->t_ev[2 * ctx->t_count + 1];
        ctx->t_count++;
    }
    int rc;
    if (ctx->cfg.env_kind == FUTBOL_ENV_V1)
        rc = launch_v1(ctx->N, ctx->epw, ctx->v1_def, (const V1Params*)ctx->d_params, ctx->B, ctx->v1, out64, what, actions,
                       mask, obs, reward, done, term, 0, nsteps, (hipStream_t)stream);
    else
        rc = launch_v0((const V0Params*)ctx->d_params, ctx->B, ctx->v0, out64, what, actions, mask, obs, reward,
                       done, term, 0, nsteps, (hipStream_t)stream);
    g_launch_events = LaunchEvents{};
    if (rc) {
        hipError_t e = hipGetLastError();
        return fail(ctx, FUTBOL_EHIP, std::string("kernel launch failed: ") + hipGetErrorString(e));
    }
    return FUTBOL_OK;
}

extern "C" int futbol_reset(FutbolCtx* ctx, const uint8_t* mask, void* obs, void* stream)
{
    if (!ctx) return FUTBOL_EINVAL;
    return launch(ctx, 1, nullptr, mask, obs, nullptr, nullptr, nullptr, stream);
}

extern "C" int futbol_step(FutbolCtx* ctx, const uint8_t* actions, void* obs, void* reward, uint8_t* done,
                           void* terminal_obs, void* stream)
{
    if (!ctx) return FUTBOL_EINVAL;
    if (!actions || !obs || !reward || !done) return fail(ctx, FUTBOL_EINVAL, "null buffer");
    int rc = launch(ctx, 0, actions, nullptr, obs, reward, done, terminal_obs, stream);
    if (rc == FUTBOL_OK) ctx->steps_since_clear += (double)ctx->B;
    return rc;
}

extern "C" int futbol_rollout(FutbolCtx* ctx, const uint8_t* actions, int32_t nsteps, void* obs, void* reward,
                              uint8_t* done, void* terminal_obs, void* stream)
{
    if (!ctx) return FUTBOL_EINVAL;
    if (!actions || !obs || !reward || !done) return fail(ctx, FUTBOL_EINVAL, "null buffer");
    if (nsteps <= 0) return fail(ctx, FUTBOL_EINVAL, "nsteps must be > 0");
    int rc = launch(ctx, 0, actions, nullptr, obs, reward, done, terminal_obs, stream, nsteps);
    if (rc == FUTBOL_OK) ctx->steps_since_clear += (double)ctx->B * nsteps;
    return rc;
}

extern "C" int futbol_fill_actions(FutbolCtx* ctx, uint64_t seed, uint64_t step, uint8_t* actions, void* stream)
{
    if (!ctx || !actions) return FUTBOL_EINVAL;
    FB_CHECK_HIP(ctx, hipSetDevice(ctx->device));
    int nvals = 5;  // MultiDiscrete([5, 5] * N) (envs_v1/futbol_env.py:78-79)
    if (ctx->cfg.env_kind == FUTBOL_ENV_V0) nvals = ctx->cfg.action_as_int0 ? 16 : 4;  // Discrete(16) / Tuple(4, 4)
    unsigned long long* ctr = step == ~(uint64_t)0 ? ctx->d_invalid + 1 : nullptr;
    if (launch_fill_actions(seed, step, ctr, (uint32_t)ctx->env_base, ctx->B, ctx->act_dim, nvals, actions,
                            (hipStream_t)stream))
        return fail(ctx, FUTBOL_EHIP, "fill_actions launch failed");
    return FUTBOL_OK;
}

extern "C" int futbol_fill_actions_steps(FutbolCtx* ctx, uint64_t seed, uint64_t step, int32_t nsteps,
                                         uint8_t* actions, void* stream)
{
    if (!ctx || !actions || nsteps <= 0 || nsteps > 65535) return FUTBOL_EINVAL;
    FB_CHECK_HIP(ctx, hipSetDevice(ctx->device));
    int nvals = 5;
    if (ctx->cfg.env_kind == FUTBOL_ENV_V0) nvals = ctx->cfg.action_as_int0 ? 16 : 4;
    unsigned long long* ctr = step == ~(uint64_t)0 ? ctx->d_invalid + 2 : nullptr;
    if (launch_fill_actions_steps(seed, step, nsteps, ctr, (uint32_t)ctx->env_base, ctx->B, ctx->act_dim, nvals,
                                  actions, (hipStream_t)stream))
        return fail(ctx, FUTBOL_EHIP, "fill_actions_steps launch failed");
    return FUTBOL_OK;
}

extern "C" int futbol_episode_stats(FutbolCtx* ctx, double* out3, int32_t clear, void* stream)
{
    if (!ctx || !out3) return FUTBOL_EINVAL;
    FB_CHECK_HIP(ctx, hipSetDevice(ctx->device));
    double* sr = ctx->cfg.env_kind == FUTBOL_ENV_V1 ? ctx->v1.stat_ret : ctx->v0.stat_ret;
    uint32_t* sc = ctx->cfg.env_kind == FUTBOL_ENV_V1 ? ctx->v1.stat_cnt : ctx->v0.stat_cnt;
    if (launch_episode_stats(sr, sc, ctx->B, ctx->steps_since_clear, out3, clear, sr, sc, (hipStream_t)stream))
        return fail(ctx, FUTBOL_EHIP, "episode_stats launch failed");
    if (clear) ctx->steps_since_clear = 0.0;
    return FUTBOL_OK;
}

extern "C" int futbol_invalid_actions(FutbolCtx* ctx, uint64_t* out, void* stream)
{
    if (!ctx || !out) return FUTBOL_EINVAL;
    FB_CHECK_HIP(ctx, hipSetDevice(ctx->device));
    unsigned long long v = 0;
    FB_CHECK_HIP(ctx, hipMemcpyAsync(&v, ctx->d_invalid, sizeof(v), hipMemcpyDeviceToHost, (hipStream_t)stream));
    FB_CHECK_HIP(ctx, hipStreamSynchronize((hipStream_t)stream));
    *out = v;
    return FUTBOL_OK;
}

extern "C" int futbol_state_bytes(const FutbolCtx* ctx, size_t* bytes)
{
    if (!ctx || !bytes) return FUTBOL_EINVAL;
    *bytes = ctx->state_bytes;
    return FUTBOL_OK;
}

extern "C" int futbol_state_field(const FutbolCtx* ctx, int32_t index, const char** name, size_t* offset,
                                  int32_t* type_code, int64_t* count)
{
    if (!ctx || index < 0 || index >= (int32_t)ctx->fields.size()) return FUTBOL_EINVAL;
    const Field& f = ctx->fields[index];
    if (name) *name = f.name;
    if (offset) *offset = f.offset;
    if (type_code) *type_code = f.type;
    if (count) *count = f.count;
    return FUTBOL_OK;
}

extern "C" int futbol_get_state(FutbolCtx* ctx, void* dst, int32_t dst_is_host, void* stream)
{
    if (!ctx || !dst) return FUTBOL_EINVAL;
    FB_CHECK_HIP(ctx, hipSetDevice(ctx->device));
    FB_CHECK_HIP(ctx, hipMemcpyAsync(dst, ctx->d_state, ctx->state_bytes,
                                     dst_is_host ? hipMemcpyDeviceToHost : hipMemcpyDeviceToDevice,
                                     (hipStream_t)stream));
    if (dst_is_host) FB_CHECK_HIP(ctx, hipStreamSynchronize((hipStream_t)stream));
    return FUTBOL_OK;
}

extern "C" int futbol_set_state(FutbolCtx* ctx, const void* src, int32_t src_is_host, void* stream)
{
    if (!ctx || !src) return FUTBOL_EINVAL;
    FB_CHECK_HIP(ctx, hipSetDevice(ctx->device));
    FB_CHECK_HIP(ctx, hipMemcpyAsync(ctx->d_state, src, ctx->state_bytes,
                                     src_is_host ? hipMemcpyHostToDevice : hipMemcpyDeviceToDevice,
                                     (hipStream_t)stream));
    if (src_is_host) FB_CHECK_HIP(ctx, hipStreamSynchronize((hipStream_t)stream));
    return FUTBOL_OK;
}

extern "C" int futbol_debug_stamps(FutbolCtx* ctx, uint64_t* host_out, int64_t n, int32_t clear)
{
    if (!ctx || !host_out) return FUTBOL_EINVAL;
    if (!ctx->d_stamps) return fail(ctx, FUTBOL_EUNSUPPORTED, "not a FUTBOL_STAMPS diagnostic build / not v1");
    const size_t bytes = (size_t)((ctx->B + 63) / 64) * kStampStride * 8;
    if ((size_t)n * 8 < bytes) return fail(ctx, FUTBOL_EINVAL, "stamps buffer too small");
#ifdef FUTBOL_CRUMBS
    memcpy(host_out, ctx->d_stamps, bytes);  // host memory: readable even after a device fault
    (void)clear;
    return FUTBOL_OK;
#endif
    FB_CHECK_HIP(ctx, hipSetDevice(ctx->device));
    FB_CHECK_HIP(ctx, hipDeviceSynchronize());
    FB_CHECK_HIP(ctx, hipMemcpy(host_out, ctx->d_stamps, bytes, hipMemcpyDeviceToHost));
    if (clear) FB_CHECK_HIP(ctx, hipMemset(ctx->d_stamps, 0, bytes));
    return FUTBOL_OK;
}

extern "C" int futbol_stream_copy(const void* src, void* dst, uint64_t bytes, void* stream)
{
    if (!src || !dst || (bytes & 15u)) return fail(nullptr, FUTBOL_EINVAL, "stream_copy: null buffer or bytes % 16");
    return launch_stream_copy(src, dst, (size_t)bytes, (hipStream_t)stream) == 0 ? FUTBOL_OK : FUTBOL_EHIP;
}

extern "C" int futbol_solver_layout(int32_t number_of_player, int32_t* out, int32_t n)
{
    if (!out || n < 1) return fail(nullptr, FUTBOL_EINVAL, "solver_layout: null out or n < 1");
    if (!v1_supported(number_of_player)) return fail(nullptr, FUTBOL_EINVAL, "solver_layout: number_of_player");
    int32_t o[8];
    layout_v1(number_of_player, o);
    for (int i = 0; i < n; ++i) out[i] = i < 8 ? o[i] : 0;
    return FUTBOL_OK;
}
