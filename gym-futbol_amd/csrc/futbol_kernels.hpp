// futbol_kernels.hpp -- launch interface between the C ABI (futbol_capi.hip)
// and the env kernels (futbol_v1.hip, futbol_v0.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stddef.h>
#include <stdint.h>
#include "futbol_state.hpp"

namespace futbol {

// diagnostic stamps buffer (FUTBOL_STAMPS builds): u64 slots per one-wave block
constexpr int kStampStride = 32;

// The 16 distinct bounds of the 12 segment cpBBs (taken from sl/sb/sr/st): the
// circle-vs-segment-BB test of segment s is  cl <= r_s && l_s <= cr && cb <= t_s && b_s <= ct.
struct BBT {
    double r1, rW1, rm1, rW3;   // r_s values
    double lm1, lW1, lm3, lWp1; // l_s values
    double tlo, tH, t1, thi;    // t_s values
    double bm1, bhi, bH, blo;   // b_s values
};

// Per-context constants of an envs_v1 `Futbol` (kernel argument, < 2 KB).
struct V1Params {
    double W, H;                                  // Futbol(width, height)
    double sax[12], say[12], sbx[12], sby[12];    // _setup_walls segments 0..11 (futbol_env.py:182-234)
    double sl[12], sb[12], sr[12], st[12];        // their cpBBs (radius 1 included)
    BBT bbt;
    double fx[21], fy[21];                        // formation of bodies A.., B.., ball (team.py:52-112)
    double L2[12], rL2[12];                       // |b - a|^2 of each segment and RN(1 / that)
    double dtv[3];                                // dt per dt code: {0, 1e-4, 0.1}
    double rdt[3];                                // RN(1 / dt)
    double damp[3];                               // cpfpow(damping 0.95, dt)
    double biasc[3];                              // 1 - cpfpow(collisionBias, dt)
    double slop;                                  // collisionSlop (0.1f)
    double clamp2_player, clamp2_ball;            // largest s with RN(sqrt(s)) <= vmax (limit_velocity)
    double form_vb;                               // formation micro-step: |v_bias| bound of the no-contact fast path
    uint64_t seed;
    uint32_t env_base;                            // global id of env 0
    int B;
    int K_done;                                   // steps until current_time > total_time
    int auto_reset;
};

struct V0Params {
    double length, width, goal_size, player_speed, shoot_speed;
    int ty_lo, ty_hi;                             // randint bounds of target_y (:306)
    int shoot_lo, shoot_hi;                       // randint bounds of the shot speed (:367)
    int one_goal_end, only_reward_goal, random_opp, action_as_int;
    uint64_t seed;
    uint32_t env_base;
    int B;
    int K_done;                                   // steps until time >= game_time
    int auto_reset;
};

// Kernel timing (futbol_kernel_timing): when `start` is set, the next env-step launch
// goes through hipExtLaunchKernelGGL, whose events are stamped by the dispatch itself
// (kernel begin / end, no marker packets around it).  Set by the C ABI, host thread-local.
struct LaunchEvents {
    hipEvent_t start = nullptr, stop = nullptr;
};
extern thread_local LaunchEvents g_launch_events;

template <typename... KArgs, typename... Args>
inline void launch_kernel(void (*k)(KArgs...), dim3 grid, dim3 block, hipStream_t stream, Args... args)
{
    static_assert(sizeof...(KArgs) == sizeof...(Args), "kernel argument count");
    if (g_launch_events.start)
        hipExtLaunchKernelGGL(k, grid, block, 0, stream, g_launch_events.start, g_launch_events.stop, 0,
                              static_cast<KArgs>(args)...);
    else
        hipLaunchKernelGGL(k, grid, block, 0, stream, static_cast<KArgs>(args)...);
}

// P: device pointer to the context's V1Params (wave-uniform scalar loads).  what 0 = step (nsteps
// consecutive steps per launch: the open-loop rollout, futbol_rollout), 1 = reset
int launch_v1(int N, int epw, int def, const V1Params* P, int B, const V1Ptrs& st, int out64, int what,
              const uint8_t* actions, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term,
              int init, int nsteps, hipStream_t stream);
int v1_supported(int N);
int v1_supported_epw(int epw);
size_t v1_spill_slots(int N);
int layout_v1(int N, int32_t* o);  // 8 values, futbol_solver_layout
bool v1_is_default_geometry(int N, const V1Params& p);

int launch_v0(const V0Params* P, int B, const V0Ptrs& st, int out64, int what, const uint8_t* actions,
              const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, int nsteps,
              hipStream_t stream);

int launch_fill_actions(uint64_t seed, uint64_t step, unsigned long long* step_ctr, uint32_t env_base, int B,
                        int adim, int nvals, uint8_t* actions, hipStream_t stream);
int launch_fill_actions_steps(uint64_t seed, uint64_t step0, int nsteps, unsigned long long* ctr, uint32_t env_base,
                              int B, int adim, int nvals, uint8_t* actions, hipStream_t stream);
int launch_stream_copy(const void* src, void* dst, size_t bytes, hipStream_t stream);
int launch_episode_stats(const double* stat_ret, const uint32_t* stat_cnt, int B, double steps, double* out3,
                         int clear, double* stat_ret_w, uint32_t* stat_cnt_w, hipStream_t stream);

}  // namespace futbol
