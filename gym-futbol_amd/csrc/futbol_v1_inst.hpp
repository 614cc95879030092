// futbol_v1_inst.hpp -- the per-team-size launch function of the envs_v1 kernels.
//
// Every futbol_v1_n<N>_e64.hip translation unit expands FUTBOL_V1_INSTANCE(N) once: one
// TU per team size, so the ten instances (number_of_player = 1..10, the range
// envs_v1/futbol_env.py:63-65 + team.py:52-112 accept) compile in parallel.
// 64 envs per one-wave block; def: the default-field instance (compile-time geometry,
// futbol_v1_params.hpp).
#pragma once
#include "futbol_v1_impl.hpp"

namespace futbol {
// the step kernel instance for the output type / geometry / rollout flags (ROLL: nsteps > 1)
template <int N, typename OT>
inline void launch_v1_step(const V1Params* P, int B, const V1Ptrs& st, int def, const uint8_t* actions, void* obs,
                           void* reward, uint8_t* done, void* term, int nsteps, hipStream_t stream)
{
    constexpr int E = 64;
    const dim3 grid((B + E - 1) / E), block(E);
    OT *o = (OT*)obs, *r = (OT*)reward, *t = (OT*)term;
    if (nsteps > 1) {
        if (def) launch_kernel(v1_step_kernel<N, E, OT, true, true>, grid, block, stream, P, st, actions, o, r, done, t, nsteps);
        else launch_kernel(v1_step_kernel<N, E, OT, false, true>, grid, block, stream, P, st, actions, o, r, done, t, nsteps);
    } else {
        if (def) launch_kernel(v1_step_kernel<N, E, OT, true, false>, grid, block, stream, P, st, actions, o, r, done, t, 1);
        else launch_kernel(v1_step_kernel<N, E, OT, false, false>, grid, block, stream, P, st, actions, o, r, done, t, 1);
    }
}
}  // namespace futbol

#define FUTBOL_V1_INSTANCE(NP)                                                                                   \
    namespace futbol {                                                                                           \
    int launch_v1_n##NP##_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, int def,          \
                              const uint8_t* actions, const uint8_t* mask, void* obs, void* reward, uint8_t* done, \
                              void* term, int init, int nsteps, hipStream_t stream)                              \
    {                                                                                                            \
        constexpr int N = NP, E = 64;                                                                            \
        const dim3 grid((B + E - 1) / E), block(E);                                                              \
        if (what == 0) {                                                                                         \
            if (out64) launch_v1_step<N, double>(P, B, st, def, actions, obs, reward, done, term, nsteps, stream); \
            else launch_v1_step<N, float>(P, B, st, def, actions, obs, reward, done, term, nsteps, stream);      \
        } else {                                                                                                 \
            if (out64)                                                                                           \
                hipLaunchKernelGGL((v1_reset_kernel<N, E, double>), grid, block, 0, stream, P, st, mask,         \
                                   (double*)obs, init);                                                          \
            else                                                                                                 \
                hipLaunchKernelGGL((v1_reset_kernel<N, E, float>), grid, block, 0, stream, P, st, mask,          \
                                   (float*)obs, init);                                                           \
        }                                                                                                        \
        return hipGetLastError() == hipSuccess ? 0 : -1;                                                         \
    }                                                                                                            \
    /* the solver layout THIS translation unit was compiled with (futbol_solver_layout) */                      \
    void layout_v1_n##NP##_e64(int32_t* o)                                                                       \
    {                                                                                                            \
        constexpr int N = NP;                                                                                    \
        o[0] = V1Shape<N>::K;                                                                                    \
        o[1] = KXN<N>;                                                                                           \
        o[2] = CKN<N>;                                                                                           \
        o[3] = CBN<N>;                                                                                           \
        o[4] = V1Shape<N>::P;                                                                                    \
        o[5] = V1Shape<N>::ONE_ROWS ? 1 : 0;                                                                     \
        o[6] = kSolveComponents<N> ? 1 : 0;                                                                      \
        o[7] = kSqBatch<N> ? 1 : 0;                                                                              \
    }                                                                                                            \
    }
