// futbol_v1_inst.hpp -- the per-team-size launch function of the envs_v1 kernels.
//
// Every futbol_v1_n<N>_e64.hip translation unit expands FUTBOL_V1_INSTANCE(N) once: one
// TU per team size, so the ten instances (number_of_player = 1..10, the range
// envs_v1/futbol_env.py:63-65 + team.py:52-112 accept) compile in parallel.
// 64 envs per one-wave block; def: the default-field instance (compile-time geometry,
// futbol_v1_params.hpp).
#pragma once
#include "futbol_v1_impl.hpp"

#define FUTBOL_V1_INSTANCE(NP)                                                                                   \
    namespace futbol {                                                                                           \
    int launch_v1_n##NP##_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, int def,          \
                              const uint8_t* actions, const uint8_t* mask, void* obs, void* reward, uint8_t* done, \
                              void* term, int init, int nsteps, hipStream_t stream)                              \
    {                                                                                                            \
        constexpr int N = NP, E = 64;                                                                            \
        const dim3 grid((B + E - 1) / E), block(E);                                                              \
        if (what == 0) {                                                                                         \
            if (out64) {                                                                                         \
                if (def)                                                                                         \
                    launch_kernel(v1_step_kernel<N, E, double, true>, grid, block, stream, P, st, actions,       \
                                  (double*)obs, (double*)reward, done, (double*)term, nsteps);                   \
                else                                                                                             \
                    launch_kernel(v1_step_kernel<N, E, double, false>, grid, block, stream, P, st, actions,      \
                                  (double*)obs, (double*)reward, done, (double*)term, nsteps);                   \
            } else {                                                                                             \
                if (def)                                                                                         \
                    launch_kernel(v1_step_kernel<N, E, float, true>, grid, block, stream, P, st, actions,        \
                                  (float*)obs, (float*)reward, done, (float*)term, nsteps);                      \
                else                                                                                             \
                    launch_kernel(v1_step_kernel<N, E, float, false>, grid, block, stream, P, st, actions,       \
                                  (float*)obs, (float*)reward, done, (float*)term, nsteps);                      \
            }                                                                                                    \
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
    }
