// futbol_v1_n3_e64.hip -- instantiation of the envs_v1 kernels for N = 3 players per team,
// 64 envs per one-wave block (one translation unit per team size: they compile in parallel).
// def: the default-field instance (compile-time geometry, futbol_v1_params.hpp).
#include "futbol_v1_impl.hpp"

namespace futbol {

int launch_v1_n3_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, int def,
                      const uint8_t* actions, const uint8_t* mask, void* obs, void* reward, uint8_t* done,
                      void* term, int init, hipStream_t stream)
{
    constexpr int N = 3, E = 64;
    const dim3 grid((B + E - 1) / E), block(E);
    if (what == 0) {
        if (out64) {
            if (def)
                launch_kernel(v1_step_kernel<N, E, double, true>, grid, block, stream, P, st, actions, (double*)obs,
                              (double*)reward, done, (double*)term);
            else
                launch_kernel(v1_step_kernel<N, E, double, false>, grid, block, stream, P, st, actions, (double*)obs,
                              (double*)reward, done, (double*)term);
        } else {
            if (def)
                launch_kernel(v1_step_kernel<N, E, float, true>, grid, block, stream, P, st, actions, (float*)obs,
                              (float*)reward, done, (float*)term);
            else
                launch_kernel(v1_step_kernel<N, E, float, false>, grid, block, stream, P, st, actions, (float*)obs,
                              (float*)reward, done, (float*)term);
        }
    } else {
        if (out64)
            hipLaunchKernelGGL((v1_reset_kernel<N, E, double>), grid, block, 0, stream, P, st, mask, (double*)obs,
                               init);
        else
            hipLaunchKernelGGL((v1_reset_kernel<N, E, float>), grid, block, 0, stream, P, st, mask, (float*)obs,
                               init);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace futbol
