// futbol_v1_n2.hip -- instantiation of the envs_v1 kernels for N = 2 players per team
// (one translation unit per N so they compile in parallel).
#include "futbol_v1_impl.hpp"

namespace futbol {

int launch_v1_n2(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* actions,
                 const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init,
                 hipStream_t stream)
{
    constexpr int N = 2;
    const dim3 grid((B + 63) / 64), block(64);
    if (what == 0) {
        if (out64)
            hipLaunchKernelGGL((v1_step_kernel<N, double>), grid, block, 0, stream, P, st, actions, (double*)obs,
                               (double*)reward, done, (double*)term);
        else
            hipLaunchKernelGGL((v1_step_kernel<N, float>), grid, block, 0, stream, P, st, actions, (float*)obs,
                               (float*)reward, done, (float*)term);
    } else {
        if (out64)
            hipLaunchKernelGGL((v1_reset_kernel<N, double>), grid, block, 0, stream, P, st, mask, (double*)obs, init);
        else
            hipLaunchKernelGGL((v1_reset_kernel<N, float>), grid, block, 0, stream, P, st, mask, (float*)obs, init);
    }
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

size_t v1_spill_slots_n2() { return V1Shape<2>::P - V1Shape<2>::K; }

}  // namespace futbol
