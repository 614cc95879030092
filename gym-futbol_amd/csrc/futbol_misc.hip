// futbol_misc.hip -- synthetic action generation and episode-statistics reduction.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "futbol_kernels.hpp"
#include "futbol_rng.hpp"

namespace futbol {

// Synthetic-policy actions of one env-step: action j = (w * nvals) >> 32 with w = word j % 4 of
// Philox block j / 4 of (seed, env, event = step, tag 1) -- four actions per block.
__device__ __forceinline__ void synthetic_actions(uint64_t seed, uint32_t env_id, uint32_t step, int adim, int nvals,
                                                  uint8_t* out)
{
    const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
    for (int b = 0; b * 4 < adim; ++b) {
        const Philox4 p = philox4x32_10((uint32_t)b, step, env_id, 1u, k0, k1);
        for (int q = 0; q < 4 && b * 4 + q < adim; ++q)
            out[b * 4 + q] = (uint8_t)(((unsigned long long)p.x[q] * (unsigned)nvals) >> 32);
    }
}


// actions[i] = synthetic_actions(seed, env_base + i, step):
// the benchmark's "left agent" (random_action() for the left team, envs_v1/futbol_env.py:306-307).
// fill_ctr != nullptr: the step is this launch's index among the context's counter-driven fills
// (0, 1, 2, ...): every block adds 1 to the counter and divides the old value by the grid size,
// which is exact because such launches are stream-ordered among themselves.  The counter is
// independent of the step kernel, so a fill can run on a second stream concurrently with a step,
// and a captured hipGraph draws fresh actions at every replay.
__global__ void __launch_bounds__(256) fill_actions_kernel(uint64_t seed, uint32_t step, unsigned long long* fill_ctr,
                                                           uint32_t env_base, int B, int adim, int nvals,
                                                           uint8_t* __restrict__ actions)
{
    __shared__ uint32_t s_step;
    if (fill_ctr) {
        if (threadIdx.x == 0) s_step = (uint32_t)(atomicAdd(fill_ctr, 1ull) / gridDim.x);
        __syncthreads();
    }
    const int env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= B) return;
    const uint32_t s = fill_ctr ? s_step : step;
    synthetic_actions(seed, env_base + (uint32_t)env, s, adim, nvals, actions + (size_t)env * adim);
}
int launch_fill_actions(uint64_t seed, uint64_t step, unsigned long long* step_ctr, uint32_t env_base, int B,
                        int adim, int nvals, uint8_t* actions, hipStream_t stream)
{
    hipLaunchKernelGGL(fill_actions_kernel, dim3((B + 255) / 256), dim3(256), 0, stream, seed, (uint32_t)step,
                       step_ctr, env_base, B, adim, nvals, actions);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// actions[t][i][j] for t < nsteps: the fills of steps step0 .. step0 + nsteps - 1 in one launch
// (grid.y = nsteps).  fill_ctr != nullptr: step0 = *fill_ctr, a step counter that
// advance_counter_kernel moves on by nsteps right after, in stream order (one plain load per
// thread here; a per-block atomic would serialise tens of thousands of same-address atomics).
__global__ void __launch_bounds__(256) fill_actions_steps_kernel(uint64_t seed, uint32_t step0,
                                                                 const unsigned long long* fill_ctr,
                                                                 uint32_t env_base, int B, int adim, int nvals,
                                                                 uint8_t* __restrict__ actions)
{
    const int env = blockIdx.x * blockDim.x + threadIdx.x;
    if (env >= B) return;
    const uint32_t t = blockIdx.y;
    const uint32_t s = (fill_ctr ? (uint32_t)*fill_ctr : step0) + t;
    synthetic_actions(seed, env_base + (uint32_t)env, s, adim, nvals, actions + ((size_t)t * B + env) * adim);
}

__global__ void advance_counter_kernel(unsigned long long* ctr, unsigned long long by) { *ctr += by; }

int launch_fill_actions_steps(uint64_t seed, uint64_t step0, int nsteps, unsigned long long* ctr, uint32_t env_base,
                              int B, int adim, int nvals, uint8_t* actions, hipStream_t stream)
{
    hipLaunchKernelGGL(fill_actions_steps_kernel, dim3((B + 255) / 256, nsteps), dim3(256), 0, stream, seed,
                       (uint32_t)step0, ctr, env_base, B, adim, nvals, actions);
    if (ctr) hipLaunchKernelGGL(advance_counter_kernel, dim3(1), dim3(1), 0, stream, ctr, (unsigned long long)nsteps);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// One block, fixed reduction order: reproducible sums.
__global__ void __launch_bounds__(1024) episode_stats_kernel(const double* __restrict__ ret,
                                                             const uint32_t* __restrict__ cnt, int B, double steps,
                                                             double* __restrict__ out3, int clear,
                                                             double* ret_w, uint32_t* cnt_w)
{
    __shared__ double sr[1024];
    __shared__ double sc[1024];
    double a = 0.0, c = 0.0;
    for (int i = threadIdx.x; i < B; i += blockDim.x) {
        a += ret[i];
        c += (double)cnt[i];
    }
    sr[threadIdx.x] = a;
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) {
            sr[threadIdx.x] += sr[threadIdx.x + s];
            sc[threadIdx.x] += sc[threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        out3[0] = sr[0];
        out3[1] = sc[0];
        out3[2] = steps;
    }
    if (clear) {
        __syncthreads();
        for (int i = threadIdx.x; i < B; i += blockDim.x) {
            ret_w[i] = 0.0;
            cnt_w[i] = 0;
        }
    }
}

int launch_episode_stats(const double* stat_ret, const uint32_t* stat_cnt, int B, double steps, double* out3,
                         int clear, double* stat_ret_w, uint32_t* stat_cnt_w, hipStream_t stream)
{
    hipLaunchKernelGGL(episode_stats_kernel, dim3(1), dim3(1024), 0, stream, stat_ret, stat_cnt, B, steps, out3,
                       clear, stat_ret_w, stat_cnt_w);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

// HBM copy ceiling (measurement only: bench.py's roofline.copy_ceiling_gbs, SURVEY 8(d) "a measured
// stream-copy ceiling"): 16 bytes per lane, four independent loads in flight per lane, then four
// stores; blocks of 256 lanes cover 16 KB each.  bytes must be a multiple of 16.
__global__ void __launch_bounds__(256) stream_copy_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst,
                                                          size_t n)
{
    const size_t i0 = (size_t)blockIdx.x * 1024 + threadIdx.x;
    uint4 a[4];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (i0 + (size_t)k * 256 < n) a[k] = src[i0 + (size_t)k * 256];
#pragma unroll
    for (int k = 0; k < 4; ++k)
        if (i0 + (size_t)k * 256 < n) dst[i0 + (size_t)k * 256] = a[k];
}

int launch_stream_copy(const void* src, void* dst, size_t bytes, hipStream_t stream)
{
    const size_t n = bytes / 16;
    const size_t blocks = (n + 1023) / 1024;
    if (blocks == 0) return 0;
    if (blocks > 0x7fffffffull) return -1;
    hipLaunchKernelGGL(stream_copy_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, (const uint4*)src, (uint4*)dst,
                       n);
    return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace futbol
