// futbol_rng.hpp -- counter-based RNG of the vectorised envs (device + host).
//
// Every stochastic call of the reference (python `random`, gym's
// `MultiDiscrete.sample`, `np.random.normal`) becomes one Philox4x32-10 block
// addressed by (seed, global env id, per-env event counter, draw index j):
//   key = {seed_lo, seed_hi},  counter = {j, event, env_id, tag}
// tag 0 = env stream, tag 1 = synthetic left-agent actions (benchmark policy).
// Draw conversions: SURVEY.md Appendix C.  Because the counter carries the
// GLOBAL env id, an env's trajectory does not depend on how envs are sharded
// over GPUs (tests/test_distributed_gloo.py, tests/test_gpu_v1_parity.py::test_sharding_invariance).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "futbol_math.hpp"

namespace futbol {

struct Philox4 {
    uint32_t x[4];
};

__host__ __device__ inline Philox4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                 uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c1 ^ k0;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c3 ^ k1;
        c1 = (uint32_t)p1;
        c3 = (uint32_t)p0;
        c0 = n0;
        c2 = n2;
    }
    Philox4 o;
    o.x[0] = c0;
    o.x[1] = c1;
    o.x[2] = c2;
    o.x[3] = c3;
    return o;
}

__host__ __device__ inline double u53(uint32_t a, uint32_t b)
{
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// One env's draw stream inside one event.
struct Stream {
    uint32_t k0, k1, env, event, j, tag;

    __host__ __device__ Stream(uint64_t seed, uint32_t env_id, uint32_t ev, uint32_t tg = 0)
        : k0((uint32_t)seed), k1((uint32_t)(seed >> 32)), env(env_id), event(ev), j(0), tag(tg) {}

    __host__ __device__ inline Philox4 next() { return philox4x32_10(j++, event, env, tag, k0, k1); }

    // the blocks of the next n draws, without consuming them (the v0 kernel computes them at a
    // converged point and lets each exclusive branch take its draws by position; skip() then
    // consumes what the lane's branch used)
    template <int n>
    __host__ __device__ inline void lookahead(Philox4 (&b)[n]) const
    {
#pragma unroll
        for (int i = 0; i < n; ++i) b[i] = philox4x32_10(j + (uint32_t)i, event, env, tag, k0, k1);
    }
    __host__ __device__ inline void skip(uint32_t n) { j += n; }
    // the block of draw index pos of this stream (absolute, consumed or not)
    __host__ __device__ inline Philox4 block(uint32_t pos) const { return philox4x32_10(pos, event, env, tag, k0, k1); }

    __host__ __device__ static inline double uniform01_of(const Philox4& p) { return u53(p.x[0], p.x[1]); }
    // random.choice over n items / gym MultiDiscrete.sample for one component
    __host__ __device__ static inline int choice_of(const Philox4& p, int n)
    {
        const double u = uniform01_of(p);
        int k = (int)floor(u * (double)n);
        return k > n - 1 ? n - 1 : k;
    }
    __host__ __device__ static inline int randint_of(const Philox4& p, int a, int b) { return a + choice_of(p, b - a + 1); }
    // CPython random.uniform: a + (b - a) * random()
    __host__ __device__ static inline double uniform_of(const Philox4& p, double a, double b)
    {
        const double u = uniform01_of(p);
        return a + (b - a) * u;
    }

    __host__ __device__ inline double uniform01() { return uniform01_of(next()); }
    __host__ __device__ inline int choice(int n) { return choice_of(next(), n); }
    __host__ __device__ inline int randint(int a, int b) { return randint_of(next(), a, b); }
    __host__ __device__ inline double uniform(double a, double b) { return uniform_of(next(), a, b); }
    // np.random.normal(mu, sigma): Box-Muller on one block
    __host__ __device__ inline double normal(double mu, double sigma) { return normal_of(next(), mu, sigma); }
    // the same from an already drawn block (the v0 kernel draws it in order and transforms it later)
    __host__ __device__ static inline double normal_of(const Philox4& p, double mu, double sigma)
    {
        const double a = u53(p.x[0], p.x[1]);
        const double b = u53(p.x[2], p.x[3]);
        const double z = sqrt(-2.0 * pm_log(1.0 - a)) * pm_cos(6.283185307179586 * b);
        return mu + sigma * z;
    }
};

}  // namespace futbol
