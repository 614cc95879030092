/*
 * oracle_rng.h -- TEST INFRASTRUCTURE ONLY (never linked into the product).
 *
 * The RNG-tape contract shared by the oracle, the golden generator
 * (tests/golden/gen_v0_golden.py, which feeds the same draws to the real
 * reference through monkey-patched `random` / `np.random`) and the HIP kernels.
 * SURVEY.md Appendix C.
 *
 * One "draw" = one Philox4x32-10 block:
 *   key     = { seed_lo32, seed_hi32 }
 *   counter = { j, event, env_id, tag }
 *     j      program-order draw index inside one event
 *     event  per-env counter, +1 for every step() and every reset()
 *     env_id global env id (shard invariant)
 *     tag    0 = env stream, 1 = synthetic benchmark/left-agent actions
 *            (4 actions per block: action j = (word j%4 of block j/4) * n >> 32)
 *
 * Conversions (fixed, identical everywhere):
 *   U        = ((x0>>5)*2^26 + (x1>>6)) / 2^53               in [0,1)
 *   choice n = min(floor(U*n), n-1)
 *   randint(a,b) = a + choice(b-a+1)
 *   uniform(a,b) = a + (b-a)*U          (CPython random.uniform form)
 *   normal(mu,sigma) = mu + sigma*Z,  Z = sqrt(-2 ln(1-U1)) * cos(2 pi U2)
 *                      U1 from (x0,x1), U2 from (x2,x3); ln and cos are the
 *                      specified +,-,*,/-only orc_pm_log / orc_pm_sincos
 *                      (oracle_math.h), so Z is the same double everywhere
 */
#ifndef ORACLE_RNG_H
#define ORACLE_RNG_H
#include <stdint.h>
#include <math.h>
#include "oracle_math.h"

static inline void oracle_philox4x32_10(const uint32_t ctr_in[4], const uint32_t key_in[2], uint32_t out[4])
{
    uint32_t c0 = ctr_in[0], c1 = ctr_in[1], c2 = ctr_in[2], c3 = ctr_in[3];
    uint32_t k0 = key_in[0], k1 = key_in[1];
    for (int r = 0; r < 10; ++r) {
        if (r) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0;
        uint32_t n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

typedef struct {
    uint64_t seed;
    uint32_t env_id;
    uint32_t event;
    uint32_t j;
    uint32_t tag;
} OracleRng;

static inline void oracle_rng_block(OracleRng *g, uint32_t out[4])
{
    uint32_t ctr[4] = { g->j, g->event, g->env_id, g->tag };
    uint32_t key[2] = { (uint32_t)g->seed, (uint32_t)(g->seed >> 32) };
    oracle_philox4x32_10(ctr, key, out);
    g->j++;
}

static inline double oracle_u53(uint32_t a, uint32_t b)
{
    return ((double)(a >> 5) * 67108864.0 + (double)(b >> 6)) * (1.0 / 9007199254740992.0);
}

static inline double oracle_uniform01(OracleRng *g)
{
    uint32_t x[4];
    oracle_rng_block(g, x);
    return oracle_u53(x[0], x[1]);
}

static inline int oracle_choice(OracleRng *g, int n)
{
    double u = oracle_uniform01(g);
    int k = (int)floor(u * (double)n);
    return k > n - 1 ? n - 1 : k;
}

/* n_draws uniform integers in [0, n) from ceil(n_draws / 4) blocks: value i = (w * n) >> 32 for
   w = word i % 4 of block i / 4 (the v1 opponent's action_space.sample(), and the synthetic
   left-agent actions under tag 1) */
static inline void oracle_words_choice(OracleRng *g, int n_draws, int n, int32_t *out)
{
    uint32_t x[4];
    for (int i = 0; i < n_draws; ++i) {
        if ((i & 3) == 0) oracle_rng_block(g, x);
        out[i] = (int32_t)(((uint64_t)x[i & 3] * (uint64_t)n) >> 32);
    }
}

static inline int oracle_randint(OracleRng *g, int a, int b)
{
    return a + oracle_choice(g, b - a + 1);
}

static inline double oracle_uniform(OracleRng *g, double a, double b)
{
    double u = oracle_uniform01(g);
    return a + (b - a) * u;
}

static inline double oracle_normal(OracleRng *g, double mu, double sigma)
{
    uint32_t x[4];
    oracle_rng_block(g, x);
    double u1 = oracle_u53(x[0], x[1]);
    double u2 = oracle_u53(x[2], x[3]);
    double z = orc_tape_z(u1, u2);
    return mu + sigma * z;
}

#endif
