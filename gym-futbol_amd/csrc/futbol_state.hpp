// futbol_state.hpp -- HBM layout of a context's env state (struct of arrays).
//
// Every per-env quantity is an array over the B envs of the context, so lane
// i of a wave touches element i: all loads/stores of a wave coalesce.  Arrays
// of per-body or per-pair quantities are [k][B].
//
// v1 (envs_v1.Futbol, Nb = 2N+1 bodies in the order A0..A(N-1),B0..B(N-1),ball):
//   pxy vxy bxy       : f64 [Nb][B][2] cpBody.p, .v, .v_bias as (x, y) pairs: one 16-byte
//                                    load / store per lane and vector (half the memory
//                                    instructions of separate x and y arrays)
//   meta              : u64 [B]       packed scalars, see Meta below
//   ep_ret            : f64 [B]       running return of the current episode
//   ckey              : u16 [P][B]    arbiter cache: pair id | age << 12
//   cjn               : f64 [P][B]    arbiter cache: jnAcc of the pair's contact
//   stat_ret, stat_cnt: f64/u32 [B]   finished-episode return sum / count
// v0 (envs.FutbolEnv):
//   row2              : f64 [13][B][2] obs rows ai_1, ai_2, opp_1, opp_2, ball x 5 = 25 entries,
//                                     stored as consecutive pairs (one 16-byte access per pair)
//   view2             : f64 [4][B][2] frozen Easy_Agent views (ai_1, ai_2, opp_1, opp_2) x (x,y)
//   meta, ep_ret, score (u32 [2][B]), stat_ret, stat_cnt
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace futbol {

// meta word bit layout (u64)
//  bits  0..2  v1: ball_owner_side (0 left, 1 right) | v0: ball_owner (0..4)
//  bits  3..5  v0: last_ball_owner
//  bits  6..7  v1: dt code of the last cpSpaceStep (0 none, 1 1e-4, 2 0.1)
//  bit   6     v0: views_live,   bit 7 v0: owner row valid (a step has run since reset)
//  bits  8..17 v1: number of live arbiter-cache entries
//  bits 18..31 steps since reset (episode length so far)
//  bits 32..63 RNG event counter
struct Meta {
    uint64_t w;
    __host__ __device__ uint32_t owner() const { return (uint32_t)(w & 7u); }
    __host__ __device__ void set_owner(uint32_t o) { w = (w & ~(uint64_t)7u) | (uint64_t)(o & 7u); }
    __host__ __device__ uint32_t last_owner() const { return (uint32_t)((w >> 3) & 7u); }
    __host__ __device__ void set_last_owner(uint32_t o) { w = (w & ~((uint64_t)7u << 3)) | ((uint64_t)(o & 7u) << 3); }
    __host__ __device__ uint32_t dtcode() const { return (uint32_t)((w >> 6) & 3u); }
    __host__ __device__ void set_dtcode(uint32_t c) { w = (w & ~((uint64_t)3u << 6)) | ((uint64_t)(c & 3u) << 6); }
    __host__ __device__ bool bit(int b) const { return (w >> b) & 1u; }
    __host__ __device__ void set_bit(int b, bool v) { w = (w & ~((uint64_t)1u << b)) | ((uint64_t)(v ? 1u : 0u) << b); }
    __host__ __device__ uint32_t ncache() const { return (uint32_t)((w >> 8) & 0x3ffu); }
    __host__ __device__ void set_ncache(uint32_t n) { w = (w & ~((uint64_t)0x3ffu << 8)) | ((uint64_t)(n & 0x3ffu) << 8); }
    __host__ __device__ uint32_t steps() const { return (uint32_t)((w >> 18) & 0x3fffu); }
    __host__ __device__ void set_steps(uint32_t s) { w = (w & ~((uint64_t)0x3fffu << 18)) | ((uint64_t)(s & 0x3fffu) << 18); }
    __host__ __device__ uint32_t event() const { return (uint32_t)(w >> 32); }
    __host__ __device__ void set_event(uint32_t e) { w = (w & 0xffffffffull) | ((uint64_t)e << 32); }
};

constexpr int kMaxSteps = 0x3fff;
constexpr int kNSeg = 12;

__host__ __device__ constexpr int v1_nbodies(int N) { return 2 * N + 1; }
__host__ __device__ constexpr int v1_npairs(int N) { return v1_nbodies(N) * kNSeg + v1_nbodies(N) * (v1_nbodies(N) - 1) / 2; }

struct V1Ptrs {
    double2 *pxy, *vxy, *bxy;  // [Nb][B]
    uint64_t* meta;
    double* ep_ret;
    uint16_t* ckey;
    double* cjn;
    double* stat_ret;
    uint32_t* stat_cnt;
    double* spill;        // contact records beyond the LDS capacity: [B][P - K][8]
    unsigned long long* invalid;  // count of clamped out-of-range actions
    unsigned long long* stamps;   // diagnostic builds only (FUTBOL_STAMPS): [blocks][16] cycle sums
};

struct V0Ptrs {
    double2* row;   // [13][B]: (row entry 2q, 2q + 1) pairs of the [25] rows (entry 25: pad)
    double2* view;  // [4][B]: (x, y) of each frozen view
    uint64_t* meta;
    double* ep_ret;
    uint32_t* score;  // [2][B]
    double* stat_ret;
    uint32_t* stat_cnt;
    unsigned long long* invalid;
};

}  // namespace futbol
