// futbol_v1_impl.hpp -- envs_v1 `Futbol` step as one HIP kernel for gfx950.
//
// Reference: gym_futbol/envs_v1/futbol_env.py (step :427-483), team.py,
// ball.py, player.py, and the Chipmunk2D 7.0.x cpSpaceStep that pymunk 5.6
// runs under them.  One env per lane; the lane keeps
// its env's bodies in registers (fp64, like cpFloat), reads/writes the SoA
// state once per step (coalesced), draws the opponent's actions and every
// other random choice from a counter-based Philox stream, and implements
// DummyVecEnv's auto-reset in the same launch.
//
// Exactness: -ffp-contract=off, only correctly rounded + - * / sqrt, and the
// reference's operation order everywhere, so results are bit-identical to the
// CPU oracle (tests/test_gpu_v1_parity.py).  Division by a constant c uses
// q0 = x*rc, r = fma(-q0, c, x), q = fma(r, rc, q0) with rc = RN(1/c)
// (Markstein's correction; equal to the IEEE quotient for every constant divisor the
// default-geometry kernels use on 6e6 random and near-midpoint samples each,
// tests/test_cdiv.py).
//
// Contacts: narrowphase over all Nb*12 circle-segment and Nb(Nb-1)/2
// circle-circle pairs in the canonical order with exact
// broadphase rejections (cpBBIntersects; an "interior" test that provably
// rejects all 12 segments at once).  A body's candidate segments are
// compacted into a per-lane bit mask and visited in ascending order, so a wave
// iterates max-over-lanes candidates, not the union.  Contact records live in
// LDS (K slots per lane, lane-contiguous: conflict-free) and beyond K in a
// global spill area, so there is no capacity limit.  The sequential-impulse
// solve keeps v / v_bias in LDS (double2, per-lane dynamic body index).  The
// persistent arbiter cache is a compact per-env list of (pair, age, jnAcc);
// its first CK entries are preloaded into registers with independent loads.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <type_traits>
#include "futbol_kernels.hpp"
#include "futbol_math.hpp"
#include "futbol_v1_params.hpp"
#include "futbol_rng.hpp"
#include "futbol_state.hpp"
#include "futbol_util.hpp"

namespace futbol {

// ---- reference constants, envs_v1/futbol_env.py:19-50, player.py:7, ball.py:7
constexpr double kPlayerR = 1.5, kBallR = 1.0, kSegR = 1.0;
constexpr double kPlayerMinv = 1.0 / 20.0, kBallMinv = 1.0 / 10.0;
constexpr double kPlayerVmax = 10.0, kBallVmax = 25.0;
constexpr double kE = 0.2;  // elasticity of players and ball; segments 0
// arbiter-cache entries preloaded into registers: FUTBOL_CK_SMALL (6) for N < 5, FUTBOL_CK_LARGE (4) for
// N = 5 (a lane with more than CKN entries sends its whole wave through the batched lookup loops; 8
// until round 5, when the hit-mask lookups made those loops cheap for 5v5: 8 -> 4 entries, 50.1 ->
// 49.3 us; 3 equal, 2 and 6 no gain)
#ifndef FUTBOL_CK_LARGE
#define FUTBOL_CK_LARGE 4
#endif
#ifndef FUTBOL_CK_SMALL
#define FUTBOL_CK_SMALL 6
#endif
// N >= 6: 2 (register pressure: those instances run at the 512-VGPR limit with spills, where code
// generation failed the instance matrix test with 8, DESIGN.md section 6 "compiler")
#ifndef FUTBOL_CK_BIG
#define FUTBOL_CK_BIG 2
#endif
template <int N>
constexpr int CKN = N >= 6 ? FUTBOL_CK_BIG : (N >= 5 ? FUTBOL_CK_LARGE : FUTBOL_CK_SMALL);
// entries beyond CKN read per batch of independent loads: each batch is one memory round trip on
// the lane's lookup and filter loops (10v10 189 -> 174 us with 4 instead of 1, -2% more with 8;
// 5v5 neutral)
#ifndef FUTBOL_CBN_LARGE
#define FUTBOL_CBN_LARGE 8
#endif
template <int N>
constexpr int CBN = N >= 5 ? FUTBOL_CBN_LARGE : 4;
// spill records (slots past the LDS ones) an item of the split solve holds in registers for its
// 10 sweeps: read from the global spill area once, written back once.  The 5v5 instance spills on
// 13% of its waves (4 measured best: 2 / 6 slower), 10v10 (2 LDS slots) on most (2 best, 4 neutral);
// 2v2 almost never.  Records past these still go through the global loop.
#ifndef FUTBOL_SPILL_REGS
#define FUTBOL_SPILL_REGS 4
#endif
#ifndef FUTBOL_SPILL_REGS_BIG  // N >= 6 (10v10 with 4 LDS slots: 0 -> 2 -> 4, 166 -> 161.5 -> 158.8 us)
#define FUTBOL_SPILL_REGS_BIG 4
#endif
#ifndef FUTBOL_SPILL_REGS2
#define FUTBOL_SPILL_REGS2 0
#endif
// (N = 6..10 share one count; N = 1, 3, 4 rarely spill: none)
template <int N>
constexpr int KXN = N == 5 ? FUTBOL_SPILL_REGS : (N >= 6 ? FUTBOL_SPILL_REGS_BIG : (N == 2 ? FUTBOL_SPILL_REGS2 : 0));
// envs_v1's exact squares (glibc pow) as one batch per site with LDS-staged tables (N <= 5), or one
// body / player at a time with the tables read from global memory (N >= 6: the large instances run at
// the register limit, where the batches' arrays added spills and the code-generation faults moved in)
#ifndef FUTBOL_SQ_BATCH_MAX  // diagnostic knob (the round-4 N = 6 build batched every N's squares)
#define FUTBOL_SQ_BATCH_MAX 5
#endif
template <int N>
constexpr bool kSqBatch = N <= FUTBOL_SQ_BATCH_MAX;
// (N >= FUTBOL_POW_CALL_MIN: the per-body glibc squares' slow path as a call, glibc_pow2_full_call)
#ifndef FUTBOL_POW_CALL_MIN
#define FUTBOL_POW_CALL_MIN 99
#endif
template <int N>
constexpr bool kPowCall = N >= FUTBOL_POW_CALL_MIN;

// Diagnostic build only (-DFUTBOL_STAMPS, bench.py --stamps): per-wave s_memtime at phase
// boundaries, accumulated into st.stamps[wave][slot] (kStampStride slots per wave: 0-10 phases,
// 11-14 the launch snapshot, 15 solver records, 16-23 sub-phases: 16-19 space_step, 20-21 the action
// phase's squares and player loop, 22 the cache lookups).  Never compiled into the product.
#ifdef FUTBOL_STAMPS
#define FUTBOL_STAMP(slot)                                                                                \
    do {                                                                                                  \
        __builtin_amdgcn_s_waitcnt(0);                                                                    \
        const unsigned long long _t = __builtin_amdgcn_s_memtime();                                      \
        __builtin_amdgcn_s_waitcnt(0);                                                                    \
        if ((threadIdx.x & 63) == 0 && st_stamps) {                                                       \
            atomicAdd(&st_stamps[(size_t)(blockIdx.x * EPW / 64) * kStampStride + (slot)], _t - _stamp_prev);                            \
        }                                                                                                 \
        _stamp_prev = _t;                                                                                 \
    } while (0)
// wave-uniform event counts for the tail study (slots 26-31): added once per wave by lane 0
#define FUTBOL_STAT(slot, val)                                                                            \
    do {                                                                                                  \
        const unsigned long long _v = (unsigned long long)(val);                                          \
        if ((threadIdx.x & 63) == 0 && st_stamps)                                                         \
            atomicAdd(&st_stamps[(size_t)(blockIdx.x * EPW / 64) * kStampStride + (slot)], _v);           \
    } while (0)
#else
#define FUTBOL_STAMP(slot) do { } while (0)
#define FUTBOL_STAT(slot, val) do { } while (0)
#endif

// Diagnostic builds only.
// -DFUTBOL_BOUNDS (FUTBOL_BUILD_VARIANT=bounds): index checks that set bit 40 + code of the
// invalid-action counter and clamp the index instead of faulting.
// -DFUTBOL_CRUMBS (FUTBOL_BUILD_VARIANT=crumbs): every wave publishes the last phase it entered
// into host-coherent memory (system scope), readable after a device fault.
#ifdef FUTBOL_BOUNDS
#define FB_BOUND(L, cond, code, fix)                                                                     \
    do {                                                                                                  \
        if (!(cond)) {                                                                                    \
            atomicOr((L).dbg, 1ull << (40 + (code)));                                                     \
            fix;                                                                                          \
        }                                                                                                 \
    } while (0)
#else
#define FB_BOUND(L, cond, code, fix) do { } while (0)
#endif
#ifdef FUTBOL_CRUMBS
#define FUTBOL_CRUMB(L, k)                                                                                \
    do {                                                                                                  \
        if (((L).lane & 63) == 0)                                                                         \
            __hip_atomic_store(&(L).crumbs[(size_t)blockIdx.x * 16], (unsigned long long)(k),            \
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);                              \
        __threadfence_system();                                                                           \
    } while (0)
#else
#define FUTBOL_CRUMB(L, k) do { } while (0)
#endif

// the split solve works per connected component of an env's contact graph: body labels in 4-bit
// fields (Nb <= 16), slot masks in kSlotBits-bit fields of a u64 (8 bits for Nb <= 8, 4 bits for
// the 5v5 instance's 4 LDS slots).  Enabled for N <= 3: the 5v5 instance measured 2% slower with
// it (its tail waves are envs past the LDS record slots, solved as one item anyway), 10v10 has
// more bodies than 4-bit labels hold
template <int N>
constexpr int kSlotBits = 2 * N + 1 <= 8 ? 8 : 4;
template <int N>
constexpr bool kSolveComponents = 2 * N + 1 <= 8;

#ifndef FUTBOL_K2
#define FUTBOL_K2 7
#endif
#ifndef FUTBOL_K5
#define FUTBOL_K5 4
#endif
// N = 8..10 (one set of solver rows): as many slots as keep a block within 40 KB (4 blocks per CU);
// records past the slots are re-read from the global spill area in every sweep (10v10: 2 -> 4 slots,
// 175 -> 166 us)
#ifndef FUTBOL_K8
#define FUTBOL_K8 5
#endif
#ifndef FUTBOL_K9
#define FUTBOL_K9 4
#endif
#ifndef FUTBOL_K10
#define FUTBOL_K10 4
#endif
// One set of solver rows (N >= FUTBOL_ONE_ROWS_MIN, round 4): the LDS holds Nb + 1 rows per lane
// instead of 2 Nb + 1 -- the narrowphase stages positions, then velocities, in the same rows (each
// record's bounce is a second pass over the contact work list), and the split solve runs the v half
// and then the v_bias half on them.  It brings N = 8..10 from 3 one-wave blocks per CU (53 KB of LDS
// each: 65 536 envs in two rounds of waves) to 4 (one round); the halves cost nothing extra there, since
// 2 x (envs with contacts) items took two rounds of the wave's lanes anyway.
#ifndef FUTBOL_ONE_ROWS_MIN
#define FUTBOL_ONE_ROWS_MIN 8
#endif
template <int N>
struct V1Shape {
    static constexpr int Nb = 2 * N + 1;
    static constexpr int BALL = 2 * N;
    static constexpr int P = v1_npairs(N);
    static constexpr bool ONE_ROWS = N >= FUTBOL_ONE_ROWS_MIN;
    static constexpr int NROWS = ONE_ROWS ? Nb + 1 : 2 * Nb + 1;
    // LDS contact-record slots per lane: 4 one-wave blocks per CU must fit in 160 KB
    // (40 KB per block: K * 4 KB of records + (2 Nb + 1) KB of solver velocity rows + the segment table;
    // N = 8..10: Nb + 1 KB of rows, ONE_ROWS)
    static constexpr int K = N == 1 ? 8 : (N == 2 ? FUTBOL_K2 : (N == 3 ? 6 : (N == 4 ? 5 : (N == 5 ? FUTBOL_K5 :
                             (N == 6 ? 3 : (N == 7 ? 2 : (N == 8 ? FUTBOL_K8 : (N == 9 ? FUTBOL_K9 : FUTBOL_K10))))))));
};

__device__ __forceinline__ double minv_of(int k, int ball) { return k == ball ? kBallMinv : kPlayerMinv; }

// correctly rounded x / c for a constant c > 0 with rc = RN(1/c).  The quotient has x's sign
// (c > 0), which copysign restores for x = -0 (the correction step alone would give +0) -- a
// bit operation instead of a compare and select
__device__ __forceinline__ double cdiv(double x, double c, double rc)
{
    const double q0 = x * rc;
    const double r = __builtin_fma(-q0, c, x);
    return __builtin_copysign(__builtin_fma(r, rc, q0), x);
}

struct SegLds {
    double ax, ay, sdx, sdy, L2, rL2;
};

// EPW = envs (active lanes) per one-wave block.  Fewer than 64 leaves lanes idle but
// puts several waves on each SIMD at B = 65536, which hides latency and balances
// the per-wave work (the kernel ends with its slowest wave).
template <int N, int EPW>
struct Scratch {
    using S = V1Shape<N>;
    // LDS contact slots per lane: the same at every EPW, so that 64/EPW times as many blocks fit per CU
    static constexpr int K = S::K;
    // contact record s of lane l: rec[s][0][l] = (nx, ny), [1] = (nMass, info bits),
    // [2] = (bias, -bounce), [3] = (jBias, jnAcc): element h of [2] / [3] belongs to half h of
    // the split solve (h = 0: v_bias / jBias chain, h = 1: v / jnAcc chain)
    double2 rec[K][4][EPW];
    // solver rows, one double2 per body and lane: rows[k] = body k's v_bias (k < Nb),
    // rows[Nb] = the static body Z (v = v_bias = +0 forever: its inverse mass is 0), rows[2 Nb - k]
    // = body k's v.  A record's row offset off = k * ROW (Z: Nb * ROW) addresses half h's row
    // as rows[0] + off (h = 0) or rows[2 Nb] - off (h = 1): both halves reach Z with no select.
    // During the narrowphase the same rows stage the bodies' positions (v_bias rows) and
    // velocities (v rows) for the per-lane dynamic body index.
    // (S::ONE_ROWS: rows[k] is body k's v, then v_bias, in turn; Z = rows[Nb])
    double2 rows[S::NROWS][EPW];
    double minv[S::Nb + 1];  // inverse mass by row: players, ball, Z = 0
    // split solve work list (+ a spare entry): env column (6 bits) | LDS record slots (8) << 6 | dt code of
    // the env's previous cpSpaceStep (warm-start dt ratio, 2) << 14 | the env's record count << 16
    uint32_t item[EPW + 1];
    SegLds seg[kNSeg];

    __device__ __forceinline__ double2& vb(int k, int l) { return rows[k][l]; }
    __device__ __forceinline__ double2& v(int k, int l) { return rows[S::ONE_ROWS ? k : 2 * S::Nb - k][l]; }
};

// info word (64 bits, stored as the bits of a double; only the low 32 are used):
//   a (5 bits) | bcode (6 bits: body id, or 32 + segment) << 5 | pair << 11 | normal << 20
__device__ __forceinline__ long long pack_info(int a, int bcode, int pair, bool normal)
{
    return (long long)(uint32_t)(a | (bcode << 5) | (pair << 11) | ((normal ? 1 : 0) << 20));
}
// solver row offsets of a record's bodies: k * ROW for body k, Nb * ROW (the static row Z) for a
// segment's static body
template <int N, int EPW>
__device__ __forceinline__ void info_rows(unsigned long long info, uint32_t& ao, uint32_t& bo)
{
    constexpr uint32_t ROW = EPW * (uint32_t)sizeof(double2);
    const uint32_t lo = (uint32_t)info;
    const uint32_t a = lo & 31u, bcode = (lo >> 5) & 63u;
    ao = a * ROW;
    bo = (bcode < 32u ? bcode : (uint32_t)V1Shape<N>::Nb) * ROW;
}
// the info word `contact` stores for arbiter id pid (its bodies follow from the id: segment arbiters
// body * 12 + segment, circle pairs Nb * 12 + row-major pair index), so that a record's flag can be set
// without reading the record back (a spill record is a global round trip)
template <int N>
__device__ __forceinline__ long long info_of_pid(int pid, bool normal)
{
    using S = V1Shape<N>;
    const bool segc = pid < S::Nb * kNSeg;
    const int q = pid - S::Nb * kNSeg;
    int i = 0;
    sfor<1, S::Nb - 1>([&](auto K) {
        constexpr int k = K;
        i += q >= k * S::Nb - k * (k + 1) / 2 ? 1 : 0;
    });
    const int as = pid / kNSeg;
    const int a = segc ? as : i;
    const int bcode = segc ? 32 + (pid - as * kNSeg) : q - (i * S::Nb - i * (i + 1) / 2) + i + 1;
    return pack_info(a, bcode, pid, normal);
}
// Record lookups by arbiter id from the hit masks (slot_of, info_of_pid below) instead of scans that
// read every record back -- the owner's cache attach, the lookups past the preloaded entries and the
// cache filter -- and the cache update's spill reads in batches: the 5v5 instance (4 LDS record slots:
// the crowded envs' records spill), 50.6 -> 50.1 us.  Measured slower where spill records are rare
// (2v2 22.26 -> 22.66 us, 3v3 +1.4%: the hit masks are live through the solve), and every build
// variant of the 10v10 kernel with it had lost-value findings (the liveness gate, section 6): the
// other instances keep the scans
#ifndef FUTBOL_HM_MIN
#define FUTBOL_HM_MIN 5
#endif
#ifndef FUTBOL_HM_MAX
#define FUTBOL_HM_MAX 5
#endif
template <int N>
constexpr bool kHitMask = N >= FUTBOL_HM_MIN && N <= FUTBOL_HM_MAX;
// null record (slots between a lane's contact count and the wave's): both bodies static (a = Z)
template <int N>
__device__ __forceinline__ long long null_info()
{
    return pack_info(V1Shape<N>::Nb, 32, 0, false);
}

// element env of row k of a [rows][B] array, the scalar-base form (kScalarBase<N> below): the row's
// base is wave-uniform (scalar registers) and the lane's part one 32-bit byte offset shared by every
// row and field, so that the accesses take the saddr form of global_load / store instead of a 64-bit
// vector address per row and field, which the kernels otherwise compute at the state loads and keep
// live until the stores: 10v10 143.0 -> 137.2 us (scratch 756 -> 664 B per lane, PMC traffic 270 ->
// 252 MB per launch), 7v7 -1.5%; 2v2 +2.7%, 5v5 +3.5%, 3v3 +0.5% (the bases then crowd the scalar
// registers), so N <= 5 keep the plain indexing (at their call sites, verbatim: the N <= 5 code is
// unchanged, and so are its ISA-gate results)
#ifndef FUTBOL_SBASE_MIN
#define FUTBOL_SBASE_MIN 6
#endif
template <int N>
constexpr bool kScalarBase = N >= FUTBOL_SBASE_MIN;
template <typename T>
__device__ __forceinline__ T& soa(T* base, int k, int B, int env)
{
    return *reinterpret_cast<T*>(reinterpret_cast<char*>(base + (size_t)k * (size_t)B) + (uint32_t)env * (uint32_t)sizeof(T));
}

// The step's final stores address every row again through a copy of the lane's env index that the
// compiler cannot see through (an empty asm): otherwise it reuses the 64-bit row addresses computed for
// the step's loads, and keeps them -- 2 VGPRs per row and field, from the loads at the top to the stores
// at the end -- live through the whole step (N >= 6: spilled to scratch).  Recomputed at the stores they
// are one add each (FUTBOL_OPAQUE_MIN, round 6).  Measured (profiles/r06/ab/c2/, two runs each): 10v10
// 137.4 -> 129.7 us (scratch 664 -> 400 B per lane), 9v9 113.5 -> 106.6, 8v8 100.9 -> 96.8; 6v6 and 5v5
// equal, 2v2 22.15 -> 22.48 (+1.5%), 7v7 slower (its build needed the ISA gate's max-ilp fallback): N >= 8
#ifndef FUTBOL_OPAQUE_MIN
#define FUTBOL_OPAQUE_MIN 8
#endif
template <int N>
constexpr bool kOpaqueStore = N >= FUTBOL_OPAQUE_MIN;
#ifndef FUTBOL_OPAQUE_PRE_MIN
#define FUTBOL_OPAQUE_PRE_MIN 99
#endif
template <int N>
constexpr bool kOpaquePre = N >= FUTBOL_OPAQUE_PRE_MIN;
__device__ __forceinline__ int opaque_lane(int x)
{
    asm volatile("" : "+v"(x));
    return x;
}

// global spill record (slot s >= K): 8 doubles [nx, ny, nMass, info, bias, -bounce, jBias, jnAcc]
// (the LDS record's four double2 in order), at spill[env][s - K][f]: a record is one 64-byte line,
// so the solve's per-sweep re-reads of an item's spill records stay in a few cache lines
template <int N, int EPW>
struct Lane {
    using S = V1Shape<N>;
    static constexpr int KL = Scratch<N, EPW>::K;
    Scratch<N, EPW>* sh;
    double* spill;
    uint16_t* ckey;
    double* cjn;
    int lane, env, B;
#ifdef FUTBOL_BOUNDS
    unsigned long long* dbg;
#endif
#ifdef FUTBOL_CRUMBS
    unsigned long long* crumbs;
#endif

    __device__ __forceinline__ double* sp(int s, int f) const
    {
        int t = s - KL;
        FB_BOUND(*this, t >= 0 && t < S::P - KL, 0, t = 0);
        return spill + ((size_t)env * (S::P - KL) + t) * 8 + f;
    }
    // record s as 4 double2 (any slot)
    __device__ __forceinline__ double2 get(int s, int q) const
    {
        if (s < KL) return sh->rec[s][q][lane];
        return make_double2(*sp(s, 2 * q), *sp(s, 2 * q + 1));
    }
    __device__ __forceinline__ void put(int s, int q, double2 x) const
    {
        if (s < KL) sh->rec[s][q][lane] = x;
        else {
            *sp(s, 2 * q) = x.x;
            *sp(s, 2 * q + 1) = x.y;
        }
    }
    __device__ __forceinline__ int get_info(int s) const { return (int)__double_as_longlong(get(s, 1).y); }
    // the info word of record s alone (no read of the record: see info_of_pid)
    __device__ __forceinline__ void put_info(int s, long long info) const
    {
        if (s < KL) sh->rec[s][1][lane].y = __longlong_as_double(info);
        else *sp(s, 3) = __longlong_as_double(info);
    }
    __device__ __forceinline__ double get_jn(int s) const { return get(s, 3).y; }
    __device__ __forceinline__ void set_rec(int s, double nx, double ny, double nm, double bi, double bo, double j,
                                            long long info) const
    {
        const double2 r0 = make_double2(nx, ny), r1 = make_double2(nm, __longlong_as_double(info)),
                      r2 = make_double2(bi, -bo), r3 = make_double2(0.0, j);
        if (s < KL) {  // one branch for the four fields
            sh->rec[s][0][lane] = r0;
            sh->rec[s][1][lane] = r1;
            sh->rec[s][2][lane] = r2;
            sh->rec[s][3][lane] = r3;
        } else {
            *sp(s, 0) = r0.x;
            *sp(s, 1) = r0.y;
            *sp(s, 2) = r1.x;
            *sp(s, 3) = r1.y;
            *sp(s, 4) = r2.x;
            *sp(s, 5) = r2.y;
            *sp(s, 6) = r3.x;
            *sp(s, 7) = r3.y;
        }
    }
};

// One half of cpArbiterApplyImpulse for one contact (frictionless: players, ball and segments
// have friction 0 except the segments' 1, and u = a.u * b.u = 0, so no tangent impulse and no
// rotation).  The normal impulse's two accumulators are independent chains:
//   h = 0: jbn = (bias - vbn) * nMass, jBias = max(jBias + jbn, 0), applied to v_bias;
//   h = 1: jn = -(bounce + vrn) * nMass, jnAcc = max(jnAcc + jn, 0), applied to v,
// with c = bias / -bounce from the record: (c - vn) * nMass.  For h = 1 this is
// ((-bounce) - vrn) * nMass, which differs from -(bounce + vrn) * nMass at most in the sign of
// a zero; jnAcc + (+-0) is the same double for every jnAcc >= +0, so the results are identical.
// ra / rb: rows of a and b in this half (rb = Z for a segment: mb = 0 keeps it +0).
__device__ __forceinline__ void apply_half(double2* ra, double2* rb, double nx, double ny, double nMass, double c,
                                           double ma, double mb, double& acc)
{
    const double2 va = *ra, vb = *rb;
    const double vn = (vb.x - va.x) * nx + (vb.y - va.y) * ny;
    const double j = (c - vn) * nMass;
    const double old = acc;
    const double t = old + j;
    const double nacc = t > 0.0 ? t : 0.0;
    acc = nacc;
    const double d = nacc - old;
    const double jx = nx * d, jy = ny * d;
    *ra = make_double2(va.x + (-jx) * ma, va.y + (-jy) * ma);
    *rb = make_double2(vb.x + jx * mb, vb.y + jy * mb);
}

// cpArbiterApplyCachedImpulse for one contact (v half; only NORMAL arbiters are warm started)
__device__ __forceinline__ void warm_half(double2* ra, double2* rb, double nx, double ny, double jn, double dt_coef,
                                          double ma, double mb)
{
    const double jx = (nx * jn) * dt_coef, jy = (ny * jn) * dt_coef;
    const double2 va = *ra;
    *ra = make_double2(va.x + (-jx) * ma, va.y + (-jy) * ma);
    const double2 vb = *rb;
    *rb = make_double2(vb.x + jx * mb, vb.y + jy * mb);
}

template <int N>
struct Env {
    using S = V1Shape<N>;
    double px[S::Nb], py[S::Nb], vx[S::Nb], vy[S::Nb], bx[S::Nb], by[S::Nb];
    Meta meta;
};

// ---------------------------------------------------------------------------
// narrowphase (cpCollision.c CircleToCircle / CircleToSegment), exact op order
__device__ __forceinline__ bool cc_test(double ax, double ay, double ra, double bx_, double by_, double rb,
                                        double& nx, double& ny, double& p1x, double& p1y, double& p2x,
                                        double& p2y)
{
    const double mind = ra + rb;
    const double dx = bx_ - ax, dy = by_ - ay;
    const double d2 = dx * dx + dy * dy;
    if (!(d2 < mind * mind)) return false;
    const double d = sqrt(d2);
    if (d != 0.0) {
        const double inv = 1.0 / d;
        nx = dx * inv;
        ny = dy * inv;
    } else {
        nx = 1.0;
        ny = 0.0;
    }
    p1x = ax + nx * ra;
    p1y = ay + ny * ra;
    p2x = bx_ + nx * (-rb);
    p2y = by_ + ny * (-rb);
    return true;
}

// CircleToCircle's contact for a pair already known to collide (dist^2 < (ra + rb)^2)
__device__ __forceinline__ void cc_contact(double ax, double ay, double ra, double bx_, double by_, double rb,
                                           double& nx, double& ny, double& p1x, double& p1y, double& p2x,
                                           double& p2y)
{
    const double dx = bx_ - ax, dy = by_ - ay;
    const double d = sqrt(dx * dx + dy * dy);
    if (d != 0.0) {
        const double inv = 1.0 / d;
        nx = dx * inv;
        ny = dy * inv;
    } else {
        nx = 1.0;
        ny = 0.0;
    }
    p1x = ax + nx * ra;
    p1y = ay + ny * ra;
    p2x = bx_ + nx * (-rb);
    p2y = by_ + ny * (-rb);
}

__device__ __forceinline__ bool cc_hit(double ax, double ay, double ra, double bx_, double by_, double rb)
{
    const double mind = ra + rb;
    const double dx = bx_ - ax, dy = by_ - ay;
    return dx * dx + dy * dy < mind * mind;
}

// closest point of segment (sa, sa + sd) to c; t = dot(sd, c - sa) / |sd|^2 clamped
__device__ __forceinline__ void seg_closest(double cx, double cy, double sax, double say, double sdx, double sdy,
                                            double L2, double rL2, double& qx, double& qy)
{
    double t = cdiv(sdx * (cx - sax) + sdy * (cy - say), L2, rL2);
    t = t < 0.0 ? 0.0 : (t > 1.0 ? 1.0 : t);
    qx = sax + sdx * t;
    qy = say + sdy * t;
}

// CircleToSegment's contact for a pair already known to collide (the same closest point and d2)
__device__ __forceinline__ void cs_contact(double cx, double cy, double rc, const SegLds& g, double& nx, double& ny,
                                           double& p1x, double& p1y, double& p2x, double& p2y)
{
    double qx, qy;
    seg_closest(cx, cy, g.ax, g.ay, g.sdx, g.sdy, g.L2, g.rL2, qx, qy);
    const double dx = qx - cx, dy = qy - cy;
    const double d = sqrt(dx * dx + dy * dy);
    if (d != 0.0) {
        const double inv = 1.0 / d;
        nx = dx * inv;
        ny = dy * inv;
    } else {  // segment->tn
        const double inv = 1.0 / sqrt(g.L2);
        nx = -g.sdy * inv;
        ny = g.sdx * inv;
    }
    p1x = cx + nx * rc;
    p1y = cy + ny * rc;
    p2x = qx + nx * (-kSegR);
    p2y = qy + ny * (-kSegR);
}

__device__ __forceinline__ bool cs_hit(const V1Params& P, int s, double cx, double cy, double rc)
{
    double qx, qy;
    seg_closest(cx, cy, P.sax[s], P.say[s], P.sbx[s] - P.sax[s], P.sby[s] - P.say[s], P.L2[s], P.rL2[s],
                qx, qy);
    const double mind = rc + kSegR;
    const double dx = qx - cx, dy = qy - cy;
    return dx * dx + dy * dy < mind * mind;
}

// ball within reach of no wall/goal segment: provably rejects all 12 segment tests
// (every segment lies on x<=0, x>=W, y<=0 or y>=H; the test needs distance < rc+1)
__device__ __forceinline__ bool far_from_segments(double x, double y, double reach, double W, double H)
{
    return (x > reach) & (x < W - reach) & (y > reach) & (y < H - reach);
}

// ---------------------------------------------------------------------------
// cpSpaceStep(dt) for one env.  dtc: 1 -> 1e-4, 2 -> 0.1
// the first CK arbiter-cache entries (ck = pair | age << 12, 0xffff = none; cj = jnAcc), loaded
// unconditionally (c < CK <= P is always in bounds) so that the loads carry no dependence on
// ncache and can be issued together with the body state at the top of the kernel
template <int N, int EPW>
__device__ __forceinline__ void load_cache_pre(const Lane<N, EPW>& L, uint32_t ncache, uint32_t (&ck)[CKN<N>],
                                               double (&cj)[CKN<N>])
{
    static_assert(CKN<N> <= V1Shape<N>::P, "preloaded cache entries must lie inside the [P][B] arrays");
    // (N >= FUTBOL_OPAQUE_PRE_MIN: the addresses computed afresh, not kept from the step's first call for the
    // restart phases' -- 10v10: 32 B less scratch per lane)
    const int env = kOpaquePre<N> ? opaque_lane(L.env) : L.env;
#pragma unroll
    for (int c = 0; c < CKN<N>; ++c) {
        if constexpr (kScalarBase<N>) {
            const uint32_t k = soa(L.ckey, c, L.B, env);
            const double j = soa(L.cjn, c, L.B, env);
            ck[c] = (uint32_t)c < ncache ? k : 0xffffu;
            cj[c] = (uint32_t)c < ncache ? j : 0.0;
        } else {
        const uint32_t k = L.ckey[(size_t)c * L.B + L.env];
        const double j = L.cjn[(size_t)c * L.B + L.env];
        ck[c] = (uint32_t)c < ncache ? k : 0xffffu;
        cj[c] = (uint32_t)c < ncache ? j : 0.0;
        }
    }
}

// ck / cj: the preloaded cache entries (load_cache_pre) of the env's CURRENT cache
template <int N, int EPW>
__device__ __forceinline__ void space_step(const V1Params& P, const Lane<N, EPW>& L, Env<N>& e, int dtc,
                                           const uint32_t (&ck)[CKN<N>], const double (&cj)[CKN<N>],
                                           bool& goal, bool& pre_aged
#ifdef FUTBOL_STAMPS
                                           , unsigned long long* st_stamps, unsigned long long& _stamp_prev
#endif
)
{
    using S = V1Shape<N>;
    const double dt = dtc == 2 ? P.dtv[2] : P.dtv[1];
    const double rdt = dtc == 2 ? P.rdt[2] : P.rdt[1];
    const uint32_t pc = e.meta.dtcode();
    const double biasCoef = dtc == 2 ? P.biasc[2] : P.biasc[1];
    const double damping = dtc == 2 ? P.damp[2] : P.damp[1];
    const double slop = P.slop, W = P.W, H = P.H;
    e.meta.set_dtcode(dtc);
    // (kOpaqueStore: the env index through an empty asm, so that the arbiter-cache and spill-record
    // addresses of this cpSpaceStep are computed here, not reused from the step's first loads)
    const int B = L.B, env = kOpaqueStore<N> ? opaque_lane(L.env) : L.env;
    uint32_t ncache = e.meta.ncache();
    FB_BOUND(L, ncache <= (uint32_t)S::P, 1, ncache = S::P);

    uint32_t touched = 0;  // preloaded entries matched by this step's contacts

    // cpBodyUpdatePosition
    sfor<S::Nb>([&](auto K) {
        constexpr int k = K;
        e.px[k] = e.px[k] + (e.vx[k] + e.bx[k]) * dt;
        e.py[k] = e.py[k] + (e.vy[k] + e.by[k]) * dt;
        e.bx[k] = 0.0;
        e.by[k] = 0.0;
    });
    // ball_contact_goal (envs_v1/futbol_env.py:291-296) of the step's space.step(0.1): the positions
    // are final here (the solve changes velocities only); the caller scores with it
    goal = false;
    if (dtc == 2 && !far_from_segments(e.px[S::BALL], e.py[S::BALL], 2.0, W, H)) {
        for (int s = 6; s < 12; ++s) goal = goal || cs_hit(P, s, e.px[S::BALL], e.py[S::BALL], kBallR);
    }

    FUTBOL_CRUMB(L, 10 + dtc);
    FUTBOL_STAMP(dtc == 2 ? 16 : 9);
    // bodies' positions (v_bias rows) and velocities (v rows) staged in LDS for the dynamic body
    // (and env column) indices of the contact work list; the solver prologue overwrites both
    Scratch<N, EPW>* const sh_ = L.sh;
    const int ln_ = L.lane;
    sfor<S::Nb>([&](auto K) {
        constexpr int k = K;
        sh_->vb(k, ln_) = make_double2(e.px[k], e.py[k]);
        if constexpr (!S::ONE_ROWS) sh_->v(k, ln_) = make_double2(e.vx[k], e.vy[k]);
    });
    // collide in canonical order; cpArbiterUpdate + preStep folded in (needs pre-damping v)
    int n = 0;
    constexpr int KLs = Lane<N, EPW>::KL;
    // (1) circle-segment hits of all bodies, (body, segment) ascending: cpBBIntersects from the
    // 16 distinct segment bounds as a 12-bit field per body in 60-bit words (5 bodies per word),
    // then the exact CircleToSegment test of every candidate bit (the body indexed dynamically
    // through the LDS rows staged above) into a hit word per 5 bodies
    FUTBOL_STAMP(dtc == 2 ? 17 : 9);
    constexpr int BPW = 5;
    constexpr int NWS = (S::Nb + BPW - 1) / BPW;
    uint64_t hsw[NWS];
    sfor<NWS>([&](auto WD) {
        constexpr int w = WD;
        constexpr int i0 = w * BPW, i1 = (w + 1) * BPW < S::Nb ? (w + 1) * BPW : S::Nb;
        uint64_t cand = 0;
        sfor<i0, i1>([&](auto I) {
            constexpr int i = I;
            constexpr double ri = i == S::BALL ? kBallR : kPlayerR;
            const double cl = e.px[i] - ri, cb = e.py[i] - ri, cr = e.px[i] + ri, ct = e.py[i] + ri;
            // every segment's cpBB lies within 1 of the field border: exact reject of all 12
            const bool interior = (cl > 1.0) & (cr < W - 1.0) & (cb > 1.0) & (ct < H - 1.0);
            const BBT& T = P.bbt;
            // each of the 16 distinct bounds contributes the set of segments whose cpBB uses it;
            // a segment is a candidate when all four of its bounds hold (the AND of four sets):
            //   segment:  0  1  2  3  4  5  6  7  8  9 10 11
            //   right:   r1 r1 W1 W1 W1 W1 m1 r1 r1 W3 W3 W3   (cl <= r)
            //   left:    m1 m1 m1 W1 W1 m1 m3 m3 m3 Wp W1 W1   (l <= cr)
            //   top:     lo  H  H lo  H  1 hi lo hi hi lo hi   (cb <= t)
            //   bottom:  m1 hi  H m1 hi m1 lo lo hi lo lo hi   (b <= ct)
            const uint32_t xr = (cl <= T.r1 ? 0x183u : 0u) | (cl <= T.rW1 ? 0x03cu : 0u) |
                                (cl <= T.rm1 ? 0x040u : 0u) | (cl <= T.rW3 ? 0xe00u : 0u);
            const uint32_t xl = (T.lm1 <= cr ? 0x027u : 0u) | (T.lW1 <= cr ? 0xc18u : 0u) |
                                (T.lm3 <= cr ? 0x1c0u : 0u) | (T.lWp1 <= cr ? 0x200u : 0u);
            const uint32_t yt = (cb <= T.tlo ? 0x489u : 0u) | (cb <= T.tH ? 0x016u : 0u) |
                                (cb <= T.t1 ? 0x020u : 0u) | (cb <= T.thi ? 0xb40u : 0u);
            const uint32_t yb = (T.bm1 <= ct ? 0x029u : 0u) | (T.bhi <= ct ? 0x912u : 0u) |
                                (T.bH <= ct ? 0x004u : 0u) | (T.blo <= ct ? 0x6c0u : 0u);
            const uint32_t c = xr & xl & yt & yb;
            cand |= interior ? 0ull : (uint64_t)c << (kNSeg * (i - i0));
        });
        uint64_t hitm = 0;
        while (cand) {
            const int bit = __builtin_ctzll(cand);
            cand &= cand - 1;
            const int bi = bit / kNSeg;
            const int sg = bit - bi * kNSeg;
            const int i = i0 + bi;
            const double2 pi_ = sh_->vb(i, ln_);
            const double ri = i == S::BALL ? kBallR : kPlayerR;
            const SegLds g = sh_->seg[sg];
            double qx, qy;
            seg_closest(pi_.x, pi_.y, g.ax, g.ay, g.sdx, g.sdy, g.L2, g.rL2, qx, qy);
            const double mind = ri + kSegR;
            const double dx = qx - pi_.x, dy = qy - pi_.y;
            hitm |= (dx * dx + dy * dy < mind * mind) ? 1ull << bit : 0ull;
        }
        hsw[w] = hitm;
    });

    // (2) circle-circle hits, pairs (i, j > i) in row-major order q (arbiter id Nb * 12 + q):
    // cpBBIntersects && dist^2 < (ri + rj)^2 (CircleToCircle's own expressions), branch-free
    constexpr int PCC = S::Nb * (S::Nb - 1) / 2;
    constexpr int NPW = (PCC + 63) / 64;
    uint64_t hpw[NPW];
    sfor<NPW>([&](auto Q) { hpw[Q] = 0; });
    sfor<S::Nb>([&](auto I) {
        constexpr int i = I;
        constexpr double ri = i == S::BALL ? kBallR : kPlayerR;
        const double cl = e.px[i] - ri, cb = e.py[i] - ri, cr = e.px[i] + ri, ct = e.py[i] + ri;
        sfor<i + 1, S::Nb>([&](auto J) {
            constexpr int j = J;
            constexpr double rj = j == S::BALL ? kBallR : kPlayerR;
            constexpr int q = i * S::Nb - i * (i + 1) / 2 + (j - i - 1);
            // (non-short-circuit & : every operand is computed anyway; `&&` became a divergent
            // branch per pair in the instances built without the phi-folding threshold, N >= 4)
            const bool bb = (cl <= e.px[j] + rj) & (e.px[j] - rj <= cr) & (cb <= e.py[j] + rj) & (e.py[j] - rj <= ct);
            const double mind = ri + rj;
            const double dx = e.px[j] - e.px[i], dy = e.py[j] - e.py[i];
            hpw[q / 64] |= (bb & (dx * dx + dy * dy < mind * mind)) ? 1ull << (q % 64) : 0ull;
        });
    });
    FUTBOL_STAMP(dtc == 2 ? 18 : 9);

    // (2b) connected components of the env's contact graph for the split solve (Nb <= 8): two
    // records are connected when they share a dynamic body (segments are the static body, whose
    // velocity rows stay +0 whatever is applied to them), and the sequential-impulse solve of one
    // component never reads a row another component writes -- so each component is solved as its
    // own chain, in canonical record order, with results bit-identical to solving the env's whole
    // list in order.  cslots: byte c = the LDS record slots (< 8) of the component labelled c
    // (labels: the lowest body of each component, 4-bit fields of `lab`, merged per pair hit).
    uint64_t cslots = 0;
    if constexpr (kSolveComponents<N>) {
        constexpr int FW = kSlotBits<N>;                  // slot-mask field width
        constexpr uint32_t FM = (1u << FW) - 1u;
        using LabT = std::conditional_t<(S::Nb <= 8), uint32_t, uint64_t>;
        constexpr LabT ONES = (LabT)0x1111111111111111ull, SEVENS = (LabT)0x7777777777777777ull,
                       EIGHTS = (LabT)0x8888888888888888ull;
        LabT lab = 0;
        uint64_t osp = 0;  // field k: the record slots whose first body is k
        int r = 0;
        sfor<S::Nb>([&](auto K) {  // body k's segment records: slots [r, r + count)
            constexpr int k = K;
            const uint32_t bits = (uint32_t)(hsw[k / BPW] >> (kNSeg * (k % BPW))) & 0xfffu;
            const int cnt = __popc(bits);
            const uint32_t rng = r < FW ? (((1u << (cnt < FW ? cnt : FW)) - 1u) << r) & FM : 0u;
            osp |= (uint64_t)rng << (FW * k);
            lab |= (LabT)k << (4 * k);
            r += cnt;
        });
        sfor<NPW>([&](auto Q) {
            uint64_t h = hpw[Q];
            while (h) {
                const int q = Q * 64 + __builtin_ctzll(h);
                h &= h - 1;
                int i = 0;
                sfor<1, S::Nb - 1>([&](auto K) {
                    constexpr int k = K;
                    i += q >= k * S::Nb - k * (k + 1) / 2 ? 1 : 0;
                });
                const int j = q - (i * S::Nb - i * (i + 1) / 2) + i + 1;
                osp |= (uint64_t)(r < FW ? 1u << r : 0u) << (FW * i);
                ++r;
                // union: every field labelled max(ci, cj) becomes min(ci, cj) (SWAR zero-field test)
                const LabT ci = (lab >> (4 * i)) & 15u, cj = (lab >> (4 * j)) & 15u;
                const LabT lo = ci < cj ? ci : cj, hi = ci < cj ? cj : ci;
                const LabT x = lab ^ (hi * ONES);
                const LabT z = ~(((x & SEVENS) + SEVENS) | x) & EIGHTS;
                const LabT fm = (z >> 3) * 15u;
                lab = (lab & ~fm) | ((lo * ONES) & fm);
            }
        });
        sfor<S::Nb>([&](auto K) {
            constexpr int k = K;
            cslots |= ((osp >> (FW * k)) & FM) << (FW * (uint32_t)((lab >> (4 * k)) & 15u));
        });
    }

    // (3) contacts and records.  A hit's record slot is its rank in canonical order (segment hits,
    // then pair hits).  The hits of all active lanes are one work list: lane l's hits occupy
    // entries [base_l, base_l + hits_l) of a table in the static row Z (unused until the solve),
    // and active lane w computes entries w, w + A, ... -- the contact of one (env, hit) each,
    // written into slot r of env column o -- so a wave computes ceil(total hits / A) contacts per
    // lane instead of max-over-lanes(hits).  The owners then attach the cached jnAcc / NORMAL
    // state (their preloaded cache entries are registers).  Beyond the table's capacity the
    // lanes compute their own contacts (same arithmetic, same records).
    int nh = 0;
    sfor<NWS>([&](auto WD) { nh += __popcll(hsw[WD]); });
    sfor<NPW>([&](auto Q) { nh += __popcll(hpw[Q]); });
    constexpr int kTableCap = EPW * (int)sizeof(double2) / 4;  // u32 entries in row Z
    uint32_t base = 0, total = 0;
#pragma unroll
    for (int b = 0; b < 9; ++b) {  // wave exclusive prefix of nh (nh <= P < 512)
        const uint64_t mb = __ballot((nh >> b) & 1);
        base += __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u)) << b;
        total += (uint32_t)__popcll(mb) << b;
    }
    auto pid_of = [&](int word, int bit, bool segw) {  // arbiter id of a hit bit
        return segw ? word * BPW * kNSeg + bit : S::Nb * kNSeg + word * 64 + bit;
    };
    // the record slot of arbiter pid (its rank among this step's hits, which are the records in
    // canonical order), or -1 when it is not a contact of this step: a test of the hit masks instead of
    // a scan of the records (whose spill lines are a global round trip each)
    auto slot_of = [&](int pid) -> int {
        constexpr int SW = BPW * kNSeg;  // segment hit bits per word
        const bool segc = pid < S::Nb * kNSeg;
        const int q = pid - S::Nb * kNSeg;
        const int w = segc ? pid / SW : NWS + (q >> 6);
        const int bit = segc ? pid - (pid / SW) * SW : (q & 63);
        uint64_t word = 0;
        int pre = 0;
        sfor<NWS>([&](auto WD) {
            constexpr int x = WD;
            word = w == x ? hsw[x] : word;
            pre += x < w ? __popcll(hsw[x]) : 0;
        });
        sfor<NPW>([&](auto Q) {
            constexpr int x = NWS + (int)Q;
            word = w == x ? hpw[Q] : word;
            pre += x < w ? __popcll(hpw[Q]) : 0;
        });
        const bool hit = (word >> bit) & 1ull;
        return hit ? pre + __popcll(word & ((1ull << bit) - 1ull)) : -1;
    };
    // the contact and record of hit `pid` of env column o (env id oenv), record slot r
    auto contact = [&](int o, int oenv, int pid, int r, bool attach) {
        // CircleToSegment (circle a, segment sg: the second body is the static one) and
        // CircleToCircle (pair a < j: a is a player, the ball is the last body) share one
        // expression chain from the circle's centre to the other point -- the segment's closest
        // point q with radius 1, or body j's centre with its radius -- so every lane of the work
        // list runs one sqrt, one division and one preStep whatever the type of its contact
        const bool segc = pid < S::Nb * kNSeg;
        const int q = pid - S::Nb * kNSeg;
        int i = 0;
        sfor<1, S::Nb - 1>([&](auto K) {
            constexpr int k = K;
            i += q >= k * S::Nb - k * (k + 1) / 2 ? 1 : 0;
        });
        const int as = pid / kNSeg;
        const int a = segc ? as : i;
        const int sg = segc ? pid - as * kNSeg : 0;
        const int j = segc ? a : q - (i * S::Nb - i * (i + 1) / 2) + i + 1;  // (segment: any valid row)
        // (S::ONE_ROWS: the rows hold positions only now; the bounce is the second pass below)
        const double2 pa = sh_->vb(a, o), pb = sh_->vb(j, o);
        const double2 va = S::ONE_ROWS ? make_double2(0.0, 0.0) : sh_->v(a, o);
        const double2 vbj = S::ONE_ROWS ? make_double2(0.0, 0.0) : sh_->v(j, o);
        const SegLds g = sh_->seg[sg];
        double qx, qy;
        seg_closest(pa.x, pa.y, g.ax, g.ay, g.sdx, g.sdy, g.L2, g.rL2, qx, qy);
        const bool ball_a = a == S::BALL, ball_j = j == S::BALL;
        const double ra = ball_a ? kBallR : kPlayerR;
        const double rb = segc ? kSegR : (ball_j ? kBallR : kPlayerR);
        const double ox = segc ? qx : pb.x, oy = segc ? qy : pb.y;
        const double dx = ox - pa.x, dy = oy - pa.y;
        const double d = sqrt(dx * dx + dy * dy);
        double nx, ny;
        if (d != 0.0) {
            const double inv = 1.0 / d;
            nx = dx * inv;
            ny = dy * inv;
        } else if (segc) {  // segment->tn
            const double inv = 1.0 / sqrt(g.L2);
            nx = -g.sdy * inv;
            ny = g.sdx * inv;
        } else {
            nx = 1.0;
            ny = 0.0;
        }
        const double p1x = pa.x + nx * ra, p1y = pa.y + ny * ra;
        const double p2x = ox + nx * (-rb), p2y = oy + ny * (-rb);
        const double apx = pa.x, apy = pa.y, avx = va.x, avy = va.y;
        const double bpx = segc ? 0.0 : pb.x, bpy = segc ? 0.0 : pb.y;   // the static body's p = (0, 0)
        const double bvx_ = segc ? 0.0 : vbj.x, bvy_ = segc ? 0.0 : vbj.y;
        constexpr double nmSB = 1.0 / (kBallMinv + 0.0), nmSP = 1.0 / (kPlayerMinv + 0.0);
        constexpr double nmCB = 1.0 / (kPlayerMinv + kBallMinv), nmCP = 1.0 / (kPlayerMinv + kPlayerMinv);
        const double nMass = segc ? (ball_a ? nmSB : nmSP) : (ball_j ? nmCB : nmCP);
        const double ee = segc ? kE * 0.0 : kE * kE;
        const int bcode = segc ? 32 + sg : j;
        // cpArbiterUpdate + preStep (needs the pre-damping v)
        const double r1x = p1x - apx, r1y = p1y - apy;
        const double r2x = p2x - bpx, r2y = p2y - bpy;
        const double bdx = bpx - apx, bdy = bpy - apy;
        const double dist = ((r2x - r1x) + bdx) * nx + ((r2y - r1y) + bdy) * ny;
        double m = dist + slop;
        m = (0.0 < m) ? 0.0 : m;
        const double bias = cdiv(-biasCoef * m, dt, rdt);
        const double bounce = ((bvx_ - avx) * nx + (bvy_ - avy) * ny) * ee;
        double jn = 0.0;
        bool normal = false;
        if (attach) {  // own record: the preloaded cache entries
#pragma unroll
            for (int c = 0; c < CKN<N>; ++c)
                if ((int)(ck[c] & 0x3ffu) == pid) {
                    jn = cj[c];
                    normal = (ck[c] >> 12) == 0;  // touched by the previous step: NORMAL -> warm start
                    touched |= 1u << c;
                }
        }
        FB_BOUND(L, r < S::P && pid < S::P, 5, r = S::P - 1);
        const double2 q0 = make_double2(nx, ny), q1 = make_double2(nMass, __longlong_as_double(pack_info(a, bcode, pid, normal))),
                      q2 = make_double2(bias, -bounce), q3 = make_double2(0.0, jn);
        if (r < KLs) {
            sh_->rec[r][0][o] = q0;
            sh_->rec[r][1][o] = q1;
            sh_->rec[r][2][o] = q2;
            sh_->rec[r][3][o] = q3;
        } else {
            double2* sp0 = (double2*)(L.spill + ((size_t)oenv * (S::P - KLs) + (r - KLs)) * 8);
            sp0[0] = q0;
            sp0[1] = q1;
            sp0[2] = q2;
            sp0[3] = q3;
        }
    };
    // S::ONE_ROWS: the bounce of record r of env column o (hit pid), from the velocities staged over
    // the positions -- CircleToSegment / CircleToCircle's bounce expression of `contact`, unchanged
    auto bounce_rec = [&](int o, int oenv, int pid, int r) {
        const bool segc = pid < S::Nb * kNSeg;
        const int q = pid - S::Nb * kNSeg;
        int i = 0;
        sfor<1, S::Nb - 1>([&](auto K) {
            constexpr int k = K;
            i += q >= k * S::Nb - k * (k + 1) / 2 ? 1 : 0;
        });
        const int a = segc ? pid / kNSeg : i;
        const int j = segc ? a : q - (i * S::Nb - i * (i + 1) / 2) + i + 1;
        const double2 va = sh_->v(a, o), vbj = sh_->v(j, o);
        const double bvx_ = segc ? 0.0 : vbj.x, bvy_ = segc ? 0.0 : vbj.y;
        const double ee = segc ? kE * 0.0 : kE * kE;
        double* sp_ = r < KLs ? nullptr : L.spill + ((size_t)oenv * (S::P - KLs) + (r - KLs)) * 8;
        const double2 nn = r < KLs ? sh_->rec[r][0][o] : *(const double2*)sp_;
        const double bounce = ((bvx_ - va.x) * nn.x + (bvy_ - va.y) * nn.y) * ee;
        if (r < KLs) sh_->rec[r][2][o].y = -bounce;
        else sp_[5] = -bounce;
    };
    auto stage_velocities = [&]() {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        sfor<S::Nb>([&](auto K) {
            constexpr int k = K;
            sh_->v(k, ln_) = make_double2(e.vx[k], e.vy[k]);
        });
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    };
    n = nh;
    if (dtc == 2) {
        FUTBOL_STAT(26, total);
        FUTBOL_STAT(27, total > (uint32_t)kTableCap ? 1 : 0);
        FUTBOL_STAT(28, __ballot(ncache > (uint32_t)CKN<N>) ? 1 : 0);
        FUTBOL_STAT(29, __ballot(n > KLs) ? 1 : 0);
    }
    if (total <= (uint32_t)kTableCap) {
        uint32_t* const table = reinterpret_cast<uint32_t*>(&sh_->rows[S::Nb][0]);
        {   // publish this lane's hits: (lane | arbiter id << 6 | slot << 16)
            uint32_t r = 0;
            sfor<NWS>([&](auto WD) {
                uint64_t h = hsw[WD];
                while (h) {
                    const int bit = __builtin_ctzll(h);
                    h &= h - 1;
                    table[base + r] = (uint32_t)ln_ | ((uint32_t)pid_of(WD, bit, true) << 6) | (r << 16);
                    ++r;
                }
            });
            sfor<NPW>([&](auto Q) {
                uint64_t h = hpw[Q];
                while (h) {
                    const int bit = __builtin_ctzll(h);
                    h &= h - 1;
                    table[base + r] = (uint32_t)ln_ | ((uint32_t)pid_of(Q, bit, false) << 6) | (r << 16);
                    ++r;
                }
            });
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const uint64_t live = __ballot(1);
        const uint32_t A = (uint32_t)__popcll(live);
        const uint32_t w0 = __builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
        for (uint32_t it = w0; it < total; it += A) {
            const uint32_t en = table[it];
            const int o = (int)(en & 63u);
            contact(o, env - ln_ + o, (int)((en >> 6) & 1023u), (int)(en >> 16), false);
        }
        if constexpr (S::ONE_ROWS) {  // velocities over the positions (row Z keeps the table), bounces
            stage_velocities();
            for (uint32_t it = w0; it < total; it += A) {
                const uint32_t en = table[it];
                const int o = (int)(en & 63u);
                bounce_rec(o, env - ln_ + o, (int)((en >> 6) & 1023u), (int)(en >> 16));
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // the owner attaches the cached jnAcc and the NORMAL (warm start) flag to its records: the
        // hits in canonical order are the records in slot order, so nothing is read back
        if constexpr (kHitMask<N>) {
        int s = 0;
        auto attach_rec = [&](int pid) {
            double jn = 0.0;
            bool hit = false, normal = false;
#pragma unroll
            for (int c = 0; c < CKN<N>; ++c)
                if ((int)(ck[c] & 0x3ffu) == pid) {
                    jn = cj[c];
                    hit = true;
                    normal = (ck[c] >> 12) == 0;
                    touched |= 1u << c;
                }
            if (hit) {
                L.put(s, 3, make_double2(0.0, jn));
                if (normal) L.put_info(s, info_of_pid<N>(pid, true));
            }
            ++s;
        };
        sfor<NWS>([&](auto WD) {
            uint64_t h = hsw[WD];
            while (h) {
                const int bit = __builtin_ctzll(h);
                h &= h - 1;
                attach_rec(pid_of(WD, bit, true));
            }
        });
        sfor<NPW>([&](auto Q) {
            uint64_t h = hpw[Q];
            while (h) {
                const int bit = __builtin_ctzll(h);
                h &= h - 1;
                attach_rec(pid_of(Q, bit, false));
            }
        });
        } else {
        for (int s = 0; s < n; ++s) {
            const double2 r1 = L.get(s, 1);
            const int pid = (int)((__double_as_longlong(r1.y) >> 11) & 511);
            double jn = 0.0;
            bool hit = false, normal = false;
#pragma unroll
            for (int c = 0; c < CKN<N>; ++c)
                if ((int)(ck[c] & 0x3ffu) == pid) {
                    jn = cj[c];
                    hit = true;
                    normal = (ck[c] >> 12) == 0;
                    touched |= 1u << c;
                }
            if (hit) {
                L.put(s, 3, make_double2(0.0, jn));
                if (normal)
                    L.put(s, 1, make_double2(r1.x, __longlong_as_double(__double_as_longlong(r1.y) | (1ll << 20))));
            }
        }
        }
    } else {  // more hits than table entries: every lane computes its own contacts
        int r = 0;
        sfor<NWS>([&](auto WD) {
            uint64_t h = hsw[WD];
            while (h) {
                const int bit = __builtin_ctzll(h);
                h &= h - 1;
                contact(ln_, env, pid_of(WD, bit, true), r, true);
                ++r;
            }
        });
        sfor<NPW>([&](auto Q) {
            uint64_t h = hpw[Q];
            while (h) {
                const int bit = __builtin_ctzll(h);
                h &= h - 1;
                contact(ln_, env, pid_of(Q, bit, false), r, true);
                ++r;
            }
        });
        if constexpr (S::ONE_ROWS) {  // velocities over the positions, then this lane's bounces
            stage_velocities();
            int r2 = 0;
            sfor<NWS>([&](auto WD) {
                uint64_t h = hsw[WD];
                while (h) {
                    const int bit = __builtin_ctzll(h);
                    h &= h - 1;
                    bounce_rec(ln_, env, pid_of(WD, bit, true), r2);
                    ++r2;
                }
            });
            sfor<NPW>([&](auto Q) {
                uint64_t h = hpw[Q];
                while (h) {
                    const int bit = __builtin_ctzll(h);
                    h &= h - 1;
                    bounce_rec(ln_, env, pid_of(Q, bit, false), r2);
                    ++r2;
                }
            });
        }
    }

    FUTBOL_CRUMB(L, 40 + dtc);
    FUTBOL_STAMP(dtc == 2 ? 4 : 9);
    // cache entries beyond the preloaded ones: read in batches of CBN independent loads, each
    // batch matched against every contact of this step.  Pairs are unique in the cache and among
    // the contacts (survivors are the entries no contact touched), so a contact matches at most
    // one entry, and none beyond CK if it matched a preloaded one.
    if (ncache > (uint32_t)CKN<N>) {
        for (uint32_t c0 = CKN<N>; c0 < ncache; c0 += CBN<N>) {
            uint32_t key[CBN<N>];
            double jn[CBN<N>];
#pragma unroll
            for (int i = 0; i < CBN<N>; ++i) {
                const uint32_t c = c0 + i < (uint32_t)S::P ? c0 + i : (uint32_t)S::P - 1;  // in bounds
                const uint32_t k = L.ckey[(size_t)c * B + env];
                jn[i] = L.cjn[(size_t)c * B + env];
                key[i] = c0 + i < ncache ? k : 0xffffu;
            }
            if constexpr (kHitMask<N>) {
#pragma unroll
            for (int i = 0; i < CBN<N>; ++i) {
                const int pid = (int)(key[i] & 0x3ffu);
                const int s = key[i] != 0xffffu ? slot_of(pid) : -1;
                if (s >= 0) {
                    L.put(s, 3, make_double2(0.0, jn[i]));
                    if ((key[i] >> 12) == 0) L.put_info(s, info_of_pid<N>(pid, true));
                }
            }
            } else {
            for (int s = 0; s < n; ++s) {
                const int pair = (L.get_info(s) >> 11) & 511;
#pragma unroll
                for (int i = 0; i < CBN<N>; ++i) {
                    if ((int)(key[i] & 0x3ffu) == pair) {
                        const double2 r1 = L.get(s, 1);
                        L.put(s, 3, make_double2(0.0, jn[i]));
                        if ((key[i] >> 12) == 0)
                            L.put(s, 1, make_double2(r1.x, __longlong_as_double(__double_as_longlong(r1.y) | (1ll << 20))));
                    }
                }
            }
            }
        }
    }

    FUTBOL_STAMP(dtc == 2 ? 22 : 9);
    // cpBodyUpdateVelocity + the reference's limit_velocity callback (ball.py:49-56, player.py:45-52):
    // l = Vec2d.length = sqrt(vx**2 + vy**2) with Python's `**2` = glibc pow(x, 2), and
    // l > vmax  <=>  s2 > T (T = largest double whose rounded sqrt is <= vmax).  x*x decides every
    // body whose s2 is clearly below T; the exact squares are computed (glibc_pow2_need: only the
    // near-midpoint ones take glibc's path) for the bodies that may clamp, whose scale uses them
    if constexpr (kSqBatch<N>) {
        double vq[2 * S::Nb], vsq[2 * S::Nb];
        uint64_t vneed = 0;
        sfor<S::Nb>([&](auto K) {
            constexpr int k = K;
            e.vx[k] = e.vx[k] * damping + 0.0 * dt;
            e.vy[k] = e.vy[k] * damping + 0.0 * dt;
            vq[2 * k] = e.vx[k];
            vq[2 * k + 1] = e.vy[k];
            const double thr = k == S::BALL ? P.clamp2_ball : P.clamp2_player;
            // |pow - x*x| <= 1 ulp per square: below T (1 - 2^-40) neither s2 exceeds T
            vneed |= (uint64_t)(e.vx[k] * e.vx[k] + e.vy[k] * e.vy[k] > thr * (1.0 - 0x1.0p-40)) * (3ull << (2 * k));
        });
        // (the LDS rows are free here: the narrowphase's staging is consumed, the solve's not yet written)
        static_assert(sizeof(L.sh->rows) >= (size_t)kPowTabBytes, "pow tables fit the solver rows");
        glibc_pow2_need_lds<2 * S::Nb>(vq, vsq, vneed, &L.sh->rows[0][0]);
        sfor<S::Nb>([&](auto K) {
            constexpr int k = K;
            const double s2 = vsq[2 * k] + vsq[2 * k + 1];
            const double thr = k == S::BALL ? P.clamp2_ball : P.clamp2_player;
            if (((vneed >> (2 * k)) & 1u) && s2 > thr) {
                constexpr double vmax = k == S::BALL ? kBallVmax : kPlayerVmax;
                const double sc = vmax / sqrt(s2);
                e.vx[k] = e.vx[k] * sc;
                e.vy[k] = e.vy[k] * sc;
            }
        });
    } else {  // N >= 6: one body at a time, tables from global memory (few live registers)
        sfor<S::Nb>([&](auto K) {
            constexpr int k = K;
            e.vx[k] = e.vx[k] * damping + 0.0 * dt;
            e.vy[k] = e.vy[k] * damping + 0.0 * dt;
            const double thr = k == S::BALL ? P.clamp2_ball : P.clamp2_player;
            const bool near = e.vx[k] * e.vx[k] + e.vy[k] * e.vy[k] > thr * (1.0 - 0x1.0p-40);
            const double vq[2] = {e.vx[k], e.vy[k]};
            double vsq[2];
            glibc_pow2_need_t<2, kPowCall<N>>(vq, vsq, near ? 3ull : 0ull);
            const double s2 = vsq[0] + vsq[1];
            if (near && s2 > thr) {
                constexpr double vmax = k == S::BALL ? kBallVmax : kPlayerVmax;
                const double sc = vmax / sqrt(s2);
                e.vx[k] = e.vx[k] * sc;
                e.vy[k] = e.vy[k] * sc;
            }
        });
    }

    FUTBOL_STAMP(dtc == 2 ? 5 : 9);
    {
        // Sequential-impulse solve (cpSpaceStep: warm start, then 10 iterations over the arbiters
        // in canonical order), split in two independent halves per env -- the v_bias / jBias chain
        // and the v / jnAcc chain (apply_half) -- and per connected component of the env's contact
        // graph (cslots above), spread over the wave's active lanes: the (env, component) pairs
        // are compacted into a work list of 2 C items (env, component, half), and lane w solves
        // item w (then w + A, ... when 2 C exceeds the A active lanes).  Each item is one lane's
        // serial chain of (10 + warm start) x records half-applications of its component, so the
        // wave's critical path is its largest component, not its most crowded env, and lanes
        // without contacts do the other items.  When the components would not fit one round of
        // the active lanes, every env is one item (its whole record list).  Records live in LDS
        // and past the K LDS slots in the global spill area (an env with spill records is always
        // one item); rows and records of env e are column e of the block's LDS arrays; an item
        // shorter than the wave's longest is padded with null applications on the static row.
        Scratch<N, EPW>* sh = L.sh;
        const int ln = L.lane;
        constexpr int KL = Lane<N, EPW>::KL;
        const int nf = n < KL ? n : KL;  // records in LDS; slots >= KL are in the global spill
        const uint64_t act = __ballot(n > 0);
        const uint64_t live = __ballot(1);
        const int A = __popcll(live);
        const int w = (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(live >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)live, 0u));
        const uint64_t whole = n > 0 ? (1ull << nf) - 1ull : 0ull;  // the env's LDS slots as one item
        uint64_t cm = whole;
        uint32_t cbase = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
        int total = __popcll(act);
        // slot-mask field width: the component fields, or one 8-bit field holding all K <= 8 LDS slots
        // of a whole-env item (a 4-bit field would drop slot 4 of the N = 4 instance's K = 5)
        constexpr int FW = kSolveComponents<N> ? kSlotBits<N> : 8;
        static_assert(kSolveComponents<N> || KL <= 8, "whole-env items hold at most 8 LDS slots");
        constexpr int NFLD = kSolveComponents<N> ? (FW == 8 ? 8 : S::Nb) : 1;  // slot-mask fields
        if constexpr (kSolveComponents<N>) {
            const uint64_t cc = n > KL ? whole : cslots;
            // nonzero fields of cc (components of this env), then their wave prefix
            uint64_t nzb;
            if constexpr (FW == 8)
                nzb = ((cc | ((cc & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full)) >> 7) & 0x0101010101010101ull;
            else
                nzb = ((cc | ((cc & 0x7777777777777777ull) + 0x7777777777777777ull)) >> 3) & 0x1111111111111111ull;
            const int nc = __popcll(nzb);
            uint32_t cb = 0, ct = 0;
#pragma unroll
            for (int b = 0; b < 5; ++b) {  // nc <= 16
                const uint64_t mb = __ballot((nc >> b) & 1);
                cb += __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u)) << b;
                ct += (uint32_t)__popcll(mb) << b;
            }
            if (2 * (int)ct <= A) {  // components fit one round of items
                cm = cc;
                cbase = cb;
                total = (int)ct;
            }
        }
        // two halves per env (N = 4..7): when more than A / 2 envs have contacts the items take two
        // rounds of the lanes, each as long as its longest item -- so the items are published longest
        // first (envs with spill records, then K, K - 1, ... LDS records), and each round runs for its
        // own longest item (mr below): round 2 holds the short ones.  Item order does not change any
        // result (an item is one lane's serial chain over its own env's rows)
        constexpr bool kSortItems = !kSolveComponents<N> && !S::ONE_ROWS;
        if constexpr (kSortItems) {
            const int cls = n > KL ? 0 : KL + 1 - n;
            uint32_t before = 0, pos = 0;
#pragma unroll
            for (int v = 0; v <= KL; ++v) {
                const uint64_t mb = __ballot(n > 0 && cls == v);
                const uint32_t r = __builtin_amdgcn_mbcnt_hi((uint32_t)(mb >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mb, 0u));
                pos = cls == v ? before + r : pos;
                before += (uint32_t)__popcll(mb);
            }
            cbase = pos;
        }
        // the wave's longest item (records): m
        int msz = 0;
#pragma unroll
        for (int b = 0; b < NFLD; ++b) {
            const int c = __popc((uint32_t)(cm >> (FW * b)) & ((1u << FW) - 1u));
            msz = c > msz ? c : msz;
        }
        int m = 0;
#pragma unroll
        for (int b = 3; b >= 0; --b) {
            const int t = m | (1 << b);
            if (t <= KL && __ballot(msz >= t)) m = t;
        }
        const bool spill = __ballot(n > KL) != 0;
#ifdef FUTBOL_STAMPS
        if ((threadIdx.x & 63) == 0 && st_stamps && dtc == 2)
            atomicAdd(&st_stamps[(size_t)(blockIdx.x * EPW / 64) * kStampStride + 15], (unsigned long long)m);
#endif
        if (m > 0) {
            // every lane publishes its rows (a lane without contacts writes its own, unused,
            // column: no divergent branch) and its items (the others write the spare entry EPW)
            sfor<S::Nb>([&](auto K) {
                constexpr int k = K;
                sh->v(k, ln) = make_double2(e.vx[k], e.vy[k]);
                if constexpr (!S::ONE_ROWS) sh->vb(k, ln) = make_double2(0.0, 0.0);
            });
            sh->rows[S::Nb][ln] = make_double2(0.0, 0.0);
            {
                const uint32_t tail = (uint32_t)ln | ((uint32_t)pc << 14) | ((uint32_t)(n < 65535 ? n : 65535) << 16);
                int idx = 0;
#pragma unroll
                for (int b = 0; b < NFLD; ++b) {
                    const uint32_t byte = (uint32_t)(cm >> (FW * b)) & ((1u << FW) - 1u);
                    const uint32_t slot = byte ? cbase + (uint32_t)idx : (uint32_t)EPW;
                    sh->item[slot] = tail | (byte << 6);
                    idx += byte ? 1 : 0;
                }
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            FUTBOL_STAMP(dtc == 2 ? 19 : 9);
            // two row sets: one pass, items (env / component, half) with the halves on different lanes;
            // S::ONE_ROWS: pass 0 runs the v halves on the v rows, pass 1 the v_bias halves on the same
            // rows (re-staged as v_bias = +0), one item per env / component per pass
            constexpr int NPASS = S::ONE_ROWS ? 2 : 1;
            const int items = S::ONE_ROWS ? total : 2 * total;
            constexpr uint32_t ROW = EPW * (uint32_t)sizeof(double2);
            const double coef2 = dt / P.dtv[2], coef1 = dt / P.dtv[1];  // dt / prev_dt, prev_dt != 0
#pragma unroll 1
            for (int pass = 0; pass < NPASS; ++pass) {
            if (S::ONE_ROWS && pass == 1) {  // the v results out, v_bias = +0 in
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                sfor<S::Nb>([&](auto K) {
                    constexpr int k = K;
                    const double2 v = sh->v(k, ln);
                    e.vx[k] = v.x;
                    e.vy[k] = v.y;
                    sh->vb(k, ln) = make_double2(0.0, 0.0);
                });
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            }
            for (int i0 = 0; i0 < items; i0 += A) {
                const int it_ = i0 + w;
                int mr = m;  // this round's longest item
                if (kSortItems && items > A) {
                    const uint32_t e0 = it_ < items ? sh->item[it_ >> 1] : 0u;
                    const int sz = __popc((e0 >> 6) & 0xffu);
                    mr = 0;
#pragma unroll
                    for (int b = 3; b >= 0; --b) {
                        const int t = mr | (1 << b);
                        if (t <= KL && __ballot(sz >= t)) mr = t;
                    }
                }
                if (it_ < items) {
                    const int m = mr;
                    const uint32_t ent = sh->item[S::ONE_ROWS ? it_ : it_ >> 1];
                    const int ie = (int)(ent & 63u);
                    const int h = S::ONE_ROWS ? 1 - pass : it_ & 1;
                    // cpArbiterApplyCachedImpulse's dt ratio of THIS env (its previous step may have
                    // been a 1e-4 reset micro-step)
                    const uint32_t ipc = (ent >> 14) & 3u;
                    const double dt_coef = ipc == 2 ? coef2 : (ipc == 1 ? coef1 : 0.0);
                    char* const base = (char*)&sh->rows[S::ONE_ROWS ? 0 : (h ? 2 * S::Nb : 0)][ie];
                    const int sgn = S::ONE_ROWS ? 1 : (h ? -1 : 1);
                    const double* const mtab = sh->minv;
                    auto row = [&](uint32_t off) { return (double2*)(base + sgn * (int)off); };
                    auto mass = [&](uint32_t off) { return mtab[off / ROW]; };
                    auto info_of = [&](double x) { return (unsigned long long)__double_as_longlong(x); };
                    // the env's spill records (beyond the LDS slots): global, indexed by its env id
                    const int ienv = env - ln + ie;
                    auto spp = [&](int s, int f) {
                        int t = s - KL;
                        FB_BOUND(L, t >= 0 && t < S::P - KL, 0, t = 0);
                        return L.spill + ((size_t)ienv * (S::P - KL) + t) * 8 + f;
                    };
                    const int nie = spill ? (int)(ent >> 16) : 0;  // env ie's record count
                    // the item's LDS records in registers for the whole solve (m is wave-uniform: the
                    // q < m guards are scalar branches): only the two body rows of each half-
                    // application go through LDS on the serial chain.  Record q of the item is the
                    // q-th slot of its mask; past its last one, a null application on the static
                    // row Z (whose rows stay +0: inverse mass 0) whose accumulator is dropped.
                    double qnx[KL], qny[KL], qnm[KL], qc[KL], qacc[KL], qma[KL], qmb[KL];
                    double2 *qra[KL], *qrb[KL];
                    bool qwarm[KL];
                    int qslot[KL];
                    uint32_t mk = (ent >> 6) & 0xffu;
                    sfor<KL>([&](auto Q) {
                        constexpr int q = Q;
                        if (q < m) {
                            const bool has = mk != 0u;
                            const int sl = (int)(__builtin_ctz(mk | 0x100u) & 7u);  // slot 0 (a real record) when !has
                            mk &= mk - 1u;
                            const double2 r0 = sh->rec[sl][0][ie], r1 = sh->rec[sl][1][ie], r2 = sh->rec[sl][2][ie],
                                          r3 = sh->rec[sl][3][ie];
                            const unsigned long long info = info_of(r1.y);
                            uint32_t ao, bo;
                            info_rows<N, EPW>(info, ao, bo);
                            ao = has ? ao : (uint32_t)S::Nb * ROW;
                            bo = has ? bo : (uint32_t)S::Nb * ROW;
                            qnx[q] = r0.x;
                            qny[q] = r0.y;
                            qnm[q] = r1.x;
                            qc[q] = h ? r2.y : r2.x;
                            qacc[q] = h ? r3.y : r3.x;
                            qra[q] = row(ao);
                            qrb[q] = row(bo);
                            qma[q] = mass(ao);
                            qmb[q] = mass(bo);
                            qwarm[q] = has && h && ((info >> 20) & 1);
                            qslot[q] = has ? sl : -1;
                        }
                    });
                    // the first KX spill records in registers too (wave-uniform count mx; past the
                    // item's own records, null applications on Z with zero operands)
                    constexpr int KX = KXN<N>;
                    constexpr int KXa = KX > 0 ? KX : 1;
                    double xnx[KXa], xny[KXa], xnm[KXa], xc[KXa], xacc[KXa], xma[KXa], xmb[KXa];
                    double2 *xra[KXa], *xrb[KXa];
                    bool xwarm[KXa], xhas[KXa];
                    int mx = 0;
                    if constexpr (KX > 0) {
                        if (spill) {
                            const int nsx = nie > KL ? (nie - KL < KX ? nie - KL : KX) : 0;
#pragma unroll
                            for (int b = 2; b >= 0; --b) {
                                const int t = mx | (1 << b);
                                if (t <= KX && __ballot(nsx >= t)) mx = t;
                            }
                            sfor<KX>([&](auto X) {
                                constexpr int x = X;
                                if (x < mx) {
                                    const bool has = x < nsx;
                                    // a lane without this record reads its env's first spill line (in
                                    // bounds) and discards it
                                    const double2* sp = (const double2*)spp(has ? KL + x : KL, 0);
                                    const double2 d0 = sp[0], d1 = sp[1], d2 = sp[2], d3 = sp[3];
                                    const unsigned long long info = info_of(d1.y);
                                    uint32_t ao, bo;
                                    info_rows<N, EPW>(info, ao, bo);
                                    xhas[x] = has;
                                    xra[x] = row(has ? ao : (uint32_t)S::Nb * ROW);
                                    xrb[x] = row(has ? bo : (uint32_t)S::Nb * ROW);
                                    xma[x] = has ? mass(ao) : 0.0;
                                    xmb[x] = has ? mass(bo) : 0.0;
                                    xnx[x] = has ? d0.x : 0.0;
                                    xny[x] = has ? d0.y : 0.0;
                                    xnm[x] = has ? d1.x : 0.0;
                                    xc[x] = has ? (h ? d2.y : d2.x) : 0.0;
                                    xacc[x] = has ? (h ? d3.y : d3.x) : 0.0;
                                    xwarm[x] = has && h && ((info >> 20) & 1);
                                }
                            });
                        }
                    }
                    const int sx0 = KL + mx;  // first spill slot the global loops handle
                    // warm start (cpArbiterApplyCachedImpulse), v half only, record order
                    sfor<KL>([&](auto Q) {
                        constexpr int q = Q;
                        if (q < m && qwarm[q]) warm_half(qra[q], qrb[q], qnx[q], qny[q], qacc[q], dt_coef, qma[q], qmb[q]);
                    });
                    if constexpr (KX > 0) {
                        sfor<KX>([&](auto X) {
                            constexpr int x = X;
                            if (x < mx && xwarm[x]) warm_half(xra[x], xrb[x], xnx[x], xny[x], xacc[x], dt_coef, xma[x], xmb[x]);
                        });
                    }
                    if (h) {
                        for (int s = sx0; s < nie; ++s) {
                            const unsigned long long info = info_of(*spp(s, 3));
                            if ((info >> 20) & 1) {
                                uint32_t ao, bo;
                                info_rows<N, EPW>(info, ao, bo);
                                warm_half(row(ao), row(bo), *spp(s, 0), *spp(s, 1), *spp(s, 7), dt_coef, mass(ao),
                                          mass(bo));
                            }
                        }
                    }
                    for (int itr = 0; itr < 10; ++itr) {
                        sfor<KL>([&](auto Q) {
                            constexpr int q = Q;
                            if (q < m) apply_half(qra[q], qrb[q], qnx[q], qny[q], qnm[q], qc[q], qma[q], qmb[q], qacc[q]);
                        });
                        if constexpr (KX > 0) {
                            sfor<KX>([&](auto X) {
                                constexpr int x = X;
                                if (x < mx) apply_half(xra[x], xrb[x], xnx[x], xny[x], xnm[x], xc[x], xma[x], xmb[x], xacc[x]);
                            });
                        }
                        for (int s = sx0; s < nie; ++s) {
                            const unsigned long long info = info_of(*spp(s, 3));
                            uint32_t ao, bo;
                            info_rows<N, EPW>(info, ao, bo);
                            double* const accp = spp(s, 6 + h);
                            double acc = *accp;
                            apply_half(row(ao), row(bo), *spp(s, 0), *spp(s, 1), *spp(s, 2), *spp(s, 4 + h), mass(ao),
                                       mass(bo), acc);
                            *accp = acc;
                        }
                    }
                    sfor<KL>([&](auto Q) {  // jBias / jnAcc back into the record (the arbiter cache reads jnAcc)
                        constexpr int q = Q;
                        if (q < m && qslot[q] >= 0) {
                            if (h) sh->rec[qslot[q]][3][ie].y = qacc[q];
                            else sh->rec[qslot[q]][3][ie].x = qacc[q];
                        }
                    });
                    if constexpr (KX > 0) {
                        sfor<KX>([&](auto X) {  // and into the spill lines
                            constexpr int x = X;
                            if (x < mx && xhas[x]) *spp(KL + x, 6 + h) = xacc[x];
                        });
                    }
                }
            }
            }  // passes
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            // (a lane without contacts reads back the v it published and v_bias = +0)
            sfor<S::Nb>([&](auto K) {
                constexpr int k = K;
                const double2 vb = sh->vb(k, ln);
                if constexpr (!S::ONE_ROWS) {
                    const double2 v = sh->v(k, ln);
                    e.vx[k] = v.x;
                    e.vy[k] = v.y;
                }
                e.bx[k] = vb.x;
                e.by[k] = vb.y;
            });
        }
    }

    FUTBOL_CRUMB(L, 60 + dtc);
    FUTBOL_STAMP(dtc == 2 ? 6 : 9);
    // cpSpaceArbiterSetFilter + store jnAcc: survivors (untouched, age+1 < 3) then this step's contacts.
    // A lane that scored will restart from formation with the contact-free micro-step
    // (formation_step: its guard is decided by this step's final v_bias), whose only effect on
    // the cache is one more filter with no contact: it is applied here (ages + 1 more, survivors
    // age + 2 < 3), so that the restart does not read the cache back
    bool fok = goal;
    sfor<S::Nb>([&](auto K) {
        constexpr int k = K;
        fok = fok & (__builtin_fabs(e.bx[k]) < P.form_vb) & (__builtin_fabs(e.by[k]) < P.form_vb);
    });
    pre_aged = fok;
    const uint32_t xa = fok ? 1u : 0u;
    uint32_t w = 0;
#pragma unroll
    for (int c = 0; c < CKN<N>; ++c) {
        if ((uint32_t)c < ncache) {
            const uint32_t key = ck[c], age = key >> 12;
            if (!((touched >> c) & 1u) && age + 1 + xa < 3) {
                FB_BOUND(L, w < (uint32_t)S::P, 6, w = S::P - 1);
                L.ckey[(size_t)w * B + env] = (uint16_t)((key & 0x3ffu) | ((age + 1 + xa) << 12));
                FB_BOUND(L, w < (uint32_t)S::P, 6, w = S::P - 1);
                L.cjn[(size_t)w * B + env] = cj[c];
                ++w;
            }
        }
    }
    // (batches of CBN loads; in-place compaction is safe: w <= c for every entry c, and a batch
    // is loaded before any of its survivors is written)
    for (uint32_t c0 = CKN<N>; c0 < ncache; c0 += CBN<N>) {
        uint32_t key[CBN<N>];
        double jn[CBN<N>];
#pragma unroll
        for (int i = 0; i < CBN<N>; ++i) {
            const uint32_t c = c0 + i < (uint32_t)S::P ? c0 + i : (uint32_t)S::P - 1;
            key[i] = L.ckey[(size_t)c * B + env];
            jn[i] = L.cjn[(size_t)c * B + env];
        }
#pragma unroll
        for (int i = 0; i < CBN<N>; ++i) {
            if (c0 + i < ncache) {
                const int pair = (int)(key[i] & 0x3ffu);
                const uint32_t age = key[i] >> 12;
                bool t = false;
                if constexpr (kHitMask<N>) {
                    t = slot_of(pair) >= 0;
                } else {
                    for (int s = 0; s < n; ++s) t |= ((L.get_info(s) >> 11) & 511) == pair;
                }
                if (!t && age + 1 + xa < 3) {
                    FB_BOUND(L, w < (uint32_t)S::P, 6, w = S::P - 1);
                    L.cjn[(size_t)w * B + env] = jn[i];
                    FB_BOUND(L, w < (uint32_t)S::P, 6, w = S::P - 1);
                    L.ckey[(size_t)w * B + env] = (uint16_t)(pair | ((age + 1 + xa) << 12));
                    ++w;
                }
            }
        }
    }
    auto put_entry = [&](long long info, double jn) {
        FB_BOUND(L, w < (uint32_t)S::P, 6, w = S::P - 1);
        L.ckey[(size_t)w * B + env] = (uint16_t)(((info >> 11) & 511) | (xa << 12));
        FB_BOUND(L, w < (uint32_t)S::P, 6, w = S::P - 1);
        L.cjn[(size_t)w * B + env] = jn;
        ++w;
    };
    if constexpr (kHitMask<N>) {
    const int nl = n < KLs ? n : KLs;
    for (int s = 0; s < nl; ++s)
        put_entry(__double_as_longlong(L.sh->rec[s][1][ln_].y), L.sh->rec[s][3][ln_].y);
    // spill records: their info and jnAcc in batches of 8 independent loads (one round trip each)
    for (int s0 = KLs; s0 < n; s0 += 8) {
        double inf[8], jq[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const int s = s0 + i < n ? s0 + i : n - 1;
            inf[i] = *L.sp(s, 3);
            jq[i] = *L.sp(s, 7);
        }
#pragma unroll
        for (int i = 0; i < 8; ++i)
            if (s0 + i < n) put_entry(__double_as_longlong(inf[i]), jq[i]);
    }
    } else {
    for (int s = 0; s < n; ++s) put_entry(L.get_info(s), L.get_jn(s));
    }
    FB_BOUND(L, w <= (uint32_t)S::P, 2, w = S::P);
    e.meta.set_ncache(w);
    FUTBOL_CRUMB(L, 70 + dtc);
    FUTBOL_STAMP(dtc == 2 ? 7 : 9);
}

// cpSpaceStep(1e-4) right after _position_to_initial (v = 0, p = formation), when provably no
// pair collides (every |v_bias| component below P.form_vb, futbol_v1_params.hpp): the same state
// space_step computes with zero contacts -- positions integrated with the carried v_bias (D.2),
// v_bias cleared, v = +0 damped (+0), no solve, and the arbiter cache filtered (every entry
// untouched: age + 1, dropped at 3, compacted in order).  Returns false, having changed nothing,
// when the guard fails; the caller then runs space_step.  No LDS, no wave-level operation: it
// runs on whichever lanes need it (a goal lane's restart costs a few hundred cycles instead of a
// whole narrowphase).
template <int N, int EPW>
__device__ __forceinline__ bool formation_step(const V1Params& P, const Lane<N, EPW>& L, Env<N>& e,
                                               bool cache_done = false)
{
    using S = V1Shape<N>;
    bool ok = true;
    sfor<S::Nb>([&](auto K) {
        constexpr int k = K;
        ok = ok & (__builtin_fabs(e.bx[k]) < P.form_vb) & (__builtin_fabs(e.by[k]) < P.form_vb);
    });
    if (!ok) return false;
    const double dt = P.dtv[1], damping = P.damp[1];
    sfor<S::Nb>([&](auto K) {  // cpBodyUpdatePosition, cpBodyUpdateVelocity (s2 = 0: no clamp)
        constexpr int k = K;
        e.px[k] = e.px[k] + (e.vx[k] + e.bx[k]) * dt;
        e.py[k] = e.py[k] + (e.vy[k] + e.by[k]) * dt;
        e.bx[k] = 0.0;
        e.by[k] = 0.0;
        e.vx[k] = e.vx[k] * damping + 0.0 * dt;
        e.vy[k] = e.vy[k] * damping + 0.0 * dt;
    });
    e.meta.set_dtcode(1);
    if (cache_done) return true;  // the previous step's cache update already applied this filter
    // cpSpaceArbiterSetFilter with no contact: survivors keep their order, age + 1 < 3
    const uint32_t ncache = e.meta.ncache();
    const int B = L.B, env = L.env;
    uint32_t w = 0;
    for (uint32_t c0 = 0; c0 < ncache; c0 += 4) {
        uint32_t key[4];
        double jn[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {  // 4 independent loads, clamped in bounds
            const uint32_t c = c0 + i < (uint32_t)S::P ? c0 + i : (uint32_t)S::P - 1;
            key[i] = L.ckey[(size_t)c * B + env];
            jn[i] = L.cjn[(size_t)c * B + env];
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t age = key[i] >> 12;
            if (c0 + i < ncache && age + 1 < 3) {
                L.ckey[(size_t)w * B + env] = (uint16_t)((key[i] & 0x3ffu) | ((age + 1) << 12));
                L.cjn[(size_t)w * B + env] = jn[i];
                ++w;
            }
        }
    }
    e.meta.set_ncache(w);
    return true;
}

// ---------------------------------------------------------------------------
template <int N>
__device__ __forceinline__ void position_to_initial(const V1Params& P, Env<N>& e)
{
    sfor<V1Shape<N>::Nb>([&](auto K) {
        constexpr int k = K;
        e.px[k] = P.fx[k];
        e.py[k] = P.fy[k];
        e.vx[k] = 0.0;
        e.vy[k] = 0.0;
    });
}

// _get_observation (envs_v1/futbol_env.py:154-180): [ball, A0.., B0..] x [x, y, vx, vy]
template <int N, typename OT>
__device__ __forceinline__ void write_obs(const Env<N>& e, OT* o)
{
    using S = V1Shape<N>;
    constexpr double r525 = 1.0 / 52.5, r555 = 1.0 / 55.5, r34 = 1.0 / 34.0, r25 = 1.0 / 25.0, r10 = 1.0 / 10.0;
    o[0] = (OT)cdiv(e.px[S::BALL] - 52.5, 52.5, r525);
    o[1] = (OT)cdiv(e.py[S::BALL] - 34.0, 34.0, r34);
    o[2] = (OT)cdiv(e.vx[S::BALL] - 0.0, 25.0, r25);
    o[3] = (OT)cdiv(e.vy[S::BALL] - 0.0, 25.0, r25);
    sfor<2 * N>([&](auto K) {
        constexpr int k = K;
        o[4 + 4 * k + 0] = (OT)cdiv(e.px[k] - 52.5, 55.5, r555);
        o[4 + 4 * k + 1] = (OT)cdiv(e.py[k] - 34.0, 34.0, r34);
        o[4 + 4 * k + 2] = (OT)cdiv(e.vx[k] - 0.0, 10.0, r10);
        o[4 + 4 * k + 3] = (OT)cdiv(e.vy[k] - 0.0, 10.0, r10);
    });
}

// The step kernel's v_bias loads for N >= FUTBOL_LATE_BIAS_MIN: issued after the action phase (the
// first use is the position update) instead of with the rest of the state, so that 2 Nb doubles are
// not live through _process_action's player loop at the register limit (one more memory round trip)
// (10v10: 158.8 -> 146.3 us, 5v5: 53.0 -> 51.8 us; 2v2 has no spills to save)
#ifndef FUTBOL_LATE_BIAS_MIN
#define FUTBOL_LATE_BIAS_MIN 5
#endif
template <int N>
constexpr bool kLateBias = N >= FUTBOL_LATE_BIAS_MIN;
// diagnostic only (the round-4 "latec" build): the preloaded arbiter-cache
// entries loaded after the action phase too
#ifndef FUTBOL_LATE_CACHE_MIN
#define FUTBOL_LATE_CACHE_MIN 99
#endif
template <int N>
constexpr bool kLateCache = N >= FUTBOL_LATE_CACHE_MIN;

template <int N, bool BIAS = true>
__device__ __forceinline__ void load_bodies(const V1Ptrs& st, int env, int B, Env<N>& e)
{
    if constexpr (kScalarBase<N>) {
        sfor<V1Shape<N>::Nb>([&](auto K) {
            constexpr int k = K;
            const double2 p = soa(st.pxy, k, B, env), v = soa(st.vxy, k, B, env);
            e.px[k] = p.x;
            e.py[k] = p.y;
            e.vx[k] = v.x;
            e.vy[k] = v.y;
            if constexpr (BIAS) {
                const double2 vb = soa(st.bxy, k, B, env);
                e.bx[k] = vb.x;
                e.by[k] = vb.y;
            }
        });
        return;
    }
    sfor<V1Shape<N>::Nb>([&](auto K) {
        constexpr int k = K;
        const size_t o = (size_t)k * B + env;
        const double2 p = st.pxy[o], v = st.vxy[o];
        e.px[k] = p.x;
        e.py[k] = p.y;
        e.vx[k] = v.x;
        e.vy[k] = v.y;
        if constexpr (BIAS) {
            const double2 vb = st.bxy[o];
            e.bx[k] = vb.x;
            e.by[k] = vb.y;
        }
    });
}
template <int N>
__device__ __forceinline__ void load_bias(const V1Ptrs& st, int env, int B, Env<N>& e)
{
    sfor<V1Shape<N>::Nb>([&](auto K) {
        constexpr int k = K;
        const double2 vb = kScalarBase<N> ? soa(st.bxy, k, B, env) : st.bxy[(size_t)k * B + env];
        e.bx[k] = vb.x;
        e.by[k] = vb.y;
    });
}
template <int N>
__device__ __forceinline__ void load_env(const V1Ptrs& st, int env, int B, Env<N>& e)
{
    e.meta.w = st.meta[env];
    load_bodies<N>(st, env, B, e);
}

template <int N>
__device__ __forceinline__ void store_env(const V1Ptrs& st, int env_, int B, const Env<N>& e)
{
    const int env = kOpaqueStore<N> ? opaque_lane(env_) : env_;
    if constexpr (kScalarBase<N>) {
        sfor<V1Shape<N>::Nb>([&](auto K) {
            constexpr int k = K;
            soa(st.pxy, k, B, env) = make_double2(e.px[k], e.py[k]);
            soa(st.vxy, k, B, env) = make_double2(e.vx[k], e.vy[k]);
            soa(st.bxy, k, B, env) = make_double2(e.bx[k], e.by[k]);
        });
        soa(st.meta, 0, B, env) = e.meta.w;
        return;
    }
    sfor<V1Shape<N>::Nb>([&](auto K) {
        constexpr int k = K;
        const size_t o = (size_t)k * B + env;
        st.pxy[o] = make_double2(e.px[k], e.py[k]);
        st.vxy[o] = make_double2(e.vx[k], e.vy[k]);
        st.bxy[o] = make_double2(e.bx[k], e.by[k]);
    });
    st.meta[env] = e.meta.w;
}

// the block's segment table in LDS (per-lane dynamic segment index in the collide loop), in two
// halves: fetch_seg issues lane s's loads (lanes 0..11) and store_seg writes them with the solver's
// inverse-mass table and synchronises -- so that the step kernel can issue these loads ahead of
// the state's and wait for them alone
__device__ __forceinline__ SegLds fetch_seg(const V1Params& P)
{
    const int s = threadIdx.x < kNSeg ? (int)threadIdx.x : 0;
    SegLds g;
    g.ax = P.sax[s];
    g.ay = P.say[s];
    g.sdx = P.sbx[s] - P.sax[s];
    g.sdy = P.sby[s] - P.say[s];
    g.L2 = P.L2[s];
    g.rL2 = P.rL2[s];
    return g;
}
template <int N, int EPW>
__device__ __forceinline__ void store_seg(const SegLds& g, Scratch<N, EPW>& sh)
{
    const int s = threadIdx.x;
    if (s < kNSeg) sh.seg[s] = g;
    if (s <= V1Shape<N>::Nb)  // inverse masses by solver row (Player/Ball mass, static Z)
        sh.minv[s] = s == V1Shape<N>::Nb ? 0.0 : (s == V1Shape<N>::BALL ? kBallMinv : kPlayerMinv);
    __syncthreads();
}
template <int N, int EPW>
__device__ __forceinline__ void load_seg_table(const V1Params& P, Scratch<N, EPW>& sh)
{
    store_seg<N, EPW>(fetch_seg(P), sh);
}

// Futbol.reset (envs_v1/futbol_env.py:146-150): owner draw, formation, space.step(1e-4)
template <int N, int EPW>
__device__ __forceinline__ void do_reset(const V1Params& P, const V1Params* __restrict__ R, const Lane<N, EPW>& L,
                                         Env<N>& e
#ifdef FUTBOL_STAMPS
                                         , unsigned long long* st_stamps, unsigned long long& _stamp_prev
#endif
)
{
    const uint32_t ev = e.meta.event();
    e.meta.set_event(ev + 1);
    Stream rs(R->seed, R->env_base + (uint32_t)L.env, ev, 0);
    e.meta.set_owner((uint32_t)rs.choice(2));
    e.meta.set_steps(0);
    position_to_initial<N>(P, e);
    if (formation_step<N, EPW>(P, L, e)) return;
    uint32_t ck[CKN<N>];
    double cj[CKN<N>];
    load_cache_pre<N, EPW>(L, e.meta.ncache(), ck, cj);
    bool goal_, pre_;
    space_step<N, EPW>(P, L, e, 1, ck, cj, goal_, pre_
#ifdef FUTBOL_STAMPS
                  , st_stamps, _stamp_prev
#endif
    );
}

// Team.get_pass_target_teammate (team.py:136-180) for player `me` of team `side`:
// returns the teammate's position.
// The pass-target draws of one step's player loop (N >= 3).  A passing player (touching the ball,
// key 4) makes one draw (random.choices over its teammates) plus one when an arrow is held and some
// teammate lies that way, at the lane's next stream positions; no other call in the loop draws.
// So a lane's pass draws are the consecutive positions j0, j0 + 1, ... from the loop's start, and
// nearly every lane makes at most two (one passer per step).  Their blocks are computed once per
// step for the whole wave, at a converged point, instead of inside each passing player's
// divergent branch (which some lane of a 5v5 wave enters for most players: 5.6 k of the wave's
// 96.6 k cycles per step); a draw past j0 + 1 (a second passer) computes its own block.
// N = 3..5 (5v5 51.0 -> 50.4 us, 3v3 29.4 -> 28.6 us); 10v10 measured 2% slower with it (twenty
// players: more lanes with a second passer, more registers), N >= 6 keeps the blocks in the branch
template <int N>
constexpr bool kPassDraws = N >= 3 && N <= 5;
struct PassDraws {
    uint32_t j0;
    uint32_t a0, b0, a1, b1;  // words 0 and 1 of the blocks at j0 and j0 + 1 (all choice_of reads)
    __device__ __forceinline__ int choice(Stream& rs, int n)
    {
        const uint32_t x = rs.j++;
        uint32_t a = x == j0 ? a0 : a1, b = x == j0 ? b0 : b1;
        if (x - j0 > 1u) {  // rare: a later passer of the same lane
            const Philox4 p = rs.block(x);
            a = p.x[0];
            b = p.x[1];
        }
        const int k = (int)floor(u53(a, b) * (double)n);
        return k > n - 1 ? n - 1 : k;
    }
};

template <int N, int side, int me, int NSQ>
__device__ __forceinline__ void pass_target(const Env<N>& e, Stream& rs, PassDraws& pd, int ar, double& tx, double& ty,
                                            const double (&sq)[NSQ], double& sx, double& sy)
{
    constexpr int base = side * N;
    if constexpr (N == 1) {
        tx = e.px[base];
        ty = e.py[base];
        sx = sq[2 * base];
        sy = sq[2 * base + 1];
        return;
    } else {
        // random.choices over teammates != self.  With one teammate (N = 2) every choice of this
        // function is over one item: floor(u * 1) = 0 for every u in [0, 1), so the draw only
        // advances the stream (no Philox block is computed) -- the same values and draw order
        int t;
        if constexpr (N - 1 == 1) {
            rs.skip(1);
            t = 0;
        } else {
            t = kPassDraws<N> ? pd.choice(rs, N - 1) : rs.choice(N - 1);
        }
        t = t >= me ? t + 1 : t;
        if (ar != 0) {
            const double x0 = e.px[base + me], y0 = e.py[base + me];
            auto dir_ok = [&](double mx, double my) {
                return ((ar == 1) & (my > 0)) | ((ar == 2) & (mx > 0)) | ((ar == 3) & (my < 0)) | ((ar == 4) & (mx < 0));
            };
            int cnt = 0;
            sfor<N>([&](auto Q) {
                constexpr int q = Q;
                cnt += dir_ok(e.px[base + q] - x0, e.py[base + q] - y0) ? 1 : 0;
            });
            if (cnt > 0) {
                int pick;
                if constexpr (N - 1 == 1) {  // cnt = 1 (self never qualifies: strict inequalities)
                    rs.skip(1);
                    pick = 0;
                } else {
                    pick = kPassDraws<N> ? pd.choice(rs, cnt) : rs.choice(cnt);
                }
                sfor<N>([&](auto Q) {
                    constexpr int q = Q;
                    if (dir_ok(e.px[base + q] - x0, e.py[base + q] - y0)) {
                        if (pick == 0) t = q;
                        --pick;
                    }
                });
            }
        }
        // select teammate t's position as tx = sum_q [q == t] * px[q] (exact: one term is
        // 1 * px, the others +-0), so LLVM cannot turn it into a scratch-memory lookup table
        tx = 0.0;
        ty = 0.0;
        sx = 0.0;
        sy = 0.0;
        sfor<N>([&](auto Q) {
            constexpr int q = Q;
            const double sel = q == t ? 1.0 : 0.0;
            tx = __builtin_fma(sel, e.px[base + q], tx);
            ty = __builtin_fma(sel, e.py[base + q], ty);
            if constexpr (kSqBatch<N>) {
                sx = __builtin_fma(sel, sq[2 * (base + q)], sx);  // the target's squares (ball - teammate)^2
                sy = __builtin_fma(sel, sq[2 * (base + q) + 1], sy);
            }
        });
    }
}

// ---------------------------------------------------------------------------
// Futbol.step (envs_v1/futbol_env.py:427-483) + DummyVecEnv auto-reset
// P: geometry / physics constants (a constexpr object in the default-field instance,
// the context's device copy otherwise); R: the context's device params (runtime fields)
template <int N, int EPW, typename OT>
__device__ __forceinline__ void v1_step_body(const V1Params& P, const V1Params* __restrict__ R, Scratch<N, EPW>& sh,
                                             V1Ptrs st, const uint8_t* __restrict__ actions, OT* __restrict__ obs,
                                             OT* __restrict__ reward, uint8_t* __restrict__ done_out,
                                             OT* __restrict__ term_obs)
{
    using S = V1Shape<N>;
    constexpr int BL = S::BALL;
    const int B = R->B;
    // lanes past B (last block) shadow env B-1's loads, which are in bounds, and return
    // after the segment table's barrier without storing anything
    const int env_raw = blockIdx.x * EPW + threadIdx.x;
    const bool live = env_raw < B;
    const int env = live ? env_raw : B - 1;
    const Lane<N, EPW> L{&sh, st.spill, st.ckey, st.cjn, (int)threadIdx.x, env, B
#ifdef FUTBOL_BOUNDS
                         , st.invalid
#endif
#ifdef FUTBOL_CRUMBS
                         , st.stamps
#endif
    };
#ifdef FUTBOL_STAMPS
    unsigned long long* st_stamps = st.stamps;
    unsigned long long _stamp_prev = __builtin_amdgcn_s_memtime();
    const unsigned long long _wave_real0 = __builtin_amdgcn_s_memrealtime(), _wave_cyc0 = _stamp_prev;
#endif
    // every HBM read of the step is issued here, in one batch (one memory round trip per step),
    // in the order of first use: the segment table (waited for alone at its LDS store), the
    // actions and the meta word (the opponent's draws need only these), then the body state,
    // the first CK arbiter-cache entries and the running return
    const SegLds seg_g = fetch_seg(P);
    uint32_t araw[2 * N];
    if constexpr ((2 * N) % 4 == 0) {
        const uint32_t* a32 = (const uint32_t*)(actions + (kScalarBase<N> ? (size_t)((uint32_t)env * (uint32_t)(2 * N)) : (size_t)env * (2 * N)));
        sfor<(2 * N) / 4>([&](auto W4) {
            constexpr int w = W4;
            const uint32_t x = a32[w];
            sfor<4>([&](auto Q) { araw[4 * w + Q] = (x >> (8 * Q)) & 0xffu; });
        });
    } else {
        const uint16_t* a16 = (const uint16_t*)(actions + (kScalarBase<N> ? (size_t)((uint32_t)env * (uint32_t)(2 * N)) : (size_t)env * (2 * N)));
        sfor<N>([&](auto W2) {
            constexpr int w = W2;
            const uint32_t x = a16[w];
            araw[2 * w] = x & 0xffu;
            araw[2 * w + 1] = x >> 8;
        });
    }
    Env<N> e;
    e.meta.w = kScalarBase<N> ? soa(st.meta, 0, B, env) : st.meta[env];
    load_bodies<N, !kLateBias<N>>(st, env, B, e);
    uint32_t ck[CKN<N>];
    double cj[CKN<N>];
    if constexpr (!kLateCache<N>) load_cache_pre<N, EPW>(L, e.meta.ncache(), ck, cj);
    const double ep_ret0 = kScalarBase<N> ? soa(st.ep_ret, 0, B, env) : st.ep_ret[env];
    // lanes past B (last block) run the action phase on their shadow copy of env B-1 in
    // registers only (no store, no counter) and leave after the segment table is in LDS
    const double W = P.W, H = P.H;
    FUTBOL_CRUMB(L, 1);
    FUTBOL_STAMP(0);

    const uint32_t ev = e.meta.event();
    e.meta.set_event(ev + 1);
    Stream rs(R->seed, R->env_base + (uint32_t)env, ev, 0);

    // actions: left team from HBM, right team = action_space.sample() (:306-307, :429)
    int arrow[2 * N], key[2 * N];
    int bad = 0;
    sfor<2 * N>([&](auto I) {
        constexpr int i = I;
        int a = (int)araw[i];
        bad += a > 4;
        a = a > 4 ? 4 : a;
        if constexpr (i & 1) key[i >> 1] = a; else arrow[i >> 1] = a;
    });
    {   // action_space.sample(): 2N uniform integers in [0, 5), four per Philox block, (w * 5) >> 32
        Philox4 blk;
        sfor<2 * N>([&](auto I) {
            constexpr int i = I;
            if constexpr (i % 4 == 0) blk = rs.next();
            const int a = (int)(((uint64_t)blk.x[i % 4] * 5ull) >> 32);
            if constexpr (i & 1) key[N + (i >> 1)] = a; else arrow[N + (i >> 1)] = a;
        });
    }
#ifdef FUTBOL_DIAG_EARLY_ATOMIC  // diagnostic builds only: the round-3 position of the count (see below)
    if (bad && live) atomicAdd(st.invalid, (unsigned long long)bad);
#endif
    FUTBOL_STAMP(1);

    // _ball_to_team_distance_arr(team_A), ball_init (:433-435)
    double d0[N];
    sfor<N>([&](auto I) {
        constexpr int i = I;
        const double dx = e.px[i] - e.px[BL], dy = e.py[i] - e.py[BL];
        d0[i] = sqrt(dx * dx + dy * dy);
    });
    const double bix = e.px[BL], biy = e.py[BL];

    // positions do not change during the action loop: one contact test per player
    bool touch[2 * N];
    sfor<2 * N>([&](auto K) {
        constexpr int k = K;
        touch[k] = cc_hit(e.px[BL], e.py[BL], kBallR, e.px[k], e.py[k], kPlayerR);
    });

    // _process_action per player, then owner update (:309-422, :447-453).
    // Shoot, press and pass all apply S * d / |d| for one direction d (shoot: goal - ball,
    // S = 120; press: ball - player, S = 40; pass: teammate - ball, S = 100), so each
    // player computes ONE sqrt and two divisions on the selected operands, and every
    // branch outcome is applied with exact selects (no +-0 additions) -- identical
    // results to the reference's five-way branch, without executing all of its arms.
    uint32_t owner = e.meta.owner();
    PassDraws pd{};
    if constexpr (kPassDraws<N>) {
        pd.j0 = rs.j;
        bool anyp = false;
        sfor<2 * N>([&](auto K) { anyp = anyp | (bool)((int)(key[K] == 4) & (int)touch[K]); });
        if (__ballot(anyp)) {  // wave-uniform: both blocks for every lane of a wave with a passer
            const Philox4 p0 = rs.block(pd.j0), p1 = rs.block(pd.j0 + 1);
            pd.a0 = p0.x[0];
            pd.b0 = p0.x[1];
            pd.a1 = p1.x[0];
            pd.b1 = p1.x[1];
        }
    }
    // get_vec's magnitude (envs_v1/futbol_env.py:56-59), np.sqrt(vec[0]**2 + vec[1]**2) with glibc
    // pow squares: the direction S * d / |d| feeds the state (round 3 squared with x*x here, and one
    // 5v5 env in 8 192 flipped an outcome within 600 steps: tests/test_oracle_modes.py).  Positions
    // do not change in the loop, so every candidate d is known now -- ball - player k (press; a
    // pass to teammate k squares k - ball, the same squares) and goal - ball (shoot) -- and their
    // exact squares are one batch: the near-midpoint ones of the squares some lane may use
    constexpr int NSQ = kSqBatch<N> ? 4 * N + 3 : 1;  // (N >= 6: per player, in the loop below)
    double sqin[NSQ], sq[NSQ];
    uint64_t sqneed = 0;
    if constexpr (kSqBatch<N>) {
        uint32_t pass_side = 0, shoot_side = 0;
        sfor<2 * N>([&](auto K) {
            constexpr int k = K;
            constexpr int side = k < N ? 0 : 1;
            pass_side |= (uint32_t)((key[k] == 4) & touch[k]) << side;
            shoot_side |= (uint32_t)((key[k] == 2) & touch[k]) << side;
        });
        sfor<2 * N>([&](auto K) {
            constexpr int k = K;
            constexpr int side = k < N ? 0 : 1;
            sqin[2 * k] = e.px[BL] - e.px[k];
            sqin[2 * k + 1] = e.py[BL] - e.py[k];
            const bool press = (key[k] == 3) & !touch[k] & (arrow[k] == 0);
            sqneed |= (uint64_t)(press | (bool)((pass_side >> side) & 1u)) * (3ull << (2 * k));
        });
        sqin[4 * N] = W - e.px[BL];      // shoot of side 0 (goal at x = W)
        sqin[4 * N + 1] = 0.0 - e.px[BL];  // side 1 (goal at x = 0)
        sqin[4 * N + 2] = H / 2 - e.py[BL];
        sqneed |= ((uint64_t)(shoot_side & 1u) << (4 * N)) | ((uint64_t)(shoot_side >> 1) << (4 * N + 1)) |
                  ((uint64_t)(shoot_side != 0) << (4 * N + 2));
    }
    // (the solver rows are free from the step's start until space_step's narrowphase stages the
    // bodies in them: nothing is kept in them across steps or ROLL iterations)
    static_assert(!kSqBatch<N> || sizeof(sh.rows) >= (size_t)kPowTabBytes, "pow tables fit the solver rows");
    if constexpr (kSqBatch<N>)
        glibc_pow2_need_lds<NSQ>(sqin, sq, sqneed, &sh.rows[0][0]);  // (rows: unused until space_step)
    FUTBOL_STAMP(20);
    sfor<2 * N>([&](auto K) {
        constexpr int k = K;
        constexpr int side = k < N ? 0 : 1;
        const int ar = arrow[k], ky = key[k];
        const bool tk = touch[k];
        const int fx = ar == 2 ? 1 : (ar == 4 ? -1 : 0);
        const int fy = ar == 1 ? 1 : (ar == 3 ? -1 : 0);
        const bool move = ky <= 1;                      // noop / dash (:331-341)
        const bool shoot = (ky == 2) & tk;              // (:344-368)
        const bool press = (ky == 3) & !tk & (ar == 0); // (:371-391)
        const bool pass = (ky == 4) & tk;               // (:394-419)
        double tx = 0.0, ty = 0.0, tsx = 0.0, tsy = 0.0;
        if constexpr (N == 2) {
            // one teammate: get_pass_target_teammate always returns it (team.py:136-180); its
            // draws are one-item choices (floor(u * 1) = 0) that only advance the stream: one,
            // plus one when an arrow is held and the teammate lies strictly that way
            constexpr int mate = side * N + (1 - (k - side * N));
            const double mx = e.px[mate] - e.px[k], my = e.py[mate] - e.py[k];
            const bool way = ((ar == 1) & (my > 0)) | ((ar == 2) & (mx > 0)) | ((ar == 3) & (my < 0)) | ((ar == 4) & (mx < 0));
            tx = e.px[mate];
            ty = e.py[mate];
            tsx = sq[2 * mate];
            tsy = sq[2 * mate + 1];
            rs.skip(pass ? (way ? 2u : 1u) : 0u);
        } else {
#ifdef FUTBOL_DIAG_NOPASS  // diagnostic only (wrong results): the cost of the pass-target draws
            tx = e.px[side * N];
            ty = e.py[side * N];
#else
            if (pass) pass_target<N, side, k - side * N>(e, rs, pd, ar, tx, ty, sq, tsx, tsy);
#endif
        }
        const double gx = side == 0 ? W : 0.0, gy = H / 2;
        const double ox = press ? e.px[k] : e.px[BL], oy = press ? e.py[k] : e.py[BL];
        const double qx = press ? e.px[BL] : (shoot ? gx : tx), qy = press ? e.py[BL] : (shoot ? gy : ty);
        const double dx = qx - ox, dy = qy - oy;
        double sx, sy;
        if constexpr (kSqBatch<N>) {
            sx = press ? sq[2 * k] : (shoot ? sq[4 * N + side] : tsx);
            sy = press ? sq[2 * k + 1] : (shoot ? sq[4 * N + 2] : tsy);
        } else {  // N >= 6: this player's two squares (tables from global memory)
            const double q2[2] = {dx, dy};
            double s2[2];
            glibc_pow2_need_t<2, kPowCall<N>>(q2, s2, (press | shoot | pass) ? 3ull : 0ull);
            sx = s2[0];
            sy = s2[1];
            (void)tsx;
            (void)tsy;
        }
        const double mag = sqrt(sx + sy);
        const double S = press ? 40.0 : (shoot ? 120.0 : 100.0);
        const double fdx = S * dx / mag, fdy = S * dy / mag;
        // player velocity: move impulse (f * arrow) / m, or the press impulse
        const int f = ky == 0 ? 20 : 40;
        const double mvx = e.vx[k] + (double)(f * fx) * kPlayerMinv, mvy = e.vy[k] + (double)(f * fy) * kPlayerMinv;
        const double pvx = e.vx[k] + fdx * kPlayerMinv, pvy = e.vy[k] + fdy * kPlayerMinv;
        e.vx[k] = move ? mvx : (press ? pvx : e.vx[k]);
        e.vy[k] = move ? mvy : (press ? pvy : e.vy[k]);
        // ball velocity: dribble (ball takes the player's velocity) or a kick (v/2 or v/10, + impulse)
        const double D = shoot ? 2.0 : 10.0, rD = shoot ? 0.5 : 0.1;
        const double kvx = cdiv(e.vx[BL], D, rD) + fdx * kBallMinv, kvy = cdiv(e.vy[BL], D, rD) + fdy * kBallMinv;
        const bool dribble = move & tk, kick = shoot | pass;
        e.vx[BL] = dribble ? e.vx[k] : (kick ? kvx : e.vx[BL]);
        e.vy[BL] = dribble ? e.vy[k] : (kick ? kvy : e.vy[BL]);
        owner = tk ? (uint32_t)side : owner;
    });
    FUTBOL_STAMP(21);

    // check_and_fix_out_bounds (:247-287), before physics
    bool out = false;
    if (!far_from_segments(e.px[BL], e.py[BL], 2.0, W, H)) {
        int w = -1;
        for (int s = 0; s < 6; ++s)
            if (w < 0 && cs_hit(P, s, e.px[BL], e.py[BL], kBallR)) w = s;
        if (w >= 0) {
            out = true;
            const double bx0 = e.px[BL], by0 = e.py[BL];
            double dbx = 0, dby = 0, dpx = 0, dpy = 0;
            if (w <= 1) { dbx = 3.5; dpx = 1; }
            else if (w == 3 || w == 4) { dbx = -3.5; dpx = -1; }
            else if (w == 2) { dby = -3.5; dpy = -1; }
            else { dby = 3.5; dpy = 1; }
            e.px[BL] = bx0 + dbx;
            e.py[BL] = by0 + dby;
            e.vx[BL] = 0.0;
            e.vy[BL] = 0.0;
            // random.choice of the new owner team's players (one draw either way)
            const int pick = rs.choice(N) + (owner == 1 ? 0 : N);
            owner = owner == 1 ? 0 : 1;
            sfor<2 * N>([&](auto Q) {
                constexpr int q = Q;
                if (q == pick) {
                    e.px[q] = bx0 + dpx;
                    e.py[q] = by0 + dpy;
                    e.vx[q] = 0.0;
                    e.vy[q] = 0.0;
                }
            });
        }
    }
    e.meta.set_owner(owner);
    FUTBOL_STAT(30, __popcll(__ballot(out)));
    // the segment table's loads were issued with the state's; every lane of the block is here
    store_seg<N, EPW>(seg_g, sh);
    if (!live) return;
    if constexpr (kLateBias<N>) load_bias<N>(st, env, B, e);
    if constexpr (kLateCache<N>) load_cache_pre<N, EPW>(L, e.meta.ncache(), ck, cj);
    FUTBOL_CRUMB(L, 3);
    FUTBOL_STAMP(2);

    // Up to three cpSpaceSteps per call, through ONE inlined call site:
    //   phase 0: space.step(TIME_STEP) of this step            (:459)
    //   phase 1: _position_to_initial after a goal, step(1e-4) (:474, :129-144)
    //   phase 2: DummyVecEnv auto-reset -> reset(), step(1e-4) (:146-150)
    double r = 0.0, ret = 0.0;
    bool goal = false, done = false, pre_aged = false;
#pragma unroll 1
    for (int ph = 0; ph < 3; ++ph) {
        if (ph == 1 && !goal) continue;
        if (ph == 2 && !(done && R->auto_reset)) continue;
        if (ph == 1) position_to_initial<N>(P, e);
        if (ph == 2) {
            if (term_obs) write_obs<N, OT>(e, term_obs + (size_t)env * (4 * S::Nb));
            st.stat_ret[env] = st.stat_ret[env] + ret;
            st.stat_cnt[env] = st.stat_cnt[env] + 1;
            ret = 0.0;
            const uint32_t ev2 = e.meta.event();
            e.meta.set_event(ev2 + 1);
            rs = Stream(R->seed, R->env_base + (uint32_t)env, ev2, 0);
            e.meta.set_owner((uint32_t)rs.choice(2));
            e.meta.set_steps(0);
            position_to_initial<N>(P, e);
        }
        FUTBOL_STAMP(ph == 0 ? 3 : 9);
        // the restart micro-steps: the per-lane no-contact path unless a v_bias is huge (after a
        // goal, phase 0 has already filtered the cache for it when its guard holds)
        if (ph == 0 || !formation_step<N, EPW>(P, L, e, ph == 1 && pre_aged)) {
            if (ph != 0) load_cache_pre<N, EPW>(L, e.meta.ncache(), ck, cj);  // the cache the previous phase left behind
            bool goal_ph;
            space_step<N, EPW>(P, L, e, ph == 0 ? 2 : 1, ck, cj, goal_ph, pre_aged
#ifdef FUTBOL_STAMPS
                          , st_stamps, _stamp_prev
#endif
            );
            if (ph == 0) goal = goal_ph;
        }
        if (ph == 0) {
            if (!out) {  // get_team_reward + get_ball_reward (:493-515)
                double mx = 0.0;
                sfor<N>([&](auto I) {
                    constexpr int i = I;
                    const double dx = e.px[i] - e.px[BL], dy = e.py[i] - e.py[BL];
                    const double diff = d0[i] - sqrt(dx * dx + dy * dy);
                    if constexpr (N == 5) {
                        if constexpr (i == 3) mx = diff;
                        if constexpr (i == 4) mx = diff > mx ? diff : mx;
                    } else {
                        if (i == 0 || diff > mx) mx = diff;
                    }
                });
                r = r + mx * 10;
                const double gx = W, gy = H / 2;
                const double ax_ = e.px[BL] - gx, ay_ = e.py[BL] - gy;
                const double ix_ = bix - gx, iy_ = biy - gy;
                r = r + (sqrt(ix_ * ix_ + iy_ * iy_) - sqrt(ax_ * ax_ + ay_ * ay_)) * 10;
            }
            // ball_contact_goal (:291-296), tested by space_step on the final positions; a goal
            // restarts from formation, the episode goes on
            if (goal) r = r + (e.px[BL] > W - 2 ? 1000.0 : -1000.0);
            FUTBOL_STAT(31, __popcll(__ballot(goal)));
            // current_time += 0.1; done = current_time > total_time
            uint32_t steps = e.meta.steps() + 1;
            steps = steps > (uint32_t)kMaxSteps ? (uint32_t)kMaxSteps : steps;  // saturate (no auto-reset)
            e.meta.set_steps(steps);
            done = (int)steps >= R->K_done;
            ret = ep_ret0 + r;
            if (done && !R->auto_reset) {
                if ((int)steps == R->K_done) {
                    st.stat_ret[env] = st.stat_ret[env] + ret;
                    st.stat_cnt[env] = st.stat_cnt[env] + 1;
                }
                ret = 0.0;
            }
        } else if (ph == 1) {
            e.meta.set_owner((uint32_t)rs.choice(2));  // random.choice(["left","right"]) (:475)
        }
        FUTBOL_STAMP(ph == 0 ? 8 : 9);
    }
    FUTBOL_CRUMB(L, 80);
    const int eo = kOpaqueStore<N> ? opaque_lane(env) : env;  // (the step's output addresses, computed here)
    if constexpr (kScalarBase<N>) {
        write_obs<N, OT>(e, obs + (size_t)((uint32_t)eo * (uint32_t)(4 * S::Nb)));
        soa(st.ep_ret, 0, B, eo) = ret;
        soa(reward, 0, B, eo) = (OT)r;
        soa(done_out, 0, B, eo) = done ? 1 : 0;
    } else {
    write_obs<N, OT>(e, obs + (size_t)eo * (4 * S::Nb));
    st.ep_ret[eo] = ret;
    reward[eo] = (OT)r;
    done_out[eo] = done ? 1 : 0;
    }
    store_env<N>(st, env, B, e);
    // The clamped-action count (futbol_invalid_actions) is the step's last memory operation, where no
    // value is live.  It used to follow the action decode, amid ~60 loads in flight and every state
    // register live: the atomic optimizer turns a divergent atomicAdd into a wave reduction and a
    // one-lane `if` nested in the `if (bad)`, and at their shared join the register allocator placed
    // live-range-split copies (v_accvgpr_write aN, vM of per-lane addresses and state) BEFORE the exec
    // restore, where they run with the inner `if`'s exec mask -- no lane at all when no action was
    // out of range -- so the AGPRs kept stale values that were read back later: the round-3 wrong
    // velocities (N = 9), wrong positions and illegal address (N = 7) and the step-19 divergence
    // (N = 3) of DESIGN.md section 6.  scripts/isa_exec_check.py finds the pattern in the code objects
    // (tests/test_isa_exec.py).  (Lanes past B returned before the solve: no count.)
#ifndef FUTBOL_DIAG_EARLY_ATOMIC
    if (bad) atomicAdd(st.invalid, (unsigned long long)bad);
#endif
    FUTBOL_CRUMB(L, 99);
    FUTBOL_STAMP(10);
#ifdef FUTBOL_STAMPS
    // snapshot of THIS launch (overwritten every launch): start / end realtime (100 MHz),
    // wave cycles, and where the wave ran (HW_ID: wave, simd, cu, sh, se | XCC_ID << 32)
    if ((threadIdx.x & 63) == 0 && st_stamps) {
        unsigned long long* w = &st_stamps[(size_t)(blockIdx.x * EPW / 64) * kStampStride];
        const unsigned long long real1 = __builtin_amdgcn_s_memrealtime();
        const unsigned long long cyc1 = __builtin_amdgcn_s_memtime();
        const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);
        const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);
        w[11] = _wave_real0;
        w[12] = real1;
        w[13] = cyc1 - _wave_cyc0;
        w[14] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    }
#endif
}

// DEF: the registered ids' default field (v1_default_geometry<N>), constants as immediates.
// nsteps > 1: an open-loop rollout (futbol_rollout): the block's envs run nsteps consecutive
// env-steps in one launch, step k reading actions[k] and writing obs[k] / reward[k] / done[k] /
// term_obs[k] (each slice [B][...]); every step is the same step body with its own state load and
// store.  Blocks never wait for each other between steps, so a wave's slow step is averaged out
// over its own next steps instead of holding the whole grid.  ROLL = false (futbol_step): one step
// and no loop around the body (the loop measured +7% on the 2v2 step: 21.4 -> 22.9 us).
// experiments only: e.g. -DFUTBOL_V1_STEP_ATTR="__attribute__((amdgpu_waves_per_eu(2)))"
#ifndef FUTBOL_V1_STEP_ATTR
#define FUTBOL_V1_STEP_ATTR
#endif
template <int N, int EPW, typename OT, bool DEF, bool ROLL>
__global__ void __launch_bounds__(EPW) FUTBOL_V1_STEP_ATTR v1_step_kernel(const V1Params* __restrict__ R, V1Ptrs st,
                                                      const uint8_t* __restrict__ actions, OT* __restrict__ obs,
                                                      OT* __restrict__ reward, uint8_t* __restrict__ done_out,
                                                      OT* __restrict__ term_obs, int nsteps)
{
    // 4 blocks per CU (160 KB of LDS) up to N = 7 and with one row set, 3 blocks otherwise
    // (FUTBOL_LDS_BLOCKS_PER_CU: an A/B build that trades blocks per CU for LDS record slots)
#ifndef FUTBOL_LDS_BLOCKS_PER_CU
    static_assert(sizeof(Scratch<N, EPW>) <= (N <= 7 || V1Shape<N>::ONE_ROWS ? 160 * 1024 / 4 : 160 * 1024 / 3),
                  "LDS per block");
#else
    static_assert(sizeof(Scratch<N, EPW>) <= 160 * 1024 / FUTBOL_LDS_BLOCKS_PER_CU, "LDS per block");
#endif
    __shared__ Scratch<N, EPW> sh;
    using S = V1Shape<N>;
    if constexpr (!ROLL) {
        if constexpr (DEF) {
            constexpr V1Params G = v1_default_geometry<N>();
            v1_step_body<N, EPW, OT>(G, R, sh, st, actions, obs, reward, done_out, term_obs);
        } else {
            v1_step_body<N, EPW, OT>(*R, R, sh, st, actions, obs, reward, done_out, term_obs);
        }
        return;
    }
    const size_t B = (size_t)R->B;
#pragma unroll 1
    for (int k = 0; k < nsteps; ++k) {
        const uint8_t* a = actions + (size_t)k * B * (2 * N);
        OT* o = obs + (size_t)k * B * (4 * S::Nb);
        OT* t = term_obs ? term_obs + (size_t)k * B * (4 * S::Nb) : nullptr;
        if constexpr (DEF) {
            constexpr V1Params G = v1_default_geometry<N>();
            v1_step_body<N, EPW, OT>(G, R, sh, st, a, o, reward + (size_t)k * B, done_out + (size_t)k * B, t);
        } else {
            v1_step_body<N, EPW, OT>(*R, R, sh, st, a, o, reward + (size_t)k * B, done_out + (size_t)k * B, t);
        }
    }
}

// futbol_create (init=1: Futbol.__init__, which ends in reset()) / futbol_reset (masked)
template <int N, int EPW, typename OT>
__global__ void __launch_bounds__(EPW) v1_reset_kernel(const V1Params* __restrict__ R, V1Ptrs st,
                                                      const uint8_t* __restrict__ mask, OT* __restrict__ obs,
                                                      int init)
{
    using S = V1Shape<N>;
    const V1Params& P = *R;
    __shared__ Scratch<N, EPW> sh;
    load_seg_table<N, EPW>(P, sh);
    const int env = blockIdx.x * EPW + threadIdx.x;
    const int B = R->B;
    if (env >= B) return;
    if (mask && !mask[env]) return;
    const Lane<N, EPW> L{&sh, st.spill, st.ckey, st.cjn, (int)threadIdx.x, env, B
#ifdef FUTBOL_BOUNDS
                         , st.invalid
#endif
#ifdef FUTBOL_CRUMBS
                         , st.stamps
#endif
    };
    Env<N> e;
    if (init) {
        sfor<S::Nb>([&](auto K) {
            constexpr int k = K;
            e.px[k] = P.fx[k];
            e.py[k] = P.fy[k];
            e.vx[k] = e.vy[k] = e.bx[k] = e.by[k] = 0.0;
        });
        e.meta.w = 0;
        st.stat_ret[env] = 0.0;
        st.stat_cnt[env] = 0;
    } else {
        load_env<N>(st, env, B, e);
    }
    st.ep_ret[env] = 0.0;
#ifdef FUTBOL_STAMPS
    unsigned long long* st_stamps = nullptr;
    unsigned long long _stamp_prev = 0;
#endif
    do_reset<N, EPW>(P, R, L, e
#ifdef FUTBOL_STAMPS
                , st_stamps, _stamp_prev
#endif
    );
    if (obs) write_obs<N, OT>(e, obs + (size_t)env * (4 * S::Nb));
    store_env<N>(st, env, B, e);
}

}  // namespace futbol
