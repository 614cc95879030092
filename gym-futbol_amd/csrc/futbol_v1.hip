// futbol_v1.hip -- dispatch of the envs_v1 kernels over team sizes and envs-per-wave.
#include "futbol_kernels.hpp"
#include "futbol_v1_impl.hpp"
#include <string.h>

namespace futbol {

#define FUTBOL_DECL(n)                                                                                    \
    int launch_v1_n##n##_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, int def,     \
                             const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, \
                             void* term, int init, int nsteps, hipStream_t stream);                   \
    void layout_v1_n##n##_e64(int32_t* o);
FUTBOL_DECL(1)
FUTBOL_DECL(2)
FUTBOL_DECL(3)
FUTBOL_DECL(4)
FUTBOL_DECL(5)
FUTBOL_DECL(6)
FUTBOL_DECL(7)
FUTBOL_DECL(8)
FUTBOL_DECL(9)
FUTBOL_DECL(10)
#undef FUTBOL_DECL

int launch_v1(int N, int epw, int def, const V1Params* P, int B, const V1Ptrs& st, int out64, int what,
              const uint8_t* actions, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term,
              int init, int nsteps, hipStream_t stream)
{
    if (epw != 64) return -2;
    switch (N) {
#define FUTBOL_CASE(n)                                                                                    \
    case n:                                                                                               \
        return launch_v1_n##n##_e64(P, B, st, out64, what, def, actions, mask, obs, reward, done, term, init, nsteps, \
                                    stream);
    FUTBOL_CASE(1) FUTBOL_CASE(2) FUTBOL_CASE(3) FUTBOL_CASE(4) FUTBOL_CASE(5)
    FUTBOL_CASE(6) FUTBOL_CASE(7) FUTBOL_CASE(8) FUTBOL_CASE(9) FUTBOL_CASE(10)
#undef FUTBOL_CASE
    default: return -2;
    }
}

// futbol_solver_layout: the constants of the team size's own translation unit
int layout_v1(int N, int32_t* o)
{
    switch (N) {
#define FUTBOL_CASE(n) case n: layout_v1_n##n##_e64(o); return 0;
    FUTBOL_CASE(1) FUTBOL_CASE(2) FUTBOL_CASE(3) FUTBOL_CASE(4) FUTBOL_CASE(5)
    FUTBOL_CASE(6) FUTBOL_CASE(7) FUTBOL_CASE(8) FUTBOL_CASE(9) FUTBOL_CASE(10)
#undef FUTBOL_CASE
    default: return -1;
    }
}

// the runtime-built geometry equals the compile-time default field of the default-field kernel
bool v1_is_default_geometry(int N, const V1Params& p)
{
    V1Params g{};
    switch (N) {
#define FUTBOL_CASE(n) case n: g = v1_default_geometry<n>(); break;
    FUTBOL_CASE(1) FUTBOL_CASE(2) FUTBOL_CASE(3) FUTBOL_CASE(4) FUTBOL_CASE(5)
    FUTBOL_CASE(6) FUTBOL_CASE(7) FUTBOL_CASE(8) FUTBOL_CASE(9) FUTBOL_CASE(10)
#undef FUTBOL_CASE
    default: return false;
    }
    V1Params q = p;  // runtime fields are not part of the geometry
    q.seed = 0;
    q.env_base = 0;
    q.B = 0;
    q.K_done = 0;
    q.auto_reset = 0;
    return memcmp(&q, &g, sizeof(V1Params)) == 0;
}

// every number_of_player the reference's Team formation implements (team.py:52-112: N <= 10;
// larger teams print "unimplemented" and fail)
int v1_supported(int N) { return N >= 1 && N <= 10; }
int v1_supported_epw(int epw) { return epw == 64; }

// spill slots needed in the worst case: the pairs past the LDS record slots of the kernel's OWN
// translation unit (layout_v1), not this one's V1Shape -- an A/B build of one TU with fewer slots
// (FUTBOL_K5=3) would otherwise index past the allocation
size_t v1_spill_slots(int N)
{
    int32_t o[8];
    if (layout_v1(N, o)) return 0;
    switch (N) {
#define FUTBOL_CASE(n) case n: return (size_t)(V1Shape<n>::P - (o[0] < V1Shape<n>::P ? o[0] : V1Shape<n>::P));
    FUTBOL_CASE(1) FUTBOL_CASE(2) FUTBOL_CASE(3) FUTBOL_CASE(4) FUTBOL_CASE(5)
    FUTBOL_CASE(6) FUTBOL_CASE(7) FUTBOL_CASE(8) FUTBOL_CASE(9) FUTBOL_CASE(10)
#undef FUTBOL_CASE
    default: return 0;
    }
}

}  // namespace futbol
