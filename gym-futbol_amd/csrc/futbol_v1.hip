// futbol_v1.hip -- dispatch of the envs_v1 kernels over team sizes and envs-per-wave.
#include "futbol_kernels.hpp"
#include "futbol_v1_impl.hpp"
#include <string.h>

namespace futbol {

#define FUTBOL_DECL(n)                                                                                    \
    int launch_v1_n##n##_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, int def,     \
                             const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, \
                             void* term, int init, hipStream_t stream);
FUTBOL_DECL(1)
FUTBOL_DECL(2)
FUTBOL_DECL(3)
FUTBOL_DECL(5)
FUTBOL_DECL(10)
#undef FUTBOL_DECL

int launch_v1(int N, int epw, int def, const V1Params* P, int B, const V1Ptrs& st, int out64, int what,
              const uint8_t* actions, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term,
              int init, hipStream_t stream)
{
    if (epw != 64) return -2;
    switch (N) {
    case 1: return launch_v1_n1_e64(P, B, st, out64, what, def, actions, mask, obs, reward, done, term, init, stream);
    case 2: return launch_v1_n2_e64(P, B, st, out64, what, def, actions, mask, obs, reward, done, term, init, stream);
    case 3: return launch_v1_n3_e64(P, B, st, out64, what, def, actions, mask, obs, reward, done, term, init, stream);
    case 5: return launch_v1_n5_e64(P, B, st, out64, what, def, actions, mask, obs, reward, done, term, init, stream);
    case 10: return launch_v1_n10_e64(P, B, st, out64, what, def, actions, mask, obs, reward, done, term, init, stream);
    default: return -2;
    }
}

// the runtime-built geometry equals the compile-time default field of the default-field kernel
bool v1_is_default_geometry(int N, const V1Params& p)
{
    V1Params g{};
    switch (N) {
    case 1: g = v1_default_geometry<1>(); break;
    case 2: g = v1_default_geometry<2>(); break;
    case 3: g = v1_default_geometry<3>(); break;
    case 5: g = v1_default_geometry<5>(); break;
    case 10: g = v1_default_geometry<10>(); break;
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

int v1_supported(int N) { return N == 1 || N == 2 || N == 3 || N == 5 || N == 10; }
int v1_supported_epw(int epw) { return epw == 64; }

// spill slots needed in the worst case (largest EPW = fewest LDS slots)
size_t v1_spill_slots(int N)
{
    switch (N) {
    case 1: return V1Shape<1>::P - V1Shape<1>::K;
    case 2: return V1Shape<2>::P - V1Shape<2>::K;
    case 3: return V1Shape<3>::P - V1Shape<3>::K;
    case 5: return V1Shape<5>::P - V1Shape<5>::K;
    case 10: return V1Shape<10>::P - V1Shape<10>::K;
    default: return 0;
    }
}

}  // namespace futbol
