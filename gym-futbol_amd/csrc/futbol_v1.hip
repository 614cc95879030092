// futbol_v1.hip -- dispatch of the envs_v1 kernels over the supported team sizes.
#include "futbol_kernels.hpp"

namespace futbol {

#define FUTBOL_V1_DECL(n)                                                                                   \
    int launch_v1_n##n(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a,   \
                       const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init,   \
                       hipStream_t stream);                                                                 \
    size_t v1_spill_slots_n##n();
FUTBOL_V1_DECL(1)
FUTBOL_V1_DECL(2)
FUTBOL_V1_DECL(3)
FUTBOL_V1_DECL(5)
FUTBOL_V1_DECL(10)

int launch_v1(int N, const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* actions,
              const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream)
{
#define FUTBOL_V1_CASE(n) \
    case n: return launch_v1_n##n(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    switch (N) {
        FUTBOL_V1_CASE(1)
        FUTBOL_V1_CASE(2)
        FUTBOL_V1_CASE(3)
        FUTBOL_V1_CASE(5)
        FUTBOL_V1_CASE(10)
    default: return -2;
    }
}

int v1_supported(int N) { return N == 1 || N == 2 || N == 3 || N == 5 || N == 10; }

size_t v1_spill_slots(int N)
{
    switch (N) {
    case 1: return v1_spill_slots_n1();
    case 2: return v1_spill_slots_n2();
    case 3: return v1_spill_slots_n3();
    case 5: return v1_spill_slots_n5();
    case 10: return v1_spill_slots_n10();
    default: return 0;
    }
}

}  // namespace futbol
