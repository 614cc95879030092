// futbol_v1.hip -- dispatch of the envs_v1 kernels over team sizes and envs-per-wave.
#include "futbol_kernels.hpp"
#include "futbol_v1_impl.hpp"

namespace futbol {

int launch_v1_n1_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);
int launch_v1_n1_e32(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);
int launch_v1_n2_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);
int launch_v1_n2_e32(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);
int launch_v1_n3_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);
int launch_v1_n3_e32(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);
int launch_v1_n5_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);
int launch_v1_n5_e32(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);
int launch_v1_n10_e64(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);
int launch_v1_n10_e32(const V1Params* P, int B, const V1Ptrs& st, int out64, int what, const uint8_t* a, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term, int init, hipStream_t stream);

int launch_v1(int N, int epw, const V1Params* P, int B, const V1Ptrs& st, int out64, int what,
              const uint8_t* actions, const uint8_t* mask, void* obs, void* reward, uint8_t* done, void* term,
              int init, hipStream_t stream)
{
    if (N == 1 && epw == 64) return launch_v1_n1_e64(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    if (N == 1 && epw == 32) return launch_v1_n1_e32(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    if (N == 2 && epw == 64) return launch_v1_n2_e64(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    if (N == 2 && epw == 32) return launch_v1_n2_e32(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    if (N == 3 && epw == 64) return launch_v1_n3_e64(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    if (N == 3 && epw == 32) return launch_v1_n3_e32(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    if (N == 5 && epw == 64) return launch_v1_n5_e64(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    if (N == 5 && epw == 32) return launch_v1_n5_e32(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    if (N == 10 && epw == 64) return launch_v1_n10_e64(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    if (N == 10 && epw == 32) return launch_v1_n10_e32(P, B, st, out64, what, actions, mask, obs, reward, done, term, init, stream);
    return -2;
}

int v1_supported(int N) { return N == 1 || N == 2 || N == 3 || N == 5 || N == 10; }
int v1_supported_epw(int epw) { return epw == 64 || epw == 32; }

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
