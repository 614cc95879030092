// futbol_util.hpp -- compile-time loops.
//
// Per-lane arrays (the env's bodies) must only ever be indexed by
// compile-time constants, or the compiler moves them to scratch memory.
// `sfor<N>(f)` calls f(integral_constant<int, i>) for i = 0..N-1 and is
// guaranteed to unroll, whatever the loop body's size.
#pragma once
#include <hip/hip_runtime.h>
#include <utility>

namespace futbol {

template <int Off, class F, int... Is>
__device__ __forceinline__ void sfor_impl(F&& f, std::integer_sequence<int, Is...>)
{
    (f(std::integral_constant<int, Off + Is>{}), ...);
}

// i = Begin .. End-1
template <int Begin, int End, class F>
__device__ __forceinline__ void sfor(F&& f)
{
    if constexpr (End > Begin) sfor_impl<Begin>(f, std::make_integer_sequence<int, End - Begin>{});
}

template <int End, class F>
__device__ __forceinline__ void sfor(F&& f)
{
    sfor<0, End>(f);
}

}  // namespace futbol
