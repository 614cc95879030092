// The round-4 kx6 fault, replayed on the host: glibc pow(x, 2) of env 93's press
// direction (5v5, step 5) with kPowLog staged as the miscompiled stage_pow_tables wrote it.
//   hipcc -O0 -ffp-contract=off -I gym-futbol_amd/csrc -o /tmp/t scripts/kx6_table_repro.cpp && /tmp/t
#include <cstdio>
#include <cstring>
#include <cstdint>
#include "futbol_math.hpp"
using namespace futbol;
int main() {
    double x = -34.6387302914942;  // dx of env 93, body 5, step 5 (press: ball - player)
    double L[384]; uint64_t E[256];
    memcpy(L, kPowLog, sizeof L); memcpy(E, kPowExp, sizeof E);
    double good = glibc_pow2_full(x, L, E);
    // the kx6 staging bug: the first double of every chunk c = 128 + w gets the high word of chunk 64 + w's first double
    for (int w = 0; w < 64; ++w) {
        uint32_t* dst = (uint32_t*)&L[2 * (128 + w)];
        const uint32_t* src = (const uint32_t*)&kPowLog[2 * (64 + w)];
        dst[1] = src[1];
    }
    double bad = glibc_pow2_full(x, L, E);
    printf("L256 %a (%a)  L128 %a  corrupted L256 %a\n", kPowLog[256], kPowLog[256], kPowLog[128], L[256]);
    printf("x*x %.17g glibc %.17g corrupted-table %.17g\n", x * x, good, bad);
}

