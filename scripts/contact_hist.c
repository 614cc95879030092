/* scripts/contact_hist.c -- diagnostic (uses the test-only oracle): distribution of contact
 * records per env-step and of its max over each 64-env wave, 2v2 random play.
 *   gcc -O2 -std=c11 -ffp-contract=off -fopenmp -Ioracle scripts/contact_hist.c \
 *       oracle/futbol_v1_oracle.c oracle/futbol_v0_oracle.c -lm -o /tmp/contact_hist
 *   /tmp/contact_hist 16384 600 [N]
 * Left actions from an LCG, right team and resets from the oracle's own RNG tape. */
#include "futbol_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
int main(int argc, char **argv) {
    int B = argc > 1 ? atoi(argv[1]) : 65536, T = argc > 2 ? atoi(argv[2]) : 300, N = argc > 3 ? atoi(argv[3]) : 2;
    OrcV1 *e = malloc(sizeof(OrcV1) * B);
    double obs[64]; double r;
    for (int b = 0; b < B; ++b) { orc_v1_init(&e[b], N, 105, 68, 30, 7, b); orc_v1_reset(&e[b], obs); }
    long hist[64] = {0}, whist[64] = {0};
    unsigned s = 1;
    for (int t = 0; t < T; ++t) {
        int wmax = 0;
        for (int b = 0; b < B; ++b) {
            int32_t a[64];
            for (int k = 0; k < 2 * N; ++k) { s = s * 1103515245u + 12345u; a[k] = (s >> 16) % 5; }
            int d = orc_v1_step(&e[b], a, obs, &r);
            if (d) orc_v1_reset(&e[b], obs);
            int n = 0;
            for (int p = 0; p < e[b].P; ++p) n += e[b].arb_inlist[p] ? 1 : 0;
            hist[n]++;
            if (n > wmax) wmax = n;
            if ((b & 63) == 63) { whist[wmax]++; wmax = 0; }
        }
    }
    printf("per env-step contacts:\n");
    for (int i = 0; i < 64; ++i) if (hist[i]) printf("  %2d %ld\n", i, hist[i]);
    printf("per wave-step max:\n");
    for (int i = 0; i < 64; ++i) if (whist[i]) printf("  %2d %ld\n", i, whist[i]);
}
