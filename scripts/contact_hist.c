/* scripts/contact_hist.c -- diagnostic (uses the test-only oracle): distribution of contact
 * records per env-step and of its max over each 64-env wave, random play; plus the solver
 * work of the two SIMT organisations of the sequential-impulse loop:
 *   "per-lane list": a wave sweeps max-over-lanes(records) slots (the kernels' solver);
 *   "static slots":  a wave sweeps, per body k, max-over-lanes(segment contacts of k) slots,
 *                    then every circle pair that any lane has in contact.
 *   gcc -O2 -std=c11 -ffp-contract=off -fopenmp -Ioracle scripts/contact_hist.c \
 *       oracle/futbol_v1_oracle.c oracle/futbol_v0_oracle.c -lm -o /tmp/contact_hist
 *   /tmp/contact_hist 16384 600 [N]
 * Left actions from an LCG, right team and resets from the oracle's own RNG tape. */
#include "futbol_oracle.h"
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define WAVE 64
#define NH (ORC_MAXP + 1)

int main(int argc, char **argv) {
    int B = argc > 1 ? atoi(argv[1]) : 65536, T = argc > 2 ? atoi(argv[2]) : 300, N = argc > 3 ? atoi(argv[3]) : 2;
    if (N < 1 || N > ORC_MAXN || B % WAVE) {
        fprintf(stderr, "need 1 <= N <= %d and B a multiple of %d\n", ORC_MAXN, WAVE);
        return 1;
    }
    const int Nb = 2 * N + 1, nwave = B / WAVE;
    OrcV1 *e = malloc(sizeof(OrcV1) * B);
    double obs[4 * ORC_MAXB]; double r;
    for (int b = 0; b < B; ++b) { orc_v1_init(&e[b], N, 105, 68, 30, 7, b); orc_v1_reset(&e[b], obs); }
    static long hist[NH], whist[NH], shist[NH], phist[NH];
    double sum_maxn = 0, sum_seg = 0, sum_pair = 0, sum_step_maxn = 0, sum_step_seg = 0, sum_step_pair = 0;
    unsigned s = 1;
    for (int t = 0; t < T; ++t) {
        int step_maxn = 0;
        double step_union = 0, step_seg = 0, step_pair = 0;
        for (int w = 0; w < nwave; ++w) {
            int wmax = 0, segmax[ORC_MAXB] = {0};
            static int pair_any[ORC_MAXP];
            memset(pair_any, 0, sizeof(pair_any));
            for (int l = 0; l < WAVE; ++l) {
                const int b = w * WAVE + l;
                int32_t a[2 * ORC_MAXN];
                for (int k = 0; k < 2 * N; ++k) { s = s * 1103515245u + 12345u; a[k] = (s >> 16) % 5; }
                int d = orc_v1_step(&e[b], a, obs, &r);
                if (d) orc_v1_reset(&e[b], obs);
                int n = 0, cseg[ORC_MAXB] = {0};
                for (int p = 0; p < e[b].P; ++p) {
                    if (!e[b].arb_inlist[p]) continue;
                    ++n;
                    if (p < Nb * ORC_NSEG) ++cseg[p / ORC_NSEG];
                    else pair_any[p] = 1;
                }
                hist[n]++;
                if (n > wmax) wmax = n;
                for (int k = 0; k < Nb; ++k) if (cseg[k] > segmax[k]) segmax[k] = cseg[k];
            }
            int su = 0, pu = 0;
            for (int k = 0; k < Nb; ++k) su += segmax[k];
            for (int p = Nb * ORC_NSEG; p < ORC_MAXP; ++p) pu += pair_any[p];
            whist[wmax]++;
            shist[su]++;
            phist[pu]++;
            sum_maxn += wmax;
            sum_seg += su;
            sum_pair += pu;
            if (wmax > step_maxn) step_maxn = wmax;
            /* static-slot cost in units of a per-lane-list record: a segment slot ~1/2, a pair slot ~1/2
               of the LDS-row record (registers, static bodies) -- printed separately below */
            if (0.5 * su + 0.5 * pu > step_union) { step_union = 0.5 * su + 0.5 * pu; step_seg = su; step_pair = pu; }
        }
        sum_step_maxn += step_maxn;
        sum_step_seg += step_seg;
        sum_step_pair += step_pair;
    }
    printf("per env-step contacts:\n");
    for (int i = 0; i < NH; ++i) if (hist[i]) printf("  %2d %ld\n", i, hist[i]);
    printf("per wave-step max over lanes (per-lane list slots):\n");
    for (int i = 0; i < NH; ++i) if (whist[i]) printf("  %2d %ld\n", i, whist[i]);
    printf("per wave-step static segment slots (sum over bodies of max over lanes):\n");
    for (int i = 0; i < NH; ++i) if (shist[i]) printf("  %2d %ld\n", i, shist[i]);
    printf("per wave-step static pair slots (pairs in contact in any lane):\n");
    for (int i = 0; i < NH; ++i) if (phist[i]) printf("  %2d %ld\n", i, phist[i]);
    const double nws = (double)nwave * T;
    printf("mean per wave-step: list slots %.3f, static segment slots %.3f, static pair slots %.3f\n",
           sum_maxn / nws, sum_seg / nws, sum_pair / nws);
    printf("mean per step of the slowest wave: list slots %.3f; static (seg, pair) of the costliest wave %.3f, %.3f\n",
           sum_step_maxn / T, sum_step_seg / T, sum_step_pair / T);
    free(e);
    return 0;
}
