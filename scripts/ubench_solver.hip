// ubench_solver.hip -- cycles per half-application of the split sequential-impulse solve
// (futbol_v1_impl.hpp apply_half), in isolation: one wave per SIMD, each lane one item with M
// records over Nb = 5 body rows + the static row, 10 sweeps.  Variants:
//   0: the kernel's loop (rows read after the previous record's writes)
//   1: + the v-half rows on a column swizzled by 8 (the two halves of an env on different banks)
//   2: (no swizzle) next record's rows prefetched before this record's writes, forwarded by loop-invariant
//      alias masks
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o ubench_solver scripts/ubench_solver.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CHECK(x)                                                                                      \
    do {                                                                                              \
        hipError_t e_ = (x);                                                                          \
        if (e_ != hipSuccess) {                                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));                 \
            exit(1);                                                                                  \
        }                                                                                             \
    } while (0)

constexpr int NB = 5, NROW = 2 * NB + 1, EPW = 64;
constexpr unsigned ROW = EPW * 16;

template <int I, int E>
struct SF {
    template <class F>
    __device__ __forceinline__ static void run(F&& f)
    {
        if constexpr (I < E) {
            f(std::integral_constant<int, I>{});
            SF<I + 1, E>::run(f);
        }
    }
};

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

template <int M, int VAR>
__global__ void __launch_bounds__(64) k_solve(const int* __restrict__ pairs, double* out, unsigned long long* cyc)
{
    __shared__ double2 rows[NROW][EPW];
    const int ln = threadIdx.x;
    for (int k = 0; k < NROW; ++k) rows[k][ln] = make_double2(k == NB ? 0.0 : 0.1 * k + ln, k == NB ? 0.0 : -0.3 * k);
    __syncthreads();
    // item: env column = partner pairs (lane 2i, 2i+1 = the two halves of env i)
    const int e = ln >> 1, h = ln & 1;
    const int col = (VAR == 1 && h) ? (e ^ 8) : e;
    char* base = (char*)&rows[h ? 2 * NB : 0][col];
    const int sgn = h ? -1 : 1;
    double2* ra[M];
    double2* rb[M];
    double nx[M], ny[M], nm[M], c[M], acc[M], ma[M], mb[M];
    SF<0, M>::run([&](auto Q) {
        constexpr int q = Q;
        const int p = pairs[(blockIdx.x * 32 + e) * M + q];
        const int a = p & 15, b = p >> 4;  // b = NB: static
        ra[q] = (double2*)(base + sgn * (int)(a * ROW));
        rb[q] = (double2*)(base + sgn * (int)(b * ROW));
        nx[q] = 0.6;
        ny[q] = 0.8;
        nm[q] = 10.0;
        c[q] = h ? -0.01 : 0.02;
        acc[q] = 0.0;
        ma[q] = a == 4 ? 0.1 : 0.05;
        mb[q] = b == NB ? 0.0 : (b == 4 ? 0.1 : 0.05);
    });
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    if constexpr (VAR < 2) {
        for (int it = 0; it < 10; ++it)
            SF<0, M>::run([&](auto Q) {
                constexpr int q = Q;
                apply_half(ra[q], rb[q], nx[q], ny[q], nm[q], c[q], ma[q], mb[q], acc[q]);
            });
    } else if constexpr (VAR == 3 || VAR == 4) {
        // forwarding by loop-invariant 32-bit lane masks and v_bfi_b32 (no SGPR masks)
        uint32_t mab[M], maa[M], mbb[M], mba[M];
        SF<0, M>::run([&](auto Q) {
            constexpr int q = Q;
            constexpr int nq = q + 1 < M ? q + 1 : 0;
            mab[q] = ra[nq] == rb[q] ? ~0u : 0u;
            maa[q] = ra[nq] == ra[q] ? ~0u : 0u;
            mbb[q] = rb[nq] == rb[q] ? ~0u : 0u;
            mba[q] = rb[nq] == ra[q] ? ~0u : 0u;
        });
        auto bsel = [](uint32_t m, double x, double y) {  // m ? x : y, bitwise
            const unsigned long long xi = __double_as_longlong(x), yi = __double_as_longlong(y);
            const uint32_t lo = ((uint32_t)xi & m) | ((uint32_t)yi & ~m);
            const uint32_t hi = ((uint32_t)(xi >> 32) & m) | ((uint32_t)(yi >> 32) & ~m);
            return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
        };
        double2 ca = *ra[0], cb = *rb[0];
        for (int it = 0; it < 10; ++it)
            SF<0, M>::run([&](auto Q) {
                constexpr int q = Q;
                constexpr int nq = q + 1 < M ? q + 1 : 0;
                const double2 la = *ra[nq], lb = *rb[nq];
                if constexpr (VAR == 4) __builtin_amdgcn_sched_barrier(0);  // issue the prefetch first
                const double vn = (cb.x - ca.x) * nx[q] + (cb.y - ca.y) * ny[q];
                const double j = (c[q] - vn) * nm[q];
                const double old = acc[q];
                const double t = old + j;
                const double nacc = t > 0.0 ? t : 0.0;
                acc[q] = nacc;
                const double d = nacc - old;
                const double jx = nx[q] * d, jy = ny[q] * d;
                const double2 na = make_double2(ca.x + (-jx) * ma[q], ca.y + (-jy) * ma[q]);
                const double2 nb = make_double2(cb.x + jx * mb[q], cb.y + jy * mb[q]);
                *ra[q] = na;
                *rb[q] = nb;
                ca = make_double2(bsel(mab[q], nb.x, bsel(maa[q], na.x, la.x)), bsel(mab[q], nb.y, bsel(maa[q], na.y, la.y)));
                cb = make_double2(bsel(mbb[q], nb.x, bsel(mba[q], na.x, lb.x)), bsel(mbb[q], nb.y, bsel(mba[q], na.y, lb.y)));
            });
    } else {
        bool fab[M], faa[M], fbb[M], fba[M];
        SF<0, M>::run([&](auto Q) {
            constexpr int q = Q;
            constexpr int nq = q + 1 < M ? q + 1 : 0;
            fab[q] = ra[nq] == rb[q];
            faa[q] = ra[nq] == ra[q];
            fbb[q] = rb[nq] == rb[q];
            fba[q] = rb[nq] == ra[q];
        });
        double2 ca = *ra[0], cb = *rb[0];
        for (int it = 0; it < 10; ++it)
            SF<0, M>::run([&](auto Q) {
                constexpr int q = Q;
                constexpr int nq = q + 1 < M ? q + 1 : 0;
                const double2 la = *ra[nq], lb = *rb[nq];
                const double vn = (cb.x - ca.x) * nx[q] + (cb.y - ca.y) * ny[q];
                const double j = (c[q] - vn) * nm[q];
                const double old = acc[q];
                const double t = old + j;
                const double nacc = t > 0.0 ? t : 0.0;
                acc[q] = nacc;
                const double d = nacc - old;
                const double jx = nx[q] * d, jy = ny[q] * d;
                const double2 na = make_double2(ca.x + (-jx) * ma[q], ca.y + (-jy) * ma[q]);
                const double2 nb = make_double2(cb.x + jx * mb[q], cb.y + jy * mb[q]);
                *ra[q] = na;
                *rb[q] = nb;
                ca = fab[q] ? nb : (faa[q] ? na : la);
                cb = fbb[q] ? nb : (fba[q] ? na : lb);
            });
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    double s = 0;
    for (int q = 0; q < M; ++q) s += acc[q];
    for (int k = 0; k < NROW; ++k) s += rows[k][ln].x + rows[k][ln].y;
    out[blockIdx.x * 64 + ln] = s;
}

template <int M, int VAR>
static void run(const int* d_pairs, double* out, unsigned long long* cyc, const char* name)
{
    CHECK(hipMemset(cyc, 0, 8));
    hipLaunchKernelGGL((k_solve<M, VAR>), dim3(1024), dim3(64), 0, 0, d_pairs, out, cyc);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemset(cyc, 0, 8));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL((k_solve<M, VAR>), dim3(1024), dim3(64), 0, 0, d_pairs, out, cyc);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipDeviceSynchronize());
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long c;
    CHECK(hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost));
    printf("%-28s M=%d  cycles/half-application %.1f   kernel %.2f us\n", name, M, (double)c / 1024 / (10.0 * M),
           ms * 1e3);
}

template <int V>
static void compare(const int* d, double* o1, double* o2, unsigned long long* cyc)
{
    hipLaunchKernelGGL((k_solve<4, 0>), dim3(1024), dim3(64), 0, 0, d, o1, cyc);
    hipLaunchKernelGGL((k_solve<4, V>), dim3(1024), dim3(64), 0, 0, d, o2, cyc);
    CHECK(hipDeviceSynchronize());
    static double h1[1024 * 64], h2[1024 * 64];
    CHECK(hipMemcpy(h1, o1, sizeof(h1), hipMemcpyDeviceToHost));
    CHECK(hipMemcpy(h2, o2, sizeof(h2), hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 1024 * 64; ++i) bad += h1[i] != h2[i];
    printf("variant 0 vs %d (M=4) differing lanes: %d\n", V, bad);
}

int main()
{
    // random records: a in 0..4, b in {0..4} \ {a} or static (NB), as in a crowded env
    const int n = 1024 * 32 * 8;
    int* h = (int*)malloc(n * sizeof(int));
    unsigned s = 12345;
    for (int i = 0; i < n; ++i) {
        s = s * 1103515245u + 12345u;
        const int a = (s >> 16) % 5;
        s = s * 1103515245u + 12345u;
        int b = (s >> 16) % 6;
        if (b == a) b = NB;
        if (b == 5) b = NB;
        h[i] = a | (b << 4);
    }
    int* d;
    double* out;
    unsigned long long* cyc;
    CHECK(hipMalloc(&d, n * sizeof(int)));
    CHECK(hipMalloc(&out, 1024 * 64 * sizeof(double)));
    CHECK(hipMalloc(&cyc, 8));
    CHECK(hipMemcpy(d, h, n * sizeof(int), hipMemcpyHostToDevice));
    double* out2;
    CHECK(hipMalloc(&out2, 1024 * 64 * sizeof(double)));
    compare<2>(d, out, out2, cyc);
    compare<3>(d, out, out2, cyc);
    compare<4>(d, out, out2, cyc);
    run<4, 4>(d, out, cyc, "prefetch first, bfi");
    run<2, 4>(d, out, cyc, "prefetch first, bfi");
    run<1, 4>(d, out, cyc, "prefetch first, bfi");
    run<8, 4>(d, out, cyc, "prefetch first, bfi");
    run<4, 0>(d, out, cyc, "kernel loop");
    run<4, 2>(d, out, cyc, "prefetch/forward");
    run<4, 3>(d, out, cyc, "prefetch/forward bfi");
    run<2, 0>(d, out, cyc, "kernel loop");
    run<2, 3>(d, out, cyc, "prefetch/forward bfi");
    run<1, 0>(d, out, cyc, "kernel loop");
    run<1, 3>(d, out, cyc, "prefetch/forward bfi");
    run<8, 0>(d, out, cyc, "kernel loop");
    run<8, 2>(d, out, cyc, "prefetch/forward");
    run<8, 3>(d, out, cyc, "prefetch/forward bfi");
    return 0;
}
