// ubench_select.hip -- cost of the compare -> select idioms of the env step kernels at one wave
// per SIMD (the step kernels' occupancy), each as 8 independent compare/select pairs per iteration:
//
//   cmpsel_vcc  v_cmp_le_f64 vcc + v_cndmask_b32 (int constant), the pairs serialised through VCC
//               (what LLVM emits for `x <= c ? K : 0u` bound masks)
//   cmpsel_sg   the same compares into 8 SGPR pairs first, then the 8 cndmasks
//   subsign_c   exact sign test without VCC: t = c - x (v_add_f64), m = t.hi >> 31 (arithmetic),
//               r = K & ~m  (x <= c  <=>  c - x >= +0 for finite x, c with c != -0)
//   icmpsel     v_cmp_eq_u32 vcc + v_cndmask_b32 (integer compare -> select)
//   cmpsel64    compiler fp64 select after an fp64 compare on the selected value's own chain
//
//   hipcc --offload-arch=gfx950 -O3 -o ubench_select scripts/ubench_select.hip && ./ubench_select
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

constexpr int ITERS = 2048;

#define V8 "+v"(r0), "+v"(r1), "+v"(r2), "+v"(r3), "+v"(r4), "+v"(r5), "+v"(r6), "+v"(r7)

__global__ void __launch_bounds__(64) k_cmpsel_vcc(double* out, unsigned long long* cyc, double s)
{
    const double x = threadIdx.x * 0.25;
    unsigned r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
    const unsigned K = 0x183u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_cmp_le_f64 vcc, %8, %9\n v_cndmask_b32 %0, 0, %10, vcc\n"
            "v_cmp_le_f64 vcc, %8, %9\n v_cndmask_b32 %1, 0, %10, vcc\n"
            "v_cmp_le_f64 vcc, %8, %9\n v_cndmask_b32 %2, 0, %10, vcc\n"
            "v_cmp_le_f64 vcc, %8, %9\n v_cndmask_b32 %3, 0, %10, vcc\n"
            "v_cmp_le_f64 vcc, %8, %9\n v_cndmask_b32 %4, 0, %10, vcc\n"
            "v_cmp_le_f64 vcc, %8, %9\n v_cndmask_b32 %5, 0, %10, vcc\n"
            "v_cmp_le_f64 vcc, %8, %9\n v_cndmask_b32 %6, 0, %10, vcc\n"
            "v_cmp_le_f64 vcc, %8, %9\n v_cndmask_b32 %7, 0, %10, vcc\n"
            : V8
            : "v"(x), "s"(s), "v"(K)
            : "vcc");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = (double)(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7);
}

__global__ void __launch_bounds__(64) k_cmpsel_sg(double* out, unsigned long long* cyc, double s)
{
    const double x = threadIdx.x * 0.25;
    unsigned r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
    const unsigned K = 0x183u;
    unsigned long long m0, m1, m2, m3, m4, m5, m6, m7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_cmp_le_f64 %8, %16, %17\n v_cmp_le_f64 %9, %16, %17\n v_cmp_le_f64 %10, %16, %17\n"
            "v_cmp_le_f64 %11, %16, %17\n v_cmp_le_f64 %12, %16, %17\n v_cmp_le_f64 %13, %16, %17\n"
            "v_cmp_le_f64 %14, %16, %17\n v_cmp_le_f64 %15, %16, %17\n"
            "v_cndmask_b32 %0, 0, %18, %8\n v_cndmask_b32 %1, 0, %18, %9\n v_cndmask_b32 %2, 0, %18, %10\n"
            "v_cndmask_b32 %3, 0, %18, %11\n v_cndmask_b32 %4, 0, %18, %12\n v_cndmask_b32 %5, 0, %18, %13\n"
            "v_cndmask_b32 %6, 0, %18, %14\n v_cndmask_b32 %7, 0, %18, %15\n"
            : V8, "=&s"(m0), "=&s"(m1), "=&s"(m2), "=&s"(m3), "=&s"(m4), "=&s"(m5), "=&s"(m6), "=&s"(m7)
            : "v"(x), "s"(s), "v"(K));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = (double)(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7);
}

// the subsign idiom written in C (what the kernels would use): the compiler's own code
__global__ void __launch_bounds__(64) k_subsign_c(double* out, unsigned long long* cyc, double s)
{
    double x = threadIdx.x * 0.25;
    unsigned acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        unsigned r = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            const double t = (s + q) - x;
            int m = (int)(__double_as_longlong(t) >> 32) >> 31;
            asm volatile("" : "+v"(m));  // keep the sign mask a VGPR value (LLVM folds it to cmp+cndmask)
            r |= (0x183u << q) & ~(unsigned)m;
        }
        acc ^= r;
        asm volatile("" : "+v"(x), "+v"(acc));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = (double)acc;
}

// the compare idiom written in C, same work as k_subsign_c
__global__ void __launch_bounds__(64) k_cmpsel_c(double* out, unsigned long long* cyc, double s)
{
    double x = threadIdx.x * 0.25;
    unsigned acc = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        unsigned r = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) r |= x <= s + q ? 0x183u << q : 0u;
        acc ^= r;
        asm volatile("" : "+v"(x), "+v"(acc));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = (double)acc;
}

__global__ void __launch_bounds__(64) k_icmpsel(double* out, unsigned long long* cyc, double s)
{
    const unsigned x = threadIdx.x & 7u;
    unsigned r0 = 0, r1 = 0, r2 = 0, r3 = 0, r4 = 0, r5 = 0, r6 = 0, r7 = 0;
    const unsigned K = 0x183u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_cmp_eq_u32 vcc, 3, %8\n v_cndmask_b32 %0, 0, %9, vcc\n"
            "v_cmp_eq_u32 vcc, 3, %8\n v_cndmask_b32 %1, 0, %9, vcc\n"
            "v_cmp_eq_u32 vcc, 3, %8\n v_cndmask_b32 %2, 0, %9, vcc\n"
            "v_cmp_eq_u32 vcc, 3, %8\n v_cndmask_b32 %3, 0, %9, vcc\n"
            "v_cmp_eq_u32 vcc, 3, %8\n v_cndmask_b32 %4, 0, %9, vcc\n"
            "v_cmp_eq_u32 vcc, 3, %8\n v_cndmask_b32 %5, 0, %9, vcc\n"
            "v_cmp_eq_u32 vcc, 3, %8\n v_cndmask_b32 %6, 0, %9, vcc\n"
            "v_cmp_eq_u32 vcc, 3, %8\n v_cndmask_b32 %7, 0, %9, vcc\n"
            : V8
            : "v"(x), "v"(K)
            : "vcc");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = (double)(r0 ^ r1 ^ r2 ^ r3 ^ r4 ^ r5 ^ r6 ^ r7);
}

typedef void (*Kern)(double*, unsigned long long*, double);

static void run(const char* name, Kern k, int pairs_per_iter)
{
    const int blocks = 1024;
    double* out;
    unsigned long long* cyc;
    CHECK(hipMalloc(&out, (size_t)blocks * 64 * sizeof(double)));
    CHECK(hipMalloc(&cyc, sizeof(unsigned long long)));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, out, cyc, 3.0);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemset(cyc, 0, sizeof(unsigned long long)));
    const int reps = 5;
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, out, cyc, 3.0);
    CHECK(hipDeviceSynchronize());
    unsigned long long c = 0;
    CHECK(hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost));
    printf("%-12s cycles per compare/select pair per wave: %6.2f\n", name,
           (double)c / ((double)reps * blocks) / ((double)pairs_per_iter * ITERS));
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
}

int main()
{
    run("cmpsel_vcc", k_cmpsel_vcc, 8);
    run("cmpsel_sg", k_cmpsel_sg, 8);
    run("icmpsel", k_icmpsel, 8);
    run("subsign_c", k_subsign_c, 8);
    run("cmpsel_c", k_cmpsel_c, 8);
    return 0;
}
