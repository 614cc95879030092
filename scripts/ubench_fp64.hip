// ubench_fp64.hip -- issue cost / latency of the instruction classes the env step kernel is
// made of (fp64 add/mul, v_cndmask, LDS b128 round trips), at 1, 2 and 4 waves per SIMD.
//
//   hipcc --offload-arch=gfx950 -O3 -o ubench_fp64 scripts/ubench_fp64.hip && ./ubench_fp64
//
// Each test is one kernel of 64-thread blocks; grid = waves_per_simd * 1024 blocks, so every
// SIMD of the 256 CUs holds that many waves.  Reported: in-kernel cycles (s_memtime) per
// instruction per wave, averaged over waves, and wall time per instruction.
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

// 8 independent fp64 add chains (throughput), 8 instructions per iteration
__global__ void __launch_bounds__(64) k_f64_indep(double* out, unsigned long long* cyc, double s)
{
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_add_f64 %0, %0, %8\n v_add_f64 %1, %1, %8\n v_add_f64 %2, %2, %8\n v_add_f64 %3, %3, %8\n"
            "v_add_f64 %4, %4, %8\n v_add_f64 %5, %5, %8\n v_add_f64 %6, %6, %8\n v_add_f64 %7, %7, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(s));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// 8 independent fp64 mul chains
__global__ void __launch_bounds__(64) k_f64_mul(double* out, unsigned long long* cyc, double s)
{
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
           a7 = a0 + 7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_mul_f64 %0, %0, %8\n v_mul_f64 %1, %1, %8\n v_mul_f64 %2, %2, %8\n v_mul_f64 %3, %3, %8\n"
            "v_mul_f64 %4, %4, %8\n v_mul_f64 %5, %5, %8\n v_mul_f64 %6, %6, %8\n v_mul_f64 %7, %7, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(s));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// one dependent fp64 add chain (latency), 8 per iteration
__global__ void __launch_bounds__(64) k_f64_dep(double* out, unsigned long long* cyc, double s)
{
    double a0 = threadIdx.x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n"
            "v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n v_add_f64 %0, %0, %1\n"
            : "+v"(a0)
            : "v"(s));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = a0;
}

// 8 independent fp32 adds (reference row of the guide: 4 cyc one wave alone)
__global__ void __launch_bounds__(64) k_f32_indep(double* out, unsigned long long* cyc, double s_)
{
    float s = (float)s_;
    float a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
          a7 = a0 + 7;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n"
            "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(s));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// 8 independent 32-bit v_cndmask (a select on a double = 2 of them)
__global__ void __launch_bounds__(64) k_cnd(double* out, unsigned long long* cyc, double s_)
{
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, b = (unsigned)s_;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_cmp_gt_u32 vcc, %0, %8\n"
            "v_cndmask_b32 %0, %0, %8, vcc\n v_cndmask_b32 %1, %1, %8, vcc\n v_cndmask_b32 %2, %2, %8, vcc\n"
            "v_cndmask_b32 %3, %3, %8, vcc\n v_cndmask_b32 %4, %4, %8, vcc\n v_cndmask_b32 %5, %5, %8, vcc\n"
            "v_cndmask_b32 %6, %6, %8, vcc\n v_cndmask_b32 %7, %7, %8, vcc\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(b)
            : "vcc");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// LDS round trip: ds_write_b128 of a row, then ds_read_b128 of it and one fp64 add on the value
// (the solver's read -> compute -> write pattern on one body row), 1 round trip per iteration
__global__ void __launch_bounds__(64) k_lds_rt(double* out, unsigned long long* cyc, double s)
{
    __shared__ double2 row[4][64];
    double2 v = make_double2(threadIdx.x, 1.0);
    row[0][threadIdx.x] = v;
    __syncthreads();
    volatile double* rp = &row[0][threadIdx.x].x;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS / 8; ++i) {
        const double x = rp[0], y = rp[1];
        rp[0] = x + s;
        rp[1] = y;
    }
    v = make_double2(rp[0], rp[1]);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = v.x + v.y;
}


// 8 independent v_cndmask_b32 on a lane mask held in an SGPR pair computed once (no VCC hazard)
__global__ void __launch_bounds__(64) k_cnd_sgpr(double* out, unsigned long long* cyc, double s_)
{
    unsigned a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
             a7 = a0 + 7, b = (unsigned)s_;
    unsigned long long m;
    asm volatile("v_cmp_gt_u32 %0, %1, 31" : "=s"(m) : "v"(a0));
    asm volatile("s_nop 4");
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_cndmask_b32 %0, %0, %8, %9\n v_cndmask_b32 %1, %1, %8, %9\n v_cndmask_b32 %2, %2, %8, %9\n"
            "v_cndmask_b32 %3, %3, %8, %9\n v_cndmask_b32 %4, %4, %8, %9\n v_cndmask_b32 %5, %5, %8, %9\n"
            "v_cndmask_b32 %6, %6, %8, %9\n v_cndmask_b32 %7, %7, %8, %9\n"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(b), "s"(m));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
}

// 8 independent v_cmp_lt_f64 into SGPR pairs
__global__ void __launch_bounds__(64) k_cmp64(double* out, unsigned long long* cyc, double s)
{
    double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    unsigned long long m0 = 0, m1 = 0, m2 = 0, m3 = 0, m4 = 0, m5 = 0, m6 = 0, m7 = 0;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        asm volatile(
            "v_cmp_lt_f64 %0, %8, %12\n v_cmp_lt_f64 %1, %9, %12\n v_cmp_lt_f64 %2, %10, %12\n v_cmp_lt_f64 %3, %11, %12\n"
            "v_cmp_gt_f64 %4, %8, %12\n v_cmp_gt_f64 %5, %9, %12\n v_cmp_gt_f64 %6, %10, %12\n v_cmp_gt_f64 %7, %11, %12\n"
            : "=s"(m0), "=s"(m1), "=s"(m2), "=s"(m3), "=s"(m4), "=s"(m5), "=s"(m6), "=s"(m7)
            : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(s));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = (double)(m0 ^ m1 ^ m2 ^ m3 ^ m4 ^ m5 ^ m6 ^ m7);
}

// compiler-generated fp64 selects: x = (x > s) ? x : y on 4 independent doubles
__global__ void __launch_bounds__(64) k_sel64(double* out, unsigned long long* cyc, double s)
{
    double a0 = threadIdx.x * 0.01, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
    const double y = s * 0.5;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        a0 = a0 > s ? a0 : y;
        a1 = a1 > s ? a1 : y;
        a2 = a2 > s ? a2 : y;
        a3 = a3 > s ? a3 : y;
        asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = a0 + a1 + a2 + a3;
}

// ds_read_b128 latency: dependent chain of reads (the address comes from the previous read)
__global__ void __launch_bounds__(64) k_lds_lat(double* out, unsigned long long* cyc, double s)
{
    __shared__ uint4 tab[64];
    tab[threadIdx.x] = make_uint4((threadIdx.x * 16u), 0u, 0u, 0u);  // self-loop: addr -> same addr
    __syncthreads();
    unsigned a = threadIdx.x * 16u;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS / 8; ++i) {
        uint4 v;
        asm volatile("ds_read_b128 %0, %1\n s_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(a) : "memory");
        a = v.x;
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = a;
}

// divergent-branch overhead: s_and_saveexec / s_cbranch_execz / s_or exec around 1 fp64 add, half the lanes
__global__ void __launch_bounds__(64) k_branch(double* out, unsigned long long* cyc, double s)
{
    double a0 = threadIdx.x;
    const bool odd = threadIdx.x & 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < ITERS; ++i) {
        if (odd) asm volatile("v_add_f64 %0, %0, %1" : "+v"(a0) : "v"(s));
        asm volatile("" ::: "memory");
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (threadIdx.x == 0) atomicAdd(cyc, t1 - t0);
    out[blockIdx.x * 64 + threadIdx.x] = a0;
}

typedef void (*Kern)(double*, unsigned long long*, double);

static void run(const char* name, Kern k, int insts_per_iter, int iters, int wps)
{
    const int blocks = 1024 * wps;
    double* out;
    unsigned long long* cyc;
    CHECK(hipMalloc(&out, (size_t)blocks * 64 * sizeof(double)));
    CHECK(hipMalloc(&cyc, sizeof(unsigned long long)));
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.0000001);  // warm
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemset(cyc, 0, sizeof(unsigned long long)));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const int reps = 5;
    CHECK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.0000001);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipDeviceSynchronize());
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long c = 0;
    CHECK(hipMemcpy(&c, cyc, sizeof(c), hipMemcpyDeviceToHost));
    const double n_inst = (double)insts_per_iter * iters;
    const double cyc_per_wave_inst = (double)c / ((double)reps * blocks) / n_inst;
    const double ns_per_inst = ms * 1e6 / reps / n_inst;  // wall per instruction (all waves)
    printf("%-10s waves/SIMD=%d  cycles/inst/wave=%7.2f  wall ns/inst=%7.3f  (SIMD-cycles/inst at 2.4GHz: %5.2f)\n",
           name, wps, cyc_per_wave_inst, ns_per_inst, ns_per_inst * 2.4 / wps);
    CHECK(hipFree(out));
    CHECK(hipFree(cyc));
}

int main()
{
    for (int w : {1, 2, 4}) {
        run("f64_add", k_f64_indep, 8, ITERS, w);
        run("f64_mul", k_f64_mul, 8, ITERS, w);
        run("f64_dep", k_f64_dep, 8, ITERS, w);
        run("f32_add", k_f32_indep, 8, ITERS, w);
        run("cndmask", k_cnd, 9, ITERS, w);
        run("lds_rt", k_lds_rt, 1, ITERS / 8, w);
        run("cnd_sgpr", k_cnd_sgpr, 8, ITERS, w);
        run("cmp_f64", k_cmp64, 8, ITERS, w);
        run("sel_f64", k_sel64, 4, ITERS, w);
        run("lds_lat", k_lds_lat, 1, ITERS / 8, w);
        run("branch", k_branch, 1, ITERS, w);
    }
    return 0;
}
