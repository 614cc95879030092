// pmc_calib.hip -- calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 for the access
// patterns the env-step kernels use (MI355X_MICROARCH.md: only 16 B/lane streams are
// calibrated).  Each kernel moves a known byte count over 512 MiB (past the 256 MiB
// Infinity Cache); scripts/pmc_traffic.py divides the counters by these counts.
//   rd_f64   8 B/lane coalesced loads        (SoA fp64 state read)
//   wr_f64   8 B/lane coalesced stores       (SoA fp64 state write)
//   wr_aos20 f32 obs rows, lane = row, 20 floats per row (AoS obs write, 2v2)
//   wr_u8    1 B/lane                        (done flags)
//   rd_f64x2 16 B/lane coalesced loads       (the (x, y)-pair body state read, round 3)
//   wr_f64x2 16 B/lane coalesced stores      (the (x, y)-pair body state write)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

__global__ void rd_f64(const double* __restrict__ a, double* __restrict__ out, size_t n)
{
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
    if (s == 12345.678) out[0] = s;  // never true for zero input: keeps the loads, writes nothing
}
__global__ void wr_f64(double* __restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (double)i;
}
__global__ void wr_aos20(float* __restrict__ a, size_t rows)
{
    for (size_t r = blockIdx.x * (size_t)blockDim.x + threadIdx.x; r < rows; r += (size_t)gridDim.x * blockDim.x)
#pragma unroll
        for (int k = 0; k < 20; ++k) a[r * 20 + k] = (float)k;
}
__global__ void wr_u8(unsigned char* __restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = (unsigned char)i;
}

__global__ void rd_f64x2(const double2* __restrict__ a, double* __restrict__ out, size_t n)
{
    double s = 0.0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const double2 v = a[i];
        s += v.x + v.y;
    }
    if (s == 12345.678) out[0] = s;
}
__global__ void wr_f64x2(double2* __restrict__ a, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        a[i] = make_double2((double)i, 1.0);
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

int main()
{
    const size_t bytes = (size_t)512 << 20;
    void* buf;
    double* out;
    CK(hipMalloc(&buf, bytes));
    CK(hipMalloc(&out, 64));
    CK(hipMemset(buf, 0, bytes));
    const dim3 grid(4096), block(256);
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(rd_f64, grid, block, 0, 0, (const double*)buf, out, bytes / 8);
        hipLaunchKernelGGL(wr_f64, grid, block, 0, 0, (double*)buf, bytes / 8);
        hipLaunchKernelGGL(wr_aos20, grid, block, 0, 0, (float*)buf, bytes / 80);
        hipLaunchKernelGGL(wr_u8, grid, block, 0, 0, (unsigned char*)buf, bytes);
        hipLaunchKernelGGL(rd_f64x2, grid, block, 0, 0, (const double2*)buf, out, bytes / 16);
        hipLaunchKernelGGL(wr_f64x2, grid, block, 0, 0, (double2*)buf, bytes / 16);
    }
    CK(hipDeviceSynchronize());
    printf("{\"rd_f64\": %zu, \"wr_f64\": %zu, \"wr_aos20\": %zu, \"wr_u8\": %zu, \"rd_f64x2\": %zu, \"wr_f64x2\": %zu}\n",
           bytes, bytes, (bytes / 80) * 80, bytes, bytes, bytes);
    CK(hipFree(buf));
    CK(hipFree(out));
    return 0;
}
