// Calibration of rocprofv3 FETCH_SIZE / WRITE_SIZE for the access widths the
// SIFT kernels use (MI355X_MICROARCH.md: only 16-B/lane streaming is
// calibrated).  Copies a 512 MiB buffer (past the 256 MiB Infinity Cache)
// with 4-B and 16-B per-lane loads/stores; known bytes = 512 MiB each way.
// hipcc --offload-arch=gfx950 -O3 tools/hbm_calib.hip -o tools/hbm_calib
#include <hip/hip_runtime.h>

#include <cstdio>

__global__ void copy4(const float* __restrict__ a, float* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}
__global__ void copy16(const float4* __restrict__ a, float4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) b[i] = a[i];
}

int main() {
    const size_t bytes = 512ull << 20, n = bytes / 4;
    float *a, *b;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&b, bytes) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 0, bytes);
    for (int r = 0; r < 3; r++) {
        hipLaunchKernelGGL(copy4, dim3(8192), dim3(256), 0, 0, a, b, n);
        hipLaunchKernelGGL(copy16, dim3(8192), dim3(256), 0, 0, (const float4*)a, (float4*)b, n / 4);
    }
    (void)hipDeviceSynchronize();
    printf("copied %zu bytes per kernel per launch\n", bytes);
    (void)hipFree(a);
    (void)hipFree(b);
    return 0;
}
