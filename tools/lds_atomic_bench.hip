// Microbenchmark: LDS atomic add throughput on gfx950 by type and conflict
// pattern (used to choose the descriptor histogram design).
// hipcc --offload-arch=gfx950 -O3 tools/lds_atomic_bench.hip -o /tmp/ldsab
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE, int SPREAD>
__global__ __launch_bounds__(256) void k(float* out, int iters) {
    __shared__ float hf[1024];
    __shared__ unsigned hu[1024];
    __shared__ unsigned long long h64[1024];
    for (int i = threadIdx.x; i < 1024; i += 256) {
        hf[i] = 0;
        hu[i] = 0;
        h64[i] = 0;
    }
    __syncthreads();
    unsigned x = threadIdx.x * 2654435761u + blockIdx.x;
    for (int it = 0; it < iters; it++) {
#pragma unroll
        for (int q = 0; q < 8; q++) {
            x = x * 1664525u + 1013904223u;
            // SPREAD: 0 = every lane distinct address, 1 = 8 lanes share, 2 = random over 360 bins
            const int a = SPREAD == 0 ? ((threadIdx.x * 4 + q) & 1023) : SPREAD == 1 ? ((threadIdx.x >> 3) * 8 + q) & 1023 : (x >> 8) % 360;
            if (MODE == 0) atomicAdd(&hf[a], 1.0f);
            if (MODE == 1) atomicAdd(&hu[a], 3u);
            if (MODE == 2) atomicAdd(&h64[a], 3ull);
            if (MODE == 3) hf[a] += 1.0f;  // plain RMW (racy; throughput reference)
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) out[blockIdx.x] = hf[5] + (float)hu[7] + (float)h64[9];
}

template <int MODE, int SPREAD>
void run(const char* name, float* d) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    const int iters = 256, blocks = 2048;
    hipLaunchKernelGGL((k<MODE, SPREAD>), dim3(blocks), dim3(256), 0, 0, d, 4);
    hipEventRecord(a);
    hipLaunchKernelGGL((k<MODE, SPREAD>), dim3(blocks), dim3(256), 0, 0, d, iters);
    hipEventRecord(b);
    hipEventSynchronize(b);
    float ms;
    hipEventElapsedTime(&ms, a, b);
    const double waveinstr = (double)blocks * 4 * iters * 8;
    printf("%-28s %8.3f ms  %6.2f ns per wave-instr per CU  (%.1f cyc @2.4GHz)\n", name, ms,
           ms * 1e6 / (waveinstr / 256), ms * 1e6 / (waveinstr / 256) * 2.4);
}

int main() {
    float* d;
    hipMalloc(&d, 4096 * sizeof(float));
    run<0, 0>("f32 distinct", d);
    run<1, 0>("u32 distinct", d);
    run<2, 0>("u64 distinct", d);
    run<3, 0>("f32 plain RMW distinct", d);
    run<0, 1>("f32 8-way shared", d);
    run<1, 1>("u32 8-way shared", d);
    run<2, 1>("u64 8-way shared", d);
    run<0, 2>("f32 random/360", d);
    run<1, 2>("u32 random/360", d);
    run<2, 2>("u64 random/360", d);
    return 0;
}
