// MFMA issue rates on gfx950: cycles per instruction on one SIMD (s_memtime
// around a loop of independent MFMAs, one wave per SIMD, and four waves per
// SIMD), for the instructions the matcher can use.
//   hipcc --offload-arch=gfx950 -O3 -o tools/mfma_rate tools/mfma_rate.hip && tools/mfma_rate
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef __bf16 b8 __attribute__((ext_vector_type(8)));

constexpr int kIters = 4096, kChains = 4;

// kind 0: i32_32x32x32_i8, 1: i32_16x16x64_i8, 2: f32_32x32x16_f16, 3: f32_32x32x16_bf16, 4: f32_16x16x32_f16
template <int KIND>
__global__ __launch_bounds__(256) void k_rate(int seed, unsigned long long* cyc, float* sink) {
    const int lane = threadIdx.x & 63;
    const i32x4 a = {seed + lane, seed * 3, lane, 7}, b = {lane * 5, seed, 3, lane};
    h8 ha, hb;
    b8 ba, bb;
    for (int i = 0; i < 8; i++) {
        ha[i] = (_Float16)(lane + i);
        hb[i] = (_Float16)(seed - i);
        ba[i] = (__bf16)(float)(lane + i);
        bb[i] = (__bf16)(float)(seed - i);
    }
    i32x16 c16[kChains] = {};
    i32x4 c4[kChains] = {};
    f32x16 f16a[kChains] = {};
    f32x4 f4[kChains] = {};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
#pragma unroll
        for (int c = 0; c < kChains; c++) {
            if constexpr (KIND == 0) c16[c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, c16[c], 0, 0, 0);
            if constexpr (KIND == 1) c4[c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(a, b, c4[c], 0, 0, 0);
            if constexpr (KIND == 2) f16a[c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ha, hb, f16a[c], 0, 0, 0);
            if constexpr (KIND == 3) f16a[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ba, bb, f16a[c], 0, 0, 0);
            if constexpr (KIND == 4) f4[c] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ha, hb, f4[c], 0, 0, 0);
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float s = 0;
    for (int c = 0; c < kChains; c++) {
        s += (float)c16[c][lane & 15] + (float)c4[c][lane & 3] + f16a[c][lane & 15] + f4[c][lane & 3];
    }
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

template <int KIND>
static void run(const char* name, long ops, int wpb) {
    // 256 CUs x 4 SIMDs: 1024 workgroups of wpb waves -> wpb waves per SIMD
    const int nwg = 1024, nw = nwg * wpb;
    unsigned long long* cyc;
    float* sink;
    CK(hipMalloc(&cyc, sizeof(unsigned long long) * nw));
    CK(hipMalloc(&sink, sizeof(float) * nw * 64));
    hipLaunchKernelGGL(k_rate<KIND>, dim3(nwg), dim3(64 * wpb), 0, 0, 1, cyc, sink);
    CK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    CK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_rate<KIND>, dim3(nwg), dim3(64 * wpb), 0, 0, 2, cyc, sink);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    unsigned long long* h = new unsigned long long[nw];
    CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
    double avg = 0;
    for (int i = 0; i < nw; i++) avg += (double)h[i];
    avg /= nw;
    const double n_mfma = (double)kIters * kChains;
    const double chip = (double)nw * n_mfma * ops / (ms * 1e-3) / 1e12;
    std::printf("{\"instr\": \"%s\", \"waves_per_simd\": %d, \"wave_cycles_per_mfma\": %.2f, \"simd_cycles_per_mfma\": %.2f, "
                "\"ops_per_mfma\": %ld, \"chip_tops\": %.1f, \"ms\": %.3f}\n",
                name, wpb, avg / n_mfma, avg / n_mfma / wpb, ops, chip, ms);
    delete[] h;
    CK(hipFree(cyc));
    CK(hipFree(sink));
}

int main() {
    for (int wpb : {1, 4}) {
        run<0>("v_mfma_i32_32x32x32_i8", 2L * 32 * 32 * 32, wpb);
        run<1>("v_mfma_i32_16x16x64_i8", 2L * 16 * 16 * 64, wpb);
        run<2>("v_mfma_f32_32x32x16_f16", 2L * 32 * 32 * 16, wpb);
        run<3>("v_mfma_f32_32x32x16_bf16", 2L * 32 * 32 * 16, wpb);
        run<4>("v_mfma_f32_16x16x32_f16", 2L * 16 * 16 * 32, wpb);
    }
    return 0;
}
