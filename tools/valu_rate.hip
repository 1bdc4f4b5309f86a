// VALU issue rates on gfx950 for the matcher's key ops: SIMD cycles per wave
// instruction (s_memtime around a loop of 8 independent chains), with 1, 2
// and 4 waves per SIMD, alone and beside v_mfma_i32_32x32x32_i8.
//   hipcc --offload-arch=gfx950 -O3 -o tools/valu_rate tools/valu_rate.hip && tools/valu_rate
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

constexpr int kIters = 2048, kChains = 8;

// op 0: v_add_f32, 1: v_lshl_add_u32, 2: v_max3_i32, 3: v_med3_i32, 4: v_add_u32, 5: v_max_i32,
// 6: v_max3_f32, 7: v_med3_f32, 8: v_max_f32, 9: v_mad_i32_i24, 10: v_add3_u32, 11: v_fma_f32,
// 12: v_lshlrev_b32, 13: v_max_u32, 14: v_pk_max_i16, 15: v_med3_u32,
// 16: v_pk_fma_f32, 17: v_pk_mov_b32, 18: v_pk_add_f32, 19: v_fmac_f32 (VOP2)
template <int OP, bool MFMA>
__global__ __launch_bounds__(256) void k_valu(int seed, unsigned long long* cyc, int* sink) {
    const int lane = threadIdx.x & 63;
    int x[kChains];
    float f[kChains];
    typedef float f2 __attribute__((ext_vector_type(2)));
    f2 p2[kChains];
    for (int c = 0; c < kChains; c++) {
        x[c] = seed + lane * 3 + c;
        f[c] = (float)x[c];
        p2[c] = (f2){f[c], f[c] + 1.f};
    }
    const int k1 = seed * 7 + lane, k2 = seed - lane;
    const f2 q1 = {(float)k1, 1.5f}, q2 = {0.5f, (float)seed};
    const i32x4 a = {seed + lane, seed * 3, lane, 7}, b = {lane * 5, seed, 3, lane};
    i32x16 acc = {};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < kIters; it++) {
        if constexpr (MFMA) acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc, 0, 0, 0);
#pragma unroll
        for (int c = 0; c < kChains; c++) {
            if constexpr (OP == 0) __asm__ volatile("v_add_f32 %0, %1, %0" : "+v"(f[c]) : "v"(k1));
            if constexpr (OP == 1) __asm__ volatile("v_lshl_add_u32 %0, %0, 9, %1" : "+v"(x[c]) : "v"(k1));
            if constexpr (OP == 2) __asm__ volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(k1), "v"(k2));
            if constexpr (OP == 3) __asm__ volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(k1), "v"(k2));
            if constexpr (OP == 4) __asm__ volatile("v_add_u32 %0, %0, %1" : "+v"(x[c]) : "v"(k1));
            if constexpr (OP == 5) __asm__ volatile("v_max_i32 %0, %0, %1" : "+v"(x[c]) : "v"(k1));
            if constexpr (OP == 6) __asm__ volatile("v_max3_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(k1), "v"(k2));
            if constexpr (OP == 7) __asm__ volatile("v_med3_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(k1), "v"(k2));
            if constexpr (OP == 8) __asm__ volatile("v_max_f32 %0, %0, %1" : "+v"(f[c]) : "v"(k1));
            if constexpr (OP == 9) __asm__ volatile("v_mad_i32_i24 %0, %0, 9, %1" : "+v"(x[c]) : "v"(k1));
            if constexpr (OP == 10) __asm__ volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(k1), "v"(k2));
            if constexpr (OP == 11) __asm__ volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[c]) : "v"(k1), "v"(k2));
            if constexpr (OP == 12) __asm__ volatile("v_lshlrev_b32 %0, 9, %0" : "+v"(x[c]));
            if constexpr (OP == 13) __asm__ volatile("v_max_u32 %0, %0, %1" : "+v"(x[c]) : "v"(k1));
            if constexpr (OP == 14) __asm__ volatile("v_pk_max_i16 %0, %0, %1" : "+v"(x[c]) : "v"(k1));
            if constexpr (OP == 15) __asm__ volatile("v_med3_u32 %0, %0, %1, %2" : "+v"(x[c]) : "v"(k1), "v"(k2));
            if constexpr (OP == 16) __asm__ volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p2[c]) : "v"(q1), "v"(q2));
            if constexpr (OP == 17) __asm__ volatile("v_pk_mov_b32 %0, %0, %1 op_sel:[1,0]" : "+v"(p2[c]) : "v"(q1));
            if constexpr (OP == 18) __asm__ volatile("v_pk_add_f32 %0, %0, %1" : "+v"(p2[c]) : "v"(q1));
            if constexpr (OP == 19) __asm__ volatile("v_fmac_f32 %0, %1, %2" : "+v"(f[c]) : "v"(k1), "v"(k2));
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    int s = acc[lane & 15];
    for (int c = 0; c < kChains; c++) s += x[c] + (int)f[c] + (int)p2[c][0] + (int)p2[c][1];
    sink[blockIdx.x * blockDim.x + threadIdx.x] = s;
    if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + (threadIdx.x >> 6)] = t1 - t0;
}

template <int OP, bool MFMA>
static void run(const char* name, int wps) {
    // 1024 workgroups of 4 waves (one per SIMD) x wps workgroups per CU -> wps waves per SIMD
    const int nwg = 256 * wps, nw = nwg * 4;
    unsigned long long* cyc;
    int* sink;
    CK(hipMalloc(&cyc, sizeof(unsigned long long) * nw));
    CK(hipMalloc(&sink, sizeof(int) * nw * 64));
    for (int rep = 0; rep < 2; rep++) hipLaunchKernelGGL((k_valu<OP, MFMA>), dim3(nwg), dim3(256), 0, 0, rep, cyc, sink);
    CK(hipDeviceSynchronize());
    unsigned long long* h = new unsigned long long[nw];
    CK(hipMemcpy(h, cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost));
    double avg = 0;
    for (int i = 0; i < nw; i++) avg += (double)h[i];
    avg /= nw;
    const double n = (double)kIters * kChains;
    std::printf("{\"op\": \"%s\", \"mfma_per_8\": %d, \"waves_per_simd\": %d, \"wave_cycles_per_op\": %.2f, "
                "\"simd_cycles_per_op\": %.2f}\n",
                name, (int)MFMA, wps, avg / n, avg / n / wps);
    delete[] h;
    CK(hipFree(cyc));
    CK(hipFree(sink));
}

int main() {
    for (int w : {2, 4, 6}) {
        run<0, false>("v_add_f32", w);
        run<11, false>("v_fma_f32", w);
        run<19, false>("v_fmac_f32", w);
        run<16, false>("v_pk_fma_f32", w);
        run<17, false>("v_pk_mov_b32", w);
        run<18, false>("v_pk_add_f32", w);
        run<2, false>("v_max3_i32", w);
    }
    return 0;
}
