// In-kernel shader clock probe (MI355X_MICROARCH.md, DVFS item 6: clock =
// delta s_memtime / delta s_memrealtime x 100 MHz), for pricing MFMA-busy
// counters at the clock the chip actually ran, not the 2.4 GHz peak.
//
// probe_start(seconds) launches NWG one-wave workgroups on a stream of their
// own (consecutive workgroups land on consecutive XCDs); each stamps both
// counters, sleeps in a loop until `seconds` of real time have passed, and
// stamps again.  While it runs, the caller keeps the GPU busy with the
// workload to be priced (here: back-to-back batched matcher calls).
// probe_finish() waits and returns per workgroup {cycles, realtime ticks}.
// The probe reads counters only; results go out through vector stores.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/libclock_probe.so tools/clock_probe.hip
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr int kNwg = 64;

__global__ __launch_bounds__(64) void k_probe(unsigned long long ticks, unsigned long long* __restrict__ out) {
    const unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    unsigned long long r1 = r0, t1 = t0;
    // Exit condition every wave reaches: real time, capped by an iteration count.
    for (int it = 0; it < (1 << 26) && r1 - r0 < ticks; it++) {
        __builtin_amdgcn_s_sleep(127);
        r1 = __builtin_amdgcn_s_memrealtime();
    }
    t1 = __builtin_amdgcn_s_memtime();
    r1 = __builtin_amdgcn_s_memrealtime();
    if (threadIdx.x == 0) {
        out[2 * blockIdx.x + 0] = t1 - t0;
        out[2 * blockIdx.x + 1] = r1 - r0;
    }
}

hipStream_t g_stream = nullptr;
unsigned long long* g_out = nullptr;

}  // namespace

extern "C" int probe_start(double seconds) {
    if (!g_stream && hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking) != hipSuccess) return -1;
    if (!g_out && hipMalloc(&g_out, sizeof(unsigned long long) * 2 * kNwg) != hipSuccess) return -2;
    if (hipMemsetAsync(g_out, 0, sizeof(unsigned long long) * 2 * kNwg, g_stream) != hipSuccess) return -3;
    const unsigned long long ticks = (unsigned long long)(seconds * 1e8);  // s_memrealtime: 100 MHz
    hipLaunchKernelGGL(k_probe, dim3(kNwg), dim3(64), 0, g_stream, ticks, g_out);
    return hipGetLastError() == hipSuccess ? 0 : -4;
}

// out: 2 * n doubles {cycles, realtime ticks} per workgroup; returns the count.
extern "C" int probe_finish(double* out, int n) {
    if (!g_stream) return -1;
    if (hipStreamSynchronize(g_stream) != hipSuccess) return -2;
    unsigned long long h[2 * kNwg];
    if (hipMemcpy(h, g_out, sizeof h, hipMemcpyDeviceToHost) != hipSuccess) return -3;
    const int m = n < kNwg ? n : kNwg;
    for (int i = 0; i < 2 * m; i++) out[i] = (double)h[i];
    return m;
}
