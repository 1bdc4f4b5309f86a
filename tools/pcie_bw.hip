// PCIe rates of the host-frame path's transfers, nothing else on the GPU:
// a C2 8-bit frame (1920 x 1200 = 2.30 MB) from mapped pinned host memory
// into device memory by (a) the DMA engine (hipMemcpyAsync) and (b) a copy
// kernel of G workgroups reading over PCIe (the staging copy's pattern:
// 4 x 16-byte loads in flight per thread), and 1.2 MB of results written
// back (device -> pinned) by DMA and by a kernel storing over PCIe.
// One JSON line per variant: GB/s over 200 back-to-back transfers.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));           \
            std::exit(1);                                                          \
        }                                                                          \
    } while (0)

__global__ __launch_bounds__(256) void k_copy16(const uint4* __restrict__ src, uint4* __restrict__ dst, size_t n) {
    const size_t nt = (size_t)gridDim.x * blockDim.x;
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + 3 * nt < n; i += 4 * nt) {
        const uint4 a = src[i], b = src[i + nt], c = src[i + 2 * nt], d = src[i + 3 * nt];
        dst[i] = a;
        dst[i + nt] = b;
        dst[i + 2 * nt] = c;
        dst[i + 3 * nt] = d;
    }
    for (; i < n; i += nt) dst[i] = src[i];
}

int main() {
    const size_t up = 1920 * 1200, down = 4366 * 284;  // frame bytes; keypoints + features + descriptors
    const int reps = 200;
    void *hUp, *hDown, *dUp, *dDown, *hUpDev, *hDownDev;
    CK(hipHostMalloc(&hUp, up, hipHostMallocMapped));
    CK(hipHostMalloc(&hDown, down, hipHostMallocMapped | hipHostMallocCoherent));
    CK(hipHostGetDevicePointer(&hUpDev, hUp, 0));
    CK(hipHostGetDevicePointer(&hDownDev, hDown, 0));
    CK(hipMalloc(&dUp, up));
    CK(hipMalloc(&dDown, down));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    auto run = [&](const char* name, size_t bytes, auto&& op) {
        for (int i = 0; i < 10; i++) op();
        CK(hipEventRecord(a, s));
        for (int i = 0; i < reps; i++) op();
        CK(hipEventRecord(b, s));
        CK(hipEventSynchronize(b));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, a, b));
        std::printf("{\"variant\": \"%s\", \"bytes\": %zu, \"us\": %.2f, \"GBps\": %.1f}\n", name, bytes,
                    1e3 * ms / reps, (double)bytes * reps / (ms * 1e6));
    };
    run("h2d_dma", up, [&] { CK(hipMemcpyAsync(dUp, hUp, up, hipMemcpyHostToDevice, s)); });
    for (int g : {16, 32, 64, 128, 256, 512}) {
        char name[32];
        std::snprintf(name, sizeof name, "h2d_kernel_%d", g);
        run(name, up, [&] {
            hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, s, (const uint4*)hUpDev, (uint4*)dUp, up / 16);
        });
    }
    run("d2h_dma", down, [&] { CK(hipMemcpyAsync(hDown, dDown, down, hipMemcpyDeviceToHost, s)); });
    for (int g : {32, 128, 512}) {
        char name[32];
        std::snprintf(name, sizeof name, "d2h_kernel_%d", g);
        run(name, down, [&] {
            hipLaunchKernelGGL(k_copy16, dim3(g), dim3(256), 0, s, (const uint4*)dDown, (uint4*)hDownDev, down / 16);
        });
    }
    // Both directions at once: the upload on one stream, the results on another.
    // (each round joins s2 back into s, so the events on s time both.)
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t j;
    CK(hipEventCreateWithFlags(&j, hipEventDisableTiming));
    run("duplex_kernel_64_128", up + down, [&] {
        hipLaunchKernelGGL(k_copy16, dim3(64), dim3(256), 0, s, (const uint4*)hUpDev, (uint4*)dUp, up / 16);
        hipLaunchKernelGGL(k_copy16, dim3(128), dim3(256), 0, s2, (const uint4*)dDown, (uint4*)hDownDev, down / 16);
        CK(hipEventRecord(j, s2));
        CK(hipStreamWaitEvent(s, j, 0));
    });
    CK(hipStreamSynchronize(s2));
    run("duplex_dma", up + down, [&] {
        CK(hipMemcpyAsync(dUp, hUp, up, hipMemcpyHostToDevice, s));
        CK(hipMemcpyAsync(hDown, dDown, down, hipMemcpyDeviceToHost, s2));
        CK(hipEventRecord(j, s2));
        CK(hipStreamWaitEvent(s, j, 0));
    });
    CK(hipStreamSynchronize(s2));
    CK(hipDeviceSynchronize());
    return 0;
}
