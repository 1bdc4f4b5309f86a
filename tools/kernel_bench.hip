// Isolated per-launch timing of the pyramid kernels (k_blur per radius and
// octave size, k_extrema_rows per octave) on a 1920x1200 synthetic frame,
// against a plain device-to-device copy of the same bytes.  Back-to-back
// launches on one stream, HIP events around N launches.
//   make tools/kernel_bench && tools/kernel_bench [iters]
// Prints one JSON object per line.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "sift_hip.h"
#include "sift_kernels.h"

using namespace sift_amd;
static const Frames kOne{1, 0};  // one frame per launch


#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e = (x);                                                                \
        if (e != hipSuccess) {                                                             \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
            std::exit(1);                                                                  \
        }                                                                                  \
    } while (0)

static Taps taps_for(double sigma) {
    Taps t{};
    int n = (int)std::lround(sigma * 8 + 1) | 1;
    if (n > 63) n = 63;
    double s = 0;
    std::vector<double> w(n);
    for (int i = 0; i < n; i++) {
        const double x = i - (n - 1) / 2.0;
        w[i] = std::exp(-x * x / (2 * sigma * sigma));
        s += w[i];
    }
    for (int i = 0; i < n; i++) t.w[i] = (float)(w[i] / s);
    t.n = n;
    return t;
}

// Read-pattern probes for the extrema kernel: every wave reads ROWS rows of
// all NP planes over COLS columns (dword: one column per lane, 62-column
// stride like k_extrema_rows; x4: four columns per lane, 256-column stride),
// all loads issued up front, and writes one sum per lane.
template <int NP, int ROWS, bool X4>
__global__ __launch_bounds__(256) void k_read_probe(const float* base, long planeStride, int pitch, int W, int H,
                                                    float* out) {
    constexpr int COLS = X4 ? 256 : 62;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x0 = blockIdx.x * COLS, y0 = (blockIdx.y * 4 + wave) * (ROWS - 2);
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(base), 0, (int)min((long)NP * planeStride * 4, 0x7fffffffL), 0x00020000);
    float acc = 0.f;
    if (X4) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        f4 v[ROWS][NP];
        const int xc = min(x0 + 4 * lane, W - 4);
#pragma unroll
        for (int k = 0; k < ROWS; k++)
#pragma unroll
            for (int d = 0; d < NP; d++)
                v[k][d] = __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(
                    rsrc, (unsigned)(min(y0 - 1 + k < 0 ? 0 : y0 - 1 + k, H - 1) * pitch + xc) * 4u,
                    (int)((long)d * planeStride * 4), 0));
#pragma unroll
        for (int k = 0; k < ROWS; k++)
#pragma unroll
            for (int d = 0; d < NP; d++) acc += v[k][d][0] + v[k][d][1] + v[k][d][2] + v[k][d][3];
    } else {
        float v[ROWS][NP];
        const int xc = min(max(x0 - 1 + lane, 0), W - 1);
#pragma unroll
        for (int k = 0; k < ROWS; k++)
#pragma unroll
            for (int d = 0; d < NP; d++)
                v[k][d] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                    rsrc, (unsigned)(min(y0 - 1 + k < 0 ? 0 : y0 - 1 + k, H - 1) * pitch + xc) * 4u,
                    (int)((long)d * planeStride * 4), 0));
#pragma unroll
        for (int k = 0; k < ROWS; k++)
#pragma unroll
            for (int d = 0; d < NP; d++) acc += v[k][d];
    }
    out[(blockIdx.y * gridDim.x + blockIdx.x) * 256 + threadIdx.x] = acc;
}

__global__ void k_empty(int* p) {
    if (p && threadIdx.x == 1023) p[0] = 1;
}

// Dispatch floor: a captured chain of `n` dependent empty kernels (as many
// launches as one frame's graph), replayed back to back on `ns` streams.
static void graph_floor(int n, int ns, int iters) {
    std::vector<hipStream_t> st(ns);
    for (auto& x : st) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
    std::vector<hipGraphExec_t> ex(ns);
    for (int k = 0; k < ns; k++) {
        hipGraph_t g;
        CK(hipStreamBeginCapture(st[k], hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < n; i++) hipLaunchKernelGGL(k_empty, dim3(256), dim3(256), 0, st[k], nullptr);
        CK(hipStreamEndCapture(st[k], &g));
        CK(hipGraphInstantiate(&ex[k], g, nullptr, nullptr, 0));
        CK(hipGraphDestroy(g));
    }
    for (int i = 0; i < 10; i++) CK(hipGraphLaunch(ex[i % ns], st[i % ns]));
    CK(hipDeviceSynchronize());
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, st[0]));
    for (int k = 1; k < ns; k++) CK(hipStreamWaitEvent(st[k], a, 0));
    for (int i = 0; i < iters; i++) CK(hipGraphLaunch(ex[i % ns], st[i % ns]));
    for (int k = 1; k < ns; k++) {
        hipEvent_t ev;
        CK(hipEventCreate(&ev));
        CK(hipEventRecord(ev, st[k]));
        CK(hipStreamWaitEvent(st[0], ev, 0));
    }
    CK(hipEventRecord(b, st[0]));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    std::printf("{\"kernel\": \"graph of %d empty kernels\", \"streams\": %d, \"us_per_graph\": %.3f}\n", n, ns,
                ms * 1e3 / iters);
}

template <class F>
static double time_us(int iters, hipStream_t s, F&& f);

template <int NP, int ROWS, bool X4>
static void probe(const OctGeom& g, float* out, hipStream_t s, int iters) {
    constexpr int COLS = X4 ? 256 : 62;
    dim3 grid((g.W + COLS - 1) / COLS, (g.H + 4 * (ROWS - 2) - 1) / (4 * (ROWS - 2)));
    double us = time_us(iters, s, [&] {
        hipLaunchKernelGGL((k_read_probe<NP, ROWS, X4>), grid, dim3(256), 0, s, g.base, g.planeStride, g.pitch, g.W,
                           g.H, out);
    });
    std::printf("{\"kernel\": \"read_probe\", \"x4\": %d, \"rows\": %d, \"W\": %d, \"us\": %.3f, \"GBps\": %.1f}\n",
                (int)X4, ROWS, g.W, us, 4.0 * NP * g.W * g.H / us / 1e3);
}

template <class F>
static double time_us(int iters, hipStream_t s, F&& f) {
    for (int i = 0; i < 5; i++) f();
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    CK(hipEventRecord(a, s));
    for (int i = 0; i < iters; i++) f();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    CK(hipEventDestroy(a));
    CK(hipEventDestroy(b));
    return ms * 1e3 / iters;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 200;
    const int W0 = 1920, H0 = 1200, L = 3;
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<float> host((size_t)W0 * H0);
    sift_synth_frame(0, W0, H0, host.data());

    // Pyramid buffers laid out as the detector lays them out (pitch multiple of 64).
    PyrDesc pyr{};
    pyr.nOct = 3;
    pyr.L = L;
    pyr.firstOctave = 0;
    size_t off = 0;
    int w = W0, h = H0, rowBase = 0;
    long bitBase = 0;
    for (int o = 0; o < 3; o++) {
        if (o) w /= 2, h /= 2;
        OctGeom& g = pyr.oct[o];
        g.W = w;
        g.H = h;
        g.pitch = (w + 63) / 64 * 64;
        g.planeStride = (long)g.pitch * h;
        g.base = reinterpret_cast<float*>(off);
        g.rowBase = rowBase;
        g.bitBase = bitBase;
        off += (size_t)g.planeStride * (L + 3);
        rowBase += L * h;
        bitBase += (long)L * h * w;
    }
    float* dPyr;
    CK(hipMalloc(&dPyr, off * sizeof(float)));
    CK(hipMemset(dPyr, 0, off * sizeof(float)));
    for (int o = 0; o < 3; o++) pyr.oct[o].base = dPyr + reinterpret_cast<size_t>(pyr.oct[o].base);
    float* dIn;
    CK(hipMalloc(&dIn, host.size() * sizeof(float)));
    CK(hipMemcpy(dIn, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice));
    float* dCopy;
    CK(hipMalloc(&dCopy, host.size() * sizeof(float)));

    // Fill the pyramid once (realistic planes for the extrema kernel).
    const double sigma = 1.6, k = std::pow(2.0, 1.0 / L);
    std::vector<Taps> lt(L + 3);
    for (int i = 1; i < L + 3; i++) {
        const double sp = std::pow(k, i - 1) * sigma, st = sp * k;
        lt[i] = taps_for(std::sqrt(st * st - sp * sp));
    }
    const Taps init = taps_for(std::sqrt(sigma * sigma - 0.25));
    launch_blur(dIn, W0, W0, H0, pyr.oct[0].base, pyr.oct[0].pitch, DecOut{}, init, kOne, 0, s);
    for (int o = 0; o < 3; o++) {
        const OctGeom& g = pyr.oct[o];
        for (int i = 1; i < L + 3; i++) {
            // plane L also writes the next octave's base plane (decimated)
            DecOut dec;
            if (i == L && o + 1 < 3) dec = DecOut{pyr.oct[o + 1].base, pyr.oct[o + 1].pitch, pyr.oct[o + 1].W, pyr.oct[o + 1].H};
            launch_blur(g.base + (size_t)(i - 1) * g.planeStride, g.pitch, g.W, g.H, g.base + (size_t)i * g.planeStride,
                        g.pitch, dec, lt[i], kOne, 0, s);
        }
    }
    CK(hipStreamSynchronize(s));

    const size_t planeB = (size_t)W0 * H0 * 4;
    double us = time_us(iters, s, [&] { CK(hipMemcpyAsync(dCopy, dIn, planeB, hipMemcpyDeviceToDevice, s)); });
    std::printf("{\"kernel\": \"hipMemcpyAsync d2d\", \"bytes\": %zu, \"us\": %.3f, \"GBps\": %.1f}\n", 2 * planeB, us,
                2 * planeB / us / 1e3);

    for (int o = 0; o < 3; o++) {
        const OctGeom& g = pyr.oct[o];
        for (int i = 1; i < L + 3; i++) {
            float* src = g.base + (size_t)(i - 1) * g.planeStride;
            float* dst = g.base + (size_t)i * g.planeStride;
            const double bytes = 8.0 * g.W * g.H;
            us = time_us(iters, s, [&] { launch_blur(src, g.pitch, g.W, g.H, dst, g.pitch, DecOut{}, lt[i], kOne, 0, s); });
            std::printf("{\"kernel\": \"k_blur<%d>\", \"octave\": %d, \"W\": %d, \"H\": %d, \"us\": %.3f, \"GBps\": %.1f}\n",
                        lt[i].n / 2, o, g.W, g.H, us, bytes / us / 1e3);
        }
    }
    uint2* dCand;
    Counters* dCtr;
    CK(hipMalloc(&dCand, sizeof(uint2) << 20));
    CK(hipMalloc(&dCtr, sizeof(Counters)));
    const float thr = std::floor(0.5 * 0.04 / L * 255);
    {
        double bytes = 0;
        for (int o = 0; o < 3; o++) bytes += 4.0 * (L + 3) * pyr.oct[o].W * pyr.oct[o].H;
        us = time_us(iters, s, [&] {
            CK(hipMemsetAsync(dCtr, 0, sizeof(Counters), s));
            launch_extrema_all(pyr, thr, dCand, dCtr, 1u << 20, kOne, s);
        });
        std::printf("{\"kernel\": \"k_extrema_all (3 octaves)+memset\", \"us\": %.3f, \"GBps\": %.1f}\n", us,
                    bytes / us / 1e3);
    }
    for (int ns : {1, 3})
        for (int n : {1, 8, 27}) graph_floor(n, ns, 300);
    us = time_us(iters, s, [&] { CK(hipMemsetAsync(dCtr, 0, sizeof(Counters), s)); });
    std::printf("{\"kernel\": \"memset 32B\", \"us\": %.3f}\n", us);
    return 0;
}
