// Memory-pattern ceilings for the Gaussian blur (no arithmetic): a batch of 16
// 1920x1200 fp32 frames copied (read once + written once, 295 MB moved) by
//   d2d      hipMemcpyAsync
//   flat     a grid-stride float4 copy
//   tile     the k_blur tile pattern: one TW x TH output tile per workgroup,
//            the (TW+16) x (TH+16) input window loaded as float4 (all loads
//            in flight), staged in LDS, barrier, TW x TH stored as float4
//   strip    a row-streaming pattern: a workgroup owns SW (64, 128) columns x SEG rows
//            (+16 halo rows read), one pass = 256/(SW/4) rows, loads kept D
//            passes ahead in registers, each pass staged through an LDS ring
//            with one barrier (the streaming blur's structure)
// Back-to-back launches on one stream, HIP events around N launches.
//   hipcc --offload-arch=gfx950 -O3 -o tools/blur_pattern_bench tools/blur_pattern_bench.hip
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

constexpr int W = 1920, H = 1200, NF = 16;

__global__ __launch_bounds__(256) void k_flat(const float4* __restrict__ a, float4* __restrict__ b, long n) {
    for (long i = blockIdx.x * 256L + threadIdx.x; i < n; i += (long)gridDim.x * 256) b[i] = a[i];
}

// Tile pattern: blockIdx.x -> (frame, tile), TW x TH output tiles, the
// (TW + 16) x (TH + 16) window loaded as float4 (all loads in flight), staged in
// LDS, barrier, the TW x TH interior stored as float4.
// XCD k gets a contiguous run of tiles in raster order (as the blur's
// xcd_tile): vertically adjacent tiles share an L2 for their halo rows.
__device__ __forceinline__ int xcd_tile(int b, int ntiles) {
    const int q = ntiles >> 3, rem = ntiles & 7, k = b & 7, i = b >> 3;
    return k * q + min(k, rem) + i;
}

template <int TW, int TH, int NT, bool XCD>
__global__ __launch_bounds__(NT) void k_tile(const float* __restrict__ a, float* __restrict__ b) {
    constexpr int IW = TW + 16, IH = TH + 16, NQ = IW / 4 * IH, LPT = (NQ + NT - 1) / NT, SPT = TW * TH / 4 / NT;
    __shared__ __attribute__((aligned(16))) float lds[IW * IH];
    constexpr int TX = W / TW, TY = (H + TH - 1) / TH;
    const int bid = XCD ? xcd_tile(blockIdx.x, NF * TX * TY) : blockIdx.x;
    const int f = bid / (TX * TY), t = bid % (TX * TY);
    const int x0 = (t % TX) * TW, y0 = (t / TX) * TH;
    const float* src = a + (size_t)f * W * H;
    float* dst = b + (size_t)f * W * H;
    const int tid = threadIdx.x;
    float4 v[LPT];
#pragma unroll
    for (int u = 0; u < LPT; u++) {
        const int idx = min(tid + NT * u, NQ - 1), row = idx / (IW / 4), q = idx % (IW / 4);
        const int gy = min(max(y0 - 8 + row, 0), H - 1), gx = min(max(x0 - 8 + 4 * q, 0), W - 4);
        v[u] = *reinterpret_cast<const float4*>(src + (size_t)gy * W + gx);
    }
#pragma unroll
    for (int u = 0; u < LPT; u++)
        if (tid + NT * u < NQ) *reinterpret_cast<float4*>(lds + 4 * (tid + NT * u)) = v[u];
    __syncthreads();
#pragma unroll
    for (int u = 0; u < SPT; u++) {
        const int idx = tid + NT * u, row = idx / (TW / 4), q = idx % (TW / 4);
        if (y0 + row < H)
            *reinterpret_cast<float4*>(dst + (size_t)(y0 + row) * W + x0 + 4 * q) =
                *reinterpret_cast<const float4*>(lds + (row + 8) * IW + 8 + 4 * q);
    }
}

template <int TW, int TH, int NT, bool XCD>
static void tile(const float* a, float* b, hipStream_t s, int iters);

// Strip pattern: blockIdx.x -> (frame, strip, segment).
template <int SW, int SEG, int D>
__global__ __launch_bounds__(256) void k_strip(const float* __restrict__ a, float* __restrict__ b) {
    constexpr int TPR = SW / 4, RPP = 256 / TPR;  // threads per row, rows per pass
    constexpr int NS = W / SW, NSEG = (H + SEG - 1) / SEG;
    constexpr int RING = 16 + 2 * RPP;
    __shared__ __attribute__((aligned(16))) float lds[RING * SW];
    const int f = blockIdx.x / (NS * NSEG), r = blockIdx.x % (NS * NSEG);
    const int x0 = (r % NS) * SW, ys = (r / NS) * SEG, ye = min(H, ys + SEG);
    const float* src = a + (size_t)f * W * H;
    float* dst = b + (size_t)f * W * H;
    const int tid = threadIdx.x, c = tid % TPR, rr = tid / TPR;
    const int y_first = ys - 8, passes = (ye + 8 - y_first + RPP - 1) / RPP;
    float4 ring[D];
    auto ld = [&](int p) {
        const int gy = min(max(y_first + p * RPP + rr, 0), H - 1);
        return *reinterpret_cast<const float4*>(src + (size_t)gy * W + x0 + 4 * c);
    };
#pragma unroll
    for (int d = 0; d < D; d++) ring[d] = ld(d);
    for (int p0 = 0; p0 < passes; p0 += D) {
#pragma unroll
        for (int d = 0; d < D; d++) {
            const int p = p0 + d;
            if (p < passes) {
                const float4 v = ring[d];
                ring[d] = ld(p + D);
                const int y = y_first + p * RPP + rr;
                *reinterpret_cast<float4*>(lds + ((p * RPP + rr) % RING) * SW + 4 * c) = v;
                __syncthreads();
                const int yo = y - 8;  // output row 8 rows behind (the column pass's lag)
                if (yo >= ys && yo < ye)
                    *reinterpret_cast<float4*>(dst + (size_t)yo * W + x0 + 4 * c) =
                        *reinterpret_cast<const float4*>(lds + ((p * RPP + rr - 8 + RING) % RING) * SW + 4 * c);
            }
        }
    }
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
    return ms * 1e3 / iters;
}

template <int TW, int TH, int NT, bool XCD>
static void tile(const float* a, float* b, hipStream_t s, int iters) {
    constexpr int TX = W / TW, TY = (H + TH - 1) / TH;
    const double us = time_us(iters, s, [&] {
        hipLaunchKernelGGL((k_tile<TW, TH, NT, XCD>), dim3(NF * TX * TY), dim3(NT), 0, s, a, b);
    });
    std::printf("{\"pattern\": \"tile\", \"TW\": %d, \"TH\": %d, \"threads\": %d, \"xcd\": %d, \"wgs\": %d, \"us\": %.2f, \"TBps\": %.3f}\n",
                TW, TH, NT, (int)XCD, NF * TX * TY, us, 2.0 * NF * W * H * 4 / us / 1e6);
}

template <int SW, int SEG, int D>
static void strip(const float* a, float* b, hipStream_t s, int iters) {
    constexpr int NS = W / SW, NSEG = (H + SEG - 1) / SEG;
    const double us = time_us(iters, s, [&] {
        hipLaunchKernelGGL((k_strip<SW, SEG, D>), dim3(NF * NS * NSEG), dim3(256), 0, s, a, b);
    });
    std::printf("{\"pattern\": \"strip\", \"SW\": %d, \"SEG\": %d, \"D\": %d, \"wgs\": %d, \"us\": %.2f, \"TBps\": %.3f}\n",
                SW, SEG, D, NF * NS * NSEG, us, 2.0 * NF * W * H * 4 / us / 1e6);
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 50;
    const size_t n = (size_t)NF * W * H;
    float *a, *b;
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&b, n * 4));
    CK(hipMemset(a, 0, n * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const double bytes = 2.0 * n * 4;
    double us = time_us(iters, s, [&] { CK(hipMemcpyAsync(b, a, n * 4, hipMemcpyDeviceToDevice, s)); });
    std::printf("{\"pattern\": \"d2d\", \"us\": %.2f, \"TBps\": %.3f}\n", us, bytes / us / 1e6);
    for (int g : {1024, 2048, 4096}) {
        us = time_us(iters, s, [&] {
            hipLaunchKernelGGL(k_flat, dim3(g), dim3(256), 0, s, (const float4*)a, (float4*)b, (long)(n / 4));
        });
        std::printf("{\"pattern\": \"flat\", \"wgs\": %d, \"us\": %.2f, \"TBps\": %.3f}\n", g, us, bytes / us / 1e6);
    }
    tile<64, 64, 256, false>(a, b, s, iters);
    tile<64, 64, 256, true>(a, b, s, iters);
    tile<64, 64, 512, true>(a, b, s, iters);
    tile<128, 64, 512, true>(a, b, s, iters);
    tile<192, 64, 512, true>(a, b, s, iters);
    tile<240, 32, 512, false>(a, b, s, iters);
    tile<240, 32, 512, true>(a, b, s, iters);
    tile<240, 64, 512, true>(a, b, s, iters);
    tile<128, 32, 256, true>(a, b, s, iters);
    strip<128, 300, 4>(a, b, s, iters);
    return 0;
}
