// Blur pattern A/B (review item: "column-strip tiles of 64 columns with a
// rolling LDS window"): the product blur (sift_amd::launch_blur, 64 x 64
// tiles staged whole in LDS) against a strip kernel written here: a workgroup
// owns 64 output columns x SEG rows, keeps the row-blurred rows in an LDS ring
// and streams 8 input rows per step (loaded one step ahead into registers), so
// no input row is read twice vertically inside a segment.  Same arithmetic as
// the product (pyramid.hip header comment): outputs compared bit for bit.
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
//     -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude -Ianother-cuda-sift_amd/csrc \
//     tools/blur_strip_ab.hip -Lanother-cuda-sift_amd/lib -lsift_hip \
//     -Wl,-rpath,'$ORIGIN/../another-cuda-sift_amd/lib' -o tools/blur_strip_ab     (here, after make)
//   tools/blur_strip_ab > gpurun_out/blur_strip_ab.jsonl                           (GPU box)
//
// One JSON line per (radius, kernel): us per 16-frame 1920x1200 launch, the
// algorithmic 8 B/px rate, and whether the planes equal the product's.
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "sift_kernels.h"
#include "sift_math.h"

using namespace sift_amd;

#define CHECK(x)                                                                                   \
    do {                                                                                           \
        hipError_t e_ = (x);                                                                       \
        if (e_ != hipSuccess) {                                                                    \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));      \
            exit(1);                                                                               \
        }                                                                                          \
    } while (0)

constexpr int SW = 64;  // strip width (output columns)
constexpr int NT = 128;  // threads per workgroup (2 waves)

__device__ __forceinline__ int refl(int p, int len) { return reflect101(p, len); }

template <int R, int SEG>
__global__ __launch_bounds__(NT) void k_blur_strip(const float* __restrict__ src, float* __restrict__ dst, int pitch,
                                                   int W, int H, long fs, Taps taps, int stripsX, int segsY) {
    constexpr int IW = SW + 2 * R;          // input columns of a strip
    constexpr int IWP = (IW + 3) & ~3;      // LDS row pitch
    constexpr int P = (2 * R + 7) / 8;      // production blocks ahead of the column pass
    constexpr int RING = 8 * (P + 1);       // row-blurred rows kept
    static_assert(IW <= NT, "one input column per thread");
    __shared__ __attribute__((aligned(16))) float stage[8][IWP + 4];
    __shared__ __attribute__((aligned(16))) float mid[RING][SW];
    const int tid = threadIdx.x;
    const int total = gridDim.x;
    const int t = xcd_tile(blockIdx.x, total);
    const int per_frame = stripsX * segsY;
    const int f = t / per_frame, rem = t - f * per_frame, sy = rem / stripsX, sx = rem - sy * stripsX;
    src = fptr(src, f * fs);
    dst = fptr(dst, f * fs);
    const int x0 = sx * SW, y0 = sy * SEG, y1 = min(y0 + SEG, H);
    const int cin = tid < IW ? refl(x0 - R + tid, W) : 0;  // this thread's input column
    float w[2 * R + 1];
#pragma unroll
    for (int k = 0; k <= 2 * R; k++) w[k] = taps.w[k];

    const int nout = y1 - y0, nblk = (nout + 7) / 8;
    const int nprod = nblk + P;  // production blocks: input rows y0 - R + 8b .. + 7
    float v[8];
    auto load_block = [&](int b) {
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const int ir = refl(y0 - R + 8 * b + r, H);
            v[r] = tid < IW ? src[(size_t)ir * pitch + cin] : 0.f;
        }
    };
    // Row pass of the staged block b into ring slots 8 * (b % (P + 1)).
    auto row_pass = [&](int b) {
        const int r = tid >> 4, xs = (tid & 15) * 4;
        float in[2 * R + 4];
#pragma unroll
        for (int q = 0; q < (2 * R + 4 + 3) / 4; q++) {
            const float4 c = *reinterpret_cast<const float4*>(&stage[r][xs + 4 * q]);
            if (4 * q + 0 < 2 * R + 4) in[4 * q + 0] = c.x;
            if (4 * q + 1 < 2 * R + 4) in[4 * q + 1] = c.y;
            if (4 * q + 2 < 2 * R + 4) in[4 * q + 2] = c.z;
            if (4 * q + 3 < 2 * R + 4) in[4 * q + 3] = c.w;
        }
        float o[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            float s;
            if constexpr (2 * R + 1 > 5) {
                s = 0.f;
#pragma unroll
                for (int k = 0; k <= 2 * R; k++) s = __fmaf_rn(in[u + k], w[k], s);
            } else {
                s = in[u + R] * w[R];
#pragma unroll
                for (int k = 1; k <= R; k++) s = __fmaf_rn(in[u + R - k] + in[u + R + k], w[R + k], s);
            }
            o[u] = s;
        }
        *reinterpret_cast<float4*>(&mid[8 * (b % (P + 1)) + r][xs]) = make_float4(o[0], o[1], o[2], o[3]);
    };
    // Column pass of output block j: rows y0 + 8j + 4h .. + 3, column c.
    auto col_pass = [&](int j) {
        const int c = tid & 63, h = tid >> 6;
        const int yb = 8 * j + 4 * h;  // output row offset in the segment
        // ring row of output-relative row q: input row y0 + q -> production index q + R
        float m[2 * R + 4];
#pragma unroll
        for (int k = 0; k < 2 * R + 4; k++) m[k] = mid[(yb + k) % RING][c];  // rows yb - R + k (+R offset)
#pragma unroll
        for (int u = 0; u < 4; u++) {
            float s = __fmaf_rn(m[u + R], w[R], 0.f);
#pragma unroll
            for (int k = 1; k <= R; k++) s = __fmaf_rn(m[u + R + k] + m[u + R - k], w[R + k], s);
            const int y = y0 + yb + u, x = x0 + c;
            if (y < y1 && x < W) dst[(size_t)y * pitch + x] = s;
        }
    };

    load_block(0);
    for (int b = 0; b < nprod; b++) {
#pragma unroll
        for (int r = 0; r < 8; r++)
            if (tid < IW) stage[r][tid] = v[r];
        if (b + 1 < nprod) load_block(b + 1);  // in flight during this step's passes
        __syncthreads();
        row_pass(b);
        __syncthreads();
        if (b >= P) col_pass(b - P);
    }
}

template <int R, int SEG>
float time_strip(const float* src, float* dst, int pitch, int W, int H, int nf, long fs, const Taps& taps, int reps,
                 hipStream_t s) {
    const int stripsX = (W + SW - 1) / SW, segsY = (H + SEG - 1) / SEG;
    const int grid = stripsX * segsY * nf;
    auto run = [&] {
        hipLaunchKernelGGL((k_blur_strip<R, SEG>), dim3(grid), dim3(NT), 0, s, src, dst, pitch, W, H, fs, taps, stripsX,
                           segsY);
    };
    for (int i = 0; i < 3; i++) run();
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a, s));
    for (int i = 0; i < reps; i++) run();
    CHECK(hipEventRecord(b, s));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    return ms * 1e3f / reps;
}

static Taps gauss_taps(int R) {
    Taps t{};
    t.n = 2 * R + 1;
    const double sigma = R / 4.0;
    double sum = 0;
    std::vector<double> g(t.n);
    for (int k = 0; k < t.n; k++) sum += g[k] = std::exp(-(k - R) * (k - R) / (2 * sigma * sigma));
    for (int k = 0; k < t.n; k++) t.w[k] = (float)(g[k] / sum);
    return t;
}

template <int R>
void run_radius(const float* src, float* dA, float* dB, int pitch, int W, int H, int nf, long fs, hipStream_t s,
                std::vector<float>& ha, std::vector<float>& hb) {
    const Taps taps = gauss_taps(R);
    const int reps = 20;
    const Frames fr{nf, fs};
    for (int i = 0; i < 3; i++) launch_blur(src, pitch, W, H, dA, pitch, DecOut{}, taps, fr, fs, s);
    hipEvent_t a, b;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&b));
    CHECK(hipEventRecord(a, s));
    for (int i = 0; i < reps; i++) launch_blur(src, pitch, W, H, dA, pitch, DecOut{}, taps, fr, fs, s);
    CHECK(hipEventRecord(b, s));
    CHECK(hipEventSynchronize(b));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, a, b));
    const float us_tile = ms * 1e3f / reps;
    const double bytes = 8.0 * W * H * nf;
    CHECK(hipMemcpy(ha.data(), dA, ha.size() * 4, hipMemcpyDeviceToHost));
    printf("{\"radius\": %d, \"kernel\": \"tile (product)\", \"us\": %.2f, \"GBps\": %.1f}\n", R, us_tile,
           bytes / us_tile / 1e3);
    auto strip = [&](auto seg_tag, const char* name) {
        constexpr int SEG = decltype(seg_tag)::value;
        CHECK(hipMemset(dB, 0, hb.size() * 4));
        const float us = time_strip<R, SEG>(src, dB, pitch, W, H, nf, fs, taps, reps, s);
        CHECK(hipMemcpy(hb.data(), dB, hb.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (int f = 0; f < nf; f++)
            for (int y = 0; y < H; y++)
                bad += memcmp(&ha[(size_t)f * fs / 4 + (size_t)y * pitch], &hb[(size_t)f * fs / 4 + (size_t)y * pitch],
                              (size_t)W * 4) != 0;
        printf("{\"radius\": %d, \"kernel\": \"%s\", \"us\": %.2f, \"GBps\": %.1f, \"rows_differing\": %zu}\n", R, name,
               us, bytes / us / 1e3, bad);
        fflush(stdout);
    };
    strip(std::integral_constant<int, 128>{}, "strip SEG=128");
    strip(std::integral_constant<int, 256>{}, "strip SEG=256");
    strip(std::integral_constant<int, 1200>{}, "strip SEG=1200");
}

int main() {
    const int W = 1920, H = 1200, nf = 16, pitch = 1920;
    const long fs = (long)pitch * H * 4;
    std::vector<float> h((size_t)nf * pitch * H);
    unsigned seed = 12345;
    for (auto& x : h) {
        seed = seed * 1664525u + 1013904223u;
        x = (float)(seed >> 24);
    }
    float *src, *dA, *dB;
    CHECK(hipMalloc(&src, h.size() * 4));
    CHECK(hipMalloc(&dA, h.size() * 4));
    CHECK(hipMalloc(&dB, h.size() * 4));
    CHECK(hipMemcpy(src, h.data(), h.size() * 4, hipMemcpyHostToDevice));
    hipStream_t s;
    CHECK(hipStreamCreate(&s));
    std::vector<float> ha(h.size()), hb(h.size());
    run_radius<5>(src, dA, dB, pitch, W, H, nf, fs, s, ha, hb);
    run_radius<6>(src, dA, dB, pitch, W, H, nf, fs, s, ha, hb);
    run_radius<8>(src, dA, dB, pitch, W, H, nf, fs, s, ha, hb);
    run_radius<10>(src, dA, dB, pitch, W, H, nf, fs, s, ha, hb);
    run_radius<13>(src, dA, dB, pitch, W, H, nf, fs, s, ha, hb);
    return 0;
}
