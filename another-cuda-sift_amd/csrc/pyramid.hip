// Gaussian pyramid and 3x3x3 scale-space extrema for gfx950.
//
// Replaces /root/reference/sift_cuda/image_func/{Filter,Resize,MatOps}.cu.
// Semantics follow OpenCV 4.x; the float
// operation order is the oracle's (oracle/sift_oracle.cpp gaussianBlur /
// upsample2x / isExtremum), so planes and candidate lists are bit-exact.
#include "sift_kernels.h"
#include "sift_math.h"

namespace sift_amd {

// ---------------------------------------------------------------------------
// 2x bilinear upsample (OpenCV resize INTER_LINEAR on float; firstOctave = -1).
// Reference: Resize.cu:6-64 (half-pixel bilinear, target size ignored).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void up_coeff(int d, int slen, int& s, float& a0, float& a1) {
    float f = (float)((d + 0.5) * 0.5 - 0.5);
    int si = (int)floorf(f);
    f -= (float)si;
    if (si < 0) { f = 0.f; si = 0; }
    if (si >= slen - 1) { f = 0.f; si = slen - 1; }
    s = si;
    a0 = 1.f - f;
    a1 = f;
}

__global__ __launch_bounds__(256) void k_upsample2x(const float* __restrict__ src, int spitch, int W, int H,
                                                    float* __restrict__ dst, int dpitch) {
    const int x = blockIdx.x * 64 + (threadIdx.x & 63);
    const int y = blockIdx.y * 4 + (threadIdx.x >> 6);
    if (x >= 2 * W || y >= 2 * H) return;
    int sx, sy;
    float ax0, ax1, ay0, ay1;
    up_coeff(x, W, sx, ax0, ax1);
    up_coeff(y, H, sy, ay0, ay1);
    const int sx1 = min(sx + 1, W - 1), sy1 = min(sy + 1, H - 1);
    const float* r0 = src + (size_t)sy * spitch;
    const float* r1 = src + (size_t)sy1 * spitch;
    const float h0 = r0[sx] * ax0 + r0[sx1] * ax1;
    const float h1 = r1[sx] * ax0 + r1[sx1] * ax1;
    dst[(size_t)y * dpitch + x] = h0 * ay0 + h1 * ay1;
}

void launch_upsample2x(const float* src, int spitch, int W, int H, float* dst, int dpitch, hipStream_t s) {
    dim3 grid((2 * W + 63) / 64, (2 * H + 3) / 4);
    hipLaunchKernelGGL(k_upsample2x, grid, dim3(256), 0, s, src, spitch, W, H, dst, dpitch);
}

// ---------------------------------------------------------------------------
// Separable Gaussian blur, one 64 x 32 output tile per 256-thread workgroup.
// The (32+2r) x (64+2r) input tile (reflect-101 borders, optional stride-2
// read = INTER_NEAREST octave decimation fused in) is staged once in LDS; the
// row pass writes a (32+2r) x 64 LDS tile; the column pass writes HBM.
// Row:    s = 0; s = fma(in[x-r+k], w[k], s), k = 0..n-1   (n > 5)
//         s = in[x]*w[r]; s = fma(in[x-k]+in[x+k], w[r+k], s)   (n <= 5)
// Column: s = fma(mid[y], w[r], 0); s = fma(mid[y+k]+mid[y-k], w[r+k], s)
// Reference: Filter.cu:8-51 (no LDS, vertical first, modulo per tap).
// ---------------------------------------------------------------------------
constexpr int BLUR_TW = 64;
constexpr int BLUR_TH = 32;

__global__ __launch_bounds__(256) void k_blur(const float* __restrict__ src, int spitch, int sstep, int W, int H,
                                              float* __restrict__ dst, int dpitch, float* __restrict__ copy_out,
                                              Taps taps) {
    extern __shared__ float lds[];
    const int n = taps.n, r = n >> 1;
    const int IW = BLUR_TW + 2 * r, IH = BLUR_TH + 2 * r;
    float* in = lds;
    float* mid = lds + IH * IW;
    const int x0 = blockIdx.x * BLUR_TW, y0 = blockIdx.y * BLUR_TH;
    const int tid = threadIdx.x;

    for (int ly = tid >> 6; ly < IH; ly += 4) {
        const int gy = reflect101(y0 - r + ly, H);
        const float* srow = src + (size_t)gy * sstep * spitch;
        for (int lx = tid & 63; lx < IW; lx += 64) {
            const int gx = reflect101(x0 - r + lx, W);
            in[ly * IW + lx] = srow[(size_t)gx * sstep];
        }
    }
    __syncthreads();

    if (n > 5) {
        for (int i = tid; i < IH * BLUR_TW; i += 256) {
            const int ly = i >> 6, lx = i & 63;
            const float* p = in + ly * IW + lx;
            float s = 0.f;
            for (int k = 0; k < n; k++) s = __fmaf_rn(p[k], taps.w[k], s);
            mid[i] = s;
        }
    } else {
        for (int i = tid; i < IH * BLUR_TW; i += 256) {
            const int ly = i >> 6, lx = i & 63;
            const float* p = in + ly * IW + lx + r;
            float s = p[0] * taps.w[r];
            for (int k = 1; k <= r; k++) s = __fmaf_rn(p[-k] + p[k], taps.w[r + k], s);
            mid[i] = s;
        }
    }
    __syncthreads();

    for (int i = tid; i < BLUR_TH * BLUR_TW; i += 256) {
        const int ly = i >> 6, lx = i & 63;
        const int gy = y0 + ly, gx = x0 + lx;
        if (gy < H && gx < W) {
            const float* p = mid + (ly + r) * BLUR_TW + lx;
            float s = __fmaf_rn(p[0], taps.w[r], 0.f);
            for (int k = 1; k <= r; k++) s = __fmaf_rn(p[k * BLUR_TW] + p[-k * BLUR_TW], taps.w[r + k], s);
            dst[(size_t)gy * dpitch + gx] = s;
            if (copy_out) copy_out[(size_t)gy * dpitch + gx] = in[(ly + r) * IW + lx + r];
        }
    }
}

void launch_blur(const float* src, int spitch, int sstep, int W, int H, float* dst, int dpitch, float* copy_out,
                 const Taps& taps, hipStream_t s) {
    const int r = taps.n >> 1;
    const size_t lds = sizeof(float) * ((size_t)(BLUR_TH + 2 * r) * (BLUR_TW + 2 * r) + (size_t)(BLUR_TH + 2 * r) * BLUR_TW);
    dim3 grid((W + BLUR_TW - 1) / BLUR_TW, (H + BLUR_TH - 1) / BLUR_TH);
    hipLaunchKernelGGL(k_blur, grid, dim3(256), lds, s, src, spitch, sstep, W, H, dst, dpitch, copy_out, taps);
}

// ---------------------------------------------------------------------------
// DoG + 3x3x3 extremum scan for one octave.  DoG planes D_d = G_{d+1} - G_d are
// formed in LDS for a 64 x 16 tile plus a 1-pixel halo (never written to HBM);
// every (layer 1..L, r, c) with border 5 is tested exactly as OpenCV's
// findScaleSpaceExtremaComputer: |v| > threshold and v >= (<=) all 26
// neighbours.  Hits are compacted with a wave ballot and one atomic per wave.
// Reference: MatOps.cu:39-181 (mask + full-volume CUB scan + scatter).
// ---------------------------------------------------------------------------
constexpr int EX_TW = 64;
constexpr int EX_TH = 16;
constexpr int EX_SW = EX_TW + 2;
constexpr int EX_SH = EX_TH + 2;

__global__ __launch_bounds__(256) void k_extrema(OctGeom g, int L, int o, float thr, uint2* __restrict__ cand,
                                                 Counters* __restrict__ ctr, unsigned cap) {
    extern __shared__ float dog[];  // (L+2) planes of EX_SH x EX_SW
    const int tid = threadIdx.x;
    const int x0 = blockIdx.x * EX_TW, y0 = blockIdx.y * EX_TH;
    const int W = g.W, H = g.H, pitch = g.pitch;
    const int PS = EX_SH * EX_SW;

    for (int i = tid; i < PS; i += 256) {
        const int ly = i / EX_SW, lx = i - ly * EX_SW;
        const int gy = y0 - 1 + ly, gx = x0 - 1 + lx;
        if (gy >= 0 && gy < H && gx >= 0 && gx < W) {
            const float* p = g.base + (size_t)gy * pitch + gx;
            float prev = p[0];
            for (int d = 0; d < L + 2; d++) {
                const float next = p[(size_t)(d + 1) * g.planeStride];
                dog[d * PS + i] = next - prev;
                prev = next;
            }
        } else {
            for (int d = 0; d < L + 2; d++) dog[d * PS + i] = 0.f;
        }
    }
    __syncthreads();

    const int lane = tid & 63;
    const int total = EX_TH * EX_TW * L;
    for (int base = 0; base < total; base += 256) {
        const int i = base + tid;
        bool hit = false;
        int layer = 0, r = 0, c = 0;
        if (i < total) {
            layer = 1 + i / (EX_TH * EX_TW);
            const int rem = i - (layer - 1) * (EX_TH * EX_TW);
            const int ly = rem >> 6, lx = rem & 63;
            r = y0 + ly;
            c = x0 + lx;
            if (r >= 5 && r < H - 5 && c >= 5 && c < W - 5) {
                const float* cur = dog + layer * PS + (ly + 1) * EX_SW + (lx + 1);
                const float val = cur[0];
                if (fabsf(val) > thr) {
                    hit = true;
                    if (val > 0) {
#pragma unroll
                        for (int d = -1; d <= 1; d++)
#pragma unroll
                            for (int dy = -1; dy <= 1; dy++)
#pragma unroll
                                for (int dx = -1; dx <= 1; dx++) hit &= val >= cur[d * PS + dy * EX_SW + dx];
                    } else {
#pragma unroll
                        for (int d = -1; d <= 1; d++)
#pragma unroll
                            for (int dy = -1; dy <= 1; dy++)
#pragma unroll
                                for (int dx = -1; dx <= 1; dx++) hit &= val <= cur[d * PS + dy * EX_SW + dx];
                    }
                }
            }
        }
        const unsigned long long mask = __ballot(hit);
        if (mask) {
            const int cnt = __popcll(mask);
            unsigned basepos = 0;
            if (lane == 0) basepos = atomicAdd(&ctr->cand, (unsigned)cnt);
            basepos = __shfl(basepos, 0);
            if (hit) {
                const unsigned pos = basepos + (unsigned)__popcll(mask & ((1ull << lane) - 1ull));
                if (pos < cap)
                    cand[pos] = make_uint2((unsigned)(o << 8 | layer), (unsigned)(r << 16 | c));
                else
                    atomicOr(&ctr->overflow, 1u);
            }
        }
    }
}

void launch_extrema(const PyrDesc& pyr, int o, float threshold, uint2* cand, Counters* ctr, unsigned cap,
                    hipStream_t s) {
    const OctGeom& g = pyr.oct[o];
    dim3 grid((g.W + EX_TW - 1) / EX_TW, (g.H + EX_TH - 1) / EX_TH);
    const size_t lds = sizeof(float) * (size_t)(pyr.L + 2) * EX_SH * EX_SW;
    hipLaunchKernelGGL(k_extrema, grid, dim3(256), lds, s, g, pyr.L, o, threshold, cand, ctr, cap);
}

}  // namespace sift_amd
