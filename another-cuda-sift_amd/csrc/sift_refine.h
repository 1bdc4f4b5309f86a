// adjustLocalExtrema (OpenCV 4.x sift.simd.hpp) for one 3x3x3 candidate, used
// by k_refine (keypoints.hip).  DoG values are re-formed from the Gaussian
// planes (G_{l+1} - G_l: the same single rounding as a stored DoG).  Accepted
// keypoints are de-duplicated by final grid position with a bitmap (OpenCV
// removes the same duplicates later in removeDuplicatedSorted); k_refine
// compacts them with one counter atomic per wave.
// Reference: SiftOps.cu:63-208 + collectKpts SiftOps.cu:210-235.
#pragma once
#include <climits>

#include "sift_kernels.h"
#include "sift_math.h"

namespace sift_amd {

constexpr int kBorder = 5;
constexpr int kMaxInterpSteps = 5;

__device__ __forceinline__ const OctGeom& octave_geom(const PyrDesc& pyr, int o) { return pyr.oct[o]; }

// q = {octave << 8 | layer, r << 16 | c} as the extrema kernels emit it.
// foff: byte offset of the candidate's frame arena (ctr / bitmap / out are
// already that frame's).
// Returns true for an accepted, first-of-its-position keypoint `k` (its
// dedupe bit `bit` is set); the caller appends it (wave-aggregated).
__device__ __forceinline__ bool refine_candidate(const PyrDesc& pyr, uint2 q, uint32_t* __restrict__ bitmap,
                                                 const KeypointParams& kp, long foff, RefKpt& k, long& bit) {
    const int L = pyr.L;
    const float img_scale = 1.f / 255.f;
    const float deriv_scale = img_scale * 0.5f;
    const float second_deriv_scale = img_scale;
    const float cross_deriv_scale = img_scale * 0.25f;
    const int o = (int)(q.x >> 8);
    int layer = (int)(q.x & 255);
    int r = (int)(q.y >> 16), c = (int)(q.y & 0xffff);
    const OctGeom& g = octave_geom(pyr, o);
    const float* G = fptr(g.base, foff);
    const long ps = g.planeStride;
    const int pitch = g.pitch;
    // The 3x3 neighbourhood of Gaussian planes layer-1 .. layer+2 around
    // (r, c): 12 row segments of 3 floats, one 12-byte load each (all in
    // flight together), instead of ~30 scattered dword loads per Newton step.
    // The octave (hence the plane base) differs between the lanes of a wave,
    // so these are 64-bit-address global loads: a buffer resource would be
    // divergent and cost a readfirstlane waterfall loop per load.  Every
    // block is inside the plane (|offset| <= 1 from a position >= kBorder
    // from the edges, layers 0 .. L+2).  DoG values are formed from it
    // exactly as a stored DoG (G_{l+1} - G_l, one rounding).  The block of the
    // converged position stays in registers for the contrast and edge tests.
    float D[3][3][3];  // D[s][dy][dx] = DoG at (layer - 1 + s, r - 1 + dy, c - 1 + dx)
    auto load_block = [&]() {
        float v[4][3][3];
        typedef const __attribute__((address_space(1))) float* gptr;  // global_load, not flat
        const gptr b = (gptr)(G + (long)(layer - 1) * ps + (long)(r - 1) * pitch + (c - 1));
#pragma unroll
        for (int p = 0; p < 4; p++)
#pragma unroll
            for (int dy = 0; dy < 3; dy++) {
                const gptr e = b + p * ps + dy * pitch;
                v[p][dy][0] = e[0];
                v[p][dy][1] = e[1];
                v[p][dy][2] = e[2];
            }
#pragma unroll
        for (int p = 0; p < 3; p++)
#pragma unroll
            for (int dy = 0; dy < 3; dy++)
#pragma unroll
                for (int dx = 0; dx < 3; dx++) D[p][dy][dx] = v[p + 1][dy][dx] - v[p][dy][dx];
    };

    float xi = 0, xr = 0, xc = 0;
    int it = 0;
    bool ok = true;
    for (; it < kMaxInterpSteps; it++) {
        load_block();
        const float c0 = D[1][1][1];
        const float cl = D[1][1][0], cr = D[1][1][2];
        const float cu = D[1][0][1], cd = D[1][2][1];
        const float pc = D[0][1][1], nc = D[2][1][1];
        const float dD0 = (cr - cl) * deriv_scale;
        const float dD1 = (cd - cu) * deriv_scale;
        const float dD2 = (nc - pc) * deriv_scale;
        const float v2 = c0 * 2;
        const float dxx = (cr + cl - v2) * second_deriv_scale;
        const float dyy = (cd + cu - v2) * second_deriv_scale;
        const float dss = (nc + pc - v2) * second_deriv_scale;
        const float dxy = (D[1][2][2] - D[1][2][0] - D[1][0][2] + D[1][0][0]) * cross_deriv_scale;
        const float dxs = (D[2][1][2] - D[2][1][0] - D[0][1][2] + D[0][1][0]) * cross_deriv_scale;
        const float dys = (D[2][2][1] - D[2][0][1] - D[0][2][1] + D[0][0][1]) * cross_deriv_scale;
        // Matx_FastSolveOp<float,3,1>: Cramer's rule, det from Matx_DetOp.
        const float a00 = dxx, a01 = dxy, a02 = dxs, a10 = dxy, a11 = dyy, a12 = dys, a20 = dxs, a21 = dys,
                    a22 = dss;
        const float b0 = dD0, b1 = dD1, b2 = dD2;
        float X0 = 0, X1 = 0, X2 = 0;
        float d = a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11);
        if (d != 0) {
            d = 1 / d;
            X0 = d * (b0 * (a11 * a22 - a12 * a21) - a01 * (b1 * a22 - a12 * b2) + a02 * (b1 * a21 - a11 * b2));
            X1 = d * (a00 * (b1 * a22 - a12 * b2) - b0 * (a10 * a22 - a12 * a20) + a02 * (a10 * b2 - b1 * a20));
            X2 = d * (a00 * (a11 * b2 - b1 * a21) - a01 * (a10 * b2 - b1 * a20) + b0 * (a10 * a21 - a11 * a20));
        }
        xi = -X2;
        xr = -X1;
        xc = -X0;
        if (fabsf(xi) < 0.5f && fabsf(xr) < 0.5f && fabsf(xc) < 0.5f) break;
        const float big = (float)(INT_MAX / 3);
        if (fabsf(xi) > big || fabsf(xr) > big || fabsf(xc) > big) {
            ok = false;
            break;
        }
        c += cv_round(xc);
        r += cv_round(xr);
        layer += cv_round(xi);
        if (layer < 1 || layer > L || c < kBorder || c >= g.W - kBorder || r < kBorder || r >= g.H - kBorder) {
            ok = false;
            break;
        }
    }
    if (!ok || it >= kMaxInterpSteps) return false;

    // D still holds the block of the converged (layer, r, c).
    const float c0 = D[1][1][1];
    const float cl = D[1][1][0], cr = D[1][1][2];
    const float cu = D[1][0][1], cd = D[1][2][1];
    const float pc = D[0][1][1], nc = D[2][1][1];
    const float dD0 = (cr - cl) * deriv_scale;
    const float dD1 = (cd - cu) * deriv_scale;
    const float dD2 = (nc - pc) * deriv_scale;
    float t = 0.f;
    t += dD0 * xc;
    t += dD1 * xr;
    t += dD2 * xi;
    const float contr = c0 * img_scale + t * 0.5f;
    if (fabsf(contr) * L < kp.contrastThreshold) return false;
    const float v2 = c0 * 2.f;
    const float dxx = (cr + cl - v2) * second_deriv_scale;
    const float dyy = (cd + cu - v2) * second_deriv_scale;
    const float dxy = (D[1][2][2] - D[1][2][0] - D[1][0][2] + D[1][0][0]) * cross_deriv_scale;
    const float tr = dxx + dyy;
    const float det = dxx * dyy - dxy * dxy;
    const float et = kp.edgeThreshold;
    if (det <= 0 || tr * tr * et >= (et + 1) * (et + 1) * det) return false;

    // Duplicate (same final octave/layer/r/c) -> identical keypoint: keep one.
    bit = g.bitBase + ((long)(layer - 1) * g.H + r) * g.W + c;
    const uint32_t m = 1u << (bit & 31);
    if (atomicOr(&bitmap[bit >> 5], m) & m) return false;

    k.x = ((float)c + xc) * (float)(1 << o);
    k.y = ((float)r + xr) * (float)(1 << o);
    k.octave = o + (layer << 8) + ((int)rint(((double)xi + 0.5) * 255) << 16);
    k.size = kp.sigma * pow2_via_double((layer + xi) / (float)L) * (float)(1 << o) * 2;
    k.response = fabsf(contr);
    k.o = o;
    k.layer = layer;
    k.rc = r << 16 | c;
    return true;
}

}  // namespace sift_amd
