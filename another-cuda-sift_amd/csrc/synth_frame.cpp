// Deterministic synthetic grayscale frames (SURVEY.md §8d "Synthetic frame
// generator"): low-frequency background + random anisotropic Gaussian blobs and
// rectangles (amplitude 30..200, random sign) + N(0, 3^2) noise, clamped to
// 0..255 and rounded, returned as fp32 like the reference's host image
// (/root/reference/cvUtils/ConversionImpl.hpp:8-31 converts 8U to float).
// Seed = 0x5EED0000 + frame_index through an in-repo PCG32 so the host CPU
// baseline and the GPU run see the same pixels.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <vector>

#include "sift_hip.h"

namespace {

struct Pcg32 {
    uint64_t state = 0, inc = 1;
    Pcg32(uint64_t seed, uint64_t seq) {
        inc = (seq << 1u) | 1u;
        next();
        state += seed;
        next();
    }
    uint32_t next() {
        uint64_t old = state;
        state = old * 6364136223846793005ULL + inc;
        uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((-rot) & 31));
    }
    double uniform() { return (next() >> 8) * (1.0 / 16777216.0); }
    double range(double a, double b) { return a + (b - a) * uniform(); }
    double normal() {
        double u1 = uniform(), u2 = uniform();
        if (u1 < 1e-12) u1 = 1e-12;
        return std::sqrt(-2.0 * std::log(u1)) * std::cos(2.0 * M_PI * u2);
    }
};

}  // namespace

extern "C" int sift_synth_frame(unsigned frame_index, int w, int h, float* out) {
    if (w <= 0 || h <= 0 || !out) return SIFT_HIP_ERR_INVALID;
    Pcg32 rng(0x5EED0000ull + frame_index, 0xC0FFEEull);
    std::vector<double> img((size_t)w * h);
    // Low-frequency background.
    const double fx1 = rng.range(0.5, 2.0), fy1 = rng.range(0.5, 2.0), ph1 = rng.range(0, 6.283);
    const double fx2 = rng.range(1.0, 3.0), fy2 = rng.range(1.0, 3.0), ph2 = rng.range(0, 6.283);
    for (int y = 0; y < h; y++)
        for (int x = 0; x < w; x++) {
            double u = (double)x / w, v = (double)y / h;
            img[(size_t)y * w + x] = 110.0 + 35.0 * std::sin(6.283 * (fx1 * u + 0.3 * fy1 * v) + ph1) +
                                     15.0 * std::cos(6.283 * (fx2 * u - fy2 * v) + ph2);
        }
    // One blob per ~1200 px^2: 1920 at 1920x1200 (several thousand keypoints).
    const int nblobs = (int)std::max(16.0, std::round((double)w * h / 1200.0));
    for (int b = 0; b < nblobs; b++) {
        const double cx = rng.range(0, w), cy = rng.range(0, h);
        const double amp = rng.range(30, 200) * (rng.uniform() < 0.5 ? -1.0 : 1.0);
        if (rng.uniform() < 0.3) {
            const double hw = rng.range(2, 24), hh = rng.range(2, 24);
            const int x0 = std::max(0, (int)(cx - hw)), x1 = std::min(w - 1, (int)(cx + hw));
            const int y0 = std::max(0, (int)(cy - hh)), y1 = std::min(h - 1, (int)(cy + hh));
            for (int y = y0; y <= y1; y++)
                for (int x = x0; x <= x1; x++) img[(size_t)y * w + x] += amp;
        } else {
            const double sx = rng.range(1.0, 9), sy = rng.range(1.0, 9), th = rng.range(0, 3.14159);
            const double c = std::cos(th), s = std::sin(th);
            const double ext = 3.5 * std::max(sx, sy);
            const int x0 = std::max(0, (int)(cx - ext)), x1 = std::min(w - 1, (int)(cx + ext));
            const int y0 = std::max(0, (int)(cy - ext)), y1 = std::min(h - 1, (int)(cy + ext));
            for (int y = y0; y <= y1; y++)
                for (int x = x0; x <= x1; x++) {
                    const double dx = x - cx, dy = y - cy;
                    const double u = (c * dx + s * dy) / sx, v = (-s * dx + c * dy) / sy;
                    img[(size_t)y * w + x] += amp * std::exp(-0.5 * (u * u + v * v));
                }
        }
    }
    for (size_t i = 0; i < img.size(); i++) {
        double v = std::round(img[i] + 3.0 * rng.normal());
        out[i] = (float)(v < 0 ? 0 : v > 255 ? 255 : v);
    }
    return SIFT_HIP_OK;
}
