// Device-side restatements of OpenCV's float helpers used on the SIFT path.
// Each one reproduces the operation order of OpenCV 4.x's AVX2+FMA SIMD body
// (core/mathfuncs_core.simd.hpp) with explicit __fmaf_rn, so that the HIP
// path and the CPU oracle (oracle/sift_oracle.cpp) agree bit for bit.
// Compiled with -ffp-contract=off and correctly rounded f32 div/sqrt.
#pragma once
#include <hip/hip_runtime.h>
#include <float.h>
#include <stdint.h>

namespace sift_amd {

// hal::exp32f constants (EXPTAB_SCALE = 6).  Folded in IEEE double at compile
// time exactly as the oracle folds them at run time.
constexpr double kExpPolyA0 = .9670371139572337719125840413672004409288e-2;
constexpr double kExpPrescale = 1.4426950408889634073599246810019 * (1 << 6);
constexpr double kExpPostscale = 1. / (1 << 6);
constexpr double kExpMaxVal = 3000. * (1 << 6);
constexpr float kExpA4 = (float)(1.000000000000002438532970795181890933776 / kExpPolyA0);
constexpr float kExpA3 = (float)(.6931471805521448196800669615864773144641 / kExpPolyA0);
constexpr float kExpA2 = (float)(.2402265109513301490103372422686535526573 / kExpPolyA0);
constexpr float kExpA1 = (float)(.5550339366753125211915322047004666939128e-1 / kExpPolyA0);
constexpr float kExpMin = (float)(-kExpMaxVal / kExpPrescale);
constexpr float kExpMax = (float)(kExpMaxVal / kExpPrescale);
constexpr float kExpPre = (float)kExpPrescale;
constexpr float kExpPost = (float)kExpPostscale;

// exp32f SIMD body: clamp, scale, round-half-even split, table * 2^k, degree-4
// polynomial by fma.  `tab` = expTab_f (64 floats in __constant__ memory).
__device__ __forceinline__ float cv_exp32f(float x, const float* tab) {
    x = fminf(fmaxf(x, kExpMin), kExpMax);
    x = x * kExpPre;
    float xr = __builtin_rintf(x);
    int xi = (int)xr;
    float xf = (x - xr) * kExpPost;
    float yf = tab[xi & 63];
    int t = (xi >> 6) + 127;
    t = t < 0 ? 0 : (t > 255 ? 255 : t);
    yf = yf * __int_as_float(t << 23);
    float z = xf + kExpA1;
    z = __fmaf_rn(z, xf, kExpA2);
    z = __fmaf_rn(z, xf, kExpA3);
    z = __fmaf_rn(z, xf, kExpA4);
    return z * yf;
}

// hal::fastAtan2 (v_atan_f32::compute), degrees in [0, 360).
__device__ __forceinline__ float cv_fast_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = fabsf(x), ay = fabsf(y);
    float c = fminf(ax, ay) / (fmaxf(ax, ay) + (float)DBL_EPSILON);
    float cc = c * c;
    float a = __fmaf_rn(__fmaf_rn(__fmaf_rn(cc, p7, p5), cc, p3), cc, p1) * c;
    if (!(ax >= ay)) a = 90.f - a;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// hal::magnitude32f SIMD body.  NB: __fsqrt_rn lowers to a bare v_sqrt_f32
// (~1 ulp) on gfx950; __builtin_sqrtf is the correctly rounded expansion.
__device__ __forceinline__ float cv_magnitude(float x, float y) { return __builtin_sqrtf(__fmaf_rn(x, x, y * y)); }

__device__ __forceinline__ int cv_round(float v) { return (int)__builtin_rintf(v); }
__device__ __forceinline__ int cv_floor(float v) { return (int)floorf(v); }

// powf(2, t) / cosf / sinf: one rounding from double (see oracle pow2f/cos).
__device__ __forceinline__ float pow2_via_double(float t) { return (float)exp2((double)t); }

__device__ __forceinline__ int reflect101(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - p - 2;
    return p;
}

// XCD-aware tile order.  Workgroups are dispatched round-robin over the 8
// XCDs (linear id b -> XCD b % 8) and each XCD has its own 4 MiB L2, so a
// raster tile order scatters neighbouring tiles -- whose halos overlap --
// over all eight L2s.  This bijection gives XCD k a contiguous run of tiles in
// raster order, so halo re-reads mostly hit the L2 that loaded them.
__device__ __forceinline__ int xcd_tile(int b, int ntiles) {
    const int q = ntiles >> 3, rem = ntiles & 7, k = b & 7, i = b >> 3;
    return k * q + min(k, rem) + i;
}

// Workgroup barrier ordering LDS only.  __syncthreads() also fences global
// memory, i.e. waits for every outstanding global load (vmcnt(0)) -- which
// would drain loads deliberately issued ahead across the barrier.
// Inclusive prefix sum over the 64 lanes of a wave with gfx9 DPP: row_shr
// 1/2/4/8 inside each 16-lane row, then row_bcast:15 / row_bcast:31 carry the
// row totals into the following rows (masked rows keep 0 and add nothing).
__device__ __forceinline__ int wave_incl_scan(int x) {
    x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
    x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
    x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
    x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
    x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return x;
}

// Maximum over the 64 lanes of a wave, returned to every lane: DPP row_shr
// 1/2/4/8, row_bcast:15/31 (identity -inf in masked / out-of-row lanes), then
// lane 63 broadcast through an SGPR.  No LDS round trips.
__device__ __forceinline__ float wave_max(float x) {
    const int ninf = __float_as_int(-INFINITY);
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x111, 0xf, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x112, 0xf, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x114, 0xf, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x118, 0xf, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x142, 0xa, 0xf, false)));
    x = fmaxf(x, __int_as_float(__builtin_amdgcn_update_dpp(ninf, __float_as_int(x), 0x143, 0xc, 0xf, false)));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}

__device__ __forceinline__ void lds_barrier() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

}  // namespace sift_amd
