/*
 * sift_oracle.cpp -- TEST INFRASTRUCTURE ONLY (see sift_oracle.h).
 *
 * A CPU restatement of OpenCV 4.x SIFT.  OpenCV is the third-party model the
 * reference follows ("closely follows the version by opencv",
 * /root/reference/readme.md:5); its pinned submodule (/root/reference/.gitmodules,
 * thirdparty/opencv, branch 4.x) is empty here, so every OpenCV function is
 * restated from its published source and named below as [OpenCV 4.x <file>:<func>].
 * Where the reference implements the same step, its file:line is cited too, with
 * the deviation ledger of SURVEY.md Appendix A.
 *
 * Floating-point contract (the thing the HIP path must reproduce bit-for-bit):
 *   - compiled with -ffp-contract=off; every fused multiply-add is an explicit
 *     fmaf() placed where OpenCV's AVX2+FMA3 dispatch uses v_fma/v_muladd;
 *   - transcendental helpers are OpenCV's own polynomials (exp32f, fastAtan2)
 *     restated here; cos/sin/pow go through double and round once to float.
 * Known, documented differences from a real OpenCV build are listed in DESIGN.md
 * ("Oracle: what is pinned and what is not").
 *
 * Build variants (the OpenCV-tolerance ensemble; built by
 * oracle/Makefile into separate libraries, selected in tests/oracle_binding.py):
 *   SIFT_ORACLE_VEC = 0   the pinned restatement above: every stage in the
 *                         formulas of OpenCV's SIMD bodies (the HIP path
 *                         reproduces this build bit for bit);
 *                   = 8   the AVX2 dispatch of sift.simd.hpp / core: SIMD loops
 *                         of 8 lanes with their scalar tails (orientation
 *                         histogram tail, smoothing of bins 32..35, in-place
 *                         tails of the hal calls), v_reduce_sum of v_float32x8
 *                         by two hadds, the descriptor's scalar clipped norm;
 *                   = 16  the AVX-512 (AVX512_SKX) dispatch: 16 lanes, the
 *                         512-bit v_reduce_sum;
 *   SIFT_ORACLE_CONTRACT = 1  GCC's default -ffp-contract=fast applied to
 *                         exactly the functions OpenCV compiles in the
 *                         FMA-enabled dispatch TU sift.simd.hpp
 *                         (adjustLocalExtrema with the inlined Matx33f Cramer
 *                         solve, calcOrientationHist, the peak interpolation of
 *                         findScaleSpaceExtremaT, calcSIFTDescriptor), and to
 *                         the scalar tails of the core hal calls; everything in
 *                         sift.dispatch.cpp / imgproc keeps its unfused form.
 */
#include "sift_oracle.h"

#include <algorithm>
#include <cfloat>
#include <climits>
#include <cmath>
#include <cstring>
#include <memory>
#include <utility>
#include <vector>
#ifdef _OPENMP
#include <omp.h>

#include <chrono>
#endif

#ifndef SIFT_ORACLE_VEC
#define SIFT_ORACLE_VEC 0
#endif
#ifndef SIFT_ORACLE_CONTRACT
#define SIFT_ORACLE_CONTRACT 0
#endif
#if SIFT_ORACLE_VEC != 0 && SIFT_ORACLE_VEC != 8 && SIFT_ORACLE_VEC != 16
#error "SIFT_ORACLE_VEC must be 0, 8 or 16"
#endif
// Contracted builds keep the hal helpers out of line so the caller's
// contraction setting never reaches their bodies (core's own SIMD formulas).
#if SIFT_ORACLE_CONTRACT
#define ORACLE_HAL __attribute__((noinline))
#else
#define ORACLE_HAL inline
#endif

namespace {

// [OpenCV 4.x sift.simd.hpp] constants.  Same values as the reference's
// /root/reference/sift_cuda/sift_func/SiftOps.cuh:7-13.
constexpr int   SIFT_IMG_BORDER       = 5;
constexpr int   SIFT_MAX_INTERP_STEPS = 5;
constexpr int   SIFT_ORI_HIST_BINS    = 36;
constexpr float SIFT_ORI_SIG_FCTR     = 1.5f;
constexpr float SIFT_ORI_RADIUS       = 3 * SIFT_ORI_SIG_FCTR;
constexpr float SIFT_ORI_PEAK_RATIO   = 0.8f;
constexpr int   SIFT_DESCR_WIDTH      = 4;
constexpr int   SIFT_DESCR_HIST_BINS  = 8;
constexpr float SIFT_DESCR_SCL_FCTR   = 3.f;
constexpr float SIFT_DESCR_MAG_THR    = 0.2f;
constexpr float SIFT_INT_DESCR_FCTR   = 512.f;
constexpr float SIFT_INIT_SIGMA       = 0.5f;
constexpr float SIFT_FIXPT_SCALE      = 1.f;

// cvRound / cvFloor [OpenCV 4.x core/fast_math.hpp]: round-half-even, floor.
inline int cvRoundF(float v) { return (int)lrintf(v); }
inline int cvRoundD(double v) { return (int)lrint(v); }
inline int cvFloorF(float v) { return (int)floorf(v); }

// Planes are allocated without zero-filling: every producer writes each pixel
// (in parallel loops, so the pages are first touched by the threads that fill
// them -- a serial zero-fill of fresh pages bounded the oracle's thread
// scaling).
template <class T>
struct NoInitAlloc : std::allocator<T> {
    template <class U>
    struct rebind {
        using other = NoInitAlloc<U>;
    };
    NoInitAlloc() = default;
    template <class U>
    NoInitAlloc(const NoInitAlloc<U>&) {}
    template <class U, class... A>
    void construct(U* p, A&&... a) {
        if constexpr (sizeof...(A) == 0)
            ::new ((void*)p) U;
        else
            ::new ((void*)p) U(std::forward<A>(a)...);
    }
};

struct Plane {
    int w = 0, h = 0;
    std::vector<float, NoInitAlloc<float>> d;
    void create(int W, int H) {
        w = W;
        h = H;
        d.clear();
        d.resize((size_t)W * H);
    }
    float at(int r, int c) const { return d[(size_t)r * w + c]; }
    float& at(int r, int c) { return d[(size_t)r * w + c]; }
};

// [OpenCV 4.x core:borderInterpolate] BORDER_REFLECT_101, looping for kernels
// wider than the image.  Reference equivalent: Filter.cuh:52-66 (single bounce).
inline int reflect101(int p, int len) {
    if (len == 1) return 0;
    while ((unsigned)p >= (unsigned)len) p = p < 0 ? -p : 2 * len - p - 2;
    return p;
}

// [OpenCV 4.x imgproc/smooth.dispatch.cpp: createGaussianKernels +
// getGaussianKernelBitExact].  ksize = cvRound(sigma*4*2+1)|1 for float images;
// taps from x = 1-n step 2 (twice the offset) with scale2X = -0.125/sigma^2,
// normalised by 1/(2*sum_{i<n/2} t_i + 1), mirrored, cast to float.
// Reference (6*sigma+1 taps, float expf): GaussianUtils.cc:39-68 (SURVEY A-3).
std::vector<float> gaussianTaps(double sigma) {
    int n = cvRoundD(sigma * 4 * 2 + 1) | 1;
    double scale2X = -0.125 / (sigma * sigma);
    int n2 = (n - 1) / 2;
    std::vector<double> values(n2 + 1);
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        double t = std::exp((double)(x * x) * scale2X);
        values[i] = t;
        sum += t;
    }
    sum *= 2.0;
    sum += 1.0;
    double mul1 = 1.0 / sum;
    std::vector<float> taps(n);
    for (int i = 0; i < n2; i++) {
        double t = values[i] * mul1;
        taps[i] = (float)t;
        taps[n - 1 - i] = (float)t;
    }
    taps[n2] = (float)(1.0 * mul1);
    return taps;
}

int nthreadsOr(int t) {
#ifdef _OPENMP
    return t > 0 ? t : omp_get_max_threads();
#else
    (void)t;
    return 1;
#endif
}

// [OpenCV 4.x imgproc/filter.simd.hpp] sepFilter2D(CV_32F) = RowFilter then
// SymmColumnFilter.  Row (ksize > 5, RowVec_32f_AVX): s = 0; s = fma(x[k], w[k], s)
// for k = 0..n-1 over source offsets -r..+r.  Row (ksize <= 5, SymmRowSmallVec_32f):
// s = x0*w0; s = fma(x[-k]+x[+k], w_k, s).  Column (SymmColumnVec_32f_Symm_AVX):
// s = fma(center, w_0, 0); s = fma(up_k + down_k, w_k, s) for k = 1..r.
// Reference: vertical-then-horizontal plain fma chain, Filter.cu:8-51 (SURVEY A-4).
void gaussianBlur(const Plane& src, Plane& dst, double sigma, int threads) {
    const std::vector<float> taps = gaussianTaps(sigma);
    const int n = (int)taps.size(), r = n / 2;
    const int W = src.w, H = src.h;
    Plane tmp;
    tmp.create(W, H);
    std::vector<int> xo(W + 2 * r);
    for (int i = 0; i < W + 2 * r; i++) xo[i] = reflect101(i - r, W);
#pragma omp parallel for num_threads(nthreadsOr(threads)) schedule(static)
    for (int y = 0; y < H; y++) {
        const float* S = &src.d[(size_t)y * W];
        float* T = &tmp.d[(size_t)y * W];
        if (n > 5) {
            for (int x = 0; x < W; x++) {
                float s = 0.f;
                for (int k = 0; k < n; k++) s = fmaf(S[xo[x + k]], taps[k], s);
                T[x] = s;
            }
        } else {
            for (int x = 0; x < W; x++) {
                float s = S[xo[x + r]] * taps[r];
                for (int k = 1; k <= r; k++) s = fmaf(S[xo[x + r - k]] + S[xo[x + r + k]], taps[r + k], s);
                T[x] = s;
            }
        }
    }
    dst.create(W, H);
#pragma omp parallel for num_threads(nthreadsOr(threads)) schedule(static)
    for (int y = 0; y < H; y++) {
        float* D = &dst.d[(size_t)y * W];
        const float* C = &tmp.d[(size_t)y * W];
        for (int x = 0; x < W; x++) D[x] = fmaf(C[x], taps[r], 0.f);
        for (int k = 1; k <= r; k++) {
            const float* U = &tmp.d[(size_t)reflect101(y - k, H) * W];
            const float* B = &tmp.d[(size_t)reflect101(y + k, H) * W];
            for (int x = 0; x < W; x++) D[x] = fmaf(B[x] + U[x], taps[r + k], D[x]);
        }
    }
}

// [OpenCV 4.x imgproc/resize.cpp] resize(INTER_LINEAR) to exactly 2x on float:
// fx = (float)((dx+0.5)*0.5-0.5), sx = cvFloor(fx), clamp to the edge with
// fx = 0; horizontal t = S[sx]*(1-fx) + S[sx+1]*fx, vertical
// D = S0*b0 + S1*b1 (VResizeLinearVec_32f, v_muladd on the SSE baseline = mul+add).
// Exact for integer-valued inputs.  Reference: Resize.cu:6-64 with the wrong
// target size (SURVEY A-6).
void upsample2x(const Plane& src, Plane& dst, int threads) {
    const int W = src.w, H = src.h, DW = W * 2, DH = H * 2;
    std::vector<int> xs(DW), ys(DH);
    std::vector<float> ax(DW * 2), ay(DH * 2);
    auto coeffs = [](int d, int slen, int& s, float* a) {
        float f = (float)((d + 0.5) * 0.5 - 0.5);
        int si = cvFloorF(f);
        f -= (float)si;
        if (si < 0) { f = 0; si = 0; }
        if (si >= slen - 1) { f = 0; si = slen - 1; }
        s = si;
        a[0] = 1.f - f;
        a[1] = f;
    };
    for (int d = 0; d < DW; d++) coeffs(d, W, xs[d], &ax[2 * d]);
    for (int d = 0; d < DH; d++) coeffs(d, H, ys[d], &ay[2 * d]);
    Plane hrow;
    hrow.create(DW, H);
#pragma omp parallel for num_threads(nthreadsOr(threads)) schedule(static)
    for (int y = 0; y < H; y++)
        for (int x = 0; x < DW; x++) {
            int sx = xs[x];
            int sx1 = std::min(sx + 1, W - 1);
            hrow.at(y, x) = src.at(y, sx) * ax[2 * x] + src.at(y, sx1) * ax[2 * x + 1];
        }
    dst.create(DW, DH);
#pragma omp parallel for num_threads(nthreadsOr(threads)) schedule(static)
    for (int y = 0; y < DH; y++) {
        int sy = ys[y], sy1 = std::min(sy + 1, H - 1);
        for (int x = 0; x < DW; x++) dst.at(y, x) = hrow.at(sy, x) * ay[2 * y] + hrow.at(sy1, x) * ay[2 * y + 1];
    }
}

// ---------------------------------------------------------------------------
// OpenCV's own transcendental helpers, restated (core/mathfuncs_core.simd.hpp).
// ---------------------------------------------------------------------------
const double EXPPOLY_32F_A0 = .9670371139572337719125840413672004409288e-2;
const double exp_prescale   = 1.4426950408889634073599246810019 * (1 << 6);
const double exp_postscale  = 1. / (1 << 6);
const double exp_max_val    = 3000. * (1 << 6);

struct ExpTables {
    float tab[64];
    float A1, A2, A3, A4, minval, maxval, prescale, postscale;
    ExpTables() {
        for (int j = 0; j < 64; j++) tab[j] = (float)(std::exp2((double)j / 64.0) * EXPPOLY_32F_A0);
        A4 = (float)(1.000000000000002438532970795181890933776 / EXPPOLY_32F_A0);
        A3 = (float)(.6931471805521448196800669615864773144641 / EXPPOLY_32F_A0);
        A2 = (float)(.2402265109513301490103372422686535526573 / EXPPOLY_32F_A0);
        A1 = (float)(.5550339366753125211915322047004666939128e-1 / EXPPOLY_32F_A0);
        minval = (float)(-exp_max_val / exp_prescale);
        maxval = (float)(exp_max_val / exp_prescale);
        prescale = (float)exp_prescale;
        postscale = (float)exp_postscale;
    }
};
const ExpTables& expTables() {
    static ExpTables t;
    return t;
}

// [OpenCV 4.x hal::exp32f] SIMD body (v_round, v_fma) applied to every element.
// (Its scalar tail, ((x0 + A1)*x0 + A2)*x0 ..., contracted by an FMA build,
// gives the same bits, so every variant uses this form.)
ORACLE_HAL float cvExp32f(float x) {
    const ExpTables& T = expTables();
    x = std::min(std::max(x, T.minval), T.maxval);
    x = x * T.prescale;
    int xi = (int)lrintf(x);
    float xf = (x - (float)xi) * T.postscale;
    float yf = T.tab[xi & 63];
    int t = (xi >> 6) + 127;
    t = std::min(std::max(t, 0), 255);
    uint32_t bits = (uint32_t)t << 23;
    float p2;
    std::memcpy(&p2, &bits, 4);
    yf = yf * p2;
    float z = xf + T.A1;
    z = fmaf(z, xf, T.A2);
    z = fmaf(z, xf, T.A3);
    z = fmaf(z, xf, T.A4);
    return z * yf;
}

// [OpenCV 4.x hal::fastAtan2 / v_atan_f32::compute], degrees.
ORACLE_HAL float cvFastAtan2(float y, float x) {
    static const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    static const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    static const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    static const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = std::fabs(x), ay = std::fabs(y);
    float c = std::min(ax, ay) / (std::max(ax, ay) + (float)DBL_EPSILON);
    float cc = c * c;
    float a = fmaf(fmaf(fmaf(cc, p7, p5), cc, p3), cc, p1) * c;
    if (!(ax >= ay)) a = 90.f - a;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}

// [OpenCV 4.x hal::magnitude32f] SIMD body: sqrt(fma(x, x, y*y)).
ORACLE_HAL float cvMagnitude(float x, float y) { return std::sqrt(fmaf(x, x, y * y)); }

#if SIFT_ORACLE_VEC
#if SIFT_ORACLE_CONTRACT
#pragma GCC push_options
#pragma GCC optimize("fp-contract=fast")
#endif
// [OpenCV 4.x core mathfuncs_core.simd.hpp: atan_f32] -- the scalar loop
// fastAtan32f runs when a call has fewer than 2 vectors of elements (the SIMD
// loop re-processes an overlapped last block otherwise).  Written as OpenCV
// writes it: a contracting build fuses `90.f - poly*c` into one fma, which the
// SIMD body (a = poly*c; 90 - a) does not.
__attribute__((noinline)) float cvFastAtan2Scalar(float y, float x) {
    static const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    static const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    static const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    static const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    float ax = std::fabs(x), ay = std::fabs(y);
    float a, c, c2;
    if (ax >= ay) {
        c = ay / (ax + (float)DBL_EPSILON);
        c2 = c * c;
        a = (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    } else {
        c = ax / (ay + (float)DBL_EPSILON);
        c2 = c * c;
        a = 90.f - (((p7 * c2 + p5) * c2 + p3) * c2 + p1) * c;
    }
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}
#if SIFT_ORACLE_CONTRACT
#pragma GCC pop_options
#endif

// hal::fastAtan2 over an array of n elements: SIMD body for n >= 2 vectors.
void cvFastAtan2Array(const float* Y, const float* X, float* ori, int n) {
    const bool simd = n >= 2 * SIFT_ORACLE_VEC;
    for (int k = 0; k < n; k++) ori[k] = simd ? cvFastAtan2(Y[k], X[k]) : cvFastAtan2Scalar(Y[k], X[k]);
}

// v_reduce_sum(v_float32) of the dispatch width.
float reduceSum(const float* a) {
#if SIFT_ORACLE_VEC == 8
    // intrin_avx.hpp: two _mm256_hadd_ps, then low + high 128-bit halves.
    return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
#else
    // intrin_avx512.hpp: 256-bit halves added, 128-bit halves added, two hadds.
    float h[8], q[4];
    for (int i = 0; i < 8; i++) h[i] = a[i] + a[i + 8];
    for (int i = 0; i < 4; i++) q[i] = h[i] + h[i + 4];
    return (q[0] + q[1]) + (q[2] + q[3]);
#endif
}
#endif  // SIFT_ORACLE_VEC

inline float pow2f(float t) { return (float)std::exp2((double)t); }

// ---------------------------------------------------------------------------
struct Keypoint {
    float x, y, size, angle, response;
    int octave;
};

// [OpenCV 4.x features2d/src/keypoint.cpp: KeypointGreater]
bool keypointGreater(const Keypoint& a, const Keypoint& b) {
    if (a.x != b.x) return a.x > b.x;
    if (a.y != b.y) return a.y > b.y;
    if (a.size != b.size) return a.size > b.size;
    if (a.angle != b.angle) return a.angle > b.angle;
    if (a.response != b.response) return a.response > b.response;
    if (a.octave != b.octave) return a.octave > b.octave;
    return false;
}

struct Params {
    int nfeatures, L, firstOctave, nOctaves;
    double contrastThreshold, edgeThreshold, sigma;
};

Params toParams(const sift_oracle_params* p) {
    sift_oracle_params d;
    sift_oracle_default_params(&d);
    if (!p) p = &d;
    return Params{p->nfeatures, p->nOctaveLayers, p->firstOctave, p->nOctaves,
                  p->contrastThreshold, p->edgeThreshold, p->sigma};
}

int autoOctaves(int w, int h, const Params& P) {
    // [OpenCV 4.x sift.dispatch.cpp: detectAndCompute]
    // nOctaves = cvRound(log(min(base.cols, base.rows))/log(2) - 2) - firstOctave.
    // Reference: Detector.hh:27 always uses the doubled size.
    if (P.nOctaves > 0) return P.nOctaves;
    int bw = P.firstOctave < 0 ? w * 2 : w, bh = P.firstOctave < 0 ? h * 2 : h;
    return cvRoundD(std::log((double)std::min(bw, bh)) / std::log(2.) - 2) - P.firstOctave;
}

// Wall time per stage of the last detect_and_compute call (bench.py's CPU
// baseline reports where the threads go): initial image, Gaussian pyramid, DoG,
// 3x3x3 candidates, keypoints (refine + orientation + dedupe + retainBest),
// descriptors.
double g_stage_ms[6];
struct StageClock {
    std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
    void mark(int i) {
        const auto n = std::chrono::steady_clock::now();
        g_stage_ms[i] = std::chrono::duration<double, std::milli>(n - t).count();
        t = n;
    }
};

class Sift {
public:
    Sift(const Params& P, int threads) : P_(P), threads_(threads) {}

    // [OpenCV 4.x sift.simd.hpp: createInitialImage].  Reference:
    // Detector.cu:41-60 + 235-260 (SURVEY A-2: sigma_diff always uses the x4 term).
    void initialImage(const Plane& img, Plane& base) const {
        float sigma = (float)P_.sigma;
        if (P_.firstOctave < 0) {
            float sig_diff = sqrtf(std::max(sigma * sigma - SIFT_INIT_SIGMA * SIFT_INIT_SIGMA * 4, 0.01f));
            Plane dbl;
            upsample2x(img, dbl, threads_);
            gaussianBlur(dbl, base, sig_diff, threads_);
        } else {
            float sig_diff = sqrtf(std::max(sigma * sigma - SIFT_INIT_SIGMA * SIFT_INIT_SIGMA, 0.01f));
            gaussianBlur(img, base, sig_diff, threads_);
        }
    }

    // [OpenCV 4.x sift.simd.hpp: buildGaussianPyramid].  Reference:
    // Detector.cu:62-87 (sigmas) + 262-310 (bilinear 1/2 resize, SURVEY A-5).
    void gaussianPyramid(const Plane& base, int nOctaves, std::vector<Plane>& pyr) const {
        const int L = P_.L;
        std::vector<double> sig(L + 3);
        sig[0] = P_.sigma;
        double k = std::pow(2., 1. / L);
        for (int i = 1; i < L + 3; i++) {
            double sig_prev = std::pow(k, (double)(i - 1)) * P_.sigma;
            double sig_total = sig_prev * k;
            sig[i] = std::sqrt(sig_total * sig_total - sig_prev * sig_prev);
        }
        pyr.resize(nOctaves * (L + 3));  // planes kept from the last call keep their pages (see dogPyramid)
        for (int o = 0; o < nOctaves; o++)
            for (int i = 0; i < L + 3; i++) {
                Plane& dst = pyr[o * (L + 3) + i];
                if (o == 0 && i == 0) {
                    dst = base;
                } else if (i == 0) {
                    // resize(src, dst, Size(cols/2, rows/2), 0, 0, INTER_NEAREST): pixel (2y, 2x).
                    const Plane& src = pyr[(o - 1) * (L + 3) + L];
                    dst.create(src.w / 2, src.h / 2);
#pragma omp parallel for num_threads(nthreadsOr(threads_)) schedule(static)
                    for (int y = 0; y < dst.h; y++)
                        for (int x = 0; x < dst.w; x++) dst.at(y, x) = src.at(2 * y, 2 * x);
                } else {
                    gaussianBlur(pyr[o * (L + 3) + i - 1], dst, sig[i], threads_);
                }
            }
    }

    // [OpenCV 4.x sift.simd.hpp: buildDoGPyramidComputer] dst = G[i+1] - G[i].
    // Reference: MatOps.cu:10-37.
    // The planes of `dogpyr` are reused across calls (the caller keeps it):
    // fresh 9 MB allocations every frame were first touched by the threads of
    // the loop below, and their concurrent page faults made this stage slower
    // at 16 threads than at 4 (4.2 -> 5.3 ms per C2 frame, round-5 review).
    void dogPyramid(const std::vector<Plane>& gpyr, std::vector<Plane>& dogpyr) const {
        const int L = P_.L, nOct = (int)gpyr.size() / (L + 3);
        dogpyr.resize(nOct * (L + 2));
        for (int o = 0; o < nOct; o++)
            for (int i = 0; i < L + 2; i++) {
                const Plane& a = gpyr[o * (L + 3) + i];
                const Plane& b = gpyr[o * (L + 3) + i + 1];
                Plane& d = dogpyr[o * (L + 2) + i];
                d.create(a.w, a.h);
                const long np = (long)a.d.size();
#pragma omp parallel for num_threads(nthreadsOr(threads_)) schedule(static)
                for (long k = 0; k < np; k++) d.d[k] = b.d[k] - a.d[k];
            }
    }

    // [OpenCV 4.x sift.simd.hpp: findScaleSpaceExtremaComputer, candidate test].
    // Reference test is identical: MatOps.cu:125-143 with threshold Detector.cu:362.
    bool isExtremum(const std::vector<Plane>& dog, int idx, int r, int c, int threshold) const {
        const Plane& img = dog[idx];
        const Plane& prev = dog[idx - 1];
        const Plane& next = dog[idx + 1];
        float val = img.at(r, c);
        if (!(std::fabs(val) > (float)threshold)) return false;
        if (val > 0) {
            for (const Plane* p : {&img, &prev, &next})
                for (int dy = -1; dy <= 1; dy++)
                    for (int dx = -1; dx <= 1; dx++)
                        if (!(val >= p->at(r + dy, c + dx))) return false;
        } else {
            for (const Plane* p : {&img, &prev, &next})
                for (int dy = -1; dy <= 1; dy++)
                    for (int dx = -1; dx <= 1; dx++)
                        if (!(val <= p->at(r + dy, c + dx))) return false;
        }
        return true;
    }

    int threshold() const {
        return (int)std::floor(0.5 * P_.contrastThreshold / P_.L * 255 * SIFT_FIXPT_SCALE);
    }

    // ---- sift.simd.hpp: compiled in OpenCV's FMA-enabled dispatch TU (variants:
    // contracted like GCC's default -ffp-contract=fast, see the header) ----
#if SIFT_ORACLE_CONTRACT
#pragma GCC push_options
#pragma GCC optimize("fp-contract=fast")
#endif
    // [OpenCV 4.x sift.simd.hpp: adjustLocalExtrema] with Matx33f::solve(DECOMP_LU)
    // = Matx_FastSolveOp<float,3,1> (Cramer's rule, det via Matx_DetOp<float,3>).
    // Reference: SiftOps.cu:6-208 (Gaussian elimination, no sub-pixel offset in the
    // output, different octave packing: SURVEY A-8).
    bool adjustLocalExtrema(const std::vector<Plane>& dog, Keypoint& kpt, int octv, int& layer,
                            int& r, int& c) const {
        const int L = P_.L;
        const float contrastThreshold = (float)P_.contrastThreshold;
        const float edgeThreshold = (float)P_.edgeThreshold;
        const float sigma = (float)P_.sigma;
        const float img_scale = 1.f / (255 * SIFT_FIXPT_SCALE);
        const float deriv_scale = img_scale * 0.5f;
        const float second_deriv_scale = img_scale;
        const float cross_deriv_scale = img_scale * 0.25f;

        float xi = 0, xr = 0, xc = 0, contr = 0;
        int i = 0;
        for (; i < SIFT_MAX_INTERP_STEPS; i++) {
            int idx = octv * (L + 2) + layer;
            const Plane& img = dog[idx];
            const Plane& prev = dog[idx - 1];
            const Plane& next = dog[idx + 1];
            float dD0 = (img.at(r, c + 1) - img.at(r, c - 1)) * deriv_scale;
            float dD1 = (img.at(r + 1, c) - img.at(r - 1, c)) * deriv_scale;
            float dD2 = (next.at(r, c) - prev.at(r, c)) * deriv_scale;
            float v2 = img.at(r, c) * 2;
            float dxx = (img.at(r, c + 1) + img.at(r, c - 1) - v2) * second_deriv_scale;
            float dyy = (img.at(r + 1, c) + img.at(r - 1, c) - v2) * second_deriv_scale;
            float dss = (next.at(r, c) + prev.at(r, c) - v2) * second_deriv_scale;
            float dxy = (img.at(r + 1, c + 1) - img.at(r + 1, c - 1) - img.at(r - 1, c + 1) + img.at(r - 1, c - 1)) *
                        cross_deriv_scale;
            float dxs = (next.at(r, c + 1) - next.at(r, c - 1) - prev.at(r, c + 1) + prev.at(r, c - 1)) *
                        cross_deriv_scale;
            float dys = (next.at(r + 1, c) - next.at(r - 1, c) - prev.at(r + 1, c) + prev.at(r - 1, c)) *
                        cross_deriv_scale;
            // H = [dxx dxy dxs; dxy dyy dys; dxs dys dss], b = dD.
            const float a00 = dxx, a01 = dxy, a02 = dxs, a10 = dxy, a11 = dyy, a12 = dys, a20 = dxs, a21 = dys,
                        a22 = dss;
            const float b0 = dD0, b1 = dD1, b2 = dD2;
            float X0 = 0, X1 = 0, X2 = 0;
            float det = a00 * (a11 * a22 - a21 * a12) - a01 * (a10 * a22 - a20 * a12) + a02 * (a10 * a21 - a20 * a11);
            float d = (float)(double)det;
            if (d != 0) {
                d = 1 / d;
                X0 = d * (b0 * (a11 * a22 - a12 * a21) - a01 * (b1 * a22 - a12 * b2) + a02 * (b1 * a21 - a11 * b2));
                X1 = d * (a00 * (b1 * a22 - a12 * b2) - b0 * (a10 * a22 - a12 * a20) + a02 * (a10 * b2 - b1 * a20));
                X2 = d * (a00 * (a11 * b2 - b1 * a21) - a01 * (a10 * b2 - b1 * a20) + b0 * (a10 * a21 - a11 * a20));
            }
            xi = -X2;
            xr = -X1;
            xc = -X0;
            if (std::fabs(xi) < 0.5f && std::fabs(xr) < 0.5f && std::fabs(xc) < 0.5f) break;
            if (std::fabs(xi) > (float)(INT_MAX / 3) || std::fabs(xr) > (float)(INT_MAX / 3) ||
                std::fabs(xc) > (float)(INT_MAX / 3))
                return false;
            c += cvRoundF(xc);
            r += cvRoundF(xr);
            layer += cvRoundF(xi);
            if (layer < 1 || layer > L || c < SIFT_IMG_BORDER || c >= img.w - SIFT_IMG_BORDER ||
                r < SIFT_IMG_BORDER || r >= img.h - SIFT_IMG_BORDER)
                return false;
        }
        if (i >= SIFT_MAX_INTERP_STEPS) return false;
        {
            int idx = octv * (L + 2) + layer;
            const Plane& img = dog[idx];
            const Plane& prev = dog[idx - 1];
            const Plane& next = dog[idx + 1];
            float dD0 = (img.at(r, c + 1) - img.at(r, c - 1)) * deriv_scale;
            float dD1 = (img.at(r + 1, c) - img.at(r - 1, c)) * deriv_scale;
            float dD2 = (next.at(r, c) - prev.at(r, c)) * deriv_scale;
            float t = 0.f;
            t += dD0 * xc;
            t += dD1 * xr;
            t += dD2 * xi;
            contr = img.at(r, c) * img_scale + t * 0.5f;
            if (std::fabs(contr) * L < contrastThreshold) return false;
            float v2 = img.at(r, c) * 2.f;
            float dxx = (img.at(r, c + 1) + img.at(r, c - 1) - v2) * second_deriv_scale;
            float dyy = (img.at(r + 1, c) + img.at(r - 1, c) - v2) * second_deriv_scale;
            float dxy = (img.at(r + 1, c + 1) - img.at(r + 1, c - 1) - img.at(r - 1, c + 1) + img.at(r - 1, c - 1)) *
                        cross_deriv_scale;
            float tr = dxx + dyy;
            float det = dxx * dyy - dxy * dxy;
            if (det <= 0 || tr * tr * edgeThreshold >= (edgeThreshold + 1) * (edgeThreshold + 1) * det) return false;
        }
        kpt.x = ((float)c + xc) * (float)(1 << octv);
        kpt.y = ((float)r + xr) * (float)(1 << octv);
        kpt.octave = octv + (layer << 8) + (cvRoundD(((double)xi + 0.5) * 255) << 16);
        kpt.size = sigma * pow2f((layer + xi) / (float)L) * (float)(1 << octv) * 2;
        kpt.response = std::fabs(contr);
        return true;
    }

    // [OpenCV 4.x sift.simd.hpp: calcOrientationHist].  Sequential accumulation
    // in (i, j) raster order; exp32f / fastAtan2 / magnitude32f as restated above.
    // Reference: SiftOps.cu:237-376 computes this on the DoG plane with floor bins
    // and no peak interpolation (SURVEY A-9).
    float calcOrientationHist(const Plane& img, int px, int py, int radius, float sigma, float* hist) const {
        const int n = SIFT_ORI_HIST_BINS;
        float expf_scale = -1.f / (2.f * sigma * sigma);
        float temp[SIFT_ORI_HIST_BINS + 4] = {0};
        float* temphist = temp + 2;
#if SIFT_ORACLE_VEC
        // OpenCV's structure: gather X, Y, W over the window, hal::exp32f (in
        // place), hal::fastAtan2, hal::magnitude32f (Mag = X, in place), then
        // the histogram: SIMD blocks add the rounded w*mag, the scalar tail
        // (len % VEC samples) does temphist[bin] += W[k]*Mag[k] (one fma in a
        // contracting build).
        const int maxlen = (2 * radius + 1) * (2 * radius + 1);
        std::vector<float> X(maxlen), Y(maxlen), W(maxlen), Ori(maxlen);
        int len = 0;
        for (int i = -radius; i <= radius; i++) {
            int y = py + i;
            if (y <= 0 || y >= img.h - 1) continue;
            for (int j = -radius; j <= radius; j++) {
                int x = px + j;
                if (x <= 0 || x >= img.w - 1) continue;
                X[len] = img.at(y, x + 1) - img.at(y, x - 1);
                Y[len] = img.at(y - 1, x) - img.at(y + 1, x);
                W[len] = (float)(i * i + j * j) * expf_scale;
                len++;
            }
        }
        for (int k = 0; k < len; k++) W[k] = cvExp32f(W[k]);
        cvFastAtan2Array(Y.data(), X.data(), Ori.data(), len);
        for (int k = 0; k < len; k++) X[k] = cvMagnitude(X[k], Y[k]);
        const float* Mag = X.data();
        const int simd_end = len - len % SIFT_ORACLE_VEC;
        int k = 0;
        for (; k < simd_end; k++) {
            int bin = cvRoundF((n / 360.f) * Ori[k]);
            if (bin >= n) bin -= n;
            if (bin < 0) bin += n;
            volatile float wm = W[k] * Mag[k];  // v_mul: rounded before the add
            temphist[bin] += wm;
        }
        for (; k < len; k++) {
            int bin = cvRoundF((n / 360.f) * Ori[k]);
            if (bin >= n) bin -= n;
            if (bin < 0) bin += n;
            temphist[bin] += W[k] * Mag[k];
        }
        temphist[-1] = temphist[n - 1];
        temphist[-2] = temphist[n - 2];
        temphist[n] = temphist[0];
        temphist[n + 1] = temphist[1];
        int i = 0;
        for (; i <= n - SIFT_ORACLE_VEC; i += SIFT_ORACLE_VEC)  // v_fma body
            for (int v = i; v < i + SIFT_ORACLE_VEC; v++)
                hist[v] = fmaf(temphist[v - 2] + temphist[v + 2], 1.f / 16.f,
                               fmaf(temphist[v - 1] + temphist[v + 1], 4.f / 16.f, temphist[v] * (6.f / 16.f)));
        for (; i < n; i++)  // scalar tail (bins 32..35), as OpenCV writes it
            hist[i] = (temphist[i - 2] + temphist[i + 2]) * (1.f / 16.f) +
                      (temphist[i - 1] + temphist[i + 1]) * (4.f / 16.f) + temphist[i] * (6.f / 16.f);
        float vmax = hist[0];
        for (int b = 1; b < n; b++) vmax = std::max(vmax, hist[b]);
        return vmax;
#endif
        for (int i = -radius; i <= radius; i++) {
            int y = py + i;
            if (y <= 0 || y >= img.h - 1) continue;
            for (int j = -radius; j <= radius; j++) {
                int x = px + j;
                if (x <= 0 || x >= img.w - 1) continue;
                float dx = img.at(y, x + 1) - img.at(y, x - 1);
                float dy = img.at(y - 1, x) - img.at(y + 1, x);
                float w = cvExp32f((float)(i * i + j * j) * expf_scale);
                float ori = cvFastAtan2(dy, dx);
                float mag = cvMagnitude(dx, dy);
                int bin = cvRoundF((n / 360.f) * ori);
                if (bin >= n) bin -= n;
                if (bin < 0) bin += n;
                temphist[bin] += w * mag;
            }
        }
        temphist[-1] = temphist[n - 1];
        temphist[-2] = temphist[n - 2];
        temphist[n] = temphist[0];
        temphist[n + 1] = temphist[1];
        for (int i = 0; i < n; i++)
            hist[i] = fmaf(temphist[i - 2] + temphist[i + 2], 1.f / 16.f,
                           fmaf(temphist[i - 1] + temphist[i + 1], 4.f / 16.f, temphist[i] * (6.f / 16.f)));
        float maxval = hist[0];
        for (int i = 1; i < n; i++) maxval = std::max(maxval, hist[i]);
        return maxval;
    }

    // [OpenCV 4.x sift.simd.hpp: findScaleSpaceExtremaComputer::operator()] body
    // after the candidate test: refine, orientation, one keypoint per peak.
    void processCandidate(const std::vector<Plane>& gpyr, const std::vector<Plane>& dog, int o, int i, int r, int c,
                          std::vector<Keypoint>& out) const {
        const int L = P_.L, n = SIFT_ORI_HIST_BINS;
        Keypoint kpt{};
        int r1 = r, c1 = c, layer = i;
        if (!adjustLocalExtrema(dog, kpt, o, layer, r1, c1)) return;
        float scl_octv = kpt.size * 0.5f / (float)(1 << o);
        float hist[SIFT_ORI_HIST_BINS];
        float omax = calcOrientationHist(gpyr[o * (L + 3) + layer], c1, r1, cvRoundF(SIFT_ORI_RADIUS * scl_octv),
                                         SIFT_ORI_SIG_FCTR * scl_octv, hist);
        float mag_thr = (float)(omax * SIFT_ORI_PEAK_RATIO);
        for (int j = 0; j < n; j++) {
            int l = j > 0 ? j - 1 : n - 1;
            int r2 = j < n - 1 ? j + 1 : 0;
            if (hist[j] > hist[l] && hist[j] > hist[r2] && hist[j] >= mag_thr) {
                float bin = j + 0.5f * (hist[l] - hist[r2]) / (hist[l] - 2 * hist[j] + hist[r2]);
                bin = bin < 0 ? n + bin : bin >= n ? bin - n : bin;
                kpt.angle = 360.f - (float)((360.f / n) * bin);
                if (std::fabs(kpt.angle - 360.f) < FLT_EPSILON) kpt.angle = 0.f;
                out.push_back(kpt);
            }
        }
    }

    // Rows of a plane are scanned in parallel (OpenCV's parallel_for_ over
    // rows, findScaleSpaceExtremaComputer) and concatenated in row order, so
    // the list is the sequential scan's.
    void candidates(const std::vector<Plane>& dog, int nOct, std::vector<int>& quads) const {
        const int L = P_.L, thr = threshold();
        for (int o = 0; o < nOct; o++)
            for (int i = 1; i <= L; i++) {
                const int idx = o * (L + 2) + i;
                const Plane& img = dog[idx];
                const int r0 = SIFT_IMG_BORDER, r1 = img.h - SIFT_IMG_BORDER;
                if (r1 <= r0) continue;
                std::vector<std::vector<int>> rows(r1 - r0);
#pragma omp parallel for num_threads(nthreadsOr(threads_)) schedule(static)
                for (int r = r0; r < r1; r++)
                    for (int c = SIFT_IMG_BORDER; c < img.w - SIFT_IMG_BORDER; c++)
                        if (isExtremum(dog, idx, r, c, thr)) rows[r - r0].insert(rows[r - r0].end(), {o, i, r, c});
                for (auto& v : rows) quads.insert(quads.end(), v.begin(), v.end());
            }
    }

    // [OpenCV 4.x sift.simd.hpp: calcSIFTDescriptor].  Reference:
    // SiftOps.cu:389-623 (modff truncation, x<cols bound, half(x512) output,
    // SURVEY A-10).
    void calcSIFTDescriptor(const Plane& img, float ptfx, float ptfy, float ori, float scl, float* dst) const {
        const int d = SIFT_DESCR_WIDTH, n = SIFT_DESCR_HIST_BINS;
        int ptx = cvRoundF(ptfx), pty = cvRoundF(ptfy);
        float arg = ori * (float)(M_PI / 180);
        float cos_t = (float)std::cos((double)arg);
        float sin_t = (float)std::sin((double)arg);
        float bins_per_rad = n / 360.f;
        float exp_scale = -1.f / (d * d * 0.5f);
        float hist_width = SIFT_DESCR_SCL_FCTR * scl;
        int radius = cvRoundF(hist_width * 1.4142135623730951f * (float)(d + 1) * 0.5f);
        radius = std::min(radius, (int)std::sqrt(((double)img.w) * img.w + ((double)img.h) * img.h));
        cos_t /= hist_width;
        sin_t /= hist_width;
        const int rows = img.h, cols = img.w;
        float hist[(SIFT_DESCR_WIDTH + 2) * (SIFT_DESCR_WIDTH + 2) * (SIFT_DESCR_HIST_BINS + 2)] = {0};
#if SIFT_ORACLE_VEC
        // OpenCV's structure: gather the window's samples (rotated bins, X, Y and
        // the Gaussian weight argument) in scalar code, then hal::exp32f (in
        // place), hal::fastAtan2, hal::magnitude32f (Mag = Y, in place), then the
        // trilinear accumulation (its SIMD body and scalar tail give the same
        // bits: every product there has a second use, so nothing contracts).
        const int maxlen = (2 * radius + 1) * (2 * radius + 1);
        std::vector<float> X(maxlen), Y(maxlen), W(maxlen), RB(maxlen), CB(maxlen), Ori(maxlen);
        int len = 0;
        for (int i = -radius; i <= radius; i++)
            for (int j = -radius; j <= radius; j++) {
                float c_rot = j * cos_t - i * sin_t;
                float r_rot = j * sin_t + i * cos_t;
                float rbin = r_rot + d / 2 - 0.5f;
                float cbin = c_rot + d / 2 - 0.5f;
                int r = pty + i, c = ptx + j;
                if (rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < rows - 1 && c > 0 &&
                    c < cols - 1) {
                    X[len] = img.at(r, c + 1) - img.at(r, c - 1);
                    Y[len] = img.at(r - 1, c) - img.at(r + 1, c);
                    RB[len] = rbin;
                    CB[len] = cbin;
                    W[len] = (c_rot * c_rot + r_rot * r_rot) * exp_scale;
                    len++;
                }
            }
        for (int k = 0; k < len; k++) W[k] = cvExp32f(W[k]);
        cvFastAtan2Array(Y.data(), X.data(), Ori.data(), len);
        for (int k = 0; k < len; k++) Y[k] = cvMagnitude(X[k], Y[k]);
        for (int k = 0; k < len; k++) {
            float rbin = RB[k], cbin = CB[k];
            float obin = (Ori[k] - ori) * bins_per_rad;
            float mag = Y[k] * W[k];
            int r0 = cvFloorF(rbin), c0 = cvFloorF(cbin), o0 = cvFloorF(obin);
            rbin -= (float)r0;
            cbin -= (float)c0;
            obin -= (float)o0;
            if (o0 < 0) o0 += n;
            if (o0 >= n) o0 -= n;
            float v_r1 = mag * rbin, v_r0 = mag - v_r1;
            float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
            float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
            float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
            float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
            float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
            float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
            int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
            hist[idx] += v_rco000;
            hist[idx + 1] += v_rco001;
            hist[idx + (n + 2)] += v_rco010;
            hist[idx + (n + 3)] += v_rco011;
            hist[idx + (d + 2) * (n + 2)] += v_rco100;
            hist[idx + (d + 2) * (n + 2) + 1] += v_rco101;
            hist[idx + (d + 3) * (n + 2)] += v_rco110;
            hist[idx + (d + 3) * (n + 2) + 1] += v_rco111;
        }
        if (false)
#endif
        for (int i = -radius; i <= radius; i++)
            for (int j = -radius; j <= radius; j++) {
                float c_rot = (float)j * cos_t - (float)i * sin_t;
                float r_rot = (float)j * sin_t + (float)i * cos_t;
                float rbin = r_rot + (float)(d / 2) - 0.5f;
                float cbin = c_rot + (float)(d / 2) - 0.5f;
                int r = pty + i, c = ptx + j;
                if (rbin > -1 && rbin < d && cbin > -1 && cbin < d && r > 0 && r < rows - 1 && c > 0 &&
                    c < cols - 1) {
                    float dx = img.at(r, c + 1) - img.at(r, c - 1);
                    float dy = img.at(r - 1, c) - img.at(r + 1, c);
                    float wgt = cvExp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale);
                    float gori = cvFastAtan2(dy, dx);
                    float gmag = cvMagnitude(dx, dy);
                    float obin = (gori - ori) * bins_per_rad;
                    float mag = gmag * wgt;
                    int r0 = cvFloorF(rbin), c0 = cvFloorF(cbin), o0 = cvFloorF(obin);
                    rbin -= (float)r0;
                    cbin -= (float)c0;
                    obin -= (float)o0;
                    if (o0 < 0) o0 += n;
                    if (o0 >= n) o0 -= n;
                    float v_r1 = mag * rbin, v_r0 = mag - v_r1;
                    float v_rc11 = v_r1 * cbin, v_rc10 = v_r1 - v_rc11;
                    float v_rc01 = v_r0 * cbin, v_rc00 = v_r0 - v_rc01;
                    float v_rco111 = v_rc11 * obin, v_rco110 = v_rc11 - v_rco111;
                    float v_rco101 = v_rc10 * obin, v_rco100 = v_rc10 - v_rco101;
                    float v_rco011 = v_rc01 * obin, v_rco010 = v_rc01 - v_rco011;
                    float v_rco001 = v_rc00 * obin, v_rco000 = v_rc00 - v_rco001;
                    int idx = ((r0 + 1) * (d + 2) + c0 + 1) * (n + 2) + o0;
                    hist[idx] += v_rco000;
                    hist[idx + 1] += v_rco001;
                    hist[idx + (n + 2)] += v_rco010;
                    hist[idx + (n + 3)] += v_rco011;
                    hist[idx + (d + 2) * (n + 2)] += v_rco100;
                    hist[idx + (d + 2) * (n + 2) + 1] += v_rco101;
                    hist[idx + (d + 3) * (n + 2)] += v_rco110;
                    hist[idx + (d + 3) * (n + 2) + 1] += v_rco111;
                }
            }
        float raw[128];
        for (int i = 0; i < d; i++)
            for (int j = 0; j < d; j++) {
                int idx = ((i + 1) * (d + 2) + (j + 1)) * (n + 2);
                hist[idx] += hist[idx + n];
                hist[idx + 1] += hist[idx + n + 1];
                for (int k = 0; k < n; k++) raw[(i * d + j) * n + k] = hist[idx + k];
            }
#if SIFT_ORACLE_VEC
        // Norm: VEC fma lanes, v_reduce_sum of the dispatch width.
        float acc[SIFT_ORACLE_VEC] = {0};
        for (int k = 0; k < 128; k++) acc[k % SIFT_ORACLE_VEC] = fmaf(raw[k], raw[k], acc[k % SIFT_ORACLE_VEC]);
        float nrm2 = reduceSum(acc);
#else
        // Norm: 8 fma lanes (AVX2 v_float32), reduced as v_reduce_sum.
        float acc[8] = {0};
        for (int k = 0; k < 128; k++) acc[k & 7] = fmaf(raw[k], raw[k], acc[k & 7]);
        float t0 = acc[0] + acc[4], t1 = acc[1] + acc[5], t2 = acc[2] + acc[6], t3 = acc[3] + acc[7];
        float nrm2 = (t0 + t2) + (t1 + t3);
#endif
        float thr = std::sqrt(nrm2) * SIFT_DESCR_MAG_THR;
        nrm2 = 0;
        for (int k = 0; k < 128; k++) {
            float val = std::min(raw[k], thr);
            raw[k] = val;
            nrm2 += val * val;
        }
        nrm2 = SIFT_INT_DESCR_FCTR / std::max(std::sqrt(nrm2), FLT_EPSILON);
        for (int k = 0; k < 128; k++) {
            int v = cvRoundF(raw[k] * nrm2);
            dst[k] = (float)std::min(std::max(v, 0), 255);
        }
    }

#if SIFT_ORACLE_CONTRACT
#pragma GCC pop_options
#endif
    // ---- end of sift.simd.hpp ----

    // [OpenCV 4.x sift.dispatch.cpp: calcDescriptorsComputer]
    void descriptors(const std::vector<Plane>& gpyr, const std::vector<Keypoint>& kpts, float* desc) const {
        const int L = P_.L, firstOctave = P_.firstOctave;
        const long nk = (long)kpts.size();
#pragma omp parallel for num_threads(nthreadsOr(threads_)) schedule(dynamic, 16)
        for (long i = 0; i < nk; i++) {
            const Keypoint& kpt = kpts[i];
            int octave = kpt.octave & 255;
            int layer = (kpt.octave >> 8) & 255;
            octave = octave < 128 ? octave : (-128 | octave);
            float scale = octave >= 0 ? 1.f / (float)(1 << octave) : (float)(1 << -octave);
            float size = kpt.size * scale;
            float ptx = kpt.x * scale, pty = kpt.y * scale;
            const Plane& img = gpyr[(octave - firstOctave) * (L + 3) + layer];
            float angle = 360.f - kpt.angle;
            if (std::fabs(angle - 360.f) < FLT_EPSILON) angle = 0.f;
            calcSIFTDescriptor(img, ptx, pty, angle, size * 0.5f, desc + 128 * i);
        }
    }

    // [OpenCV 4.x sift.dispatch.cpp: detectAndCompute], useProvidedKeypoints = false.
    std::vector<Keypoint> detect(const Plane& img, std::vector<Plane>& gpyr) const {
        const int L = P_.L;
        StageClock clk;
        Plane base;
        initialImage(img, base);
        clk.mark(0);
        const int nOct = autoOctaves(img.w, img.h, P_);
        gaussianPyramid(base, nOct, gpyr);
        clk.mark(1);
        // Reused across calls (dogPyramid).  The parallel loops below must see
        // the calling thread's planes, so they use this reference, not the
        // thread_local itself (each OpenMP worker has its own instance).
        static thread_local std::vector<Plane> dog_tls;
        std::vector<Plane>& dog = dog_tls;
        dogPyramid(gpyr, dog);
        clk.mark(2);
        std::vector<int> quads;
        candidates(dog, nOct, quads);
        clk.mark(3);
        const long nc = (long)quads.size() / 4;
        std::vector<std::vector<Keypoint>> per(nc);
#pragma omp parallel for num_threads(nthreadsOr(threads_)) schedule(dynamic, 64)
        for (long k = 0; k < nc; k++)
            processCandidate(gpyr, dog, quads[4 * k], quads[4 * k + 1], quads[4 * k + 2], quads[4 * k + 3], per[k]);
        std::vector<Keypoint> kpts;
        for (auto& v : per) kpts.insert(kpts.end(), v.begin(), v.end());
        (void)L;
        // KeyPointsFilter::removeDuplicatedSorted.
        std::sort(kpts.begin(), kpts.end(), keypointGreater);
        if (kpts.size() >= 2) {
            size_t i = 0;
            for (size_t j = 1; j < kpts.size(); ++j) {
                const Keypoint& a = kpts[i];
                const Keypoint& b = kpts[j];
                if (a.x != b.x || a.y != b.y || a.size != b.size || a.angle != b.angle) kpts[++i] = kpts[j];
            }
            kpts.resize(i + 1);
        }
        // KeyPointsFilter::retainBest: keep every keypoint whose response is >= the
        // nfeatures-th largest (the set nth_element + partition yields), stably.
        if (P_.nfeatures > 0 && kpts.size() > (size_t)P_.nfeatures) {
            std::vector<float> resp(kpts.size());
            for (size_t k = 0; k < kpts.size(); k++) resp[k] = kpts[k].response;
            std::nth_element(resp.begin(), resp.begin() + P_.nfeatures - 1, resp.end(), std::greater<float>());
            const float amb = resp[P_.nfeatures - 1];
            std::vector<Keypoint> kept;
            for (auto& k : kpts)
                if (k.response >= amb) kept.push_back(k);
            kpts.swap(kept);
        }
        if (P_.firstOctave < 0) {
            for (auto& kpt : kpts) {
                float scale = 1.f / (float)(1 << -P_.firstOctave);
                kpt.octave = (kpt.octave & ~255) | ((kpt.octave + P_.firstOctave) & 255);
                kpt.x *= scale;
                kpt.y *= scale;
                kpt.size *= scale;
            }
        }
        clk.mark(4);
        return kpts;
    }

    const Params& params() const { return P_; }

private:
    Params P_;
    int threads_;
};

Plane toPlane(const float* img, int w, int h) {
    Plane p;
    p.create(w, h);
    std::memcpy(p.d.data(), img, sizeof(float) * (size_t)w * h);
    return p;
}

}  // namespace

extern "C" {

const char* sift_oracle_variant(void) {
#if SIFT_ORACLE_VEC == 0
    return SIFT_ORACLE_CONTRACT ? "simd-formulas+contract" : "pinned";
#elif SIFT_ORACLE_VEC == 8
    return SIFT_ORACLE_CONTRACT ? "avx2-fma" : "avx2";
#else
    return SIFT_ORACLE_CONTRACT ? "avx512-fma" : "avx512";
#endif
}

void sift_oracle_default_params(sift_oracle_params* p) {
    p->nfeatures = 0;
    p->nOctaveLayers = 3;
    p->contrastThreshold = 0.04;
    p->edgeThreshold = 10;
    p->sigma = 1.6;
    p->firstOctave = -1;
    p->nOctaves = 0;
}

int sift_oracle_gaussian_taps(double sigma, float* taps, int cap) {
    std::vector<float> t = gaussianTaps(sigma);
    if ((int)t.size() > cap) return -1;
    std::copy(t.begin(), t.end(), taps);
    return (int)t.size();
}

int sift_oracle_num_octaves(int w, int h, const sift_oracle_params* p) { return autoOctaves(w, h, toParams(p)); }

void sift_oracle_octave_dims(int w, int h, const sift_oracle_params* p, int o, int* ow, int* oh) {
    Params P = toParams(p);
    int W = P.firstOctave < 0 ? 2 * w : w, H = P.firstOctave < 0 ? 2 * h : h;
    for (int k = 0; k < o; k++) {
        W /= 2;
        H /= 2;
    }
    *ow = W;
    *oh = H;
}

long sift_oracle_gaussian_pyramid(const float* img, int w, int h, const sift_oracle_params* p, float* planes) {
    Params P = toParams(p);
    const int nOct = autoOctaves(w, h, P);
    long total = 0;
    for (int o = 0; o < nOct; o++) {
        int ow, oh;
        sift_oracle_octave_dims(w, h, p, o, &ow, &oh);
        total += (long)ow * oh * (P.L + 3);
    }
    if (!planes) return total;
    Sift s(P, 0);
    Plane base;
    s.initialImage(toPlane(img, w, h), base);
    std::vector<Plane> gpyr;
    s.gaussianPyramid(base, nOct, gpyr);
    long off = 0;
    for (auto& pl : gpyr) {
        std::memcpy(planes + off, pl.d.data(), sizeof(float) * pl.d.size());
        off += (long)pl.d.size();
    }
    return off;
}

long sift_oracle_extrema(const float* img, int w, int h, const sift_oracle_params* p, int* quads, long cap) {
    Params P = toParams(p);
    Sift s(P, 0);
    Plane base;
    s.initialImage(toPlane(img, w, h), base);
    std::vector<Plane> gpyr, dog;
    const int nOct = autoOctaves(w, h, P);
    s.gaussianPyramid(base, nOct, gpyr);
    s.dogPyramid(gpyr, dog);
    std::vector<int> q;
    s.candidates(dog, nOct, q);
    long n = (long)q.size() / 4;
    if (quads) std::copy(q.begin(), q.begin() + 4 * std::min(n, cap), quads);
    return n;
}

long sift_oracle_detect_and_compute(const float* img, int w, int h, const sift_oracle_params* p, int threads,
                                    sift_oracle_kpt* out, float* desc, long cap) {
    Params P = toParams(p);
    Sift s(P, threads);
    static thread_local std::vector<Plane> gpyr;  // reused across calls (pages already mapped)
    std::vector<Keypoint> kpts = s.detect(toPlane(img, w, h), gpyr);
    long n = (long)kpts.size();
    long m = std::min(n, cap);
    if (out)
        for (long i = 0; i < m; i++)
            out[i] = sift_oracle_kpt{kpts[i].x, kpts[i].y, kpts[i].size, kpts[i].angle, kpts[i].response,
                                     kpts[i].octave};
    StageClock clk;
    g_stage_ms[5] = 0;
    if (desc && m > 0) {
        std::vector<Keypoint> head(kpts.begin(), kpts.begin() + m);
        s.descriptors(gpyr, head, desc);
        clk.mark(5);
    }
    return n;
}

int sift_oracle_stage_ms(double* out, int cap) {
    const int n = std::min(cap, 6);
    for (int i = 0; i < n; i++) out[i] = g_stage_ms[i];
    return 6;
}

int sift_oracle_compute_descriptors(const float* img, int w, int h, const sift_oracle_params* p,
                                    const sift_oracle_kpt* kpts, long n, float* desc) {
    Params P = toParams(p);
    Sift s(P, 0);
    Plane base;
    s.initialImage(toPlane(img, w, h), base);
    std::vector<Plane> gpyr;
    s.gaussianPyramid(base, autoOctaves(w, h, P), gpyr);
    std::vector<Keypoint> k(n);
    for (long i = 0; i < n; i++)
        k[i] = Keypoint{kpts[i].x, kpts[i].y, kpts[i].size, kpts[i].angle, kpts[i].response, kpts[i].octave};
    s.descriptors(gpyr, k, desc);
    return 0;
}

// [OpenCV 4.x core/batch_distance.cpp: batchDistance(K=2, NORM_L2)] as used by
// BFMatcher::knnMatchImpl.  Ties keep the lower train index (strict '<' insert).
// Reference: Match.cu:8-177 (fp16 (a-b)/4 squared sums, squared ratio 0.8).
void sift_oracle_knn2(const float* q, long nq, const float* t, long nt, int threads, int* idx, float* dist) {
#pragma omp parallel for num_threads(nthreadsOr(threads)) schedule(static)
    for (long i = 0; i < nq; i++) {
        float bestD[2] = {FLT_MAX, FLT_MAX};
        int bestN[2] = {-1, -1};
        const float* a = q + 128 * i;
        for (long j = 0; j < nt; j++) {
            const float* b = t + 128 * j;
            float s = 0.f;
            for (int k = 0; k < 128; k++) {
                float df = a[k] - b[k];
                s += df * df;
            }
            float dd = std::sqrt(s);
            if (dd < bestD[1]) {
                int k = 0;
                for (k = 0; k >= 0 && bestD[k] > dd; k--) {
                    bestD[k + 1] = bestD[k];
                    bestN[k + 1] = bestN[k];
                }
                bestD[k + 1] = dd;
                bestN[k + 1] = (int)j;
            }
        }
        idx[2 * i] = bestN[0];
        idx[2 * i + 1] = bestN[1];
        dist[2 * i] = bestD[0];
        dist[2 * i + 1] = bestD[1];
    }
}

}  // extern "C"
