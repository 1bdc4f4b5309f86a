// 4x4x8 SIFT descriptor for gfx950 (OpenCV 4.x sift.simd.hpp calcSIFTDescriptor).
//
// Replaces /root/reference/sift_cuda/sift_func/SiftOps.cu:454-623 (128 threads
// per keypoint, 8 shared-memory float atomics per sample, modff bins, serial
// lane-0 normalisation, half(x512) output).
//
// Four wavefronts (a 256-thread workgroup) per keypoint, several keypoints
// in flight per CU, so memory latency of one keypoint hides behind the others'
// ALU work:
//   * k_bucket_rank already computed the keypoint's window (DescJob), read
//     here with scalar loads;
//   * only samples inside the rotated 4x4-cell square are enumerated: per row
//     a conservative j-interval, a prefix sum over rows, and each lane takes a
//     contiguous run of the enumerated samples (the oracle's exact per-sample
//     test is still applied, so the set of samples is unchanged);
//   * gradients are read straight from the Gaussian plane (L1/L2 resident:
//     neighbouring keypoints share it) with bounds-checked buffer loads, four
//     samples' loads in flight per lane;
//   * each sample follows the oracle's operations (fastAtan2 polynomial,
//     magnitude, Gaussian weight, cvFloor bins, trilinear split in OpenCV's
//     order) with native v_rcp/v_sqrt/v_exp for the transcendentals (see
//     desc_atan2), and its 8 contributions go to the LDS histogram as 4
//     ds_add_u64, each carrying the orientation pair (o0, o0+1) as two u32
//     words.
// The histogram is fixed point (scale 2^S per keypoint, chosen from the
// frame's pixel range so no bin can reach 2^31): on gfx950 an LDS f32 atomic
// costs ~193 cycles per wave instruction against ~9 for u32 and ~17 for u64
// (tools/lds_atomic_bench.hip), and integer addition is
// associative, so the histogram is identical for any lane schedule
// (deterministic) and equals the exact sum of the rounded contributions.
// OpenCV sums the same float contributions sequentially in float, so
// descriptor bytes can differ from the oracle by +-1 where that rounding lands
// on a .5 boundary (tests bound the rate).  L2 norm (8 fma lanes +
// v_reduce_sum order), 0.2 clip, sequential renorm and x512 rounding are the
// oracle's float operations.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "sift_kernels.h"
#include "sift_math.h"

namespace sift_amd {

constexpr int kD = 4, kN = 8;
constexpr int kCells = (kD + 2) * (kD + 2);  // 36 spatial cells incl. the border ring
constexpr int kCellW = 10;                   // dwords per cell in each fixed-point histogram
constexpr int kMaxRows = kDescMaxRows;       // enumerated windows: side = 2R+1 <= kMaxRows
constexpr int kGroup = 4;                    // samples whose loads are in flight together (raster path)
// Consecutive samples of one row per work item (enumerated path).  Measured:
// 4-sample items -2 %, 1-sample items (dword loads per sample) 304 vs 198 us.
constexpr int kItem = 2;
// Histogram copies: lane l adds into copy l % kCopies, so lanes working on
// the same (cell, orientation) -- same LDS address, serialised atomics -- are
// spread over kCopies addresses (banks 16 apart); the epilogue sums them.
// 352 vs 381 us per 16-frame launch (1 copy), 378 (4 copies: LDS-limited occupancy).
constexpr int kCopies = 2;
constexpr int kHistWords = 2 * kCells * kCellW;  // one copy: the even- and the odd-orientation histogram
// (Measured and dropped: lane -> run permutations 5, 9, 17, 33 (equal or
// worse); the oracle's correctly rounded division / sqrt / exp32f in the
// sample loop (+16 % time, flip counts unchanged).)

// This frame's host rows (HostOut): null pointers unless the frame asked
// for them (Counters.pad[1] level, set by k_order / k_select) and the handle
// has a host region for it.
struct HostRows {
    float* k3;
    float* f4;
    uint16_t* desc;
};
// (Also moves h's device result pointers to the frame.)
__device__ __forceinline__ HostRows host_rows(HostOut& h, const Counters* ctr, unsigned frame, long foff) {
    h.k3 = fptr(h.k3, foff);
    h.f4 = fptr(h.f4, foff);
    const unsigned level = ctr->pad[1] & ((1u << kHostReqShift) - 1);
    char* r = level ? h.tab[frame] : nullptr;
    if (!r) return HostRows{nullptr, nullptr, nullptr};
    float* f4 = reinterpret_cast<float*>(r + ((12 * (size_t)h.cap + 255) & ~(size_t)255));
    return HostRows{reinterpret_cast<float*>(r), f4,
                    level > 1 ? reinterpret_cast<uint16_t*>(reinterpret_cast<char*>(f4) + 16 * (size_t)h.cap) : nullptr};
}
// Output row po's keypoint (lanes 0-2) and features (lanes 3-6) to the host rows.
__device__ __forceinline__ void host_row(const HostRows& hr, const HostOut& h, unsigned po, int t) {
    if (t < 3)
        hr.k3[(size_t)po * 3 + t] = h.k3[(size_t)po * 3 + t];
    else
        hr.f4[(size_t)po * 4 + t - 3] = h.f4[(size_t)po * 4 + t - 3];
}

struct DescGeom {
    float cos_t, sin_t, exp_scale;
    int ptx, pty, rows, cols;
};

// Rotated-grid coordinates of window sample (i, j) and its validity: the
// oracle's calcSIFTDescriptor loop body, operation for operation.
__device__ __forceinline__ bool desc_sample(const DescGeom& G, int i, int j, float& rbin, float& cbin, float& c_rot,
                                            float& r_rot) {
    c_rot = (float)j * G.cos_t - (float)i * G.sin_t;
    r_rot = (float)j * G.sin_t + (float)i * G.cos_t;
    rbin = r_rot + (float)(kD / 2) - 0.5f;
    cbin = c_rot + (float)(kD / 2) - 0.5f;
    const int r = G.pty + i, c = G.ptx + j;
    return rbin > -1 && rbin < kD && cbin > -1 && cbin < kD && r > 0 && r < G.rows - 1 && c > 0 && c < G.cols - 1;
}

// The 8 contributions of one sample, OpenCV's order and names (v_rco[r][c][o]).
// Independent pairs go through v_pk_mul_f32 / v_pk_add_f32 (each half an IEEE
// op, so every value is the oracle's): 8 VALU instead of 14.
typedef float f32x2t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void trilinear(float mag, float rbf, float cbf, float obf, float v[8]) {
    const float v_r1 = mag * rbf, v_r0 = mag - v_r1;
    const f32x2t r10 = {v_r1, v_r0};
    const f32x2t rc_1 = r10 * (f32x2t){cbf, cbf};  // (v_rc11, v_rc01)
    const f32x2t rc_0 = r10 - rc_1;                // (v_rc10, v_rc00)
    const f32x2t ob = {obf, obf};
    const f32x2t hi_a = rc_1 * ob, hi_b = rc_0 * ob;  // (v7, v3), (v5, v1)
    const f32x2t lo_a = rc_1 - hi_a, lo_b = rc_0 - hi_b;  // (v6, v2), (v4, v0)
    v[7] = hi_a[0];
    v[3] = hi_a[1];
    v[5] = hi_b[0];
    v[1] = hi_b[1];
    v[6] = lo_a[0];
    v[2] = lo_a[1];
    v[4] = lo_b[0];
    v[0] = lo_b[1];
}

// Shrink [lo, hi] to a superset of the integers j with -1 < j*s + b < kD
// (margin 1e-4 in bin units and one sample each side, so float rounding of the
// exact per-sample test can never fall outside the enumerated range).
// inv_s = 1 / s (computed once per keypoint).  Float: the bounds before
// clamping to +-(R+2) carry a relative error of a few 1e-7, i.e. < 1e-4
// samples for R <= 50, far inside the one-sample margin each side.
__device__ __forceinline__ void clip_interval(int& lo, int& hi, float s, float inv_s, float b, int R) {
    constexpr float lb = -1.f - 1e-4f, ub = kD + 1e-4f;
    if (fabsf(s) < 1e-12f) {
        if (b <= lb || b >= ub) hi = lo - 1;
        return;
    }
    float x1 = (lb - b) * inv_s, x2 = (ub - b) * inv_s;
    if (x1 > x2) {
        const float t = x1;
        x1 = x2;
        x2 = t;
    }
    x1 = fmaxf(x1, (float)(-R - 2));
    x2 = fminf(x2, (float)(R + 2));
    lo = max(lo, (int)floorf(x1) - 1);
    hi = min(hi, (int)ceilf(x2) + 1);
}

// Sample math with native gfx950 instructions (v_rcp_f32, v_sqrt_f32,
// v_exp_f32; ~1 ulp) instead of the correctly rounded / table forms the
// orientation and pyramid need for bit-exact keypoints.  Every operation is
// continuous in its inputs here (trilinear split, magnitude weights), so ulp
// differences move a descriptor entry by ~1e-7 relative and flip its rounding
// only at a .5 boundary: inside the |diff| <= 1 bar, at the same rate as the
// summation-order difference.  The fastAtan2 polynomial itself is kept.
__device__ __forceinline__ float desc_atan2(float y, float x) {
    const float p1 = 0.9997878412794807f * (float)(180 / M_PI);
    const float p3 = -0.3258083974640975f * (float)(180 / M_PI);
    const float p5 = 0.1555786518463281f * (float)(180 / M_PI);
    const float p7 = -0.04432655554792128f * (float)(180 / M_PI);
    const float ax = fabsf(x), ay = fabsf(y);
    const float c = fminf(ax, ay) * __builtin_amdgcn_rcpf(fmaxf(ax, ay) + (float)DBL_EPSILON);
    const float cc = c * c;
    float a = __fmaf_rn(__fmaf_rn(__fmaf_rn(cc, p7, p5), cc, p3), cc, p1) * c;
    if (!(ax >= ay)) a = 90.f - a;
    if (x < 0) a = 180.f - a;
    if (y < 0) a = 360.f - a;
    return a;
}
__device__ __forceinline__ float desc_magnitude(float x, float y) {
    return __builtin_amdgcn_sqrtf(__fmaf_rn(x, x, y * y));
}

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
struct JobWords {
    u32x4 w[4];
};

// kDT threads per keypoint: 4 waves for a single frame (few keypoints, the
// chip needs the parallelism inside each), 2 waves for frame batches (more
// keypoints in flight per CU: 296 vs 311 us per 8-frame launch, tools/ab_*).
// Minimum waves per SIMD (VGPR budget <= 80): 198 us vs 208 (5) and 211 (8)
// per 8-frame launch; re-swept in round 3 (5 / 7: 337 / 331 vs 334 us).
constexpr int kDescWaves = 6;
// Sum over the 64 lanes, returned to every lane (DPP, as wave_max).
__device__ __forceinline__ float wave_sum(float x) {
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x111, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x112, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x114, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x118, 0xf, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x142, 0xa, 0xf, false));
    x += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x143, 0xc, 0xf, false));
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), 63));
}
template <int kDT>
__global__ __launch_bounds__(kDT, kDescWaves) void k_descriptor(const DescJob* __restrict__ jobs, const Counters* __restrict__ ctr,
                                                   const unsigned* __restrict__ range_keys,
                                                   uint16_t* __restrict__ desc, Sidecar sidecar,
                                                   Counters* __restrict__ host_ctr, HostOut host, long fs,
                                                   unsigned nf) {
    // Two u32 fixed-point histograms so that each sample's orientation pair
    // (o0, o0+1) is one naturally aligned ds_add_u64 (low word o0, high word
    // o0+1): even o0 -> histE[cell*10 + o], odd o0 -> histO[cell*10 + 1 + o]
    // (slot 9 = orientation 8, wrapped into 0 at the end).  The per-keypoint
    // scale keeps every bin below 2^31, so no carry crosses the word boundary.
    __shared__ __attribute__((aligned(16))) unsigned histE[kCopies * kHistWords];  // copy c at c * kHistWords
    __shared__ int rowpre[kMaxRows + 4], rowlo[kMaxRows], rowln[kMaxRows];
    __shared__ float s_norm[12];
    __shared__ int s_cn[2];  // |codes|^2 of the keypoint's two halves (sidecar key bias)
    constexpr int kPer = kDT >= 128 ? 1 : 128 / kDT;  // descriptor entries per thread in the epilogue
    static_assert(kPer == 1, "the sidecar norm takes entries 0-63 / 64-127 from waves 0 / 1");

    const int tid = threadIdx.x, lane = tid & 63;
    // 1-D grid, frame = block % nf: consecutive workgroups are dispatched to
    // consecutive XCDs, so with 8 frames each frame's keypoints run on one
    // XCD (its L2 serves neighbouring keypoints' overlapping windows, in
    // row order) instead of every XCD fetching lines of every frame.
    const unsigned frame = blockIdx.x % nf, wg = blockIdx.x / nf, nwg = gridDim.x / nf;
    const long foff = frame * fs;
    jobs = fptr(jobs, foff);
    ctr = fptr(ctr, foff);
    range_keys = fptr(range_keys, foff);
    desc = fptr(desc, foff);
    sidecar.codes = fptr(sidecar.codes, foff);
    sidecar.keys = fptr(sidecar.keys, foff);
    host_ctr += frame;
    const unsigned n = ctr->final_n;
    // The frame's counters are final before this (last) kernel starts: hand
    // them to the host's pinned copy directly (no D2H copy node in the graph).
    if (wg == 0 && tid < (int)(sizeof(Counters) / 4))
        reinterpret_cast<unsigned*>(host_ctr)[tid] = reinterpret_cast<const unsigned*>(ctr)[tid];
    const HostRows hr = host_rows(host, ctr, frame, foff);
    // A single frame's grid (8192) exceeds its keypoint count: the surplus
    // workgroups leave before the pixel-range reduction below.
    if (wg >= n) return;
    // Pixel range of the frame; it bounds every Gaussian plane (convex blurs).
    unsigned kmax = 0, knmn = 0;
    for (int i = lane; i < kRangeSlots; i += 64) {
        kmax = max(kmax, range_keys[2 * i]);
        knmn = max(knmn, range_keys[2 * i + 1]);
    }
    for (int off = 32; off > 0; off >>= 1) {
        kmax = max(kmax, (unsigned)__shfl_xor((int)kmax, off));
        knmn = max(knmn, (unsigned)__shfl_xor((int)knmn, off));
    }
    const float range = (decode_range_key(kmax) + decode_range_key(knmn)) * 1.001f;
    const float bins_per_rad = kN / 360.f;

    // Plain round-robin keypoint -> workgroup (-> XCD): keypoints are in
    // (octave, layer, row) order and their cost grows with scale, so handing
    // each XCD a contiguous run (L2 locality) unbalances the XCDs -- measured
    // 10-30 % slower frames.
    // Jobs are prefetched one keypoint ahead as vector loads (lanes 0-15, one
    // dword each) and moved to SGPRs with v_readlane: a scalar load at the
    // top of each keypoint would expose a memory latency per keypoint, and a
    // scalar prefetch would be waited for by the body's first lgkmcnt(0).
    const unsigned* __restrict__ jw = reinterpret_cast<const unsigned*>(jobs);
    unsigned jnext = n ? jw[min(wg, n - 1) * 16u + (lane & 15)] : 0u;
    for (unsigned p = wg; p < n; p += nwg) {
        const unsigned jcur = jnext;
        jnext = jw[min(p + nwg, n - 1) * 16u + (lane & 15)];
        JobWords jwd;
#pragma unroll
        for (int q = 0; q < 16; q++) jwd.w[q >> 2][q & 3] = __builtin_amdgcn_readlane(jcur, q);
        const DescJob jb = __builtin_bit_cast(DescJob, jwd);
        DescGeom G;
        G.cos_t = jb.cos_t;
        G.sin_t = jb.sin_t;
        G.exp_scale = -1.f / (kD * kD * 0.5f);
        G.ptx = jb.ptx;
        G.pty = jb.pty;
        G.rows = jb.rows;
        G.cols = jb.cols;
        const int radius = jb.radius, side = 2 * radius + 1;
        const bool enumerated = side <= kMaxRows;
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(jb.img), 0, jb.rows * jb.pitch * 4, 0x00020000);

        static_assert((kCopies * kHistWords) % 4 == 0, "histograms zeroed as uint4");
        for (int i = tid; i < kCopies * kHistWords / 4; i += kDT) reinterpret_cast<uint4*>(histE)[i] = make_uint4(0u, 0u, 0u, 0u);
        if (enumerated) {
            const float inv_sin = __builtin_amdgcn_rcpf(G.sin_t), inv_cos = __builtin_amdgcn_rcpf(G.cos_t);
            for (int t = tid; t < side; t += kDT) {
                const int i = t - radius, r = G.pty + i;
                int lo = max(-radius, 1 - G.ptx), hi = min(radius, G.cols - 2 - G.ptx);
                if (r <= 0 || r >= G.rows - 1) hi = lo - 1;
                clip_interval(lo, hi, G.sin_t, inv_sin, (float)i * G.cos_t + (kD / 2 - 0.5f), radius);
                clip_interval(lo, hi, G.cos_t, inv_cos, -(float)i * G.sin_t + (kD / 2 - 0.5f), radius);
                const int len = max(hi - lo + 1, 0);
                rowlo[t] = lo;
                rowln[t] = len;
                rowpre[t + 1] = (len + kItem - 1) / kItem;  // items of kItem consecutive samples
            }
            if (tid == 0) rowpre[0] = 0;
            lds_barrier();
            if (tid < 64) {  // inclusive scan of row counts (entries 2l+1, 2l+2 of rowpre per lane)
                const int a = 2 * lane + 1 <= side ? rowpre[2 * lane + 1] : 0;
                const int b = 2 * lane + 2 <= side ? rowpre[2 * lane + 2] : 0;
                const int sum = wave_incl_scan(a + b);
                if (2 * lane + 1 <= side) rowpre[2 * lane + 1] = sum - b;
                if (2 * lane + 2 <= side) rowpre[2 * lane + 2] = sum;
            }
        }
        // Fixed-point scale 2^S with every bin < 2^31: a contribution is at most
        // the gradient magnitude <= sqrt(2) * range, and a bin collects samples
        // from a 2x2-cell rotated square of side 2*hist_width, i.e. at most
        // (2*sqrt(2)*hist_width + 2)^2 samples.
        const float nb = 2.8285f * jb.hist_width + 2.f;
        int e;
        (void)frexpf(nb * nb * 1.4143f * range + 1.f, &e);
        const int S = min(31 - e, 40);
        const float fxs = ldexpf(1.f, S);
        lds_barrier();

        // One sample from its four neighbours (l, r, u, d).  Branch-free so
        // that the kGroup samples of a group interleave (ILP): a rejected
        // sample keeps in-range bin indices and adds zeros.
        auto accum_rot = [&](float c_rot, float r_rot, bool valid, float l, float r, float u, float d) {
            // (cbin, rbin) and the squared radius as packed pairs (IEEE per half).
            const f32x2t rot = {c_rot, r_rot};
            const f32x2t bins = (rot + (f32x2t){(float)(kD / 2), (float)(kD / 2)}) - (f32x2t){0.5f, 0.5f};
            float cbin = bins[0], rbin = bins[1];
            valid = valid && rbin > -1 && rbin < kD && cbin > -1 && cbin < kD;
            const float dx = r - l, dy = u - d;
            const f32x2t sq = rot * rot;
            // exp_scale = -1/8 is a power of two, so (r2 * -1/8) * log2(e)
            // = r2 * (-log2(e) / 8) with the same single rounding: one multiply.
            const float wgt = __builtin_amdgcn_exp2f((sq[0] + sq[1]) * (-1.44269504088896341f / (kD * kD * 0.5f)));
            const float gori = desc_atan2(dy, dx);
            const float gmag = desc_magnitude(dx, dy);
            float obin = (gori - jb.angle) * bins_per_rad;
            // x 2^S (exact): the trilinear parts come out in fixed-point units.
            // A select, not a branch around the product (every operand is
            // finite: enumerated samples are in-image).
            const float mag = (gmag * wgt * fxs) * (valid ? 1.f : 0.f);
            // cvFloor in the float domain (the clamp only guards rejected
            // samples): r - floor(r) is the oracle's r - (float)cvFloor(r).
            const float r0f = fminf(fmaxf(floorf(rbin), -1.f), (float)(kD - 1));
            const float c0f = fminf(fmaxf(floorf(cbin), -1.f), (float)(kD - 1));
            const float o0f = floorf(obin);
            rbin -= r0f;
            cbin -= c0f;
            obin -= o0f;
            // obin is in (-8, 8), so o0 & 7 is OpenCV's `o0 += n if < 0, -= n
            // if >= n` wrap (two's complement).
            const int o0 = (int)o0f & (kN - 1);
            const int odd = o0 & 1;
            // Word of (cell, o0) in the parity's histogram: cell = (r0 + 1) *
            // (kD + 2) + (c0 + 1), 10 words per cell -- formed in float (small
            // exact integers, one fma chain) instead of integer multiplies.
            // Both histograms have 10 dwords per cell, so the four u64 adds of
            // a sample sit at constant offsets from hb (immediate offsets).
            const unsigned cw = (unsigned)__fmaf_rn(r0f, (float)((kD + 2) * kCellW),
                                                     __fmaf_rn(c0f, (float)kCellW, (float)((kD + 3) * kCellW)));
            unsigned* hb = histE + (lane & (kCopies - 1)) * kHistWords + cw + (unsigned)(o0 + odd * (kCells * kCellW + 1));
            float v[8];
            trilinear(mag, rbin, cbin, obin, v);
#pragma unroll
            for (int q = 0; q < 8; q += 2) {
                const int off = (q & 4 ? (kD + 2) * kCellW : 0) + (q & 2 ? kCellW : 0);
                const unsigned lo = (unsigned)v[q];  // truncation: < 2^-S per contribution
                const unsigned hi = (unsigned)v[q + 1];
                atomicAdd(reinterpret_cast<unsigned long long*>(hb + off),
                          ((unsigned long long)hi << 32) | (unsigned long long)lo);
            }
        };
        auto accumulate = [&](int i, int j, bool in, float l, float r, float u, float d) {
            float rbin, cbin, c_rot, r_rot;
            const bool valid = desc_sample(G, i, j, rbin, cbin, c_rot, r_rot) && in;
            accum_rot(c_rot, r_rot, valid, l, r, u, d);
        };
        // Gradient loads of up to kGroup samples, then their accumulation.
        // Samples outside the plane read 0 (buffer range check) and are
        // rejected by desc_sample.
        auto group = [&](const int (&gi)[kGroup], const int (&gj)[kGroup], int cnt) {
            float l[kGroup], r[kGroup], u[kGroup], d[kGroup];
#pragma unroll
            for (int t = 0; t < kGroup; t++) {
                const unsigned o = (unsigned)((G.pty + gi[t]) * jb.pitch + G.ptx + gj[t]) * 4u;
                l[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, o - 4u, 0, 0));
                r[t] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, o + 4u, 0, 0));
                u[t] = __builtin_bit_cast(float,
                                          __builtin_amdgcn_raw_buffer_load_b32(rsrc, o - 4u * jb.pitch, 0, 0));
                d[t] = __builtin_bit_cast(float,
                                          __builtin_amdgcn_raw_buffer_load_b32(rsrc, o + 4u * jb.pitch, 0, 0));
            }
#pragma unroll
            for (int t = 0; t < kGroup; t++) accumulate(gi[t], gj[t], t < cnt, l[t], r[t], u[t], d[t]);
        };

        if (enumerated) {
            // Work items of kItem (2) consecutive samples of one row: their
            // neighbours come in as one 16-byte and two 8-byte loads instead of
            // four dword loads per sample, and i * sin / i * cos are shared.  Each thread takes a contiguous run
            // of items.  Rows hold only in-image samples (the intervals are
            // clipped to 1 .. cols-2 / rows 1 .. rows-2), so validity is the
            // oracle's bin-range test alone.
            const int N = rowpre[side];
            const int run = (N + kDT - 1) / kDT;
            const int tq = tid;  // this thread's run
            const int k0 = min(N, tq * run), k1 = min(N, k0 + run);
            if (k0 < k1) {
                int lo = 0, hi = side - 1;  // last row with rowpre[row] <= k0 (non-empty)
                while (lo < hi) {
                    const int mid = (lo + hi + 1) >> 1;
                    if (rowpre[mid] <= k0) lo = mid;
                    else hi = mid - 1;
                }
                int row = lo;
                int jj = rowlo[row] + kItem * (k0 - rowpre[row]);
                int jend = rowlo[row] + rowln[row];  // exclusive
                typedef float f32x4d __attribute__((ext_vector_type(4)));
                typedef float f32x2d __attribute__((ext_vector_type(2)));
                const int pitch4 = 4 * jb.pitch;
                for (int k = k0; k < k1; k++) {
                    const int i = row - radius;
                    const int cnt = jend - jj;
                    const unsigned o = (unsigned)((G.pty + i) * jb.pitch + G.ptx + jj) * 4u;
                    // (x-1 .. x+kItem) of the row, (x .. x+kItem-1) of the rows above and below.
                    float row6[kItem + 2], up[kItem], dn[kItem];
                    {
                        const f32x4d cm = __builtin_bit_cast(f32x4d, __builtin_amdgcn_raw_buffer_load_b128(rsrc, o - 4u, 0, 0));
                        static_assert(kItem == 2, "items of two samples");
                        const f32x2d u2 = __builtin_bit_cast(f32x2d, __builtin_amdgcn_raw_buffer_load_b64(rsrc, o - pitch4, 0, 0));
                        const f32x2d d2 = __builtin_bit_cast(f32x2d, __builtin_amdgcn_raw_buffer_load_b64(rsrc, o + pitch4, 0, 0));
                        for (int t = 0; t < 2; t++) up[t] = u2[t], dn[t] = d2[t];
                        for (int t = 0; t < 4; t++) row6[t] = cm[t];
                    }
                    const float fi = (float)i, is = fi * G.sin_t, ic = fi * G.cos_t;
#pragma unroll
                    for (int t = 0; t < kItem; t++) {
                        const float fj = (float)(jj + t);
                        // desc_sample's rotation, operation for operation
                        // (c = j*cos - i*sin, r = j*sin + i*cos), packed.
                        const f32x2t pr = (f32x2t){fj, fj} * (f32x2t){G.cos_t, G.sin_t};
                        const f32x2t rot = pr + (f32x2t){-is, ic};
                        accum_rot(rot[0], rot[1], t < cnt, row6[t], row6[t + 2], up[t], dn[t]);
                        // One sample at a time: interleaving the four keeps
                        // ~90 VGPRs live (occupancy 5 instead of 8 waves/SIMD).
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    jj += kItem;
                    if (k + 1 < k1 && jj >= jend) {  // next non-empty row
                        do row++;
                        while (rowpre[row + 1] == rowpre[row]);
                        jj = rowlo[row];
                        jend = jj + rowln[row];
                    }
                }
            }
        } else {  // huge window: the full raster, rejected samples included
            const int total = side * side;
            for (int q0 = tid * kGroup; q0 < total; q0 += kDT * kGroup) {
                int gi[kGroup], gj[kGroup];
#pragma unroll
                for (int t = 0; t < kGroup; t++) {
                    const int q = min(q0 + t, total - 1);
                    gi[t] = q / side - radius;
                    gj[t] = q % side - radius;
                }
                group(gi, gj, total - q0);
            }
        }
        lds_barrier();

        // Wrap, L2 norm, 0.2 clip, renormalisation, x512 rounding.
        const float inv = ldexpf(1.f, -S);
        float val[kPer];
#pragma unroll
        for (int h = 0; h < kPer; h++) {
            const int t = min(tid + kDT * h, 127);  // threads past 128 mirror entry 127 (never stored)
            const int ii = t >> 5, jj = (t >> 3) & 3, kk = t & 7;
            const int cell = (ii + 1) * (kD + 2) + (jj + 1);
            unsigned long long hv = 0;
#pragma unroll
            for (int c = 0; c < kCopies; c++) {
                const unsigned* hE = histE + c * kHistWords;
                const unsigned* hO = hE + kCells * kCellW;
                hv += (unsigned long long)hE[cell * kCellW + kk] + hO[cell * kCellW + 1 + kk];
                if (kk == 0) hv += hO[cell * kCellW + 9];
            }
            val[h] = (float)((double)hv * (double)inv);
        }
        // Both norms as wave sums (DPP) of the entries' squares, one partial
        // per wave through LDS: two barriers instead of four and no serial
        // 128-term sum (thread 0 alone, OpenCV's order: 347.8 vs 336.9 us per
        // serialised 16-frame launch, round 6).  The float order is not
        // OpenCV's, so the scale can differ by an ulp -- inside the default
        // mode's +-1 bar (its histogram is summed in another order already;
        // the exact mode keeps OpenCV's order).
        static_assert(kPer == 1, "one entry per thread");
        const bool own = tid < 128;
        const float w1 = wave_sum(own ? val[0] * val[0] : 0.f);
        if (lane == 0) s_norm[tid >> 6] = w1;
        lds_barrier();
        const float thr = __builtin_sqrtf(s_norm[0] + s_norm[1]) * 0.2f;
        val[0] = fminf(val[0], thr);
        const float w2 = wave_sum(own ? val[0] * val[0] : 0.f);
        if (lane == 0) s_norm[4 + (tid >> 6)] = w2;
        lds_barrier();
        const float scale = 512.f / fmaxf(__builtin_sqrtf(s_norm[4] + s_norm[5]), FLT_EPSILON);
        const unsigned po = (unsigned)jb.out;  // output row (the job order may differ: JobOrder)
        int c2 = 0;  // this thread's share of |codes|^2
#pragma unroll
        for (int h = 0; h < kPer; h++) {
            int v = cv_round(val[h] * scale);
            v = v < 0 ? 0 : (v > 255 ? 255 : v);
            const _Float16 hv = (_Float16)(float)v;
            if (tid + kDT * h < 128) {
                desc[(size_t)po * 128 + tid + kDT * h] = __builtin_bit_cast(uint16_t, hv);
                if (hr.desc) hr.desc[(size_t)po * 128 + tid + kDT * h] = __builtin_bit_cast(uint16_t, hv);
                sidecar.codes[(size_t)po * 128 + tid + kDT * h] = (int8_t)(v - 128);
                c2 += (v - 128) * (v - 128);
            }
        }
        // Sidecar key bias: each wave's sum (DPP scan, total in lane 63) to
        // LDS before the barrier that ends the keypoint, thread 0 adds the
        // two after it (s_cn is next written after several more barriers).
        c2 = __builtin_amdgcn_readlane(wave_incl_scan(c2), 63);
        if (lane == 0 && tid < 128) s_cn[tid >> 6] = c2;
        if (hr.k3 && tid < 7) host_row(hr, host, po, tid);
        lds_barrier();  // sq / histograms are rewritten by the next keypoint
        if (tid == 0) sidecar.keys[po] = -(256 * (s_cn[0] + s_cn[1]) + (int)(po & 255));
    }
}

// ---------------------------------------------------------------------------
// Exact mode (sift_hip_set_descriptor_mode(h, SIFT_HIP_DESC_EXACT)): OpenCV's
// histogram bit for bit.  calcSIFTDescriptor sums each bin's float
// contributions sequentially in raster order of the window; float addition is
// not associative, so the fixed-point histogram above can land one byte off.
// Here every bin has ONE owner lane that adds its contributions in that order:
//   * one wave per keypoint (four independent waves per workgroup, private
//     LDS, no workgroup barrier inside the keypoint loop); the enumerated
//     samples are taken in chunks of 64 consecutive samples (raster order),
//     one per lane, their gradient loads two chunks ahead;
//   * each lane computes its sample with the oracle's correctly rounded math
//     (cv_exp32f table exp, fastAtan2 with IEEE division, magnitude with IEEE
//     sqrt) and OpenCV's trilinear split into 8 contributions;
//   * owners: lane = (cell 0..15, orientation pair g 0..3) adds bins 2g,
//     2g + 1; bin 8 (o0 = 7's upper bin, wrapped into bin 0 at the end as
//     OpenCV does) has its own run per cell, added by the cell's g = 0 lane;
//   * packed runs (round 6): per chunk each owner takes the popcount of its
//     ballot mask (the samples touching its cell row, column and orientation
//     pair), one wave scan of the counts gives every owner a contiguous run in
//     LDS and a table row {mask, run start}, and each sample writes, for every
//     owner it touches, the float2 that owner adds at run start + rank (rank =
//     v_mbcnt of the owner's mask below the sample); then each owner adds its
//     run in order, four entries per step.  Entries are {into bin 2g, into
//     bin 2g + 1}: even o0 writes (v_o0, v_o0+1) to pair o0 / 2, odd o0 writes
//     (+0, v_o0) to pair (o0 - 1) / 2 and (v_o0+1, +0) to pair (o0 + 1) / 2
//     (bin 8's run for o0 = 7, whose adds read the x halves only).  Runs are
//     padded to four entries with zeros: every contribution is >= +0, so
//     x + 0 = x exactly.  A sample's targets outside the 4x4 interior read a
//     null row (mask 0) whose rank lands on a trash entry.
// The walk's length is still the busiest owner's hits in the chunk (64
// consecutive samples are a thin band of the window), but a hit costs ~2.5
// instructions instead of the ~15 of the round-4 mask walk (owners pulling
// their hits by bit scans and decoding per-sample records; 1585 -> 1275 us per
// serialised 16-frame launch).
// ---------------------------------------------------------------------------
constexpr int kExactWaves = 4;
// Minimum waves per SIMD: 6 (78 VGPRs, a 12-byte spill) -- the LDS limit of
// the 4-wave workgroups; the unconstrained build took 83 VGPRs, 5 waves/SIMD:
// 923-929 vs 977-989 us per 16-frame launch (profiles/round6/exact_waves_ab.txt).
constexpr int kExactMinWaves = 6;
constexpr int kExactWG = 64 * kExactWaves;
// Inclusive prefix maximum over the 64 lanes (non-negative values; DPP as
// wave_incl_scan).
__device__ __forceinline__ int wave_incl_max(int x) {
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false));
    x = max(x, __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false));
    return x;
}
// Orders one wave's LDS writes before its later LDS reads by other lanes (LDS
// executes a wave's instructions in order; the fences keep the compiler from
// moving accesses across).
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
}
__constant__ float c_desc_exptab[64];
void upload_desc_exp_table(const float* tab64) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_desc_exptab), tab64, 64 * sizeof(float));
}

constexpr int kRunRows = 16 * 5;               // (cell, g): g = 0..3 pairs, g = 4 bin 8
constexpr int kPoolEntries = 64 * 8 + 80;  // <= 8 entries per sample + padding of 80 runs to even counts
// (Measured and dropped: the masks' picks as inline-asm v_bfi_b32 with the
// ballot SGPR as an operand -- 60 fewer VALU per chunk than the compiler's
// v_mov + v_cndmask, but descriptors went wrong on the GPU (an SGPR hazard the
// compiler cannot see inside inline asm; tests/test_gpu_batch.py).)
// Inclusive wave prefix sum with the DPP row shifts / broadcasts applied to
// the adds themselves (no zero-initialised copies): wave_incl_scan's result.
// Rows outside row_mask are not written and keep their sum.
__device__ __forceinline__ int wave_incl_scan_dpp(int x) {
    asm volatile(
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:0\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_bcast:15 row_mask:0xa bank_mask:0xf\n\t"
        "s_nop 1\n\tv_add_u32_dpp %0, %0, %0 row_bcast:31 row_mask:0xc bank_mask:0xf\n\t"
        "s_nop 1"
        : "+v"(x));
    return x;
}
__global__ __launch_bounds__(kExactWG, kExactMinWaves) void k_descriptor_exact(const DescJob* __restrict__ jobs,
                                                                    const Counters* __restrict__ ctr,
                                                                    uint16_t* __restrict__ desc, Sidecar sidecar,
                                                                    Counters* __restrict__ host_ctr, HostOut host,
                                                                    long fs, unsigned nf) {
    __shared__ float s_tab[64];
    __shared__ __attribute__((aligned(16))) float2 s_pool[kExactWaves][kPoolEntries];
    __shared__ __attribute__((aligned(16))) uint4 s_tbl[kExactWaves][kRunRows];            // {mask lo, hi, start, -}
    __shared__ unsigned short s_rowpre[kExactWaves][kMaxRows + 1];
    __shared__ signed char s_rowlo[kExactWaves][kMaxRows];
    __shared__ float s_nrm[kExactWaves][12];

    const int lane = threadIdx.x & 63, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    float2* pool = s_pool[w];
    uint4* tbl = s_tbl[w];
    unsigned short* rowpre = s_rowpre[w];
    signed char* rowlo = s_rowlo[w];
    float* raw = reinterpret_cast<float*>(pool);     // after the chunk loop
    float* s_norm = s_nrm[w];
    int* rowmap = reinterpret_cast<int*>(pool);      // inside fetch(), before a chunk's runs are written
    const unsigned frame = blockIdx.x % nf, wg = blockIdx.x / nf, nwg = gridDim.x / nf;
    const long foff = frame * fs;
    jobs = fptr(jobs, foff);
    ctr = fptr(ctr, foff);
    desc = fptr(desc, foff);
    sidecar.codes = fptr(sidecar.codes, foff);
    sidecar.keys = fptr(sidecar.keys, foff);
    host_ctr += frame;
    const unsigned n = ctr->final_n;
    static_assert(sizeof(Counters) <= 4 * kExactWG, "counters handed over by one workgroup");
    if (wg == 0 && threadIdx.x < sizeof(Counters) / 4)
        reinterpret_cast<unsigned*>(host_ctr)[threadIdx.x] = reinterpret_cast<const unsigned*>(ctr)[threadIdx.x];
    if (wg * kExactWaves >= n) return;  // workgroup-uniform
    if (w == 0) s_tab[lane] = c_desc_exptab[lane];
    lds_barrier();
    const float bins_per_rad = kN / 360.f;
    const float exp_scale = -1.f / (kD * kD * 0.5f);
    // This lane's bins: interior cell (ci, cj), orientations 2g and 2g + 1.
    const int cell = lane >> 2, g = lane & 3, ci = cell >> 2, cj = cell & 3;

    for (unsigned p = wg * kExactWaves + w; p < n; p += nwg * kExactWaves) {
        JobWords jwd;
        const unsigned* __restrict__ jw = reinterpret_cast<const unsigned*>(jobs + p);
#pragma unroll
        for (int q = 0; q < 16; q++) jwd.w[q >> 2][q & 3] = __builtin_amdgcn_readfirstlane(jw[q]);
        const DescJob jb = __builtin_bit_cast(DescJob, jwd);
        DescGeom G;
        G.cos_t = jb.cos_t;
        G.sin_t = jb.sin_t;
        G.exp_scale = exp_scale;
        G.ptx = jb.ptx;
        G.pty = jb.pty;
        G.rows = jb.rows;
        G.cols = jb.cols;
        const int radius = jb.radius, side = 2 * radius + 1;
        const bool enumerated = side <= kMaxRows;
        const __amdgpu_buffer_rsrc_t rsrc =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(jb.img), 0, jb.rows * jb.pitch * 4, 0x00020000);
        int N;
        if (enumerated) {
            const float inv_sin = __builtin_amdgcn_rcpf(G.sin_t), inv_cos = __builtin_amdgcn_rcpf(G.cos_t);
            int len2[2];
#pragma unroll
            for (int h = 0; h < 2; h++) {
                const int t = 2 * lane + h, i = t - radius, r = G.pty + i;
                int lo = max(-radius, 1 - G.ptx), hi = min(radius, G.cols - 2 - G.ptx);
                if (r <= 0 || r >= G.rows - 1 || t >= side) hi = lo - 1;
                clip_interval(lo, hi, G.sin_t, inv_sin, (float)i * G.cos_t + (kD / 2 - 0.5f), radius);
                clip_interval(lo, hi, G.cos_t, inv_cos, -(float)i * G.sin_t + (kD / 2 - 0.5f), radius);
                len2[h] = max(hi - lo + 1, 0);
                if (t < side) rowlo[t] = lo;
            }
            const int sum = wave_incl_scan(len2[0] + len2[1]);
            if (2 * lane + 1 <= side) rowpre[2 * lane + 1] = sum - len2[1];
            if (2 * lane + 2 <= side) rowpre[2 * lane + 2] = sum;
            if (lane == 0) rowpre[0] = 0;
            N = __builtin_amdgcn_readlane(sum, 63);
        } else {
            N = side * side;  // huge window: the full raster, the oracle's test per sample
        }
        wave_lds_sync();

        auto row_search = [&](int k) {
            int lo = 0, hi = side - 1;  // last row with rowpre[row] <= k
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (rowpre[mid] <= k) lo = mid;
                else hi = mid - 1;
            }
            return lo;
        };
        auto gload = [&](unsigned o) {
            return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rsrc, o, 0, 0));
        };
        const unsigned pitch4 = 4u * jb.pitch;
        struct Fetch {
            int i, j;
            float l, r, u, d;
        };
        // Gradient loads two chunks ahead of the math (unconditionally: past
        // the end they re-read an in-buffer address).  Rows of a chunk [kf, kf
        // + 64) without a per-lane search: frb is the row of sample kf; rows
        // frb+1 .. frb+64 that start inside the chunk mark their start (ds_max:
        // of several rows starting at one position -- empty rows -- the last
        // is the non-empty one) and a wave prefix maximum gives every position
        // its row.  Non-empty rows are contiguous, so 64 rows cover the chunk;
        // if not, the binary search.
        int frb = N > 0 ? __builtin_amdgcn_readfirstlane(enumerated ? row_search(0) : 0) : 0;
        auto fetch = [&](int kf) {
            Fetch f;
            if (enumerated) {
                int row;
                const bool covered = rowpre[min(frb + 65, side)] >= min(kf + 64, N);  // uniform
                if (covered) {
                    rowmap[lane] = frb;
                    wave_lds_sync();
                    const int r = frb + 1 + lane;
                    if (r < side) {
                        const int st = rowpre[r] - kf;
                        if (st >= 0 && st < 64) atomicMax(&rowmap[st], r);
                    }
                    wave_lds_sync();
                    row = wave_incl_max(rowmap[lane]);
                    wave_lds_sync();
                } else {
                    row = row_search(min(kf + lane, N - 1));
                }
                frb = __builtin_amdgcn_readlane(row, 63);
                f.i = row - radius;
                f.j = rowlo[row] + (kf + lane - rowpre[row]);
            } else {
                const int k = min(kf + lane, N - 1);
                f.i = k / side - radius;
                f.j = k % side - radius;
            }
            const unsigned o = (unsigned)((G.pty + f.i) * jb.pitch + G.ptx + f.j) * 4u;
            f.l = gload(o - 4u);
            f.r = gload(o + 4u);
            f.u = gload(o - pitch4);
            f.d = gload(o + pitch4);
            return f;
        };
        Fetch f1 = fetch(0), f2 = fetch(64);
        unsigned sel_ci[kD], sel_cj[kD], sel_g[kD];  // all ones where this lane's index is q
#pragma unroll
        for (int q = 0; q < kD; q++) {
            sel_ci[q] = ci == q ? ~0u : 0u;
            sel_cj[q] = cj == q ? ~0u : 0u;
            sel_g[q] = g == q ? ~0u : 0u;
        }
        float accA = 0.f, accB = 0.f, accW = 0.f;  // bins 2g, 2g + 1, and 8 (g = 0)
        for (int k0 = 0; k0 < N; k0 += 64) {
            // ---- sample k0 + lane: the oracle's math ----
            const int i = f1.i, j = f1.j;
            const float l = f1.l, r = f1.r, u = f1.u, d = f1.d;
            f1 = f2;
            f2 = fetch(k0 + 128);
            float rbin, cbin, c_rot, r_rot;
            const bool valid = desc_sample(G, i, j, rbin, cbin, c_rot, r_rot) && k0 + lane < N;
            const float dx = r - l, dy = u - d;
            const float wgt = cv_exp32f((c_rot * c_rot + r_rot * r_rot) * exp_scale, s_tab);
            const float gori = cv_fast_atan2(dy, dx);
            const float gmag = cv_magnitude(dx, dy);
            float obin = (gori - jb.angle) * bins_per_rad;
            const float mag = gmag * wgt;
            const int r0 = cv_floor(rbin), c0 = cv_floor(cbin);
            int o0 = cv_floor(obin);
            rbin -= (float)r0;
            cbin -= (float)c0;
            obin -= (float)o0;
            if (o0 < 0) o0 += kN;
            if (o0 >= kN) o0 -= kN;
            float v[8];
            trilinear(mag, rbin, cbin, obin, v);
            // ---- owners: masks, counts, runs ----
            // Samples touching interior cell row / column q (r0 in {q - 1, q}),
            // orientation pair q (o0 in {2q - 1, 2q, 2q + 1}; pair 0 without
            // o0 = 7, whose upper bin is bin 8) and bin 8 (o0 = 7).
            const int r0v = valid ? r0 : 64;
            unsigned long long RR[kD], CC[kD], OO[kD];
#pragma unroll
            for (int q = 0; q < kD; q++) {
                RR[q] = __builtin_amdgcn_ballot_w64((unsigned)(r0v - q + 1) < 2u);
                CC[q] = __builtin_amdgcn_ballot_w64((unsigned)(c0 - q + 1) < 2u);
                OO[q] = __builtin_amdgcn_ballot_w64(q == 0 ? (unsigned)o0 < 2u : (unsigned)(o0 - 2 * q + 1) < 3u);
            }
            const unsigned long long O7 = __builtin_amdgcn_ballot_w64(o0 == kN - 1);
            auto pick = [](const unsigned long long (&X)[kD], const unsigned (&sel)[kD]) {
                unsigned lo = (unsigned)X[0], hi = (unsigned)(X[0] >> 32);
#pragma unroll
                for (int q = 1; q < kD; q++) {
                    lo = ((unsigned)X[q] & sel[q]) | (lo & ~sel[q]);
                    hi = ((unsigned)(X[q] >> 32) & sel[q]) | (hi & ~sel[q]);
                }
                return (unsigned long long)hi << 32 | lo;
            };
            const unsigned long long RC = pick(RR, sel_ci) & pick(CC, sel_cj);
            const unsigned long long M = RC & pick(OO, sel_g);
            const unsigned long long Mw = g == 0 ? RC & O7 : 0ull;
            const int cnt = __builtin_popcountll(M), cntw = __builtin_popcountll(Mw);
            const int c2 = (cnt + 1) & ~1, w2 = (cntw + 1) & ~1;
            // Runs: every pair run, then every bin-8 run (16-bit halves of one scan).
            const int packed = c2 | w2 << 16;
            const int incl = wave_incl_scan_dpp(packed), excl = incl - packed;
            const int start = excl & 0xffff, startw = (__builtin_amdgcn_readlane(incl, 63) & 0xffff) + (excl >> 16);
            tbl[cell * 5 + g] = make_uint4((unsigned)M, (unsigned)(M >> 32), (unsigned)start, 0u);
            if (g == 0) tbl[cell * 5 + 4] = make_uint4((unsigned)Mw, (unsigned)(Mw >> 32), (unsigned)startw, 0u);
            // Padding: a run of odd count ends in a zero entry.
            if (cnt & 1) pool[start + c2 - 1] = make_float2(0.f, 0.f);
            if (cntw & 1) pool[startw + w2 - 1] = make_float2(0.f, 0.f);
            wave_lds_sync();
            // ---- samples: push each contribution pair to its owner's run ----
            const bool odd = o0 & 1;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int tci = r0 + (q >> 1), tcj = c0 + (q & 1);
                if (valid && (unsigned)tci < (unsigned)kD && (unsigned)tcj < (unsigned)kD) {
                    const int rp = (tci * kD + tcj) * 5 + (o0 >> 1);
                    const float lo = v[2 * q], hi = v[2 * q + 1];
                    const uint3 tp = *reinterpret_cast<const uint3*>(&tbl[rp]);
                    pool[__builtin_amdgcn_mbcnt_hi(tp.y, __builtin_amdgcn_mbcnt_lo(tp.x, tp.z))] =
                        make_float2(odd ? 0.f : lo, odd ? lo : hi);
                    if (odd) {
                        const uint3 ts = *reinterpret_cast<const uint3*>(&tbl[rp + 1]);
                        pool[__builtin_amdgcn_mbcnt_hi(ts.y, __builtin_amdgcn_mbcnt_lo(ts.x, ts.z))] = make_float2(hi, 0.f);
                    }
                }
            }
            wave_lds_sync();
            // ---- owners: add the runs in order ----
            const float4* run = reinterpret_cast<const float4*>(pool + start);  // (start even: 16-byte aligned)
            int k = 0;
            for (; k + 1 < c2 / 2; k += 2) {
                const float4 e0 = run[k], e1 = run[k + 1];
                accA = accA + e0.x;
                accB = accB + e0.y;
                accA = accA + e0.z;
                accB = accB + e0.w;
                accA = accA + e1.x;
                accB = accB + e1.y;
                accA = accA + e1.z;
                accB = accB + e1.w;
            }
            if (k < c2 / 2) {
                const float4 e0 = run[k];
                accA = accA + e0.x;
                accB = accB + e0.y;
                accA = accA + e0.z;
                accB = accB + e0.w;
            }
            const float4* runw = reinterpret_cast<const float4*>(pool + startw);
            for (k = 0; k < w2 / 2; k++) {  // g = 0 lanes (w2 = 0 elsewhere)
                const float4 e0 = runw[k];
                accW = accW + e0.x;
                accW = accW + e0.z;
            }
            wave_lds_sync();
        }
        // OpenCV's wrap: hist[0] += hist[8] (hist[1] += hist[9] adds +0).
        raw[cell * kN + 2 * g] = g == 0 ? accA + accW : accA;
        raw[cell * kN + 2 * g + 1] = accB;
        wave_lds_sync();
        if (lane < 8) {
            float a = 0.f;
#pragma unroll
            for (int q = 0; q < 16; q++) a = __fmaf_rn(raw[lane + 8 * q], raw[lane + 8 * q], a);
            s_norm[lane] = a;
        }
        wave_lds_sync();
        const float t0 = s_norm[0] + s_norm[4], t1 = s_norm[1] + s_norm[5], t2 = s_norm[2] + s_norm[6],
                    t3 = s_norm[3] + s_norm[7];
        const float thr = __builtin_sqrtf((t0 + t2) + (t1 + t3)) * 0.2f;
        const float v0 = fminf(raw[2 * lane], thr), v1 = fminf(raw[2 * lane + 1], thr);
        wave_lds_sync();
        raw[2 * lane] = v0;
        raw[2 * lane + 1] = v1;
        wave_lds_sync();
        if (lane == 0) {
            float nrm2 = 0.f;
            for (int q = 0; q < 128; q++) nrm2 = nrm2 + raw[q] * raw[q];
            s_norm[8] = 512.f / fmaxf(__builtin_sqrtf(nrm2), FLT_EPSILON);
        }
        wave_lds_sync();
        const float scale = s_norm[8];
        int b0 = cv_round(v0 * scale), b1 = cv_round(v1 * scale);
        b0 = b0 < 0 ? 0 : (b0 > 255 ? 255 : b0);
        b1 = b1 < 0 ? 0 : (b1 > 255 ? 255 : b1);
        const _Float16 h0 = (_Float16)(float)b0, h1 = (_Float16)(float)b1;
        const unsigned po = (unsigned)jb.out;
        const unsigned pair = (unsigned)__builtin_bit_cast(uint16_t, h0) | (unsigned)__builtin_bit_cast(uint16_t, h1) << 16;
        reinterpret_cast<unsigned*>(desc + (size_t)po * 128)[lane] = pair;
        HostOut hf = host;
        const HostRows hr = host_rows(hf, ctr, frame, foff);
        if (hr.desc) reinterpret_cast<unsigned*>(hr.desc + (size_t)po * 128)[lane] = pair;
        if (hr.k3 && lane < 7) host_row(hr, hf, po, lane);
        reinterpret_cast<unsigned short*>(sidecar.codes + (size_t)po * 128)[lane] =
            (unsigned short)((b0 - 128) & 255) | (unsigned short)(((b1 - 128) & 255) << 8);
        const int c2 = __builtin_amdgcn_readlane(wave_incl_scan((b0 - 128) * (b0 - 128) + (b1 - 128) * (b1 - 128)), 63);
        if (lane == 0) sidecar.keys[po] = -(256 * c2 + (int)(po & 255));
        wave_lds_sync();  // rowpre / raw / s_norm are rewritten by the next keypoint
    }
}

void launch_descriptor(const DescJob* jobs, const Counters* ctr, const unsigned* range_keys, uint16_t* desc,
                       Sidecar sidecar, Counters* host_ctr, HostOut host, const KeypointParams& kp, const Frames& fr,
                       hipStream_t s) {
    if (kp.descExact) {
        // One wave per keypoint; each workgroup loops over keypoints.
        const int per = fr.nf <= 1 ? 2048 : std::max(512, 8192 / fr.nf);
        hipLaunchKernelGGL(k_descriptor_exact, dim3(per * fr.nf),
                           dim3(kExactWG), 0, s, jobs, ctr, desc, sidecar, host_ctr, host, fr.stride, (unsigned)fr.nf);
        return;
    }
    // Threads per keypoint: 256 for a single frame (128: 34.6 us, 512: 47.6 vs
    // 36.1 per frame, round 3), 128 for frame batches.
    constexpr int kSingleDT = 256, kBatchDT = 128;
    if (fr.nf <= 1) {
        hipLaunchKernelGGL(k_descriptor<kSingleDT>, dim3(8192), dim3(kSingleDT), 0, s, jobs, ctr, range_keys, desc,
                           sidecar, host_ctr, host, fr.stride, 1u);
    } else {
        // Workgroups per frame: 2048 at 8 frames (16384 in all).  The bigger
        // grids this kernel once had filled every CU slot and kept the other
        // stream's pyramid kernels out; with fewer workgroups (each looping
        // over more keypoints) the two co-reside: +2-3 % frame rate
        // (tools/grid_sweep.sh).
        const int per = std::max(1024, 16384 / fr.nf);
        hipLaunchKernelGGL(k_descriptor<kBatchDT>, dim3(per * fr.nf), dim3(kBatchDT), 0, s, jobs, ctr, range_keys,
                           desc, sidecar, host_ctr, host, fr.stride, (unsigned)fr.nf);
    }
}

}  // namespace sift_amd
