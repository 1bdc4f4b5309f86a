// Keypoint stages for gfx950: sub-pixel refinement, orientation histogram,
// retainBest selection, deterministic ordering and the 4x4x8 descriptor.
//
// Replaces /root/reference/sift_cuda/sift_func/SiftOps.cu and
// /root/reference/sift_cuda/utils/CudaMemcpyUtils.cu.  Semantics follow OpenCV
// 4.x; float operation order is the oracle's
// (oracle/sift_oracle.cpp adjustLocalExtrema / calcOrientationHist /
// calcSIFTDescriptor), so refined keypoints and angles are bit-exact.  The
// descriptor histogram is accumulated in a different (parallel) order, so
// descriptor bytes may differ from the oracle by +-1 (tests/test_gpu_parity.py).
#include <hip/hip_fp16.h>

#include <algorithm>

#include <cstddef>

#include "sift_kernels.h"
#include "sift_math.h"
#include "sift_refine.h"

namespace sift_amd {

__constant__ float c_exptab[64];

void upload_exp_table(const float* tab64) {
    (void)hipMemcpyToSymbol(HIP_SYMBOL(c_exptab), tab64, 64 * sizeof(float));
}

constexpr int kOriBins = 36;
constexpr float kOriSigFctr = 1.5f;
constexpr float kOriRadius = 3 * kOriSigFctr;
constexpr float kOriPeakRatio = 0.8f;


// ---------------------------------------------------------------------------
// adjustLocalExtrema, one thread per candidate of the extrema kernel's list.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_refine(PyrDesc pyr, const uint2* __restrict__ cand, unsigned capCand,
                                                Counters* __restrict__ ctr, uint32_t* __restrict__ bitmap,
                                                RefKpt* __restrict__ out, KeypointParams kp, long fs,
                                                unsigned nf) {
    // XCD-aware mapping as k_orientation's: frame = w % nf; a frame's q XCDs
    // each take a contiguous range of its candidates (scan order: neighbours
    // share their 3x3x4 rows in one L2).
    const unsigned w = blockIdx.x, per = gridDim.x / nf;
    const unsigned frame = w % nf, l = w / nf;
    const unsigned q = (nf < 8 && 8 % nf == 0) ? 8 / nf : 1;
    const unsigned range = l % q, j = l / q, step = per / q;
    const long foff = (long)frame * fs;
    cand = fptr(cand, foff);
    ctr = fptr(ctr, foff);
    bitmap = fptr(bitmap, foff);
    out = fptr(out, foff);
    const unsigned n = min(ctr->cand, capCand);
    const unsigned span = (n + q - 1) / q, iend = min(n, (range + 1) * span);
    const int lane = threadIdx.x & 63;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    // Wave-uniform loop (the append below is a wave collective).
    for (unsigned i0 = range * span + j * blockDim.x + (threadIdx.x & ~63u); i0 < iend; i0 += step * blockDim.x) {
        const unsigned i = i0 + lane;
        RefKpt k;
        long bit = 0;
        const bool acc = i < iend && refine_candidate(pyr, cand[i], bitmap, kp, foff, k, bit);
        // One counter atomic per wave (a per-lane atomic on one address
        // serialises in L2).
        const unsigned long long mask = __ballot(acc);
        if (!mask) continue;
        unsigned wbase = 0;
        if (lane == 0) wbase = atomicAdd(&ctr->refined, (unsigned)__popcll(mask));
        wbase = __builtin_amdgcn_readfirstlane(wbase);
        if (acc) {
            const unsigned slot = wbase + (unsigned)__popcll(mask & lt_mask);
            if (slot < kp.capRefined) {
                out[slot] = k;
            } else {
                atomicOr(&ctr->overflow, 2u);
                atomicAnd(&bitmap[bit >> 5], ~(1u << (bit & 31)));  // every set bit belongs to a stored keypoint
            }
        }
    }
}

// Workgroups per frame of the keypoint kernels: a single frame gets `one`
// (>= its usual item count, one item per workgroup); a batch shares about
// `one` * 2 among its frames, each workgroup looping over several items.
static int per_frame_blocks(int one, int nf) { return nf <= 1 ? one : std::max(one / 4, 2 * one / nf); }

void launch_refine(const PyrDesc& pyr, const uint2* cand, unsigned capCand, Counters* ctr, uint32_t* bitmap,
                   RefKpt* out, const KeypointParams& kp, const Frames& fr, hipStream_t s) {
    const int per = per_frame_blocks(512, fr.nf) & ~7;
    hipLaunchKernelGGL(k_refine, dim3(per * fr.nf), dim3(256), 0, s, pyr, cand, capCand, ctr, bitmap, out, kp,
                       fr.stride, (unsigned)fr.nf);
}

// ---------------------------------------------------------------------------
// calcOrientationHist + peak search (OpenCV 4.x sift.simd.hpp), one wave64
// (a 64-thread workgroup) per refined keypoint, on the Gaussian plane of the
// refined layer.  OpenCV sums each of the 36 bins sequentially in float over
// the window's samples in raster order, so that order is kept exactly:
// samples are produced 64 at a time in raster order (lane = sample; gradients
// by bounds-checked buffer loads straight from the plane); six ballots on the
// bin bits give lane b the mask and count of bin b, a DPP wave scan of the
// counts (rounded up to 4) the start of bin b's run in an LDS buffer, and every
// sample its slot (start of its bin + its lane rank inside the bin, fetched
// from lane `bin` by shuffles); pads hold +0.0.  Lane b (< 36) then adds its
// bin's values in that order to its running sum -- OpenCV's sequential sum,
// carried in a register across chunks.  <1 KB of LDS per keypoint.
// Smoothing and peak interpolation use wave shuffles, the maximum a DPP
// reduction.
// Reference: SiftOps.cu:237-376 (DoG plane, 32-lane LDS atomics, floor bins,
// no interpolation, SURVEY A-9).
// ---------------------------------------------------------------------------
typedef unsigned u32x4_k __attribute__((ext_vector_type(4)));
struct RefWords {
    u32x4_k w[2];
};

__device__ __forceinline__ RefKpt load_ref(const RefKpt* in, unsigned k) {  // scalar (constant address space)
    const __attribute__((address_space(4))) u32x4_k* c = (const __attribute__((address_space(4))) u32x4_k*)(in + k);
    RefWords r;
    r.w[0] = c[0];
    r.w[1] = c[1];
    return __builtin_bit_cast(RefKpt, r);
}

// Gradients of one 64-sample chunk of the window (lane = sample, raster
// order); the next chunk's loads are issued before a chunk is processed.
struct OriFetch {
    int i, j;
    bool valid;
    float xl, xr, yu, yd;
};
struct OriWin {
    __amdgpu_buffer_rsrc_t rsrc;
    int r, c, radius, side, total, pitch, W, H;
    unsigned mside;  // idx / side == umulhi(idx, mside)
    float expf_scale;
};
__device__ __forceinline__ OriFetch ori_fetch(const OriWin& wn, int base, int lane) {
    OriFetch f;
    const int idx = base + lane;
    f.i = (int)__umulhi((unsigned)idx, wn.mside);
    f.j = idx - (int)__umul24((unsigned)f.i, (unsigned)wn.side);
    const int y = wn.r + f.i - wn.radius, x = wn.c + f.j - wn.radius;
    f.valid = idx < wn.total && y > 0 && y < wn.H - 1 && x > 0 && x < wn.W - 1;
    // (24-bit products: rows, pitches and window sides are < 2^24.)
    const unsigned o0 = f.valid ? (__umul24((unsigned)y, (unsigned)wn.pitch) + (unsigned)x) * 4u : 0x80000000u;
    f.xl = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wn.rsrc, o0 - 4u, 0, 0));
    f.xr = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wn.rsrc, o0 + 4u, 0, 0));
    f.yu = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wn.rsrc, o0 - 4u * wn.pitch, 0, 0));
    f.yd = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wn.rsrc, o0 + 4u * wn.pitch, 0, 0));
    return f;
}

// One chunk's weighted magnitudes sorted into bin runs in `buf` (bin b's run
// starts at the returned lane-b value, 16-byte aligned, padded with +0.0 to a
// multiple of 4; lanes >= 36 get the end of the last run).
__device__ __forceinline__ int ori_sort_chunk(const OriWin& wn, const OriFetch& cur, int lane, const float* s_exptab,
                                              const unsigned long long (&lane_nb)[6], float* buf, int& c4out) {
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    const int i = cur.i, j = cur.j;
    const bool valid = cur.valid;
    const int ii = i - wn.radius, jj = j - wn.radius;
    const float dx = cur.xr - cur.xl, dy = cur.yu - cur.yd;
    // ii^2 + jj^2 in float: small integers (< 2^24), so exactly the integer
    // sum the oracle converts (no quarter-rate / 64-bit integer multiplies).
    const float fii = (float)ii, fjj = (float)jj;
    const float w = cv_exp32f(__fmaf_rn(fii, fii, fjj * fjj) * wn.expf_scale, s_exptab);
    const float ori = cv_fast_atan2(dy, dx);
    const float mag = cv_magnitude(dx, dy);
    int bin = cv_round((kOriBins / 360.f) * ori);
    // ori is in [0, 360] (cv_fast_atan2), so bin is in [0, 36]: OpenCV's
    // "if (bin >= n) bin -= n; if (bin < 0) bin += n" reduces to bin 36 -> 0.
    bin = bin >= kOriBins ? 0 : bin;
    // Radix ranks from six ballots on the bin bits (MSB first): for each
    // key k, `less(k)` = valid samples with a smaller bin and `eq(k)` =
    // those with bin k.  A sample's slot is less(bin) + its lane rank
    // inside eq(bin) (raster order); lane b < 36 sums slots
    // [less(b), less(b) + |eq(b)|) -- no LDS counts, no scan.
    // (The bin-bit ballots need not exclude invalid lanes: vmask does below.)
    unsigned long long m[6];
#pragma unroll
    for (int bit = 0; bit < 6; bit++) m[bit] = __builtin_amdgcn_ballot_w64(((bin >> bit) & 1) != 0);
    const unsigned long long vmask = __builtin_amdgcn_ballot_w64(valid);
    // Lane b's bin mask eq(b) from the ballots (bit k of b selects m[k]
    // or its complement), its count cb and, since bins are lane
    // indices, start = the exclusive prefix of cb over lanes (DPP scan).
    // (32-bit halves: eq & (m ^ nb) is one v_bitop3_b32 per half and bit;
    // nb is 0 or all ones, the same in both halves.)
    unsigned eq_lo = (unsigned)vmask, eq_hi = (unsigned)(vmask >> 32);
#pragma unroll
    for (int bit = 0; bit < 6; bit++) {
        const unsigned nb = (unsigned)lane_nb[bit];
        // LUT 0x60 = S0 & (S1 ^ S2) (truth-table index S0 << 2 | S1 << 1 | S2)
        eq_lo = __builtin_amdgcn_bitop3_b32(eq_lo, (unsigned)m[bit], nb, 0x60);
        eq_hi = __builtin_amdgcn_bitop3_b32(eq_hi, (unsigned)(m[bit] >> 32), nb, 0x60);
    }
    const unsigned long long eq_l = ((unsigned long long)eq_hi << 32) | eq_lo;
    const int cb = __popcll(eq_l);  // lanes >= 36: no sample has that bin
    // Bins start on 16-byte boundaries (runs padded to a multiple of 4
    // with +0.0, which leaves a non-negative sum unchanged), so lane b
    // reads its run with ds_read_b128 and no bounds tests.
    const int c4 = (cb + 3) & ~3;
    const int start = wave_incl_scan(c4) - c4;
    // Pads: the run's last float4 zeroed first; the samples' stores below
    // come later in this wave's LDS order and overwrite its non-pad slots.
    if (c4 > cb) *reinterpret_cast<float4*>(buf + start + c4 - 4) = make_float4(0.f, 0.f, 0.f, 0.f);
    c4out = c4;
    // A sample's less(bin) and eq(bin) are those lane `bin` just
    // computed for its own key: three shuffles instead of a second
    // radix rank per sample.
    const int less_s = __shfl(start, bin);
    const unsigned long long eq_s = ((unsigned long long)(unsigned)__shfl((int)(eq_l >> 32), bin) << 32) |
                                    (unsigned)__shfl((int)(unsigned)eq_l, bin);
    if (valid) buf[less_s + __popcll(eq_s & lt_mask)] = w * mag;
    return start;
}

// Lane b adds its bin's run [start, end) in order (OpenCV's sequential sum).
// (Reading four float4s per LDS round trip, with +0.0 past the run, measured
// 5 % slower on 16-frame batches and equal on one frame.)
__device__ __forceinline__ float ori_add_run(float acc, const float* buf, int start, int end) {
    for (int t0 = start; t0 < end; t0 += 4) {
        const float4 v = *reinterpret_cast<const float4*>(buf + t0);
        acc = acc + v.x;
        acc = acc + v.y;
        acc = acc + v.z;
        acc = acc + v.w;
    }
    return acc;
}

__device__ __forceinline__ OriWin ori_window(const PyrDesc& pyr, const RefKpt& kpt, long foff, const OctGeom*& gout) {
    const int o = kpt.o, layer = kpt.layer;
    const OctGeom& g = octave_geom(pyr, o);
    gout = &g;
    OriWin wn;
    wn.r = kpt.rc >> 16;
    wn.c = kpt.rc & 0xffff;
    const float* img = fptr(g.base, foff) + (size_t)layer * g.planeStride;
    wn.pitch = g.pitch;
    wn.W = g.W;
    wn.H = g.H;
    const float scl_octv = kpt.size * 0.5f / (float)(1 << o);
    wn.radius = cv_round(kOriRadius * scl_octv);
    const float sigma = kOriSigFctr * scl_octv;
    wn.expf_scale = -1.f / (2.f * sigma * sigma);
    wn.side = 2 * wn.radius + 1;
    wn.total = wn.side * wn.side;
    wn.mside = (unsigned)(4294967296.0 / wn.side) + 1u;
    wn.rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(img), 0, wn.H * wn.pitch * 4, 0x00020000);
    return wn;
}

// Entries of the oriented list (refined slots + appended peaks, holes included).
__device__ __forceinline__ unsigned oriented_count(const Counters* ctr, const KeypointParams& kp) {
    return min(min(ctr->refined, kp.capRefined) + ctr->oriented, kp.capOriented);
}

// Smoothing, peaks and the oriented keypoints of one histogram (lane b < 36
// holds bin b's sum), written by the calling wave: the first peak into the
// keypoint's own slot k, the others appended after the n_ref refined slots
// (one atomic per keypoint with several peaks: a per-keypoint atomic on the
// frame's one counter serialised a single frame's 4.4k waves, 40 us).
__device__ __forceinline__ void ori_emit(float acc, const RefKpt& kpt, const OctGeom& g, int fo, int lane, unsigned k,
                                         unsigned n_ref, Counters* __restrict__ ctr, OriKpt* __restrict__ out,
                                         const KeypointParams& kp) {
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    // Circular [1 4 6 4 1]/16 smoothing (SIMD body, fma form).
    const int bl = lane < kOriBins ? lane : 0;
    const float tm2 = __shfl(acc, (bl + kOriBins - 2) % kOriBins);
    const float tm1 = __shfl(acc, (bl + kOriBins - 1) % kOriBins);
    const float tp1 = __shfl(acc, (bl + 1) % kOriBins);
    const float tp2 = __shfl(acc, (bl + 2) % kOriBins);
    const float h = __fmaf_rn(tm2 + tp2, 1.f / 16.f, __fmaf_rn(tm1 + tp1, 4.f / 16.f, acc * (6.f / 16.f)));
    const float mx = wave_max(lane < kOriBins ? h : -INFINITY);
    const float mag_thr = (float)(mx * kOriPeakRatio);
    const float hl = __shfl(h, (bl + kOriBins - 1) % kOriBins);
    const float hr = __shfl(h, (bl + 1) % kOriBins);
    const bool peak = lane < kOriBins && h > hl && h > hr && h >= mag_thr;
    const unsigned long long mask = __ballot(peak);
    if (!mask) {
        if (lane == 0) {
            OriKpt hole{};
            hole.bucket = kHoleBucket;
            out[k] = hole;
        }
        return;
    }
    const int npk = __popcll(mask), first = __builtin_ctzll(mask);
    unsigned basepos = 0;
    if (lane == 0 && npk > 1) basepos = atomicAdd(&ctr->oriented, (unsigned)(npk - 1));
    basepos = __builtin_amdgcn_readfirstlane(basepos);
    if (peak) {
        const int layer = kpt.layer, r = kpt.rc >> 16, c = kpt.rc & 0xffff;
        float bin = (float)lane + 0.5f * (hl - hr) / (hl - 2 * h + hr);
        bin = bin < 0 ? kOriBins + bin : bin >= kOriBins ? bin - kOriBins : bin;
        float angle = 360.f - (float)((360.f / kOriBins) * bin);
        if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
        OriKpt ok;
        ok.x = kpt.x;
        ok.y = kpt.y;
        ok.size = kpt.size;
        ok.angle = angle;
        ok.response = kpt.response;
        ok.octave = kpt.octave;
        if (fo < 0) {
            const float scale = 1.f / (float)(1 << -fo);
            ok.octave = (kpt.octave & ~255) | ((kpt.octave + fo) & 255);
            ok.x *= scale;
            ok.y *= scale;
            ok.size *= scale;
        }
        ok.bucket = g.rowBase + (layer - 1) * g.H + r;
        ok.sub = (c << 6) | lane;
        const unsigned pos = lane == first ? k : n_ref + basepos + (unsigned)__popcll(mask & lt_mask) - 1u;
        if (pos < kp.capOriented)
            out[pos] = ok;
        else
            atomicOr(&ctr->overflow, 4u);
    }
}

__device__ __forceinline__ void ori_clear_bit(uint32_t* bitmap, const OctGeom& g, const RefKpt& kpt) {
    // the keypoint's dedupe bit, for the next frame (no memset node)
    const int layer = kpt.layer, r = kpt.rc >> 16, c = kpt.rc & 0xffff;
    const long bit = g.bitBase + ((long)(layer - 1) * g.H + r) * g.W + c;
    atomicAnd(&bitmap[bit >> 5], ~(1u << (bit & 31)));
}

// Chunks whose gradient loads are in flight: 2, 3, 4 measured equal on one
// frame and on batches (round 2).  Two chunks sorted per step (their
// dependence chains interleaved in one wave, round 4): 140 vs 131 us per
// 16-frame launch, single frames equal.
constexpr int kOriAhead = 1;
// XCD-aware keypoint mapping (a 1-D grid of nf * per one-wave workgroups;
// the dispatcher hands workgroup w to XCD w % 8, and each XCD has its own L2).
// Frame = w % nf, so with nf a multiple of 8 every frame lives on one XCD (its
// windows are fetched into one L2): 16-frame launches fetch 209.9 MB instead
// of 270.4 (the round-4 mapping, frame = blockIdx.y with keypoints
// round-robin over blockIdx.x, put every frame's neighbouring keypoints on all
// 8 XCDs), against 192.1 MB for a perfect cache at 128-byte lines
// (tools/window_line_model.py).
__global__ __launch_bounds__(64) void k_orientation(PyrDesc pyr, const RefKpt* __restrict__ in,
                                                    Counters* __restrict__ ctr, OriKpt* __restrict__ out,
                                                    uint32_t* __restrict__ bitmap, KeypointParams kp, long fs,
                                                    unsigned nf) {
    __shared__ __attribute__((aligned(16))) float chunk[64 + 3 * kOriBins];  // bin runs padded to 4
    // Below 8 frames a frame's keypoints stay round-robin over its XCDs
    // (q = 1): single frames are latency-bound and contiguous per-XCD ranges
    // unbalance the XCDs (C2 single frame 26.7 -> 29.8 us with ranges).
    const unsigned w = blockIdx.x, per = gridDim.x / nf;
    const unsigned frame = w % nf, l = w / nf;
    const unsigned q = 1;
    const unsigned range = l % q, j = l / q, step = per / q;
    const long foff = (long)frame * fs;
    in = fptr(in, foff);
    ctr = fptr(ctr, foff);
    out = fptr(out, foff);
    bitmap = fptr(bitmap, foff);
    __shared__ float s_exptab[64];
    const int lane = threadIdx.x;
    s_exptab[lane] = c_exptab[lane];
    unsigned long long lane_nb[6];  // all ones where bit k of the lane index is 0
#pragma unroll
    for (int bit = 0; bit < 6; bit++) lane_nb[bit] = ((lane >> bit) & 1) ? 0ull : ~0ull;
    const unsigned n = min(ctr->refined, kp.capRefined);
    const int fo = pyr.firstOctave;
    const unsigned span = (n + q - 1) / q, kend = min(n, (range + 1) * span);
    for (unsigned k = range * span + j; k < kend; k += step) {
        const RefKpt kpt = load_ref(in, k);
        const OctGeom* gp;
        const OriWin wn = ori_window(pyr, kpt, foff, gp);
        if (lane == 0) ori_clear_bit(bitmap, *gp, kpt);
        float acc = 0.f;  // temphist[lane] for lane < 36
        // Loads run kOriAhead chunks ahead of the chunk being sorted (ring of
        // fetches): a large keypoint's chunks are a dependent chain, and
        // with one chunk in flight each waited for a memory round trip.
        OriFetch ring[kOriAhead];
#pragma unroll
        for (int q = 0; q < kOriAhead; q++) ring[q] = ori_fetch(wn, 64 * q, lane);
        for (int base = 0; base < wn.total; base += 64) {
            const OriFetch cur = ring[0];
#pragma unroll
            for (int q = 0; q + 1 < kOriAhead; q++) ring[q] = ring[q + 1];
            if (base + 64 * kOriAhead < wn.total) ring[kOriAhead - 1] = ori_fetch(wn, base + 64 * kOriAhead, lane);
            int c4;
            const int start = ori_sort_chunk(wn, cur, lane, s_exptab, lane_nb, chunk, c4);
            lds_barrier();
            // Lane b (< 36; others have cb = 0) adds its bin's values in order.
            acc = ori_add_run(acc, chunk, start, start + c4);
            lds_barrier();  // chunk is rewritten by the next 64 samples
        }
        ori_emit(acc, kpt, *gp, fo, lane, k, n, ctr, out, kp);
    }
}

void launch_orientation(const PyrDesc& pyr, const RefKpt* in, Counters* ctr, OriKpt* out, uint32_t* bitmap,
                        const KeypointParams& kp, const Frames& fr, hipStream_t s) {
    // One-wave workgroups per frame: 8192 for a single frame, 1024 at 8 frames.
    // Grids that fill every wave slot keep the other stream's pyramid kernels
    // out; this size lets them co-reside (+2-4 % frame rate, tools/grid_sweep.sh).
    // (512 per frame at 16 frames; 256 measured equal, round 2.)  per is a
    // multiple of 8: every XCD range gets the same number of workgroups.
    const int per = fr.nf <= 1 ? 8192 : std::max(256, 8192 / fr.nf) & ~7;
    hipLaunchKernelGGL(k_orientation, dim3(per * fr.nf), dim3(64), 0, s, pyr, in, ctr, out, bitmap, kp, fr.stride,
                       (unsigned)fr.nf);
}

// ---------------------------------------------------------------------------
// KeyPointsFilter::retainBest: response threshold = the numFeatures-th largest
// response (positive floats order like their bit patterns), by a 4-pass 8-bit
// MSB radix select in one workgroup.  Keeps every keypoint with response >= it,
// which is exactly the set OpenCV's nth_element + partition keeps.
// Reference: keeps the first numFeatures in octave order (CudaMemcpyUtils.cu:38-49).
// ---------------------------------------------------------------------------
// Radix-select digit step (wave 0 of the workgroup, all 64 lanes): the
// largest digit d with sum(hist[d' > d]) + hist[d] >= k, and k minus the
// count above it -- the sequential top-down scan of KeyPointsFilter's
// nth_element threshold, done with 4 bins per lane and a DPP scan (no
// 256-step dependent LDS loop).  No such digit: (0, k), as the loop gives.
__device__ __forceinline__ void radix_digit(const unsigned* hist, unsigned k, int lane, int& digit, unsigned& newk) {
    unsigned h[4], bsum = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        h[j] = hist[255 - 4 * lane - j];  // descending digits
        bsum += h[j];
    }
    unsigned cum = (unsigned)wave_incl_scan((int)bsum) - bsum;  // counts of the higher digits
    int dl = -1;
    unsigned kl = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        if (dl < 0 && cum + h[j] >= k) {
            dl = 255 - 4 * lane - j;
            kl = k - cum;
        }
        cum += h[j];
    }
    const unsigned long long hit = __ballot(dl >= 0);
    if (!hit) {
        digit = 0;
        newk = k;
        return;
    }
    const int src = __builtin_ctzll(hit);
    digit = __builtin_amdgcn_readlane(dl, src);
    newk = (unsigned)__builtin_amdgcn_readlane((int)kl, src);
}

__global__ __launch_bounds__(1024) void k_select(const OriKpt* __restrict__ kpts, Counters* __restrict__ ctr,
                                                 unsigned* __restrict__ zero_range, KeypointParams kp, long fs) {
    __shared__ unsigned hist[256];
    __shared__ unsigned s_prefix, s_k;
    const long foff = blockIdx.y * fs;  // frame blockIdx.y
    kpts = fptr(kpts, foff);
    ctr = fptr(ctr, foff);
    zero_range = fptr(zero_range, foff);
    const unsigned n = oriented_count(ctr, kp);
    const int tid = threadIdx.x, lane = tid & 63;
    for (int i = tid; i < 2 * kRangeSlots; i += 1024) zero_range[i] = 0u;  // next frame's range keys
    if (tid == 0) ctr->pad[1] >>= kHostReqShift;  // host results request -> level (HostOut)
    if (kp.numFeatures <= 0 || n <= (unsigned)kp.numFeatures) {
        if (tid == 0) ctr->thr_bits = 0u;
        return;
    }
    if (tid == 0) {
        s_prefix = 0;
        s_k = (unsigned)kp.numFeatures;
    }
    unsigned pmask = 0;
    for (int shift = 24; shift >= 0; shift -= 8) {
        for (int i = tid; i < 256; i += 1024) hist[i] = 0;
        __syncthreads();
        const unsigned prefix = s_prefix;
        for (unsigned i = tid; i < n; i += 1024) {
            const unsigned b = __float_as_uint(kpts[i].response);
            if ((b & pmask) == prefix) atomicAdd(&hist[(b >> shift) & 255u], 1u);
        }
        __syncthreads();
        if (tid < 64) {
            int digit;
            unsigned k;
            radix_digit(hist, s_k, lane, digit, k);
            if (tid == 0) {
                s_k = k;
                s_prefix = prefix | ((unsigned)digit << shift);
            }
        }
        pmask |= 255u << shift;
        __syncthreads();
    }
    if (tid == 0) ctr->thr_bits = s_prefix;
}

void launch_select(const OriKpt* kpts, Counters* ctr, unsigned* zero_range, const KeypointParams& kp, const Frames& fr,
                   hipStream_t s) {
    hipLaunchKernelGGL(k_select, dim3(1, fr.nf), dim3(1024), 0, s, kpts, ctr, zero_range, kp, fr.stride);
}

// ---------------------------------------------------------------------------
// Deterministic output order without a comparison sort: counting sort into
// row buckets (octave, layer, r), then rank by (c, peak) inside each bucket.
// Atomic compaction upstream makes arrival order nondeterministic; this makes
// the output order a pure function of the keypoint set.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_bucket_count(const OriKpt* __restrict__ kpts, const Counters* __restrict__ ctr,
                                                      unsigned* __restrict__ bcount, int* __restrict__ slot,
                                                      KeypointParams kp, long fs) {
    const long foff = blockIdx.y * fs;  // frame blockIdx.y
    kpts = fptr(kpts, foff);
    ctr = fptr(ctr, foff);
    bcount = fptr(bcount, foff);
    slot = fptr(slot, foff);
    const unsigned n = oriented_count(ctr, kp);
    const float thr = __uint_as_float(ctr->thr_bits);
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const OriKpt k = kpts[i];
        slot[i] = k.bucket != kHoleBucket && k.response >= thr ? (int)atomicAdd(&bcount[k.bucket], 1u) : -1;
    }
}

void launch_bucket_count(const OriKpt* kpts, const Counters* ctr, unsigned* bcount, int* slot,
                         const KeypointParams& kp, const Frames& fr, hipStream_t s) {
    hipLaunchKernelGGL(k_bucket_count, dim3(256, fr.nf), dim3(256), 0, s, kpts, ctr, bcount, slot, kp, fr.stride);
}

__global__ __launch_bounds__(1024) void k_bucket_scan(const unsigned* __restrict__ bcount, unsigned* __restrict__ boff,
                                                      Counters* __restrict__ ctr, KeypointParams kp, long fs) {
    __shared__ unsigned wsum[16];
    const long foff = blockIdx.y * fs;  // frame blockIdx.y
    bcount = fptr(bcount, foff);
    boff = fptr(boff, foff);
    ctr = fptr(ctr, foff);
    __shared__ unsigned carry_s;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (tid == 0) carry_s = 0;
    __syncthreads();
    for (int base = 0; base < kp.numBuckets; base += 1024) {
        const int i = base + tid;
        const unsigned v = i < kp.numBuckets ? bcount[i] : 0u;
        const unsigned x = (unsigned)wave_incl_scan((int)v);
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        unsigned wpre = 0, tot = 0;
        for (int k = 0; k < 16; k++) {
            if (k < w) wpre += wsum[k];
            tot += wsum[k];
        }
        const unsigned carry = carry_s;
        if (i < kp.numBuckets) boff[i] = carry + wpre + x - v;
        __syncthreads();
        if (tid == 0) carry_s = carry + tot;
        __syncthreads();
    }
    if (tid == 0) {
        const unsigned total = carry_s;
        ctr->final_n = min(total, kp.capFinal);
        if (total > kp.capFinal) atomicOr(&ctr->overflow, 8u);
    }
}

void launch_bucket_scan(unsigned* bcount, unsigned* boff, Counters* ctr, const KeypointParams& kp, const Frames& fr,
                        hipStream_t s) {
    hipLaunchKernelGGL(k_bucket_scan, dim3(1, fr.nf), dim3(1024), 0, s, bcount, boff, ctr, kp, fr.stride);
}

__global__ __launch_bounds__(256) void k_bucket_scatter(const OriKpt* __restrict__ kpts, const Counters* __restrict__ ctr,
                                                        const unsigned* __restrict__ boff, const int* __restrict__ slot,
                                                        int* __restrict__ order, KeypointParams kp, long fs) {
    const long foff = blockIdx.y * fs;  // frame blockIdx.y
    kpts = fptr(kpts, foff);
    ctr = fptr(ctr, foff);
    boff = fptr(boff, foff);
    slot = fptr(slot, foff);
    order = fptr(order, foff);
    const unsigned n = oriented_count(ctr, kp);
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const int s = slot[i];
        if (s >= 0) order[boff[kpts[i].bucket] + (unsigned)s] = (int)i;
    }
}

void launch_bucket_scatter(const OriKpt* kpts, const Counters* ctr, const unsigned* boff, const int* slot, int* order,
                           const KeypointParams& kp, const Frames& fr, hipStream_t s) {
    hipLaunchKernelGGL(k_bucket_scatter, dim3(256, fr.nf), dim3(256), 0, s, kpts, ctr, boff, slot, order, kp,
                       fr.stride);
}

// ---------------------------------------------------------------------------
// k_select + k_bucket_count + k_bucket_scan + k_bucket_scatter in ONE
// workgroup (one launch instead of four; ~10^4 keypoints per frame): the
// retainBest threshold by the same radix select, row-bucket counts by LDS
// atomics, their exclusive scan in place in LDS, and the scatter into bucket
// order.  Written to global memory: thr_bits, final_n, and for every
// non-empty bucket its count and offset (k_bucket_rank reads both and zeroes
// the counts), and order[].  Used when the buckets fit in LDS
// (kOrderMaxBuckets); the four kernels above remain for larger pyramids.
// ---------------------------------------------------------------------------
// Segment (octave, layer) of a final keypoint in the bucket order (k_order's
// job-order segments; JobOrder).
__device__ __forceinline__ int lpt_seg(int packed_octave, int fo, int L) {
    const int o = (int)(signed char)(packed_octave & 255) - fo, layer = (packed_octave >> 8) & 255;
    return o * L + layer - 1;
}

__global__ __launch_bounds__(1024) void k_order(PyrDesc pyr, const OriKpt* __restrict__ kpts, Counters* __restrict__ ctr,
                                                unsigned* __restrict__ zero_range, unsigned* __restrict__ bcount,
                                                unsigned* __restrict__ boff, int* __restrict__ slot,
                                                int* __restrict__ order, JobOrder* __restrict__ jord,
                                                KeypointParams kp, long fs) {
    extern __shared__ unsigned s_bucket[];  // counts, then exclusive offsets
    __shared__ unsigned hist[256], wsum[16];
    __shared__ unsigned s_prefix, s_k;
    __shared__ unsigned s_seg[kLptSegs];  // kept keypoints per (octave, layer) segment
    const int L = pyr.L, fo = pyr.firstOctave;
    const bool lpt = kp.descExact && L <= 8 && pyr.nOct * L <= kLptSegs;  // exact mode only (JobOrder)
    const long foff = blockIdx.y * fs;  // frame blockIdx.y
    kpts = fptr(kpts, foff);
    ctr = fptr(ctr, foff);
    zero_range = fptr(zero_range, foff);
    bcount = fptr(bcount, foff);
    boff = fptr(boff, foff);
    slot = fptr(slot, foff);
    order = fptr(order, foff);
    jord = fptr(jord, foff);
    const unsigned n = oriented_count(ctr, kp);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nb = kp.numBuckets;
    for (int i = tid; i < 2 * kRangeSlots; i += 1024) zero_range[i] = 0u;  // next frame's range keys
    for (int i = tid; i < nb; i += 1024) s_bucket[i] = 0u;
    if (tid == 0) ctr->pad[1] >>= kHostReqShift;  // host results request -> level (HostOut)
    if (tid < kLptSegs) s_seg[tid] = 0u;
    if (tid == 0) {
        s_prefix = 0;
        s_k = (unsigned)kp.numFeatures;
    }
    __syncthreads();
    // retainBest threshold (k_select's radix select)
    const bool sel = kp.numFeatures > 0 && n > (unsigned)kp.numFeatures;
    if (sel) {
        unsigned pmask = 0;
        for (int shift = 24; shift >= 0; shift -= 8) {
            for (int i = tid; i < 256; i += 1024) hist[i] = 0;
            __syncthreads();
            const unsigned prefix = s_prefix;
            for (unsigned i = tid; i < n; i += 1024) {
                const unsigned b = __float_as_uint(kpts[i].response);
                if ((b & pmask) == prefix) atomicAdd(&hist[(b >> shift) & 255u], 1u);
            }
            __syncthreads();
            if (tid < 64) {
                int digit;
                unsigned k;
                radix_digit(hist, s_k, lane, digit, k);
                if (tid == 0) {
                    s_k = k;
                    s_prefix = prefix | ((unsigned)digit << shift);
                }
            }
            pmask |= 255u << shift;
            __syncthreads();
        }
    }
    const unsigned thr_bits = sel ? s_prefix : 0u;
    if (tid == 0) ctr->thr_bits = thr_bits;
    const float thr = __uint_as_float(thr_bits);
    // counts (the slot order inside a bucket is re-ranked by k_bucket_rank).
    // Up to kOrderRegs * 1024 entries (a frame's usual count) keep their
    // bucket and slot in registers for the scatter below (one 16-byte load
    // of {response, octave, bucket, sub} per entry, no slot[] round trip);
    // larger lists go through slot[], four entries' loads in flight.
    constexpr int kOrderRegs = 8;
    static_assert(sizeof(OriKpt) == 32 && offsetof(OriKpt, response) == 16 && offsetof(OriKpt, bucket) == 24,
                  "k_order reads {response, octave, bucket, sub} as the entry's second float4");
    const bool inreg = n <= kOrderRegs * 1024u;
    int rbk[kOrderRegs], rsl[kOrderRegs];
    if (inreg) {
        float4 q[kOrderRegs];
        const float4* kq = reinterpret_cast<const float4*>(kpts);
#pragma unroll
        for (int u = 0; u < kOrderRegs; u++) q[u] = kq[2 * min(tid + 1024u * u, n - 1) + 1];
#pragma unroll
        for (int u = 0; u < kOrderRegs; u++) {
            const unsigned i = tid + 1024u * u;
            rbk[u] = __float_as_int(q[u].z);
            const bool keep = i < n && (unsigned)rbk[u] != kHoleBucket && q[u].x >= thr;
            rsl[u] = keep ? (int)atomicAdd(&s_bucket[rbk[u]], 1u) : -1;
            if (keep && lpt) atomicAdd(&s_seg[lpt_seg(__float_as_int(q[u].y), fo, L)], 1u);
        }
    } else {
        for (unsigned i0 = tid; i0 < n; i0 += 4 * 1024) {
            int bk[4], oc[4];
            float rs[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const unsigned i = min(i0 + 1024u * u, n - 1);
                bk[u] = kpts[i].bucket;
                rs[u] = kpts[i].response;
                oc[u] = kpts[i].octave;
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const unsigned i = i0 + 1024u * u;
                if (i < n) {
                    const bool keep = (unsigned)bk[u] != kHoleBucket && rs[u] >= thr;
                    slot[i] = keep ? (int)atomicAdd(&s_bucket[bk[u]], 1u) : -1;
                    if (keep && lpt) atomicAdd(&s_seg[lpt_seg(oc[u], fo, L)], 1u);
                }
            }
        }
    }
    __syncthreads();
    // Exclusive scan in place: each thread sums a contiguous run of buckets,
    // one workgroup scan of the 1024 run sums, then each run is rewritten as
    // offsets; non-empty buckets are published for k_bucket_rank.
    {
        const int per = (nb + 1023) / 1024;
        const int b0 = min(tid * per, nb), b1 = min(b0 + per, nb);
        unsigned sum = 0;
        for (int b = b0; b < b1; b++) sum += s_bucket[b];
        const unsigned x = (unsigned)wave_incl_scan((int)sum);
        if (lane == 63) wsum[w] = x;
        __syncthreads();
        unsigned run = x - sum, total = 0;
        for (int k = 0; k < 16; k++) {
            if (k < w) run += wsum[k];
            total += wsum[k];
        }
        for (int b = b0; b < b1; b++) {
            const unsigned v = s_bucket[b];
            if (v) {
                s_bucket[b] = run;
                bcount[b] = v;
                boff[b] = run;
            }
            run += v;
        }
        if (tid == 0) {
            ctr->final_n = min(total, kp.capFinal);
            ctr->pad[0] = total;  // entries of `order` (k_rank_final)
            if (total > kp.capFinal) atomicOr(&ctr->overflow, 8u);
            // Job order, longest first (JobOrder): segments in bucket order
            // give the final positions, layers high to low the job positions.
            const bool use = lpt && total <= kp.capFinal;
            jord->valid = use;
            if (use) {
                const int ns = pyr.nOct * L;
                unsigned start = 0;
                for (int sg = 0; sg < ns; sg++) {
                    jord->segStart[sg] = (int)start;
                    start += s_seg[sg];
                }
                unsigned job = 0;
                for (int l = L; l >= 1; l--)
                    for (int o = 0; o < pyr.nOct; o++) {
                        jord->jobBase[o * L + l - 1] = (int)job;
                        job += s_seg[o * L + l - 1];
                    }
            }
        }
    }
    __syncthreads();
    // scatter (slot[i] was written by this same thread above)
    if (inreg) {
#pragma unroll
        for (int u = 0; u < kOrderRegs; u++)
            if (rsl[u] >= 0) order[s_bucket[rbk[u]] + (unsigned)rsl[u]] = (int)(tid + 1024u * u);
    } else {
        for (unsigned i = tid; i < n; i += 1024) {
            const int sl = slot[i];
            if (sl >= 0) order[s_bucket[kpts[i].bucket] + (unsigned)sl] = (int)i;
        }
    }
}

bool launch_order(const PyrDesc& pyr, const OriKpt* kpts, Counters* ctr, unsigned* zero_range, unsigned* bcount,
                  unsigned* boff, int* slot, int* order, JobOrder* jord, const KeypointParams& kp, const Frames& fr,
                  hipStream_t s) {
    if (kp.numBuckets > kOrderMaxBuckets) return false;
    hipLaunchKernelGGL(k_order, dim3(1, fr.nf), dim3(1024), sizeof(unsigned) * (size_t)kp.numBuckets, s, pyr, kpts,
                       ctr, zero_range, bcount, boff, slot, order, jord, kp, fr.stride);
    return true;
}

// Descriptor job of one final keypoint: calcDescriptorsComputer (unpackOctave,
// octave scale, angle flip 360 - angle) and the head of calcSIFTDescriptor
// (cos/sin / hist_width, radius clamped to the image diagonal), computed once
// per keypoint here so the descriptor workgroup starts from scalar loads.
__device__ DescJob make_desc_job(const PyrDesc& pyr, const OriKpt& kpt, long foff) {
    DescJob j;
    int octave = kpt.octave & 255;
    const int layer = (kpt.octave >> 8) & 255;
    octave = octave < 128 ? octave : (-128 | octave);
    const float scale = octave >= 0 ? 1.f / (float)(1 << octave) : (float)(1 << -octave);
    const float size = kpt.size * scale;
    const float ptfx = kpt.x * scale, ptfy = kpt.y * scale;
    const OctGeom& g = pyr.oct[octave - pyr.firstOctave];
    j.img = fptr(g.base, foff) + (size_t)layer * g.planeStride;
    j.pitch = g.pitch;
    j.rows = g.H;
    j.cols = g.W;
    float angle = 360.f - kpt.angle;
    if (fabsf(angle - 360.f) < FLT_EPSILON) angle = 0.f;
    j.angle = angle;
    const float scl = size * 0.5f;
    j.ptx = cv_round(ptfx);
    j.pty = cv_round(ptfy);
    j.hist_width = 3.f * scl;
    int radius = cv_round(j.hist_width * 1.4142135623730951f * (float)(4 + 1) * 0.5f);
    radius = min(radius, (int)sqrt((double)g.W * g.W + (double)g.H * g.H));
    j.radius = radius;
    const float arg = angle * (float)(M_PI / 180);  // cosf/sinf via double
    j.cos_t = (float)cos((double)arg) / j.hist_width;
    j.sin_t = (float)sin((double)arg) / j.hist_width;
    j.out = 0;
    j.pad[0] = j.pad[1] = j.pad[2] = 0;
    return j;
}

// Final order inside each row bucket (rank by sub key), then write the
// keypoint's outputs (reference layout Detector.hh:54-57: float3 {x, y,
// layer}, float4 {packed octave, size, response, angle}) and its descriptor job.
__global__ __launch_bounds__(256) void k_bucket_rank(PyrDesc pyr, const OriKpt* __restrict__ kpts,
                                                     unsigned* __restrict__ bcount,
                                                     const unsigned* __restrict__ boff, const int* __restrict__ order,
                                                     const Counters* __restrict__ ctr, DescJob* __restrict__ jobs,
                                                     float* __restrict__ kpts3, float* __restrict__ feats4,
                                                     KeypointParams kp, long fs) {
    const long foff = blockIdx.y * fs;  // frame blockIdx.y
    kpts = fptr(kpts, foff);
    bcount = fptr(bcount, foff);
    boff = fptr(boff, foff);
    order = fptr(order, foff);
    ctr = fptr(ctr, foff);
    jobs = fptr(jobs, foff);
    kpts3 = fptr(kpts3, foff);
    feats4 = fptr(feats4, foff);
    const int lane = threadIdx.x & 63;
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int nwaves = gridDim.x * 4;
    const unsigned cap = kp.capFinal;
    for (int b = wave; b < kp.numBuckets; b += nwaves) {
        const unsigned cnt = bcount[b];
        if (cnt == 0) continue;
        const unsigned base = boff[b];
        for (unsigned e0 = 0; e0 < cnt; e0 += 64) {
            const unsigned e = e0 + lane;
            int idx = -1, se = 0;
            if (e < cnt) {
                idx = order[base + e];
                se = kpts[idx].sub;
            }
            unsigned rank = 0;
            for (unsigned f0 = 0; f0 < cnt; f0 += 64) {
                const unsigned f = f0 + lane;
                const int sf = f < cnt ? kpts[order[base + f]].sub : 0x7fffffff;
                const unsigned lim = min(64u, cnt - f0);
                for (unsigned l = 0; l < lim; l++) rank += (unsigned)(__shfl(sf, (int)l) < se);
            }
            const unsigned pos = base + rank;
            if (e < cnt && pos < cap) {
                const OriKpt k = kpts[idx];
                DescJob j = make_desc_job(pyr, k, foff);
                j.out = (int)pos;
                jobs[pos] = j;
                kpts3[3 * (size_t)pos + 0] = k.x;
                kpts3[3 * (size_t)pos + 1] = k.y;
                kpts3[3 * (size_t)pos + 2] = (float)((k.octave >> 8) & 255);
                reinterpret_cast<float4*>(feats4)[pos] = make_float4((float)k.octave, k.size, k.response, k.angle);
            }
        }
        if (lane == 0) bcount[b] = 0u;  // zero for the next frame (no memset node)
    }
}

// The same final order, parallel over keypoints instead of buckets (k_order
// path, where bcount/boff are rewritten every frame for every non-empty bucket
// and nothing reads an empty one): thread per position of `order`; its
// keypoint's rank inside its row bucket = bucket entries with a smaller sub
// key (buckets hold a few keypoints).  Every keypoint's chain of dependent
// loads runs at once instead of one bucket after another per wave.
__global__ __launch_bounds__(256) void k_rank_final(PyrDesc pyr, const OriKpt* __restrict__ kpts,
                                                    const unsigned* __restrict__ bcount,
                                                    const unsigned* __restrict__ boff, const int* __restrict__ order,
                                                    const Counters* __restrict__ ctr, const JobOrder* __restrict__ jord,
                                                    DescJob* __restrict__ jobs, float* __restrict__ kpts3,
                                                    float* __restrict__ feats4, KeypointParams kp, long fs) {
    const long foff = blockIdx.y * fs;  // frame blockIdx.y
    kpts = fptr(kpts, foff);
    bcount = fptr(bcount, foff);
    boff = fptr(boff, foff);
    order = fptr(order, foff);
    ctr = fptr(ctr, foff);
    jord = fptr(jord, foff);
    jobs = fptr(jobs, foff);
    kpts3 = fptr(kpts3, foff);
    feats4 = fptr(feats4, foff);
    // Every entry of `order` (a bucket straddling capFinal still has
    // positions below it); positions >= capFinal are dropped.
    const unsigned n = ctr->pad[0];
    const unsigned cap = kp.capFinal;
    const bool lpt = jord->valid != 0;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
        const OriKpt k = kpts[order[i]];
        const unsigned base = boff[k.bucket], cnt = bcount[k.bucket];
        unsigned rank = 0;
        for (unsigned f = 0; f < cnt; f++) rank += (unsigned)(kpts[order[base + f]].sub < k.sub);
        const unsigned pos = base + rank;
        if (pos < cap) {
            DescJob j = make_desc_job(pyr, k, foff);
            j.out = (int)pos;
            int q = (int)pos;
            if (lpt) {
                const int sg = lpt_seg(k.octave, pyr.firstOctave, pyr.L);
                q = jord->jobBase[sg] + ((int)pos - jord->segStart[sg]);
            }
            jobs[q] = j;
            kpts3[3 * (size_t)pos + 0] = k.x;
            kpts3[3 * (size_t)pos + 1] = k.y;
            kpts3[3 * (size_t)pos + 2] = (float)((k.octave >> 8) & 255);
            reinterpret_cast<float4*>(feats4)[pos] = make_float4((float)k.octave, k.size, k.response, k.angle);
        }
    }
}

void launch_rank_final(const PyrDesc& pyr, const OriKpt* kpts, const unsigned* bcount, const unsigned* boff,
                       const int* order, const Counters* ctr, const JobOrder* jord, DescJob* jobs, float* kpts3,
                       float* feats4, const KeypointParams& kp, const Frames& fr, hipStream_t s) {
    hipLaunchKernelGGL(k_rank_final, dim3(64, fr.nf), dim3(256), 0, s, pyr, kpts, bcount, boff, order, ctr, jord, jobs,
                       kpts3, feats4, kp, fr.stride);
}

void launch_bucket_rank(const PyrDesc& pyr, const OriKpt* kpts, unsigned* bcount, const unsigned* boff,
                        const int* order, const Counters* ctr, DescJob* jobs, float* kpts3, float* feats4,
                        const KeypointParams& kp, const Frames& fr, hipStream_t s) {
    hipLaunchKernelGGL(k_bucket_rank, dim3(per_frame_blocks(256, fr.nf), fr.nf), dim3(256), 0, s, pyr, kpts, bcount,
                       boff, order, ctr, jobs, kpts3, feats4, kp, fr.stride);
}

// ---------------------------------------------------------------------------
// Frame rows copied by a small grid on the frame's lane stream: a host-input
// frame's staging (mapped pinned host memory) into device memory before the
// frame's first kernel, and a micro-batch's frames into the lane's group
// input.  kStageWg workgroups with four 16-byte loads in flight per thread
// (1 MiB in flight, the PCIe link's rate) hold a few CUs for the transfer,
// where the first blur reading the pinned buffer itself held every tile's
// workgroup for it and slowed the other lanes;
// a runtime 2-D copy of a device frame took a slow path (0.165 vs 0.093
// ms/frame for f32 vs u8 micro-batches).  16-byte units when the rows and
// pitches allow, bytes otherwise.  `flag` (nullable): thread 0 of
// workgroup 0 stores flag_val there (a host frame's results request in its
// Counters, HostOut).
// ---------------------------------------------------------------------------
constexpr int kStageUnroll = 4;
__global__ __launch_bounds__(256) void k_copy_rows16(const char* __restrict__ src, size_t spitch, char* __restrict__ dst,
                                                     size_t dpitch, unsigned row16, unsigned n16,
                                                     unsigned* __restrict__ flag, unsigned flag_val) {
    const unsigned nt = gridDim.x * blockDim.x;
    if (flag && blockIdx.x == 0 && threadIdx.x == 0) *flag = flag_val;
    auto at = [&](unsigned i, size_t pitch) { return (size_t)(i / row16) * pitch + (size_t)(i % row16) * 16; };
    unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    for (; i + (kStageUnroll - 1) * nt < n16; i += kStageUnroll * nt) {
        uint4 v[kStageUnroll];
#pragma unroll
        for (int u = 0; u < kStageUnroll; u++) v[u] = *reinterpret_cast<const uint4*>(src + at(i + u * nt, spitch));
#pragma unroll
        for (int u = 0; u < kStageUnroll; u++) *reinterpret_cast<uint4*>(dst + at(i + u * nt, dpitch)) = v[u];
    }
    for (; i < n16; i += nt) *reinterpret_cast<uint4*>(dst + at(i, dpitch)) = *reinterpret_cast<const uint4*>(src + at(i, spitch));
}
__global__ __launch_bounds__(256) void k_copy_rows1(const unsigned char* __restrict__ src, size_t spitch,
                                                    unsigned char* __restrict__ dst, size_t dpitch, unsigned rowB,
                                                    unsigned n, unsigned* __restrict__ flag, unsigned flag_val) {
    if (flag && blockIdx.x == 0 && threadIdx.x == 0) *flag = flag_val;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x)
        dst[(size_t)(i / rowB) * dpitch + i % rowB] = src[(size_t)(i / rowB) * spitch + i % rowB];
}

void launch_copy_rows(const void* src, size_t spitch, void* dst, size_t dpitch, size_t rowB, int rows, int wgs,
                      hipStream_t s, unsigned* flag, unsigned flag_val) {
    const bool v16 = ((uintptr_t)src | (uintptr_t)dst | spitch | dpitch | rowB) % 16 == 0;
    if (v16)
        hipLaunchKernelGGL(k_copy_rows16, dim3(wgs), dim3(256), 0, s, static_cast<const char*>(src), spitch,
                           static_cast<char*>(dst), dpitch, (unsigned)(rowB / 16), (unsigned)(rowB / 16 * rows), flag, flag_val);
    else
        hipLaunchKernelGGL(k_copy_rows1, dim3(wgs), dim3(256), 0, s, static_cast<const unsigned char*>(src), spitch,
                           static_cast<unsigned char*>(dst), dpitch, (unsigned)rowB, (unsigned)(rowB * rows), flag, flag_val);
}

}  // namespace sift_amd
