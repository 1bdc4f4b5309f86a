// C ABI of libsift_hip.so: Detector state, buffer layout in HBM, the hipGraph
// of the whole fixed-shape pipeline, timing hooks and the matcher handle.
//
// Replaces /root/reference/sift_cuda/interface/Detector.cu (8 stages, 5 CUDA
// graphs with a host sync after each, a mid-pipeline count D2H, a 10-stream
// pool) with ONE graph per descriptor buffer: every data-dependent size lives
// in device counters, every launch has a fixed grid, and the only host sync
// per frame is the final 32-byte counter readback.
//
// The handle's state and the orchestration split over four translation units
// (detector_state.h): this one holds geometry, arenas, graph capture, the frame
// launch and the detector entry points.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>

#include "detector_state.h"

namespace sift_amd {
namespace det {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

namespace {

// OpenCV getGaussianKernelBitExact (same arithmetic as oracle gaussianTaps).
Taps gaussian_taps(double sigma) {
    Taps t{};
    int n = (int)lrint(sigma * 4 * 2 + 1) | 1;
    if (n > kMaxTaps) n = kMaxTaps;
    const double scale2X = -0.125 / (sigma * sigma);
    const int n2 = (n - 1) / 2;
    std::vector<double> values(n2 + 1);
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        const double v = std::exp((double)(x * x) * scale2X);
        values[i] = v;
        sum += v;
    }
    sum *= 2.0;
    sum += 1.0;
    const double mul1 = 1.0 / sum;
    for (int i = 0; i < n2; i++) {
        const float v = (float)(values[i] * mul1);
        t.w[i] = v;
        t.w[n - 1 - i] = v;
    }
    t.w[n2] = (float)(1.0 * mul1);
    t.n = n;
    return t;
}

// Compile-time A/B and instrumentation switches of the kernels (tools/ab_*.sh
// builds pass them through EXTRA_HIPFLAGS, which the Makefile also records as
// SIFT_AB_FLAGS).  Any of them makes this a non-default build:
// sift_hip_version() lists them ("build=ab ..."), and bench.py and
// __graft_entry__.smoke() refuse such a library, so a measured or tested line
// always names the code it ran.
const char* build_flags() {
#ifdef SIFT_AB_FLAGS
    return " " SIFT_AB_FLAGS;
#else
    return "";
#endif
}

}  // namespace

int setup_geometry(sift_hip_detector* d) {
    const sift_hip_config& c = d->cfg;
    d->L = c.numOctaveLayers;
    d->firstOctave = c.upscale ? -1 : 0;
    d->baseW = c.upscale ? 2 * c.col_width : c.col_width;
    d->baseH = c.upscale ? 2 * c.row_width : c.row_width;
    int nOct = c.numOctaves;
    if (nOct <= 0)  // [OpenCV 4.x sift.dispatch.cpp] cvRound(log2(min) - 2) - firstOctave
        nOct = (int)lrint(std::log((double)std::min(d->baseW, d->baseH)) / std::log(2.) - 2) - d->firstOctave;
    if (nOct < 1) nOct = 1;
    if (nOct > kMaxOctaves) return fail(SIFT_HIP_ERR_INVALID, "too many octaves");
    d->nOct = nOct;
    int W = d->baseW, H = d->baseH;
    int rowBase = 0;
    long bitBase = 0;
    size_t off = 0;
    for (int o = 0; o < nOct; o++) {
        if (o > 0) {
            W /= 2;
            H /= 2;
        }
        if (W < 1 || H < 1) return fail(SIFT_HIP_ERR_INVALID, "octave smaller than one pixel");
        OctGeom& g = d->pyr.oct[o];
        g.W = W;
        g.H = H;
        g.pitch = (W + 63) / 64 * 64;
        g.planeStride = (long)g.pitch * H;
        g.base = nullptr;  // bound to a lane's arena by bind_lane
        d->lay.octave[o] = off;
        g.rowBase = rowBase;
        g.bitBase = bitBase;
        off += (size_t)g.planeStride * (d->L + 3);
        rowBase += d->L * H;
        bitBase += (long)d->L * H * W;
    }
    d->pyr.nOct = nOct;
    d->pyr.L = d->L;
    d->pyr.firstOctave = d->firstOctave;
    d->kp.numBuckets = rowBase;
    d->bitmapWords = (size_t)(bitBase + 31) / 32;
    return SIFT_HIP_OK;
}

void setup_taps(sift_hip_detector* d) {
    const float sigma = (float)d->cfg.sigma;
    const float sig_diff = d->firstOctave < 0 ? sqrtf(std::max(sigma * sigma - 0.5f * 0.5f * 4, 0.01f))
                                              : sqrtf(std::max(sigma * sigma - 0.5f * 0.5f, 0.01f));
    d->initTaps = gaussian_taps((double)sig_diff);
    const int L = d->L;
    std::vector<double> sig(L + 3);
    sig[0] = d->cfg.sigma;
    const double k = std::pow(2., 1. / L);
    for (int i = 1; i < L + 3; i++) {
        const double sig_prev = std::pow(k, (double)(i - 1)) * d->cfg.sigma;
        const double sig_total = sig_prev * k;
        sig[i] = std::sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
    d->layerTaps.resize(L + 3);
    for (int i = 0; i < L + 3; i++) d->layerTaps[i] = gaussian_taps(sig[i]);
    // The pyramid tail for the small octaves.  (Measured alternative, round
    // 4: per-plane launches -- 752x480 sync 0.2177 vs 0.2094-0.2107 ms.)
    d->tailOct = L + 3 <= kTailMaxPlanes ? tail_first_octave(d->pyr, d->layerTaps.data(), L) : d->nOct;
    d->threshold = (float)(int)std::floor(0.5 * d->cfg.contrastThreshould / L * 255 * 1.0);
    d->kp.contrastThreshold = (float)d->cfg.contrastThreshould;
    d->kp.edgeThreshold = (float)d->cfg.edgeThreshould;
    d->kp.sigma = (float)d->cfg.sigma;
    d->kp.numFeatures = d->cfg.numFeatures;
    // Capacities sized to the frame (were fixed 1M / 2^18 / 2^19 / 65536, so a
    // small frame held 128 MiB against the reference's 84, readme.md:16).
    // Candidates: 1/8 of the scale-space samples (a 3x3x3 extremum test passes
    // ~7 % of samples of pure noise before the contrast threshold; natural and
    // synthetic frames stay far below); refined <= candidates; oriented: one
    // slot per refined keypoint + as many extra peaks; results: numFeatures
    // (+ a quarter for retainBest's response ties), or 1/32 of the pyramid's
    // pixels without a feature limit (C1 frames keep ~1/3000).  Every stage
    // clamps to its capacity and sets its overflow bit (sift_hip_overflow_flags).
    double sumPx = 0;
    for (int o = 0; o < d->nOct; o++) sumPx += (double)d->pyr.oct[o].W * d->pyr.oct[o].H;
    auto clampu = [](double v, double lo, double hi) { return (unsigned)std::max(lo, std::min(v, hi)); };
    d->capCand = clampu(sumPx * L / 8, 16384, 1u << 20);
    d->kp.capRefined = std::min(d->capCand, 1u << 18);
    d->kp.capOriented = 2 * d->kp.capRefined;
    const int nfeat = d->cfg.numFeatures;
    d->kp.capFinal = d->cfg.maxKeypoints > 0 ? (unsigned)d->cfg.maxKeypoints
                     : nfeat > 0             ? clampu(nfeat + std::max(nfeat / 4, 512), 1024, 65536)
                                             : clampu(sumPx / 32, 4096, 65536);
    // LDS patch bounds: scl_octv = sigma * 2^((layer + xi) / L) <= sigma * 2^((L + 0.5) / L).
    // Larger radii (not reachable from accepted keypoints) fall back to HBM reads.
    const double sclMax = d->cfg.sigma * std::pow(2.0, (L + 0.5) / L);
    d->kp.oriRmax = (int)lrint(4.5 * sclMax) + 1;
    d->kp.descRmax = std::min((int)lrint(3.0 * sclMax * 1.4142135623730951 * 2.5) + 1, 60);
    // Valid descriptor samples lie in a rotated square of side 5 * hist_width.
    const double hw = 3.0 * sclMax;
    d->kp.descNrec = std::min((int)std::ceil((5.0 * hw + 3.0) * (5.0 * hw + 3.0)), 8192);
}

void upload_exp_tab() {
    const double A0 = .9670371139572337719125840413672004409288e-2;
    float tab[64];
    for (int j = 0; j < 64; j++) tab[j] = (float)(std::exp2((double)j / 64.0) * A0);
    upload_exp_table(tab);
    upload_desc_exp_table(tab);
}

// Points the handle's buffer views (stream, frame-0 arena pointers, host
// counters) at lane k.  Every entry point binds the lane it works on: the
// submitting lane for a new frame (idx 0: launches address frame 0's arena),
// the current frame's lane and arena for accessors (idx: its arena in a
// micro-batch, which offsets the results views and host counters).
void bind_lane(sift_hip_detector* d, int k, int idx) {
    Lane& L = d->lanes[k];
    const ArenaLayout& a = d->lay;
    char* A = L.arena;
    d->ln = k;
    d->stream = L.stream;
    d->dInput = reinterpret_cast<float*>(A + a.input);
    d->dUp = d->firstOctave < 0 ? reinterpret_cast<float*>(A + a.up) : nullptr;
    d->dPyr = reinterpret_cast<float*>(A + a.pyr);
    for (int o = 0; o < d->nOct; o++) d->pyr.oct[o].base = d->dPyr + a.octave[o];
    d->dCand = reinterpret_cast<uint2*>(A + a.cand);
    d->dRef = reinterpret_cast<RefKpt*>(A + a.ref);
    d->dOri = reinterpret_cast<OriKpt*>(A + a.ori);
    d->dSlot = reinterpret_cast<int*>(A + a.slot);
    d->dOrder = reinterpret_cast<int*>(A + a.order);
    d->dJobs = reinterpret_cast<DescJob*>(A + a.jobs);
    d->dJord = reinterpret_cast<JobOrder*>(A + a.jord);
    d->dRange = reinterpret_cast<unsigned*>(A + a.range);
    d->dBcount = reinterpret_cast<unsigned*>(A + a.bcount);
    d->dBoff = reinterpret_cast<unsigned*>(A + a.boff);
    d->dBitmap = reinterpret_cast<uint32_t*>(A + a.bitmap);
    d->dCtr = reinterpret_cast<Counters*>(A + a.ctr);
    char* R = A + (size_t)idx * d->afs;
    for (int b = 0; b < d->kSlots; b++) {
        d->dKpts3[b] = reinterpret_cast<float*>(R + a.k3[b]);
        d->dFeats4[b] = reinterpret_cast<float*>(R + a.f4[b]);
        d->dDesc[b] = reinterpret_cast<uint16_t*>(R + a.desc[b]);
        d->dSide[b] = Sidecar{reinterpret_cast<int8_t*>(R + a.codes[b]), reinterpret_cast<int*>(R + a.ckeys[b])};
    }
    d->hCtr = L.hCtr + idx;
    d->hCtrDev = L.hCtrDev + idx;
}

// Results of frame f (lane and slot from its record), without binding.
const uint16_t* frame_desc(const sift_hip_detector* d, long long f) {
    const auto& r = d->frecs[f & (kFrameRing - 1)];
    return reinterpret_cast<const uint16_t*>(d->lanes[r.lane].arena + (size_t)r.idx * d->afs + d->lay.desc[r.slot]);
}
const Counters& frame_counters(const sift_hip_detector* d, long long f, int i) {
    const auto& r = d->frecs[f & (kFrameRing - 1)];
    return d->lanes[r.lane].hCtr[(size_t)r.slot * d->lanes[r.lane].B + r.idx + i];
}

// Per-handle allocations shared by the lanes: the upload ring and the frame
// arena layout (the lanes themselves: add_lane).
int allocate(sift_hip_detector* d) {
    HIPCHK(hipSetDevice(d->device));
    d->allocated = true;
    // The pyramid tail is an optimisation: without the LDS it asks for (a
    // device whose opt-in limit is lower, or a refused attribute) the small
    // octaves take the per-plane blur launches instead.
    if (d->tailOct < d->nOct) {
        int optin = 0;
        if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, d->device) != hipSuccess ||
            optin < (int)(sizeof(float) * kTailLdsFloats) || tail_init() != hipSuccess) {
            (void)hipGetLastError();
            d->tailOct = d->nOct;
        }
    }
    HIPCHK(hipEventCreateWithFlags(&d->evIn, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&d->evOut, hipEventDisableTiming));
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    d->inPitch = (W + 63) / 64 * 64;
    if (d->firstOctave < 0) d->upPitch = (2 * W + 63) / 64 * 64;
    size_t pyrFloats = 0;
    for (int o = 0; o < d->nOct; o++) pyrFloats += (size_t)d->pyr.oct[o].planeStride * (d->L + 3);
    const unsigned capO = d->kp.capOriented, capF = d->kp.capFinal;

    // Frame arena: every per-frame buffer at a 256-B aligned offset; B arenas
    // back to back per lane.  Zeroed once at allocation; afterwards the
    // kernels keep the scratch zero for the next frame (first blur: counters,
    // k_order / k_select: range keys, k_bucket_rank: bucket counts,
    // k_orientation: dedupe bits), so the frame graph has no memset node.
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (std::max<size_t>(bytes, 1) + 255) & ~(size_t)255;
        return o;
    };
    ArenaLayout& a = d->lay;
    a.input = take(sizeof(float) * (size_t)d->inPitch * H);  // blank warm-up frame / u8 -> f32 scratch
    a.up = d->firstOctave < 0 ? take(sizeof(float) * (size_t)d->upPitch * 2 * H) : 0;
    a.pyr = take(sizeof(float) * pyrFloats);
    a.cand = take(sizeof(uint2) * d->capCand);
    a.ref = take(sizeof(RefKpt) * d->kp.capRefined);
    a.ori = take(sizeof(OriKpt) * capO);
    a.slot = take(sizeof(int) * capO);
    a.order = take(sizeof(int) * capO);
    a.jobs = take(sizeof(DescJob) * capF);
    a.jord = take(sizeof(JobOrder));
    a.range = take(sizeof(unsigned) * 2 * 2 * kRangeSlots);  // one set per frame parity
    a.bcount = take(sizeof(unsigned) * (size_t)d->kp.numBuckets);
    a.boff = take(sizeof(unsigned) * (size_t)d->kp.numBuckets);
    a.bitmap = take(sizeof(uint32_t) * d->bitmapWords);
    a.ctr = take(sizeof(Counters));
    for (int b = 0; b < d->kSlots; b++) {
        a.k3[b] = take(sizeof(float) * 3 * (size_t)capF);
        a.f4[b] = take(sizeof(float) * 4 * (size_t)capF);
        a.desc[b] = take(sizeof(uint16_t) * 128 * (size_t)capF);
        a.codes[b] = take(128 * (size_t)capF);
        a.ckeys[b] = take(sizeof(int) * (size_t)capF);
    }
    d->afs = (long)off;
    upload_exp_tab();
    return SIFT_HIP_OK;
}

int build_graphs(sift_hip_detector* d);

// A new compute lane: stream, zeroed arenas, host counters, events and the
// captured graphs (bound on return).
int add_lane(sift_hip_detector* d, int B, int nslots) {
    if (d->nLanes >= kMaxLanes) return fail(SIFT_HIP_ERR_STATE, "no lane left");
    const int k = d->nLanes;
    Lane& L = d->lanes[k];
    d->nLanes++;  // from here the destructor releases what the lane holds
    L.B = B;
    L.nslots = nslots;
    HIPCHK(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking));
    if (hipMalloc((void**)&L.arena, (size_t)d->afs * B) != hipSuccess)
        return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the frame arenas failed");
    HIPCHK(hipMemsetAsync(L.arena, 0, (size_t)d->afs * B, L.stream));
    const size_t nh = (size_t)nslots * B;
    HIPCHK(hipHostMalloc((void**)&L.hCtr, sizeof(Counters) * nh, hipHostMallocMapped | hipHostMallocCoherent));
    memset(L.hCtr, 0, sizeof(Counters) * nh);
    HIPCHK(hipHostGetDevicePointer((void**)&L.hCtrDev, L.hCtr, 0));
    if (hipMalloc((void**)&L.dHostTab, sizeof(char*) * nh) != hipSuccess)
        return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the host results table failed");
    HIPCHK(hipMemsetAsync(L.dHostTab, 0, sizeof(char*) * nh, L.stream));
    for (int b = 0; b < d->kSlots; b++) {
        HIPCHK(hipEventCreateWithFlags(&L.evFrame[b], hipEventDisableTiming));
        HIPCHK(hipEventRecord(L.evFrame[b], L.stream));
    }
    std::fill(std::begin(L.hostFrame), std::end(L.hostFrame), -1LL);
    // The lane's host-input staging, sized for f32 rows of pitch inPitch (an
    // 8-bit frame uses the first quarter with a byte pitch of inPitch); its
    // events start complete.
    const size_t inBytes = sizeof(float) * (size_t)d->inPitch * d->cfg.row_width;
    for (int i = 0; i < Lane::kInSlots; i++) {
        HIPCHK(hipHostMalloc(&L.hStage[i], inBytes, hipHostMallocMapped | hipHostMallocNonCoherent));
        HIPCHK(hipEventCreateWithFlags(&L.evRead[i], hipEventDisableTiming));
        HIPCHK(hipEventRecord(L.evRead[i], L.stream));
    }
    bind_lane(d, k);
    for (int i = 0; i < B; i++)
        for (int b = 0; b < d->kSlots; b++)
            register_sidecar(d, fptr(d->dDesc[b], (long)i * d->afs),
                             Sidecar{fptr(d->dSide[b].codes, (long)i * d->afs), fptr(d->dSide[b].keys, (long)i * d->afs)},
                             (int)d->kp.capFinal);
    if (d->hostWant)
        if (int rc = ensure_host_res(d, L)) return rc;
    if (int rc = build_graphs(d)) return rc;
    L.ready = true;
    return SIFT_HIP_OK;
}

// The first kernel reads the caller's image (upload ring slot or a device
// pointer); it stays outside the graph so the graph never bakes a user pointer.
// Pixel-range keys by frame parity p (frame f uses p = f & 1; k_select zeroes
// the other set for the next frame).
unsigned* range_keys(sift_hip_detector* d, int p) { return d->dRange + (size_t)p * 2 * kRangeSlots; }

// pitch in elements of the frame's format (bytes for SIFT_HIP_U8); nf frames
// at byte stride sfs.
void enqueue_head(sift_hip_detector* d, const void* img, int pitch, int fmt, int parity, int nf, long sfs) {
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    const bool u8 = fmt == SIFT_HIP_U8;
    const Frames fr{nf, d->afs};
    const double inB = (double)W * H * (u8 ? 1 : 4) * nf;
    // Counters first: the initial blur accumulates the frame's pixel range.
    if (d->firstOctave < 0) {
        d->timed("upsample", inB + (double)W * H * 16 * nf, [&] {
            if (u8)
                launch_upsample2x_u8((const uint8_t*)img, pitch, W, H, d->dUp, d->upPitch, fr, sfs, d->stream);
            else
                launch_upsample2x((const float*)img, pitch, W, H, d->dUp, d->upPitch, fr, sfs, d->stream);
        });
    } else {
        const OctGeom& g = d->pyr.oct[0];
        d->timed("blur_init", inB + (double)W * H * 4 * nf, [&] {
            long s = sfs;
            if (u8) {
                if (launch_blur_u8((const uint8_t*)img, pitch, W, H, g.base, g.pitch, d->initTaps, fr, sfs, d->stream,
                                   range_keys(d, parity), d->dCtr))
                    return;
                launch_u8_to_f32((const uint8_t*)img, pitch, W, H, d->dInput, d->inPitch, fr, sfs, d->stream);
                img = d->dInput;
                pitch = d->inPitch;
                s = d->afs;
            }
            launch_blur((const float*)img, pitch, W, H, g.base, g.pitch, DecOut{}, d->initTaps, fr, s, d->stream,
                        range_keys(d, parity), d->dCtr);
        });
    }
}

// Pyramid tail: octaves d->tailOct.. in one launch (one workgroup per frame,
// planes in LDS), none when every octave is too large for it.
void left_tail(sift_hip_detector* d, int nf, hipStream_t s) {
    if (d->tailOct >= d->nOct) return;
    double bytes = 0;
    for (int o = d->tailOct; o < d->nOct; o++)
        bytes += (double)d->pyr.oct[o].W * d->pyr.oct[o].H * 4 * (o == d->tailOct ? 1 + (d->L + 2) : (d->L + 2)) * nf;
    d->timed("pyr_tail", bytes, [&] { launch_blur_tail(d->pyr, d->layerTaps.data(), d->L, d->tailOct, Frames{nf, d->afs}, s); });
}

// The frame pipeline after the head, as the stages tool/perf.cu replays one
// at a time (sift_hip_replay_stage): pyramid (blur jobs), extrema, refine,
// orientation, order (retainBest + deterministic order + descriptor jobs),
// descriptor.  `parity` = the frame's range-key set (frame parity).
void enqueue_pyramid(sift_hip_detector* d, int nf, int parity) {
    hipStream_t s = d->stream;
    const int L = d->L;
    const Frames fr{nf, d->afs};
    if (d->firstOctave < 0) {
        const OctGeom& g = d->pyr.oct[0];
        d->timed("blur_init", (double)g.W * g.H * 8 * nf, [&] {
            launch_blur(d->dUp, d->upPitch, g.W, g.H, g.base, g.pitch, DecOut{}, d->initTaps, fr, d->afs, s,
                        range_keys(d, parity), d->dCtr);
        });
    }
    static const char* blurNames[kMaxOctaves] = {"blur_o0", "blur_o1", "blur_o2", "blur_o3", "blur_o4", "blur_o5",
                                                 "blur_o6", "blur_o7", "blur_o8", "blur_o9", "blur_o10", "blur_o11",
                                                 "blur_o12", "blur_o13", "blur_o14", "blur_o15"};
    // Blur jobs (o, i): plane i of octave o from plane i-1 (plane 0 of octave
    // o+1 is written by job (o, L) as it stores: the INTER_NEAREST half-size
    // copy of plane L).  List-scheduled in (o, i) order: a job is ready once
    // its input plane's job has been launched (stream order); the two oldest
    // ready jobs share one launch when their radii have a pair kernel -- with
    // L = 3, (o, 4) + (o+1, 1) and (o, 5) + (o+1, 2): 11 launches instead of 15
    // for three octaves.
    struct Job {
        int o, i;
        BlurDesc b;
        double bytes;
    };
    std::vector<Job> jobs;
    // Octaves from d->tailOct on: one pyramid-tail launch after the jobs
    // (launch_blur_tail; their base plane is written by job (tailOct - 1, L)).
    for (int o = 0; o < d->tailOct; o++) {
        const OctGeom& g = d->pyr.oct[o];
        for (int i = 1; i < L + 3; i++) {
            Job j{o, i, {}, 0};
            j.b.src = g.base + (size_t)(i - 1) * g.planeStride;
            j.b.spitch = g.pitch;
            j.b.dst = g.base + (size_t)i * g.planeStride;
            j.b.dpitch = g.pitch;
            j.b.W = g.W;
            j.b.H = g.H;
            j.b.taps = &d->layerTaps[i];
            j.bytes = (double)g.W * g.H * 8 * nf;
            if (i == L && o + 1 < d->nOct) {
                const OctGeom& n = d->pyr.oct[o + 1];
                j.b.dec = DecOut{n.base, n.pitch, n.W, n.H};
                j.bytes += (double)n.W * n.H * 4 * nf;
            }
            jobs.push_back(j);
        }
    }
    auto idx = [&](int o, int i) { return o * (L + 2) + (i - 1); };
    std::vector<bool> done(jobs.size(), false);
    auto ready = [&](size_t k) {
        const Job& j = jobs[k];
        if (done[k]) return false;
        if (j.i >= 2) return (bool)done[idx(j.o, j.i - 1)];
        return j.o == 0 || (bool)done[idx(j.o - 1, L)];
    };
    if (jobs.empty()) left_tail(d, nf, s);
    for (size_t left = jobs.size(); left > 0;) {
        int a = -1, b = -1;
        for (size_t k = 0; k < jobs.size() && b < 0; k++)
            if (ready(k)) (a < 0 ? a : b) = (int)k;
        const Job& ja = jobs[a];
        bool paired = false;
        if (b >= 0) {
            const Job& jb = jobs[b];
            char name[16];
            snprintf(name, sizeof name, "blur_o%d+o%d", ja.o, jb.o);
            d->timed(name, ja.bytes + jb.bytes, [&] { paired = launch_blur_pair(ja.b, jb.b, fr, s); });
            if (paired) {
                done[b] = true;
                left--;
            }
        }
        if (!paired) {
            d->timed(blurNames[ja.o], ja.bytes, [&] {
                launch_blur(ja.b.src, ja.b.spitch, ja.b.W, ja.b.H, ja.b.dst, ja.b.dpitch, ja.b.dec,
                            *ja.b.taps, fr, d->afs, s);
            });
        }
        done[a] = true;
        left--;
    }
    if (!jobs.empty()) left_tail(d, nf, s);
}

void enqueue_extrema(sift_hip_detector* d, int nf) {
    hipStream_t s = d->stream;
    const int L = d->L;
    const Frames fr{nf, d->afs};
    double exBytes = 0;
    for (int o = 0; o < d->nOct; o++) exBytes += (double)d->pyr.oct[o].W * d->pyr.oct[o].H * 4 * (L + 3) * nf;
    d->timed("extrema", exBytes, [&] {
        if (!launch_extrema_all(d->pyr, d->threshold, d->dCand, d->dCtr, d->capCand, fr, s))
            for (int o = 0; o < d->nOct; o++)
                launch_extrema(d->pyr, o, d->threshold, d->dCand, d->dCtr, d->capCand, fr, s);
    });
}

void enqueue_refine(sift_hip_detector* d, int nf) {
    const Frames fr{nf, d->afs};
    d->timed("refine", 0, [&] {
        launch_refine(d->pyr, d->dCand, d->capCand, d->dCtr, d->dBitmap, d->dRef, d->kp, fr, d->stream);
    });
}

void enqueue_orientation(sift_hip_detector* d, int nf) {
    const Frames fr{nf, d->afs};
    d->timed("orientation", 0,
             [&] { launch_orientation(d->pyr, d->dRef, d->dCtr, d->dOri, d->dBitmap, d->kp, fr, d->stream); });
}

void enqueue_order(sift_hip_detector* d, int slot, int nf) {
    hipStream_t s = d->stream;
    const int parity = slot & 1;
    const Frames fr{nf, d->afs};
    if (d->kp.numBuckets <= kOrderMaxBuckets) {
        d->timed("order", 0, [&] {
            launch_order(d->pyr, d->dOri, d->dCtr, range_keys(d, parity ^ 1), d->dBcount, d->dBoff, d->dSlot, d->dOrder,
                         d->dJord, d->kp, fr, s);
        });
    } else {
        d->timed("select", 0, [&] { launch_select(d->dOri, d->dCtr, range_keys(d, parity ^ 1), d->kp, fr, s); });
        d->timed("bucket_count", 0,
                 [&] { launch_bucket_count(d->dOri, d->dCtr, d->dBcount, d->dSlot, d->kp, fr, s); });
        d->timed("bucket_scan", 0, [&] { launch_bucket_scan(d->dBcount, d->dBoff, d->dCtr, d->kp, fr, s); });
        d->timed("bucket_scatter", 0,
                 [&] { launch_bucket_scatter(d->dOri, d->dCtr, d->dBoff, d->dSlot, d->dOrder, d->kp, fr, s); });
    }
    d->timed("bucket_rank", 0, [&] {
        if (d->kp.numBuckets <= kOrderMaxBuckets)
            launch_rank_final(d->pyr, d->dOri, d->dBcount, d->dBoff, d->dOrder, d->dCtr, d->dJord, d->dJobs, d->dKpts3[slot],
                              d->dFeats4[slot], d->kp, fr, s);
        else  // bucket_count needs zeroed counts: the bucket-parallel ranking re-zeroes them
            launch_bucket_rank(d->pyr, d->dOri, d->dBcount, d->dBoff, d->dOrder, d->dCtr, d->dJobs, d->dKpts3[slot],
                               d->dFeats4[slot], d->kp, fr, s);
    });
}

void enqueue_descriptor(sift_hip_detector* d, int slot, int nf) {
    const Frames fr{nf, d->afs};
    d->timed("descriptor", 0, [&] {
        launch_descriptor(d->dJobs, d->dCtr, range_keys(d, slot & 1), d->dDesc[slot], d->dSide[slot],
                          d->hCtrDev + (size_t)slot * d->lane().B,
                          HostOut{d->lane().dHostTab + (size_t)slot * d->lane().B, d->dKpts3[slot], d->dFeats4[slot],
                                  d->kp.capFinal},
                          d->kp, fr, d->stream);
    });
}

void enqueue_body(sift_hip_detector* d, int slot, int nf) {
    enqueue_pyramid(d, nf, slot & 1);  // kSlots is even, so slot parity = frame parity
    enqueue_extrema(d, nf);
    enqueue_refine(d, nf);
    enqueue_orientation(d, nf);
    enqueue_order(d, slot, nf);
    enqueue_descriptor(d, slot, nf);
}

int capture(sift_hip_detector* d, int slot, int nf, hipGraphExec_t* out) {
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
    enqueue_body(d, slot, nf);
    HIPCHK(hipStreamEndCapture(d->stream, &g));
    HIPCHK(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    HIPCHK(hipGraphDestroy(g));
    return SIFT_HIP_OK;
}

// The head for f32 device input (the frame's first blur, or the 2x upsample)
// as node parameters for image `img` (pitch in floats, nf frames at byte
// stride sfs): what enqueue_head launches.
void head_node(sift_hip_detector* d, HeadNode& h, const float* img, int pitch, int parity, int nf, long sfs) {
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    const Frames fr{nf, d->afs};
    if (d->firstOctave < 0) {
        head_upsample_node(h, img, pitch, W, H, d->dUp, d->upPitch, fr, sfs);
    } else {
        const OctGeom& g = d->pyr.oct[0];
        head_blur_node(h, img, pitch, W, H, g.base, g.pitch, d->initTaps, fr, sfs, range_keys(d, parity), d->dCtr);
    }
}

// head + body captured together; the graph is kept for its head node.
int capture_with_head(sift_hip_detector* d, int slot, int nf, hipGraphExec_t* out, hipGraph_t* graph,
                      hipGraphNode_t* head) {
    HIPCHK(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
    enqueue_head(d, d->dInput, d->inPitch, SIFT_HIP_F32, slot & 1, nf, d->afs);
    enqueue_body(d, slot, nf);
    HIPCHK(hipStreamEndCapture(d->stream, graph));
    size_t nroot = 0;
    HIPCHK(hipGraphGetRootNodes(*graph, nullptr, &nroot));
    if (nroot != 1) return fail(SIFT_HIP_ERR_RUNTIME, "captured frame graph: expected one root (the head)");
    HIPCHK(hipGraphGetRootNodes(*graph, head, &nroot));
    hipGraphNodeType ty;
    HIPCHK(hipGraphNodeGetType(*head, &ty));
    if (ty != hipGraphNodeTypeKernel) return fail(SIFT_HIP_ERR_RUNTIME, "captured frame graph: the head is not a kernel");
    HIPCHK(hipGraphInstantiate(out, *graph, nullptr, nullptr, 0));
    return SIFT_HIP_OK;
}

int build_graphs(sift_hip_detector* d) {
    Lane& L = d->lane();
    for (int b = 0; b < L.nslots; b++) {
        if (int rc = capture(d, b, L.B, &L.exec[b])) return rc;
        if (int rc = capture_with_head(d, b, L.B, &L.execH[b], &L.graphH[b], &L.headH[b])) return rc;
        L.headIn[b][0] = Lane::HeadIn{d->dInput, d->inPitch, d->afs};
        if (L.B > 1) {
            if (int rc = capture(d, b, 1, &L.exec1[b])) return rc;
            if (int rc = capture_with_head(d, b, 1, &L.execH1[b], &L.graphH1[b], &L.headH1[b])) return rc;
            L.headIn[b][1] = Lane::HeadIn{d->dInput, d->inPitch, d->afs};
        }
    }
    return SIFT_HIP_OK;
}

bool event_done(hipEvent_t e) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) return true;
    (void)hipGetLastError();  // hipErrorNotReady is not an error of the handle
    return false;
}

// Blank launch groups through every graph of a lane created after warm-up
// (first-launch costs, as sift_hip_warmup's blank frames pay them for lane 0).
// They take no frame numbers; slots 0..kSlots-1 in order keep the lane's
// range-key parity alternating, and the lane's next frame takes slot 0.
int warm_lane(sift_hip_detector* d) {
    Lane& L = d->lane();
    const int nb = L.B > 1 ? 2 : 1;
    for (int r = 0; r < nb; r++)
        for (int b = 0; b < L.nslots; b++) {
            HIPCHK(hipGraphLaunch(r == 0 ? L.execH[b] : L.execH1[b], L.stream));
            HIPCHK(hipEventRecord(L.evFrame[b], L.stream));
            L.nfOf[b] = r == 0 ? L.B : 1;
        }
    L.launched = (long long)nb * L.nslots;
    return SIFT_HIP_OK;
}

// Enqueues launch group d->submitted (nf frames at byte stride sfs) on the
// bound lane (pick_lane); `consumed` (nullable) is recorded once the input has
// been read.  A batch (sift_hip_detect_batch_device) is one frame number; a
// micro-batch (`numbered`) takes nf numbers, frame d->submitted + i in arena i.  With stage dumps on (single frames after warm-up) the frame's
// input is kept as float, the frame is completed synchronously and dumped.
int run_frame(sift_hip_detector* d, const void* img, int pitch, int fmt, hipEvent_t consumed, int nf, long sfs,
              bool numbered) {
    const long long f = d->submitted;
    Lane& L = d->lane();
    const int slot = (int)(L.launched % L.nslots);
    const bool dump = !d->dgDir.empty() && nf == 1 && d->firstFrame > 0;
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    if (dump) {
        if (!d->dDg && hipMalloc((void**)&d->dDg, sizeof(float) * (size_t)W * H) != hipSuccess)
            return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the stage-dump input failed");
        if (fmt == SIFT_HIP_U8)
            launch_u8_to_f32((const uint8_t*)img, pitch, W, H, d->dDg, W, Frames{1, 0}, 0, d->stream);
        else
            HIPCHK(hipMemcpy2DAsync(d->dDg, sizeof(float) * W, img, sizeof(float) * (size_t)pitch, sizeof(float) * W,
                                    H, hipMemcpyDefault, d->stream));
    }
    const bool graphs = d->useGraph && !d->timing;
    hipGraphExec_t gh = !graphs || consumed || fmt != SIFT_HIP_F32 ? nullptr
                        : nf == L.B                                  ? L.execH[slot]
                        : nf == 1                                    ? L.execH1[slot]
                                                                     : nullptr;
    // The head node of execH[slot] is re-pointed only once that exec's last
    // launch (whose completion evFrame[slot] still records) has finished: a
    // queued launch never sees its kernel arguments change.  Otherwise the
    // frame takes the separate head launch and the plain exec.
    if (gh && !event_done(L.evFrame[slot])) gh = nullptr;
    if (gh) {  // device f32 input: one launch for the whole frame, the head re-pointed at img
        const Lane::HeadIn in{img, pitch, sfs};
        Lane::HeadIn& cur = L.headIn[slot][nf == L.B ? 0 : 1];
        if (!(cur == in)) {
            HeadNode& h = d->headNode;
            head_node(d, h, static_cast<const float*>(img), pitch, slot & 1, nf, sfs);
            HIPCHK(hipGraphExecKernelNodeSetParams(gh, nf == L.B ? L.headH[slot] : L.headH1[slot], &h.p));
            cur = in;
        }
        HIPCHK(hipGraphLaunch(gh, d->stream));
    } else {
        enqueue_head(d, img, pitch, fmt, slot & 1, nf, sfs);
        if (consumed) HIPCHK(hipEventRecord(consumed, d->stream));
        hipGraphExec_t g = nf == L.B ? L.exec[slot] : (nf == 1 ? L.exec1[slot] : nullptr);
        if (graphs && g) {
            HIPCHK(hipGraphLaunch(g, d->stream));
        } else {  // timing mode, or a partial batch: the same launches, eagerly
            enqueue_body(d, slot, nf);
        }
    }
    HIPCHK(hipEventRecord(L.evFrame[slot], d->stream));
    const int nums = numbered ? nf : 1;
    L.nfOf[slot] = nf;
    L.slotFrame[slot] = f;
    L.slotNum[slot] = nums;
    L.launched++;
    L.last = f + nums - 1;
    for (int i = 0; i < nums; i++) d->frec(f + i) = sift_hip_detector::FrameRec{d->ln, slot, i};
    for (int i = 0; i < nf; i++) sidecar_refreshed(fptr(d->dDesc[slot], (long)i * d->afs));
    d->submitted = f + nums;
    if (dump) {
        HIPCHK(hipStreamSynchronize(d->stream));
        if (d->timing) d->collect_timing();
        d->current = f;
        d->curLane = d->ln;
        d->curIdx = 0;
        d->cur = slot;
        complete_counts(d);
        return dump_stage_files(d);
    }
    return SIFT_HIP_OK;
}

// Exposes frame f through the result accessors (and binds its lane).  Its
// counts are read once the frame is complete (complete_counts).
void make_current(sift_hip_detector* d, long long f) {
    d->current = f;
    d->curLane = d->frec(f).lane;
    d->curIdx = d->frec(f).idx;
    d->cur = d->frec(f).slot;
    d->countsValid = false;
    bind_lane(d, d->curLane, d->curIdx);
}

void complete_counts(sift_hip_detector* d) {
    const long long f = d->current;
    auto n = [&](long long g) {
        return g < d->firstFrame ? 0 : (int)std::min<unsigned>(frame_counters(d, g).final_n, d->kp.capFinal);
    };
    d->count = n(f);
    d->prevCount = n(f - 1);
    d->countsValid = true;
}

// Counts of the current launch group are read from the pinned host copies its
// last kernel writes: an accessor called before sift_hip_sync / sift_hip_wait
// (e.g. straight after sift_hip_detect_device) first waits for that group.  The
// previous frame may run on another lane: its counts are waited for too.
int ensure_counts(sift_hip_detector* d) {
    if (d->countsValid) return SIFT_HIP_OK;
    for (long long g : {d->current - 1, d->current})
        if (g >= d->firstFrame) {
            const auto& r = d->frec(g);
            HIPCHK(hipEventSynchronize(d->lanes[r.lane].evFrame[r.slot]));
        }
    complete_counts(d);
    return SIFT_HIP_OK;
}

int sync_lanes(sift_hip_detector* d) {
    for (int k = 0; k < d->nLanes; k++)
        if (d->lanes[k].ready) HIPCHK(hipStreamSynchronize(d->lanes[k].stream));
    if (d->timing) d->collect_timing();
    return SIFT_HIP_OK;
}

int finish_frame(sift_hip_detector* d) {
    if (int rc = run_group(d)) return rc;
    if (int rc = sync_lanes(d)) return rc;
    if (d->submitted > 0) {
        make_current(d, d->submitted - 1);
        complete_counts(d);
    }
    return SIFT_HIP_OK;
}

}  // namespace det
}  // namespace sift_amd

void sift_amd::set_last_error(const std::string& msg) { det::g_err = msg; }

// Frames the batch accessors expose for the current frame: a batch
// (sift_hip_detect_batch_device: one frame number, nfOf frames in arenas
// 0..nfOf-1), or -- for a frame of a micro-batch, which has a frame number of
// its own and whose views bind_lane already offset to its arena -- that frame
// alone (index 0).
int batch_frames_of(sift_hip_detector* d) {
    if (d->current < d->firstFrame) return 0;
    const Lane& L = d->lane();
    return L.slotNum[d->cur] > 1 ? 1 : L.nfOf[d->cur];
}

// Every entry point starts bound to the current frame's lane (the accessors
// address it); submitting entry points re-bind to the lane they pick.
#define CHECK_HANDLE(h)                                                                       \
    do {                                                                                      \
        if (!(h)) return fail(SIFT_HIP_ERR_INVALID, "null handle");                          \
        if (!(h)->allocated || !(h)->lanes[0].ready)                                          \
            return fail(SIFT_HIP_ERR_STATE, "sift_hip_warmup not called");                    \
        HIPCHK(hipSetDevice((h)->device));                                                    \
        bind_lane((h), (h)->curLane, (h)->curIdx);                                            \
    } while (0)

extern "C" {

void sift_hip_default_config(sift_hip_config* c, int w, int h) {
    c->col_width = w;
    c->row_width = h;
    c->numFeatures = 5000;
    c->numOctaveLayers = 3;
    c->contrastThreshould = 0.04;
    c->edgeThreshould = 10;
    c->sigma = 1.6;
    c->upscale = 0;
    c->numOctaves = 0;
    c->maxKeypoints = 0;
}

const char* sift_hip_version(void) {
    static char buf[512];
    int rt = 0;
    (void)hipRuntimeGetVersion(&rt);
    const char* ab = build_flags();
    snprintf(buf, sizeof buf, "abi=%d arch=gfx950 hip=%d build=%s%s", SIFT_HIP_ABI_VERSION, rt, ab[0] ? "ab" : "default",
             ab);
    return buf;
}

const char* sift_hip_last_error(void) { return g_err.c_str(); }

int sift_hip_create(const sift_hip_config* cfg, int device, sift_hip_t* out) {
    if (!cfg || !out) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *out = nullptr;
    if (cfg->col_width <= 0 || cfg->row_width <= 0) return fail(SIFT_HIP_ERR_INVALID, "image width or height not set");
    if (cfg->col_width >= 65536 || cfg->row_width >= 65536)
        return fail(SIFT_HIP_ERR_INVALID, "image dimension >= 65536 unsupported");
    if (cfg->numOctaveLayers < 1 || cfg->numOctaveLayers > 32)
        return fail(SIFT_HIP_ERR_INVALID, "numOctaveLayers out of range");
    if (!(cfg->sigma > 0)) return fail(SIFT_HIP_ERR_INVALID, "sigma must be > 0");
    auto* d = new sift_hip_detector();
    d->cfg = *cfg;
    if (device < 0) {
        if (hipGetDevice(&d->device) != hipSuccess) d->device = 0;
    } else {
        d->device = device;
    }
    int rc = setup_geometry(d);
    if (rc) {
        delete d;
        return rc;
    }
    setup_taps(d);
    *out = d;
    return SIFT_HIP_OK;
}

int sift_hip_destroy(sift_hip_t h) {
    delete h;
    return SIFT_HIP_OK;
}

int sift_hip_warmup(sift_hip_t d) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (d->allocated) return d->lanes[0].ready ? SIFT_HIP_OK : fail(SIFT_HIP_ERR_STATE, "an earlier warm-up failed");
    if (d->mb > 1) {  // a micro-batch runs the lane's B-frame graphs
        if (d->B > 1 && d->B != d->mb)
            return fail(SIFT_HIP_ERR_INVALID, "micro-batch and batch size differ (set one, or both equal)");
        d->B = d->mb;
    }
    int rc = allocate(d);
    if (rc) return rc;
    rc = add_lane(d, d->B);  // lane 0; more lanes on demand (pick_lane)
    if (rc) return rc;
    // One blank frame (batch) through each graph: first-touch, code-object load.
    const int ns = d->lanes[0].nslots;
    for (int i = 0; i < ns * (d->B > 1 ? 2 : 1); i++) {
        const int nf = i < ns ? d->B : 1;
        if ((rc = run_frame(d, d->dInput, d->inPitch, SIFT_HIP_F32, nullptr, nf, d->afs))) return rc;
        if ((rc = finish_frame(d))) return rc;
    }
    d->firstFrame = d->submitted;
    d->count = d->prevCount = 0;
    return SIFT_HIP_OK;
}

int sift_hip_num_octaves(sift_hip_t h, int* n) {
    if (!h || !n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *n = h->nOct;
    return SIFT_HIP_OK;
}

int sift_hip_octave_dims(sift_hip_t h, int o, int* w, int* hh, int* pitch) {
    if (!h || o < 0 || o >= h->nOct) return fail(SIFT_HIP_ERR_INVALID, "bad octave");
    if (w) *w = h->pyr.oct[o].W;
    if (hh) *hh = h->pyr.oct[o].H;
    if (pitch) *pitch = h->pyr.oct[o].pitch;
    return SIFT_HIP_OK;
}

int sift_hip_detect(sift_hip_t d, const float* img, size_t stride) {
    CHECK_HANDLE(d);
    long long f = 0;
    int rc = submit_host(d, img, stride, SIFT_HIP_F32, &f);
    return rc ? rc : wait_frame(d, f);
}

int sift_hip_detect_u8(sift_hip_t d, const uint8_t* img, size_t stride) {
    CHECK_HANDLE(d);
    long long f = 0;
    int rc = submit_host(d, img, stride, SIFT_HIP_U8, &f);
    return rc ? rc : wait_frame(d, f);
}

int sift_hip_submit(sift_hip_t d, const void* img, size_t stride, int format, long long* ticket) {
    CHECK_HANDLE(d);
    return submit_host(d, img, stride, format, ticket);
}

int sift_hip_wait(sift_hip_t d, long long ticket) {
    CHECK_HANDLE(d);
    return wait_frame(d, ticket);
}

int sift_hip_detect_device_fmt(sift_hip_t d, const void* img, size_t stride, int format, void* stream) {
    CHECK_HANDLE(d);
    if (!img) return fail(SIFT_HIP_ERR_INVALID, "null image");
    const int es = format_size(format);
    if (!es) return fail(SIFT_HIP_ERR_INVALID, "unknown pixel format");
    const int W = d->cfg.col_width;
    if (stride == 0) stride = (size_t)es * W;
    if (stride % es || stride < (size_t)es * W)
        return fail(SIFT_HIP_ERR_INVALID, "row stride must be a multiple of the pixel size and >= width");
    if (int rc = check_in_flight(d)) return rc;
    long long f = 0;
    if (int rc = submit_device(d, img, stride, format, stream, 1, 0, &f)) return rc;
    // Device-ordered consumers see this frame's buffers at once; counts
    // follow at sift_hip_sync / sift_hip_wait.
    make_current(d, f);
    if (stream) {
        HIPCHK(hipEventRecord(d->evOut, d->stream));
        HIPCHK(hipStreamWaitEvent((hipStream_t)stream, d->evOut, 0));
    }
    return SIFT_HIP_OK;
}

int sift_hip_submit_device(sift_hip_t d, const void* img, size_t stride, int format, void* stream, long long* ticket) {
    CHECK_HANDLE(d);
    if (!img) return fail(SIFT_HIP_ERR_INVALID, "null image");
    const int es = format_size(format);
    if (!es) return fail(SIFT_HIP_ERR_INVALID, "unknown pixel format");
    const int W = d->cfg.col_width;
    if (stride == 0) stride = (size_t)es * W;
    if (stride % es || stride < (size_t)es * W)
        return fail(SIFT_HIP_ERR_INVALID, "row stride must be a multiple of the pixel size and >= width");
    if (int rc = check_in_flight(d)) return rc;
    return submit_device(d, img, stride, format, stream, 1, 0, ticket, true);
}

int sift_hip_detect_device(sift_hip_t d, const float* img, size_t stride, void* stream) {
    return sift_hip_detect_device_fmt(d, img, stride, SIFT_HIP_F32, stream);
}

int sift_hip_set_batch(sift_hip_t d, int frames) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (frames < 1 || frames > kMaxBatch) return fail(SIFT_HIP_ERR_INVALID, "batch size out of range (1..64)");
    if (d->allocated) return fail(SIFT_HIP_ERR_STATE, "sift_hip_set_batch after sift_hip_warmup");
    d->B = frames;
    return SIFT_HIP_OK;
}

int sift_hip_set_lanes(sift_hip_t d, int lanes) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (lanes < 1 || lanes > kMaxLanes) return fail(SIFT_HIP_ERR_INVALID, "lanes out of range (1..4)");
    if (d->allocated) return fail(SIFT_HIP_ERR_STATE, "sift_hip_set_lanes after sift_hip_warmup");
    d->maxLanes = lanes;
    return SIFT_HIP_OK;
}

int sift_hip_set_micro_batch(sift_hip_t d, int frames) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (frames < 1 || frames > sift_hip_detector::kMaxMicroBatch)
        return fail(SIFT_HIP_ERR_INVALID, "micro-batch out of range (1..16)");
    if (d->allocated) return fail(SIFT_HIP_ERR_STATE, "sift_hip_set_micro_batch after sift_hip_warmup");
    d->mb = frames;
    return SIFT_HIP_OK;
}

int sift_hip_micro_batch(sift_hip_t d, int* frames) {
    if (!d || !frames) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *frames = d->mb;
    return SIFT_HIP_OK;
}

int sift_hip_set_auto_micro_batch(sift_hip_t d, int frames) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (frames < 0 || frames > sift_hip_detector::kMaxMicroBatch)
        return fail(SIFT_HIP_ERR_INVALID, "automatic micro-batch out of range (0..16)");
    if (d->allocated) return fail(SIFT_HIP_ERR_STATE, "sift_hip_set_auto_micro_batch after sift_hip_warmup");
    d->autoMb = frames;
    return SIFT_HIP_OK;
}

int sift_hip_auto_micro_batch(sift_hip_t d, int* frames) {
    if (!d || !frames) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *frames = auto_groups(d) ? d->autoMb : 0;
    return SIFT_HIP_OK;
}

int sift_hip_lanes(sift_hip_t d, int* max_lanes, int* created) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (max_lanes) *max_lanes = d->maxLanes;
    if (created) *created = d->nLanes;
    return SIFT_HIP_OK;
}

int sift_hip_set_descriptor_mode(sift_hip_t d, int mode) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (mode != SIFT_HIP_DESC_FAST && mode != SIFT_HIP_DESC_EXACT) return fail(SIFT_HIP_ERR_INVALID, "unknown descriptor mode");
    if (d->allocated) return fail(SIFT_HIP_ERR_STATE, "sift_hip_set_descriptor_mode after sift_hip_warmup");
    d->kp.descExact = mode == SIFT_HIP_DESC_EXACT;
    return SIFT_HIP_OK;
}

int sift_hip_descriptor_mode(sift_hip_t d, int* mode) {
    if (!d || !mode) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *mode = d->kp.descExact ? SIFT_HIP_DESC_EXACT : SIFT_HIP_DESC_FAST;
    return SIFT_HIP_OK;
}

int sift_hip_batch_capacity(sift_hip_t d, int* frames) {
    if (!d || !frames) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *frames = d->B;
    return SIFT_HIP_OK;
}

int sift_hip_detect_batch_device(sift_hip_t d, const void* frames, int n, size_t stride, size_t frame_stride,
                                 int format, void* stream) {
    CHECK_HANDLE(d);
    if (!frames) return fail(SIFT_HIP_ERR_INVALID, "null frames");
    if (n < 1 || n > d->B) return fail(SIFT_HIP_ERR_INVALID, "frame count outside 1..batch capacity");
    const int es = format_size(format);
    if (!es) return fail(SIFT_HIP_ERR_INVALID, "unknown pixel format");
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    if (stride == 0) stride = (size_t)es * W;
    if (stride % es || stride < (size_t)es * W)
        return fail(SIFT_HIP_ERR_INVALID, "row stride must be a multiple of the pixel size and >= width");
    if (frame_stride == 0) frame_stride = stride * H;
    if (n > 1 && frame_stride < stride * (H - 1) + (size_t)es * W)
        return fail(SIFT_HIP_ERR_INVALID, "frame stride smaller than one frame");
    if (int rc = check_in_flight(d)) return rc;
    long long f = 0;
    if (int rc = submit_device(d, frames, stride, format, stream, n, frame_stride, &f)) return rc;
    make_current(d, f);
    if (stream) {
        HIPCHK(hipEventRecord(d->evOut, d->stream));
        HIPCHK(hipStreamWaitEvent((hipStream_t)stream, d->evOut, 0));
    }
    return SIFT_HIP_OK;
}

int sift_hip_batch_frames(sift_hip_t d, int* n) {
    CHECK_HANDLE(d);
    if (!n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *n = batch_frames_of(d);
    return SIFT_HIP_OK;
}

int sift_hip_batch_results_device(sift_hip_t d, int i, int* count, int* overflow, const float** k3,
                                  const float** f4, const uint16_t** desc) {
    CHECK_HANDLE(d);
    if (i < 0 || i >= batch_frames_of(d)) return fail(SIFT_HIP_ERR_INVALID, "no such frame in the current batch");
    if (count || overflow)
        if (int rc = ensure_counts(d)) return rc;
    const Counters& c = d->hCtr[(size_t)d->cur * d->lane().B + i];
    const long o = (long)i * d->afs;
    if (count) *count = (int)std::min<unsigned>(c.final_n, d->kp.capFinal);
    if (overflow) *overflow = (int)c.overflow;
    if (k3) *k3 = fptr(d->dKpts3[d->cur], o);
    if (f4) *f4 = fptr(d->dFeats4[d->cur], o);
    if (desc) *desc = fptr(d->dDesc[d->cur], o);
    return SIFT_HIP_OK;
}

int sift_hip_batch_copy_to_host(sift_hip_t d, int i, float* k3, float* f4, uint16_t* desc, int cap, int* count) {
    int n = 0;
    const float *dk = nullptr, *df = nullptr;
    const uint16_t* dd = nullptr;
    if (int rc = sift_hip_batch_results_device(d, i, &n, nullptr, &dk, &df, &dd)) return rc;
    n = std::min(n, cap);
    if (count) *count = n;
    hipStream_t s;
    if (int rc = copy_stream(d, &s)) return rc;
    HIPCHK(hipStreamWaitEvent(s, d->lane().evFrame[d->cur], 0));
    if (n > 0) {
        if (k3) HIPCHK(hipMemcpyAsync(k3, dk, sizeof(float) * 3 * n, hipMemcpyDeviceToHost, s));
        if (f4) HIPCHK(hipMemcpyAsync(f4, df, sizeof(float) * 4 * n, hipMemcpyDeviceToHost, s));
        if (desc) HIPCHK(hipMemcpyAsync(desc, dd, sizeof(uint16_t) * 128 * n, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    return SIFT_HIP_OK;
}

int sift_hip_sync(sift_hip_t d) {
    CHECK_HANDLE(d);
    return finish_frame(d);
}

int sift_hip_num_keypoints(sift_hip_t d, int* n) {
    if (!d || !n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    if (d->allocated && d->lanes[0].ready) {
        HIPCHK(hipSetDevice(d->device));
        bind_lane(d, d->curLane, d->curIdx);
        if (int rc = ensure_counts(d)) return rc;
    }
    *n = d->count;
    return SIFT_HIP_OK;
}

int sift_hip_overflow_flags(sift_hip_t d, int* flags) {
    if (!d || !flags) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    if (d->allocated && d->lanes[0].ready) {
        HIPCHK(hipSetDevice(d->device));
        bind_lane(d, d->curLane, d->curIdx);
        if (int rc = ensure_counts(d)) return rc;
    }
    *flags = d->hCtr ? (int)d->hCtr[(size_t)d->cur * d->lane().B].overflow : 0;
    return SIFT_HIP_OK;
}

int sift_hip_capacities(sift_hip_t d, int* cand, int* refined, int* oriented, int* results) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (cand) *cand = (int)d->capCand;
    if (refined) *refined = (int)d->kp.capRefined;
    if (oriented) *oriented = (int)d->kp.capOriented;
    if (results) *results = (int)d->kp.capFinal;
    return SIFT_HIP_OK;
}

int sift_hip_results_device(sift_hip_t d, const float** k3, const float** f4, const uint16_t** desc,
                            const uint16_t** prev, int* prevCount, int* capacity) {
    CHECK_HANDLE(d);
    if (prevCount)
        if (int rc = ensure_counts(d)) return rc;
    if (k3) *k3 = d->dKpts3[d->cur];
    if (f4) *f4 = d->dFeats4[d->cur];
    if (desc) *desc = d->dDesc[d->cur];
    if (prev) *prev = d->current - 1 >= d->firstFrame ? frame_desc(d, d->current - 1) : d->dDesc[(d->cur + d->lane().nslots - 1) % d->lane().nslots];
    if (prevCount) *prevCount = d->prevCount;
    if (capacity) *capacity = (int)d->kp.capFinal;
    return SIFT_HIP_OK;
}

int sift_hip_copy_to_host(sift_hip_t d, float* k3, float* f4, uint16_t* desc, int cap) {
    CHECK_HANDLE(d);
    if (int rc = ensure_counts(d)) return rc;
    const int n = std::min(d->count, cap);
    Lane& L = d->lane();
    if (!d->hostWant)
        for (int k = 0; k < d->nLanes; k++)
            if (d->lanes[k].ready)
                if (int rc = ensure_host_res(d, d->lanes[k])) return rc;
    d->hostWant = std::max(d->hostWant, desc ? 2 : 1);
    const int region = d->cur * d->lane().B + d->curIdx;
    if (L.hRes && L.hostFrame[region] == d->current && d->current >= d->firstFrame && (!desc || L.hostDesc[region])) {
        // A host-input frame: its descriptor kernel wrote them to pinned host memory.
        HIPCHK(hipEventSynchronize(L.evFrame[d->cur]));
        float *hk3, *hf4;
        uint16_t* hdesc;
        host_res(d, L.hRes, region, &hk3, &hf4, &hdesc);
        if (n > 0) {
            if (k3) memcpy(k3, hk3, sizeof(float) * 3 * n);
            if (f4) memcpy(f4, hf4, sizeof(float) * 4 * n);
            if (desc) {  // 2.2 MB at C2: split over the copy pool (one thread: 0.100 -> 0.047 ms, C++ loop)
                if (!d->pool && 256u * n >= (1u << 20)) d->pool = new CopyPool(kCopyWorkers);
                copy_rows(d->pool, (char*)desc, 256, (const char*)hdesc, 256, 256, n);
            }
        }
        return SIFT_HIP_OK;
    }
    // On the copy stream, ordered after the current frame only: frames
    // submitted after it keep running.
    hipStream_t s;
    if (int rc = copy_stream(d, &s)) return rc;
    HIPCHK(hipStreamWaitEvent(s, d->lane().evFrame[d->cur], 0));
    if (n > 0) {
        if (k3) HIPCHK(hipMemcpyAsync(k3, d->dKpts3[d->cur], sizeof(float) * 3 * n, hipMemcpyDeviceToHost, s));
        if (f4) HIPCHK(hipMemcpyAsync(f4, d->dFeats4[d->cur], sizeof(float) * 4 * n, hipMemcpyDeviceToHost, s));
        if (desc)
            HIPCHK(hipMemcpyAsync(desc, d->dDesc[d->cur], sizeof(uint16_t) * 128 * n, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    return SIFT_HIP_OK;
}

// The current frame's results in the handle's pinned host region (the lane's
// region slot * B + idx): a host-input frame's were written there by its
// descriptor kernel (HostOut), any other frame's are copied there now over the
// copy stream.  No copy into caller memory.
int sift_hip_results_host(sift_hip_t d, const float** k3, const float** f4, const uint16_t** desc, int* count) {
    CHECK_HANDLE(d);
    if (int rc = ensure_counts(d)) return rc;
    const int n = std::min(d->count, (int)d->kp.capFinal);
    Lane& L = d->lane();
    if (!d->hostWant)
        for (int k = 0; k < d->nLanes; k++)
            if (d->lanes[k].ready)
                if (int rc = ensure_host_res(d, d->lanes[k])) return rc;
    d->hostWant = std::max(d->hostWant, desc ? 2 : 1);
    const int region = d->cur * d->lane().B + d->curIdx;
    float *hk3, *hf4;
    uint16_t* hdesc;
    host_res(d, L.hRes, region, &hk3, &hf4, &hdesc);
    if (L.hostFrame[region] == d->current && d->current >= d->firstFrame && (!desc || L.hostDesc[region])) {
        HIPCHK(hipEventSynchronize(L.evFrame[d->cur]));
    } else {
        hipStream_t s;
        if (int rc = copy_stream(d, &s)) return rc;
        HIPCHK(hipStreamWaitEvent(s, L.evFrame[d->cur], 0));
        if (n > 0) {
            HIPCHK(hipMemcpyAsync(hk3, d->dKpts3[d->cur], sizeof(float) * 3 * n, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(hf4, d->dFeats4[d->cur], sizeof(float) * 4 * n, hipMemcpyDeviceToHost, s));
            if (desc)
                HIPCHK(hipMemcpyAsync(hdesc, d->dDesc[d->cur], sizeof(uint16_t) * 128 * n, hipMemcpyDeviceToHost, s));
        }
        HIPCHK(hipStreamSynchronize(s));
        L.hostFrame[region] = d->current;
        L.hostDesc[region] = desc != nullptr;
    }
    if (k3) *k3 = hk3;
    if (f4) *f4 = hf4;
    if (desc) *desc = hdesc;
    if (count) *count = n;
    return SIFT_HIP_OK;
}

int sift_hip_results_sidecar(sift_hip_t d, const int8_t** codes, const int** keys) {
    CHECK_HANDLE(d);
    if (codes) *codes = d->dSide[d->cur].codes;
    if (keys) *keys = d->dSide[d->cur].keys;
    return SIFT_HIP_OK;
}

int sift_hip_copy_descriptors_device(sift_hip_t d, uint16_t* dst, int cap, void* stream) {
    CHECK_HANDLE(d);
    if (int rc = ensure_counts(d)) return rc;
    const int n = std::min(d->count, cap);
    hipStream_t s = stream ? (hipStream_t)stream : d->stream;
    if (s != d->stream) HIPCHK(hipStreamWaitEvent(s, d->lane().evFrame[d->cur], 0));
    if (n > 0) HIPCHK(hipMemcpyAsync(dst, d->dDesc[d->cur], sizeof(uint16_t) * 128 * n, hipMemcpyDeviceToDevice, s));
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return SIFT_HIP_OK;
}

int sift_hip_set_datagen(sift_hip_t d, const char* dir) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    d->dgDir = dir ? dir : "";
    return SIFT_HIP_OK;
}

int sift_hip_replay_stage(sift_hip_t d, const char* dump_dir, const char* stage, const char* out_dir) {
    CHECK_HANDLE(d);
    if (!dump_dir || !stage || !out_dir) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    return replay_stage(d, dump_dir, stage, out_dir);
}

int sift_hip_set_timing(sift_hip_t d, int enable) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    d->timing = enable != 0;
    d->blurReps = enable > 1 ? enable : 1;
    return SIFT_HIP_OK;
}

int sift_hip_timing_count(sift_hip_t d, int* n) {
    if (!d || !n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *n = (int)d->tagg.size();
    return SIFT_HIP_OK;
}

int sift_hip_timing_entry(sift_hip_t d, int i, const char** name, double* ms, int* launches, double* bytes) {
    if (!d || i < 0 || i >= (int)d->tagg.size()) return fail(SIFT_HIP_ERR_INVALID, "bad timing index");
    if (name) *name = d->tagg[i].name.c_str();
    if (ms) *ms = d->tagg[i].ms;
    if (launches) *launches = d->tagg[i].launches;
    if (bytes) *bytes = d->tagg[i].bytes;
    return SIFT_HIP_OK;
}

int sift_hip_timing_reset(sift_hip_t d) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    for (auto& a : d->tagg) a.ms = a.bytes = 0, a.launches = 0;
    return SIFT_HIP_OK;
}

int sift_hip_debug_gaussian(sift_hip_t d, int o, int layer, float* out) {
    CHECK_HANDLE(d);
    if (o < 0 || o >= d->nOct || layer < 0 || layer >= d->L + 3 || !out)
        return fail(SIFT_HIP_ERR_INVALID, "bad plane");
    const OctGeom& g = d->pyr.oct[o];
    HIPCHK(hipMemcpy2D(out, sizeof(float) * g.W, g.base + (size_t)layer * g.planeStride, sizeof(float) * g.pitch,
                       sizeof(float) * g.W, g.H, hipMemcpyDeviceToHost));
    return SIFT_HIP_OK;
}

int sift_hip_debug_candidates(sift_hip_t d, int* quads, int cap, int* count) {
    CHECK_HANDLE(d);
    if (int rc = ensure_counts(d)) return rc;
    const Counters& c = d->hCtr[(size_t)d->cur * d->lane().B];
    const int n = (int)std::min<unsigned>(c.cand, d->capCand);
    if (count) *count = (int)c.cand;
    const int m = std::min(n, cap);
    if (m > 0 && quads) {
        std::vector<uint2> tmp(m);
        HIPCHK(hipMemcpy(tmp.data(), d->dCand, sizeof(uint2) * m, hipMemcpyDeviceToHost));
        for (int i = 0; i < m; i++) {
            quads[4 * i] = (int)(tmp[i].x >> 8);
            quads[4 * i + 1] = (int)(tmp[i].x & 255);
            quads[4 * i + 2] = (int)(tmp[i].y >> 16);
            quads[4 * i + 3] = (int)(tmp[i].y & 0xffff);
        }
    }
    return SIFT_HIP_OK;
}

}  // extern "C"
