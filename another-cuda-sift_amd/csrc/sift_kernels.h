// Internal interface between the C-ABI orchestration (detector.hip) and the
// HIP kernel translation units.  Not installed; no torch types.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

namespace sift_amd {

constexpr int kMaxOctaves = 16;
constexpr int kMaxTaps = 63;  // r <= 31
constexpr int kMaxBatch = 64;  // frames per launch

// Frame batches: every launch processes `nf` frames.  Each frame owns one
// "frame arena" (pyramid, candidate / keypoint lists, counters, result slots)
// and the arenas sit at a fixed byte stride, so frame f's copy of any buffer
// is the frame-0 pointer + f * stride.  Kernels take the frame from the grid
// (blockIdx.y, or the XCD-ordered block index for the tiled pyramid kernels).
// nf = 1 is the single-frame pipeline.
struct Frames {
    int nf;
    long stride;  // bytes between consecutive frames' arenas
};
template <class T>
__host__ __device__ __forceinline__ T* fptr(T* p, long off) {
    return reinterpret_cast<T*>(reinterpret_cast<uintptr_t>(p) + off);
}

// Separable Gaussian taps (host-computed, OpenCV getGaussianKernel bit-exact
// recipe) passed by value so they live in the kernarg segment (scalar loads).
struct Taps {
    float w[64];
    int n;
};

// One octave of the Gaussian pyramid: (L+3) planes of H rows x pitch floats,
// plane i at base + i * planeStride.  Pitch is a multiple of 64 floats (256 B)
// so every row starts on a full HBM burst.
struct OctGeom {
    float* base;
    long planeStride;  // floats
    int W, H, pitch;
    int rowBase;   // first global row-bucket id of this octave (layers 1..L)
    long bitBase;  // first bit of this octave in the dedupe bitmap
};

struct PyrDesc {
    OctGeom oct[kMaxOctaves];
    int nOct;
    int L;
    int firstOctave;
};

// Refined keypoint (output of adjustLocalExtrema), pyramid coordinates.
struct RefKpt {
    float x, y, size, response;  // x,y,size in the detection pyramid's units
    int octave;                  // packed, pyramid octave index in low byte
    int o, layer, rc;            // rc = r << 16 | c
};

// Oriented keypoint = cv::KeyPoint after the firstOctave rescale, plus its
// deterministic sort key (row bucket, (c << 6) | peak index).
struct OriKpt {
    float x, y, size, angle, response;
    int octave;
    int bucket, sub;
};

// Per-frame counters, zeroed by the frame's first blur (no memset node).
struct Counters {
    unsigned cand;       // 3x3x3 extrema candidates
    unsigned refined;    // after adjustLocalExtrema + dedupe
    unsigned oriented;   // orientation peaks beyond each keypoint's first (appended after the refined slots)
    unsigned final_n;    // after retainBest (written by the bucket scan)
    unsigned overflow;   // bit 0 cand, 1 refined, 2 oriented, 3 final
    unsigned thr_bits;   // retainBest response threshold (float bits)
    unsigned pad[2];     // pad[0]: entries of the order list (k_order path); pad[1]: host results (HostOut)
};

// Oriented keypoint list: refined keypoint k's first peak sits in slot k (no
// atomic), further peaks are appended from slot min(refined, capRefined) on;
// a keypoint without a peak leaves a hole (bucket kHoleBucket, response 0).
constexpr unsigned kHoleBucket = 0xffffffffu;

// --- launch wrappers (implemented in pyramid.hip / keypoints.hip / match.hip) --
// sfs: byte stride between the nf source frames (the caller's frames or arenas).
void launch_upsample2x(const float* src, int spitch, int W, int H, float* dst, int dpitch, const Frames& fr, long sfs,
                       hipStream_t s);
// Pixel range of octave 0 / plane 0 (every later plane is a convex combination
// of it), accumulated by the initial blur as kRangeSlots pairs of
// order-preserving keys {max(v), max(-v)} (atomicMax spread over slots).
constexpr int kRangeSlots = 256;
// range_keys (nullable): 2 * kRangeSlots keys, zeroed before the launch.
// zero_ctr (nullable): counters to zero (the frame's first blur).
// The next octave's base plane, written by the blur of plane L of this octave
// as it stores its tiles: dst[2y][2x] -> p[y][x] for x < W, y < H (OpenCV's
// INTER_NEAREST half-size resize).  p == nullptr: none.
struct DecOut {
    float* p = nullptr;
    int pitch = 0, W = 0, H = 0;
};
void launch_blur(const float* src, int spitch, int W, int H, float* dst, int dpitch, const DecOut& dec,
                 const Taps& taps, const Frames& fr, long sfs, hipStream_t s, unsigned* range_keys = nullptr,
                 Counters* zero_ctr = nullptr);
// Kernel node parameters of the f32 head launches (the frame's first blur with
// range keys and counter zeroing, or the 2x upsample), for re-pointing a
// captured graph's head node at each frame's input.
struct HeadNode {
    hipKernelNodeParams p;
    alignas(16) unsigned char args[512];  // argument values (argv[i] -> args)
    void* argv[8];
};
void head_blur_node(HeadNode& h, const float* src, int spitch, int W, int H, float* dst, int dpitch, const Taps& taps,
                    const Frames& fr, long sfs, unsigned* range_keys, Counters* zero_ctr);
void head_upsample_node(HeadNode& h, const float* src, int spitch, int W, int H, float* dst, int dpitch,
                        const Frames& fr, long sfs);
// Two independent float blurs in one launch (no range keys / counters);
// false (nothing launched) when the radius pair has no instantiation.
struct BlurDesc {
    const float* src;
    int spitch, W, H;
    float* dst;
    int dpitch;
    DecOut dec;
    const Taps* taps;
};
bool launch_blur_pair(const BlurDesc& a, const BlurDesc& b, const Frames& fr, hipStream_t s);
// Pyramid tail (pyramid.hip): planes 1..L+2 of octaves o0..nOct-1 of each
// frame in one workgroup, in LDS, from octave o0's base plane (already in
// HBM).  tail_first_octave: the first octave from which every later octave
// fits (nOct: none).  taps[i] = the blur of plane i (i = 1..L+2).
constexpr int kTailLdsFloats = 32768;  // 128 KiB of dynamic LDS (+ ~4.6 KiB static: taps, reflection tables)
constexpr int kTailMaxPlanes = 9;           // L <= 6
struct TailDesc {
    OctGeom oct[kMaxOctaves];
    Taps taps[kTailMaxPlanes];
    int o0, nOct, L, regionX, regionY, rpad;
};
int tail_first_octave(const PyrDesc& pyr, const Taps* taps, int L);
hipError_t tail_init();  // lets the tail kernel take up to 160 KiB of dynamic LDS (once, before capture)
void launch_blur_tail(const PyrDesc& pyr, const Taps* taps, int L, int o0, const Frames& fr, hipStream_t s);
// 8-bit frames (pitches in bytes).  launch_blur_u8 returns false (nothing
// launched) for an init radius without a fused 8-bit instantiation; the caller
// then converts with launch_u8_to_f32 and uses launch_blur.
bool launch_blur_u8(const uint8_t* src, int spitch, int W, int H, float* dst, int dpitch, const Taps& taps,
                    const Frames& fr, long sfs, hipStream_t s, unsigned* range_keys, Counters* zero_ctr);
void launch_u8_to_f32(const uint8_t* src, int spitch, int W, int H, float* dst, int dpitch, const Frames& fr,
                      long sfs, hipStream_t s);
void launch_upsample2x_u8(const uint8_t* src, int spitch, int W, int H, float* dst, int dpitch, const Frames& fr,
                          long sfs, hipStream_t s);
// 3x3x3 extrema of every octave in one launch (L = 1..6; false = nothing
// launched), else per octave with launch_extrema.
bool launch_extrema_all(const PyrDesc& pyr, float threshold, uint2* cand, Counters* ctr, unsigned cap,
                        const Frames& fr, hipStream_t s);
void launch_extrema(const PyrDesc& pyr, int o, float threshold, uint2* cand, Counters* ctr, unsigned cap,
                    const Frames& fr, hipStream_t s);

struct KeypointParams {
    float contrastThreshold, edgeThreshold, sigma;
    int numFeatures;
    unsigned capRefined, capOriented, capFinal;
    int numBuckets;
    int oriRmax, descRmax;  // LDS patch bounds for orientation / descriptor radii
    int descNrec;           // LDS record bound of the descriptor's counting sort
    int descExact;          // 1: OpenCV's sequential float histogram (k_descriptor_exact)
};
void launch_refine(const PyrDesc& pyr, const uint2* cand, unsigned capCand, Counters* ctr, uint32_t* bitmap,
                   RefKpt* out, const KeypointParams& kp, const Frames& fr, hipStream_t s);
// Also clears each refined keypoint's dedupe bit (k_refine set it), so the
// bitmap is zero again for the next frame without a memset.
void launch_orientation(const PyrDesc& pyr, const RefKpt* in, Counters* ctr, OriKpt* out, uint32_t* bitmap,
                        const KeypointParams& kp, const Frames& fr, hipStream_t s);
// zero_range: the other frame buffer's 2 * kRangeSlots range keys (zeroed here
// for the next frame, so no memset node is needed).
void launch_select(const OriKpt* kpts, Counters* ctr, unsigned* zero_range, const KeypointParams& kp, const Frames& fr,
                   hipStream_t s);
// select + bucket count + scan + scatter in one single-workgroup launch;
// false (nothing launched) when the row buckets exceed kOrderMaxBuckets.
constexpr int kOrderMaxBuckets = 16384;  // 64 KiB of LDS

// Descriptor job order, longest first (exact descriptor mode): jobs are
// stored grouped by layer, highest layer (largest windows) first, octave and
// final order inside, so the descriptor grid starts its largest keypoints in
// its first residency round (a job's `out` keeps the output order).  Per
// frame, written by k_order and read by k_rank_final: per (octave, layer)
// segment its first final position and its first job index, and whether the
// order is in use.  Measured (tools/desc_mode_bench.py, two passes): exact
// mode 0.153 vs 0.156-0.157 ms per frame, single-frame sync 0.378-0.382 vs
// 0.408-0.409 ms; the default mode 0.092-0.093 vs 0.090-0.091 ms per frame
// (its per-keypoint cost varies less), so only the exact mode uses it.
constexpr int kLptSegs = kMaxOctaves * 8;  // octaves x (L <= 8) layers
struct JobOrder {
    int valid;
    int segStart[kLptSegs];
    int jobBase[kLptSegs];
};

bool launch_order(const PyrDesc& pyr, const OriKpt* kpts, Counters* ctr, unsigned* zero_range, unsigned* bcount, unsigned* boff, int* slot,
                  int* order, JobOrder* jord, const KeypointParams& kp, const Frames& fr, hipStream_t s);
void launch_bucket_count(const OriKpt* kpts, const Counters* ctr, unsigned* bcount, int* slot,
                         const KeypointParams& kp, const Frames& fr, hipStream_t s);
void launch_bucket_scan(unsigned* bcount, unsigned* boff, Counters* ctr, const KeypointParams& kp, const Frames& fr,
                        hipStream_t s);
void launch_bucket_scatter(const OriKpt* kpts, const Counters* ctr, const unsigned* boff, const int* slot,
                           int* order, const KeypointParams& kp, const Frames& fr, hipStream_t s);
// One final keypoint's descriptor window (written by k_bucket_rank, read with
// scalar loads by k_descriptor).  64 bytes.
constexpr int kDescMaxRows = 128;  // enumerated windows: 2 * radius + 1 <= kDescMaxRows
struct DescJob {
    const float* img;        // Gaussian plane (octave, layer) of the keypoint
    float cos_t, sin_t;      // cos/sin(angle) / hist_width
    float angle;             // 360 - kpt.angle (0 when that is 360)
    float hist_width;        // 3 * scl
    int ptx, pty;            // rounded keypoint position in the octave
    int rows, cols, pitch;   // plane geometry
    int radius;              // window radius (clamped to the plane diagonal)
    int out;                 // output slot (descriptor row) of this job's keypoint
    int pad[3];
};

static_assert(sizeof(DescJob) == 64, "DescJob is one 64-byte scalar load");

void launch_rank_final(const PyrDesc& pyr, const OriKpt* kpts, const unsigned* bcount, const unsigned* boff,
                       const int* order, const Counters* ctr, const JobOrder* jord, DescJob* jobs, float* kpts3, float* feats4,
                       const KeypointParams& kp, const Frames& fr, hipStream_t s);
// Results of a finished frame -> mapped pinned host buffers (host-input frames).
// Frame rows (rowB bytes, `rows` of them, pitches in bytes) copied by `wgs`
// 256-thread workgroups on the lane stream: host staging -> device, and
// micro-batch frames -> the group input (keypoints.hip).
constexpr int kStageWg = 64;      // host staging (PCIe-bound)
constexpr int kGroupCopyWg = 512; // device-to-device (HBM)
// flag (nullable): a word set to flag_val by the copy (a host frame's
// results request, Counters.pad[1]).
void launch_copy_rows(const void* src, size_t spitch, void* dst, size_t dpitch, size_t rowB, int rows, int wgs,
                      hipStream_t s, unsigned* flag = nullptr, unsigned flag_val = 0);
void launch_bucket_rank(const PyrDesc& pyr, const OriKpt* kpts, unsigned* bcount, const unsigned* boff,
                        const int* order, const Counters* ctr, DescJob* jobs, float* kpts3, float* feats4,
                        const KeypointParams& kp, const Frames& fr, hipStream_t s);
// host_ctr: device-mapped pinned host memory receiving the frames' counters
// (frame f at host_ctr[f]).
// Matcher sidecar of a descriptor buffer (written by the descriptor kernels
// beside the fp16 rows): per keypoint p its int8 codes c = v - 128 (128 B,
// row-major) and the key bias -(256 |c|^2 + (p & 255)) that the matcher's
// prep kernel would compute (match.hip).  sift_hip_match_* use it for
// detector-produced buffers instead of converting the fp16 rows.
struct Sidecar {
    int8_t* codes;
    int* keys;
};
// Host results written by the descriptor kernel itself (host-input frames of a
// handle whose caller reads results back): Counters.pad[1] carries the
// request -- high half set by the frame's staging copy (kHostReqShift), moved
// into the low half (the level: 1 keypoints + features, 2 also descriptors)
// by k_order / k_select, which clear the request; the frame's first blur keeps
// only the request half.  tab[frame] = the frame's pinned host region (null:
// none), laid out as the detector's host results (k3 | f4 at 256-aligned
// 12 cap | descriptors at + 16 cap); k3 / f4 = the slot's device results.
constexpr int kHostReqShift = 16;
struct HostOut {
    char* const* tab;
    const float* k3;
    const float* f4;
    unsigned cap;
};
void launch_descriptor(const DescJob* jobs, const Counters* ctr, const unsigned* range_keys, uint16_t* desc,
                       Sidecar side, Counters* host_ctr, HostOut host, const KeypointParams& kp, const Frames& fr,
                       hipStream_t s);

// Order-preserving unsigned key of a float (0 is below every key), so that
// atomicMax over keys is a float max with a zeroed counter as the identity.
__device__ __forceinline__ unsigned range_key(float f) {
    const unsigned u = __float_as_uint(f);
    return u & 0x80000000u ? ~u : u | 0x80000000u;
}
__device__ __forceinline__ float decode_range_key(unsigned u) {
    return __uint_as_float(u & 0x80000000u ? u & 0x7fffffffu : ~u);
}

// The C ABI's thread-local error message (sift_hip_last_error), shared by
// the translation units that implement entry points.
void set_last_error(const std::string& msg);

// Exp table (OpenCV expTab_f) uploaded once per device (orientation and
// descriptor translation units each hold a copy).
void upload_exp_table(const float* tab64);
void upload_desc_exp_table(const float* tab64);

}  // namespace sift_amd
