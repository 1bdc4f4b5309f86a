// Internal interface between the C-ABI orchestration (detector.hip) and the
// HIP kernel translation units.  Not installed; no torch types.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace sift_amd {

constexpr int kMaxOctaves = 16;
constexpr int kMaxTaps = 63;  // r <= 31

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

// Per-frame counters, zeroed by one memset node at the head of the graph.
struct Counters {
    unsigned cand;       // 3x3x3 extrema candidates
    unsigned refined;    // after adjustLocalExtrema + dedupe
    unsigned oriented;   // after orientation peaks
    unsigned final_n;    // after retainBest (written by the bucket scan)
    unsigned overflow;   // bit 0 cand, 1 refined, 2 oriented, 3 final
    unsigned thr_bits;   // retainBest response threshold (float bits)
    unsigned pad[2];
};

// --- launch wrappers (implemented in pyramid.hip / keypoints.hip / match.hip) --
void launch_upsample2x(const float* src, int spitch, int W, int H, float* dst, int dpitch, hipStream_t s);
void launch_blur(const float* src, int spitch, int sstep, int W, int H, float* dst, int dpitch, float* copy_out,
                 const Taps& taps, hipStream_t s);
void launch_extrema(const PyrDesc& pyr, int o, float threshold, uint2* cand, Counters* ctr, unsigned cap,
                    hipStream_t s);

struct KeypointParams {
    float contrastThreshold, edgeThreshold, sigma;
    int numFeatures;
    unsigned capRefined, capOriented, capFinal;
    int numBuckets;
    int oriRmax, descRmax;  // LDS patch bounds for orientation / descriptor radii
    int descNrec;           // LDS record bound of the descriptor's counting sort
};
void launch_refine(const PyrDesc& pyr, const uint2* cand, unsigned capCand, Counters* ctr, uint32_t* bitmap,
                   RefKpt* out, const KeypointParams& kp, hipStream_t s);
void launch_orientation(const PyrDesc& pyr, const RefKpt* in, Counters* ctr, OriKpt* out, const KeypointParams& kp,
                        hipStream_t s);
void launch_select(const OriKpt* kpts, Counters* ctr, const KeypointParams& kp, hipStream_t s);
void launch_bucket_count(const OriKpt* kpts, const Counters* ctr, unsigned* bcount, int* slot,
                         const KeypointParams& kp, hipStream_t s);
void launch_bucket_scan(unsigned* bcount, unsigned* boff, Counters* ctr, const KeypointParams& kp, hipStream_t s);
void launch_bucket_scatter(const OriKpt* kpts, const Counters* ctr, const unsigned* boff, const int* slot,
                           int* order, const KeypointParams& kp, hipStream_t s);
void launch_bucket_rank(const OriKpt* kpts, const unsigned* bcount, const unsigned* boff, const int* order,
                        const Counters* ctr, int* final_order, const KeypointParams& kp, hipStream_t s);
void launch_descriptor(const PyrDesc& pyr, const OriKpt* kpts, const int* final_order, const Counters* ctr,
                       float* kpts3, float* feats4, uint16_t* desc, const KeypointParams& kp, hipStream_t s);

// Exp table (OpenCV expTab_f) uploaded once per device.
void upload_exp_table(const float* tab64);
void upload_exp_table_desc(const float* tab64);

}  // namespace sift_amd
