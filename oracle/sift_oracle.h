/*
 * sift_oracle.h -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of OpenCV 4.x SIFT (features2d/src/sift.dispatch.cpp +
 * sift.simd.hpp) and of BFMatcher(NORM_L2).knnMatch(k=2).  It is the parity
 * checker for the HIP path in another-cuda-sift_amd/ and the CPU baseline leg of
 * bench.py.  Nothing in the product links, loads or calls this library.
 *
 * Parity status: UNPINNED against a real OpenCV build.  OpenCV (the third-party
 * library the reference names as its model, /root/reference/readme.md:5, pinned
 * only as git submodule "thirdparty/opencv" branch 4.x, /root/reference/.gitmodules)
 * is not present in this image and the reference ships no golden vectors
 * (/root/reference/data/readme.md is empty).  See DESIGN.md "Oracle".
 */
#ifndef SIFT_ORACLE_H
#define SIFT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One keypoint, field-for-field cv::KeyPoint minus class_id. */
typedef struct {
    float x, y;      /* pt, original-image pixels                       */
    float size;      /* diameter                                         */
    float angle;     /* degrees, 0..360                                  */
    float response;  /* |contrast|                                       */
    int   octave;    /* packed: octave & 255 | layer << 8 | xi << 16     */
} sift_oracle_kpt;

/* cv::SIFT::create() parameters + the two knobs the reference adds. */
typedef struct {
    int    nfeatures;          /* 0 = keep all (OpenCV default)           */
    int    nOctaveLayers;      /* 3                                       */
    double contrastThreshold;  /* 0.04                                    */
    double edgeThreshold;      /* 10                                      */
    double sigma;              /* 1.6                                     */
    int    firstOctave;        /* -1 = double the image (OpenCV), 0 = not */
    int    nOctaves;           /* 0 = OpenCV's auto formula               */
} sift_oracle_params;

void sift_oracle_default_params(sift_oracle_params* p);

/* Which build of the restatement this library is (oracle/Makefile):
 * "pinned" (the parity pin of the HIP path), "avx2-fma", "avx512-fma" (the
 * OpenCV-tolerance ensemble). */
const char* sift_oracle_variant(void);

/* Gaussian taps exactly as cv::getGaussianKernel(cvRound(8*sigma+1)|1, sigma, CV_32F).
 * Returns the tap count (odd) or -1 if cap is too small. */
int sift_oracle_gaussian_taps(double sigma, float* taps, int cap);

/* Number of octaves the auto formula gives for a w x h input. */
int sift_oracle_num_octaves(int w, int h, const sift_oracle_params* p);

/* Octave geometry: width/height of octave o. */
void sift_oracle_octave_dims(int w, int h, const sift_oracle_params* p, int o, int* ow, int* oh);

/* Full Gaussian pyramid.  `planes` receives nOctaves*(L+3) planes, each stored
 * densely (ow*oh floats) one after another in (octave, layer) order.
 * Returns the number of floats written, or the number needed if planes==NULL. */
long sift_oracle_gaussian_pyramid(const float* img, int w, int h,
                                  const sift_oracle_params* p, float* planes);

/* 3x3x3 scale-space extrema before refinement: (octave, layer, r, c) quadruples
 * in octave/layer/raster order.  Returns the count (writes min(count, cap)). */
long sift_oracle_extrema(const float* img, int w, int h, const sift_oracle_params* p,
                         int* quads, long cap);

/* Full detectAndCompute.  Keypoints come out in KeypointGreater order
 * (removeDuplicatedSorted) with retainBest applied as a stable filter; the
 * descriptors are the CV_32F 0..255 integers, 128 per keypoint.  Returns the
 * keypoint count; writes at most cap keypoints/descriptors (desc may be NULL).
 * `threads` <= 0 means all OpenMP threads. */
long sift_oracle_detect_and_compute(const float* img, int w, int h,
                                    const sift_oracle_params* p, int threads,
                                    sift_oracle_kpt* kpts, float* desc, long cap);

/* Descriptors for given keypoints (OpenCV's useProvidedKeypoints=false path
 * reuses this), computed on the pyramid of `img`. */
/* Wall time (ms) of the stages of the last sift_oracle_detect_and_compute call:
 * initial image, Gaussian pyramid, DoG, 3x3x3 candidates, keypoints (refine,
 * orientation, dedupe, retainBest), descriptors.  Returns 6. */
int sift_oracle_stage_ms(double* out, int cap);

int sift_oracle_compute_descriptors(const float* img, int w, int h,
                                    const sift_oracle_params* p,
                                    const sift_oracle_kpt* kpts, long n, float* desc);

/* BFMatcher(NORM_L2).knnMatch(k=2) on 128-D float descriptors: idx[2*i+{0,1}]
 * and dist[2*i+{0,1}] (sqrt L2).  Missing neighbours are -1 / FLT_MAX. */
void sift_oracle_knn2(const float* query, long nq, const float* train, long nt,
                      int threads, int* idx, float* dist);

#ifdef __cplusplus
}
#endif
#endif
