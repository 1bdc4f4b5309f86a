// sift_cuda::Detector / matchBruteForce (include/sift_cuda/Detector.hh): the
// reference's C++ surface (/root/reference/sift_cuda/interface/Detector.hh:24-96,
// /root/reference/sift_cuda/sift_func/Match.cuh:9-14) over the C ABI in
// include/sift_hip.h.  Plain C++ (g++): no HIP headers, no device code.
//
// Error behaviour mirrors the reference: CUDA_CHECK printed the error and
// exit(EXIT_FAILURE)ed (CudaMemRAII.cuh:11-19); gpuWarmUpAndAllocate returns
// false when the image size is unset (Detector.cu:22-25).
#include "sift_cuda/Detector.hh"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <memory>

#include "sift_hip.h"

namespace sift_cuda {

namespace {

void check(int rc, const char* what) {
    if (rc != SIFT_HIP_OK) {
        std::fprintf(stderr, "sift_hip error %d in %s: %s\n", rc, what, sift_hip_last_error());
        std::exit(EXIT_FAILURE);
    }
}

sift_hip_config toAbi(const CudaSiftConfig& c) {
    sift_hip_config a;
    sift_hip_default_config(&a, c.col_width, c.row_width);
    a.numFeatures = c.numFeatures;
    a.numOctaveLayers = c.numOctaveLayers;
    a.contrastThreshould = c.contrastThreshould;
    a.edgeThreshould = c.edgeThreshould;
    a.sigma = c.sigma;
    a.upscale = c.upscale ? 1 : 0;
    a.numOctaves = c.numOctaves;
    a.maxKeypoints = c.maxKeypoints;
    return a;
}

}  // namespace

Detector::Detector(const CudaSiftConfig& config) : Detector(config, -1) {}

Detector::Detector(const CudaSiftConfig& config, int device) : m_config(config) {
    if (config.col_width > 0 && config.row_width > 0) {
        const sift_hip_config a = toAbi(config);
        check(sift_hip_create(&a, device, &m_handle), "Detector::Detector");
        sift_hip_num_octaves(m_handle, &m_nOctaves);
    }
    max_kpts = config.numFeatures;
    std::cout << "nOctaves: " << m_nOctaves << ". " << config.col_width << ", " << config.row_width << std::endl;
}

Detector::~Detector() {
    if (m_handle) sift_hip_destroy(m_handle);
}

bool Detector::gpuWarmUpAndAllocate() {
    if (m_initialized) return true;
    if (!m_handle) {
        std::cerr << "Image width or height not set." << std::endl;
        return false;
    }
    check(sift_hip_warmup(m_handle), "gpuWarmUpAndAllocate");
    m_initialized = true;
    refreshViews();
    return true;
}

void Detector::refreshViews() {
    const float *k3 = nullptr, *f4 = nullptr;
    const uint16_t *desc = nullptr, *prev = nullptr;
    int prevCount = 0, cap = 0;
    check(sift_hip_results_device(m_handle, &k3, &f4, &desc, &prev, &prevCount, &cap), "results");
    device_kpts = DeviceBuffer<Float3>(reinterpret_cast<Float3*>(const_cast<float*>(k3)), (size_t)cap);
    device_features = DeviceBuffer<Float4>(reinterpret_cast<Float4*>(const_cast<float*>(f4)), (size_t)cap);
    // Writable descriptor views drop the rows' matcher sidecar (sift_hip.h).
    auto written = [](const void* p) { (void)sift_hip_descriptors_written(static_cast<const uint16_t*>(p)); };
    device_descriptor = DeviceBuffer<Half>(reinterpret_cast<Half*>(const_cast<uint16_t*>(desc)), (size_t)cap * 128, written);
    prev_descriptor = DeviceBuffer<Half>(reinterpret_cast<Half*>(const_cast<uint16_t*>(prev)), (size_t)cap * 128, written);
    sift_hip_num_keypoints(m_handle, &total_size);
    warnOverflow();
}

// A stage that hit its capacity (sift_hip_capacities) clamps and sets a bit:
// results may then be missing keypoints the reference would keep.  Reported
// on stderr once per detector and flag set (maxKeypoints raises the limit).
void Detector::warnOverflow() {
    int flags = 0;
    if (!m_handle || sift_hip_overflow_flags(m_handle, &flags) != SIFT_HIP_OK || !flags) return;
    if ((flags & ~m_overflowWarned) == 0) return;
    m_overflowWarned |= flags;
    std::fprintf(stderr,
                 "sift_cuda::Detector: capacity overflow (flags 0x%x: 1 candidates, 2 refined, 4 oriented, "
                 "8 results); keypoints were dropped -- raise CudaSiftConfig::maxKeypoints\n",
                 flags);
}

void Detector::detectAndCompute(const Imagef& image) {
    if (!m_initialized && !gpuWarmUpAndAllocate()) return;
    if (!image.m_data || image.cols() != m_config.col_width || image.rows() != m_config.row_width) {
        std::fprintf(stderr, "detectAndCompute: image is %dx%d, detector configured for %dx%d\n", image.cols(),
                     image.rows(), m_config.col_width, m_config.row_width);
        std::exit(EXIT_FAILURE);
    }
    check(sift_hip_detect(m_handle, image.m_data->data(), sizeof(float) * (size_t)image.cols()), "detectAndCompute");
    refreshViews();
}

namespace {

template <class T>
void check_shape(const Image<T>& image, const CudaSiftConfig& c, const char* what) {
    if (!image.m_data || image.cols() != c.col_width || image.rows() != c.row_width) {
        std::fprintf(stderr, "%s: image is %dx%d, detector configured for %dx%d\n", what, image.cols(), image.rows(),
                     c.col_width, c.row_width);
        std::exit(EXIT_FAILURE);
    }
}

}  // namespace

void Detector::detectAndCompute(const Image8U& image) {
    if (!m_initialized && !gpuWarmUpAndAllocate()) return;
    check_shape(image, m_config, "detectAndCompute");
    check(sift_hip_detect_u8(m_handle, image.m_data->data(), (size_t)image.cols()), "detectAndCompute");
    refreshViews();
}

long long Detector::submit(const Imagef& image) {
    if (!m_initialized && !gpuWarmUpAndAllocate()) return -1;
    check_shape(image, m_config, "submit");
    long long t = -1;
    check(sift_hip_submit(m_handle, image.m_data->data(), sizeof(float) * (size_t)image.cols(), SIFT_HIP_F32, &t),
          "submit");
    return t;
}

long long Detector::submit(const Image8U& image) {
    if (!m_initialized && !gpuWarmUpAndAllocate()) return -1;
    check_shape(image, m_config, "submit");
    long long t = -1;
    check(sift_hip_submit(m_handle, image.m_data->data(), (size_t)image.cols(), SIFT_HIP_U8, &t), "submit");
    return t;
}

long long Detector::submitDevice(const void* dev, size_t stride, bool u8, void* stream) {
    if (!m_initialized && !gpuWarmUpAndAllocate()) return -1;
    long long t = -1;
    check(sift_hip_submit_device(m_handle, dev, stride, u8 ? SIFT_HIP_U8 : SIFT_HIP_F32, stream, &t), "submitDevice");
    return t;
}

void Detector::setLanes(int lanes) {
    if (m_handle) check(sift_hip_set_lanes(m_handle, lanes), "setLanes");
}

void Detector::setAutoMicroBatch(int frames) {
    if (m_handle) check(sift_hip_set_auto_micro_batch(m_handle, frames), "setAutoMicroBatch");
}
void Detector::setMicroBatch(int frames) {
    if (m_handle) check(sift_hip_set_micro_batch(m_handle, frames), "setMicroBatch");
}

void Detector::wait(long long ticket) {
    check(sift_hip_wait(m_handle, ticket), "wait");
    refreshViews();
}

void Detector::detectAndComputeDevice(const float* dev, size_t stride, void* stream) {
    if (!m_initialized && !gpuWarmUpAndAllocate()) return;
    check(sift_hip_detect_device(m_handle, dev, stride, stream), "detectAndComputeDevice");
    check(sift_hip_sync(m_handle), "detectAndComputeDevice sync");
    refreshViews();
}

void Detector::setDataGen(const std::string& path) {
    m_debug_path = path;
    if (m_handle) check(sift_hip_set_datagen(m_handle, path.c_str()), "setDataGen");
}

void Detector::setExactDescriptors(bool exact) {
    if (m_handle)
        check(sift_hip_set_descriptor_mode(m_handle, exact ? SIFT_HIP_DESC_EXACT : SIFT_HIP_DESC_FAST),
              "setExactDescriptors");
}

void Detector::replayStage(const std::string& dump_dir, const std::string& stage, const std::string& out_dir) {
    if (!m_initialized && !gpuWarmUpAndAllocate()) return;
    check(sift_hip_replay_stage(m_handle, dump_dir.c_str(), stage.c_str(), out_dir.c_str()), "replayStage");
    refreshViews();
}

void Detector::copyToHost(bool descriptor) {
    if (!m_initialized) return;
    final_kpts.resize((size_t)total_size);
    final_features.resize((size_t)total_size);
    if (descriptor) descriptors.resize((size_t)total_size * 128);
    check(sift_hip_copy_to_host(m_handle, reinterpret_cast<float*>(final_kpts.data()),
                                reinterpret_cast<float*>(final_features.data()),
                                descriptor ? reinterpret_cast<uint16_t*>(descriptors.data()) : nullptr, total_size),
          "copyToHost");
}

Detector::HostResults Detector::hostResults(bool descriptor) {
    HostResults r;
    if (!m_initialized) return r;
    const float *k3 = nullptr, *f4 = nullptr;
    const uint16_t* desc = nullptr;
    check(sift_hip_results_host(m_handle, &k3, &f4, descriptor ? &desc : nullptr, &r.count), "hostResults");
    r.kpts = reinterpret_cast<const Float3*>(k3);
    r.features = reinterpret_cast<const Float4*>(f4);
    r.descriptors = reinterpret_cast<const Half*>(desc);
    return r;
}

namespace {

struct MatcherDeleter {
    void operator()(sift_hip_matcher* m) const { sift_hip_matcher_destroy(m); }
};

}  // namespace

std::vector<int> matchBruteForce(const DeviceBuffer<Half>& des, int num_des, const DeviceBuffer<Half>& src,
                                 int num_src) {
    thread_local std::unique_ptr<sift_hip_matcher, MatcherDeleter> matcher;
    thread_local int capQ = 0, capT = 0;
    std::vector<int> out((size_t)std::max(num_des, 0), -1);
    if (num_des <= 0) return out;
    if (!matcher || num_des > capQ || num_src > capT) {
        capQ = std::max(num_des, capQ);
        capT = std::max(std::max(num_src, 1), capT);
        sift_hip_matcher_t m = nullptr;
        check(sift_hip_matcher_create(-1, capQ, capT, 1, &m), "matchBruteForce");
        matcher.reset(m);
    }
    check(sift_hip_match_host(matcher.get(), reinterpret_cast<const uint16_t*>(des.data()), num_des,
                              reinterpret_cast<const uint16_t*>(src.data()), num_src, 0.8f, 1, out.data()),
          "matchBruteForce");
    return out;
}

}  // namespace sift_cuda
