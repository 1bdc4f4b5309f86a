// Drop-in for /root/reference/sift_cuda/interface/Detector.hh:24-96.
// Same class name, constructor, public methods and public result members;
// device members are non-owning DeviceBuffer views, host members std::vector.
// No HIP/CUDA header is included: everything goes through include/sift_hip.h.
#pragma once
#include <string>
#include <vector>

#include "sift_cuda/CudaSiftConfig.hh"
#include "sift_cuda/HostImage.hh"
#include "sift_cuda/Types.hh"

struct sift_hip_detector;

namespace sift_cuda {

class Detector {
public:
    explicit Detector(const CudaSiftConfig& config);
    // Extra: bound to an explicit device instead of the calling thread's
    // current one (one Detector per GPU, each driven by its own host thread:
    // sift_cuda/MultiDetector.hh).
    Detector(const CudaSiftConfig& config, int device);
    ~Detector();
    Detector(const Detector&) = delete;
    Detector& operator=(const Detector&) = delete;

    // Detector.cu:17-39: allocate, capture the pipeline graph, warm up.
    // Returns false when the image size is unset (as the reference does).
    bool gpuWarmUpAndAllocate();

    // Detector.cu:133-233: synchronous; results valid until the next call.
    void detectAndCompute(const Imagef& image);
    // Extra: 8-bit frame (Image8U, HostImage.hh:187); converted on the GPU,
    // results identical to the Imagef holding the same values.
    void detectAndCompute(const Image8U& image);
    // Extra: pipelined input (sift_hip_submit / sift_hip_wait).  submit()
    // stages and uploads the frame while earlier frames compute and returns a
    // ticket; wait(ticket) makes that frame's results (and its predecessor's
    // descriptors as prev_descriptor) current.  Frames in flight compute
    // concurrently on up to setLanes() compute lanes (default 2), at most two
    // per lane past the last waited one.
    long long submit(const Imagef& image);
    long long submit(const Image8U& image);
    // Extra: the same for a frame already in device memory (fp32 or 8-bit,
    // row stride in bytes), read after `hip_stream` reaches the call; the
    // buffer must stay unchanged until wait(ticket).
    long long submitDevice(const void* device_image, size_t row_stride_bytes, bool u8 = false,
                           void* hip_stream = nullptr);
    void wait(long long ticket);
    // Extra: compute lanes for frames in flight (sift_hip_set_lanes, 1..4);
    // before gpuWarmUpAndAllocate.  1 = every frame on one stream in order.
    void setLanes(int lanes);
    // Extra: submitDevice frames run in launch groups of `frames`
    // (sift_hip_set_micro_batch, 1..16); before gpuWarmUpAndAllocate.
    void setMicroBatch(int frames);
    // Extra: automatic launch groups of up to `frames` once every lane is
    // busy (sift_hip_set_auto_micro_batch; default 8, 0 = off); before
    // gpuWarmUpAndAllocate.
    void setAutoMicroBatch(int frames);
    // Extra: image already in device memory (fp32, row stride in bytes).
    void detectAndComputeDevice(const float* device_image, size_t row_stride_bytes, void* hip_stream = nullptr);

    // Detector.cu:606-634: copies total_size results (+ descriptors) to host.
    void copyToHost(bool descriptor);
    // Extra: the same rows without the copy into final_kpts / final_features /
    // descriptors -- views of the detector's pinned host results of the
    // current frame (sift_hip_results_host), valid while that frame is the
    // current or the previous one.
    struct HostResults {
        const Float3* kpts = nullptr;
        const Float4* features = nullptr;
        const Half* descriptors = nullptr;  // 128 per keypoint; null unless requested
        int count = 0;
    };
    HostResults hostResults(bool descriptor);

    // Detector.hh:48-51 debug snapshot switch: every following detectAndCompute
    // writes its stage dumps into `path` (sift_hip_set_datagen: meta.json,
    // input, every Gaussian plane, candidates, keypoints, descriptors);
    // tests/stage_check.py replays them.  An empty path switches it off.
    void setDataGen(const std::string& path);
    // Extra: OpenCV's sequential float descriptor histogram (bit-identical
    // descriptors; sift_hip_set_descriptor_mode(SIFT_HIP_DESC_EXACT)).  Call
    // before gpuWarmUpAndAllocate; the default is the fixed-point histogram.
    void setExactDescriptors(bool exact);
    // tool/perf.cu:43-100 (HostInterface.hh:11-69 run<Stage>): one stage --
    // "pyramid", "extrema", "refine", "orientation", "order", "descriptor" --
    // alone on a setDataGen dump's recorded input; its outputs go to out_dir
    // in the dump's formats (sift_hip_replay_stage).  Discards the current results.
    void replayStage(const std::string& dump_dir, const std::string& stage, const std::string& out_dir);

    int numOctaves() const { return m_nOctaves; }
    sift_hip_detector* handle() const { return m_handle; }

    // Results (Detector.hh:53-62).
    DeviceBuffer<Float3> device_kpts;      // {x, y, layer}
    DeviceBuffer<Float4> device_features;  // {octave (packed, as float), size, response, angle}
    DeviceBuffer<Half> device_descriptor;  // 128 per keypoint, values 0..255
    DeviceBuffer<Half> prev_descriptor;    // previous frame's descriptors
    std::vector<Float3> final_kpts{};
    std::vector<Float4> final_features{};
    std::vector<Half> descriptors{};
    int max_kpts = 5000;
    int total_size{0};

private:
    void refreshViews();
    void warnOverflow();
    CudaSiftConfig m_config{};
    sift_hip_detector* m_handle{nullptr};
    bool m_initialized{false};
    int m_nOctaves{0};
    int m_overflowWarned{0};  // overflow flags already reported on stderr
    std::string m_debug_path;
};

// Match.cuh:9-14: for each of the num_des rows of `des`, the index of its
// nearest row of `src` if it passes Lowe's test on squared distances
// (d1^2 < 0.8 d2^2, the reference's Match.cu:172 convention), else -1.
std::vector<int> matchBruteForce(const DeviceBuffer<Half>& des, int num_des, const DeviceBuffer<Half>& src,
                                 int num_src);

}  // namespace sift_cuda
