// Multi-GPU surface for C++ callers, an extension of the
// reference's per-frame loop (/root/reference/tool/extract_and_match_example.cc
// :62-87) -- the reference binds one Detector to the calling thread's current
// device (/root/reference/sift_cuda/interface/Detector.hh:26-29) and has no
// multi-GPU path:
//
//  * MultiDetector: frame i runs on worker i % workers(), each worker a
//    sift_cuda::Detector bound to its device and driven by its own host thread
//    (C4: 256 frames over the node's GPUs; no data-path collective).
//  * crossMatch: the 8-way match (C5) -- every device's descriptor set is
//    all-gathered (RCCL over xGMI by default) and each device matches its own
//    set against every other one in one batched launch.
//
// The all-gather and the matcher are injectable (std::function), so the
// orchestration is testable without GPUs (tests/cpp/test_multi.cpp).
// No HIP header is included: everything goes through include/sift_hip.h.
#pragma once
#include <functional>
#include <memory>
#include <vector>

#include "sift_cuda/CudaSiftConfig.hh"
#include "sift_cuda/HostImage.hh"
#include "sift_cuda/Types.hh"

namespace sift_cuda {

struct FrameResult {
    int frame = -1, worker = -1, device = -1;
    std::vector<Float3> kpts;       // {x, y, layer}
    std::vector<Float4> features;   // {packed octave, size, response, angle}
    std::vector<Half> descriptors;  // 128 per keypoint (empty unless requested)
};

// One device's detector loop (the default: sift_cuda::Detector on that device).
class FrameWorker {
public:
    virtual ~FrameWorker() = default;
    virtual int device() const = 0;
    // Runs on this worker's own host thread only.
    virtual void detect(int frame, const Image8U& image, bool descriptors, FrameResult& out) = 0;
};

// Frames of worker `w` out of `n` for `frames` frames: w, w + n, ... (C4 sharding).
std::vector<int> shardFrames(int frames, int w, int n);

class MultiDetector {
public:
    // One sift_cuda::Detector per entry of `devices` (a device may repeat: several
    // detectors, i.e. HIP streams, on one GPU); exactDescriptors: every detector
    // in the exact descriptor mode (Detector::setExactDescriptors).
    MultiDetector(const CudaSiftConfig& config, const std::vector<int>& devices, bool exactDescriptors = false);
    explicit MultiDetector(std::vector<std::unique_ptr<FrameWorker>> workers);
    ~MultiDetector();
    MultiDetector(const MultiDetector&) = delete;
    MultiDetector& operator=(const MultiDetector&) = delete;

    int workers() const { return (int)m_workers.size(); }
    FrameWorker& worker(int w) { return *m_workers[(size_t)w]; }

    // Every frame exactly once, frame i on worker i % workers(), each worker on
    // its own host thread; `sink` receives each result (calls serialised by a
    // mutex, in completion order).  Exceptions of a worker are rethrown here.
    void detectAll(const std::vector<Image8U>& frames, bool descriptors,
                   const std::function<void(FrameResult&&)>& sink);

private:
    std::vector<std::unique_ptr<FrameWorker>> m_workers;
};

// All-gather of equal-size byte blocks, rank k's block send[k] on device
// devices[k]: returns, per rank, a buffer on that rank's device holding all
// blocks (rank r at offset r * bytes).  The buffers stay owned by the gather.
using AllGatherFn = std::function<std::vector<const void*>(const std::vector<const void*>& send, size_t bytes)>;

// Batched matcher of one rank: its query set against each of the train sets
// (device pointers on that rank's device), top-1 index per query if it passes
// Lowe's ratio test (ratio on distances), else -1; one launch for all pairs.
using BatchMatchFn = std::function<std::vector<std::vector<int>>(
    int rank, const void* query, int nq, const std::vector<const void*>& trains, const std::vector<int>& nts)>;

// RCCL all-gather over `devices` (distinct GPUs; ncclCommInitAll), buffers
// allocated on first use and reused.
AllGatherFn rcclAllGather(const std::vector<int>& devices);
// Device-to-device copies instead of RCCL (several ranks on one GPU, or no RCCL).
AllGatherFn copyAllGather(const std::vector<int>& devices);
// sift_hip_match_batched on each rank's device (one matcher per rank).
BatchMatchFn hipBatchMatch(const std::vector<int>& devices, int max_rows, float ratio = 0.8f);

// C5.  Rank k holds set k: `rows` x 128 half on devices[k] (rows padded to a
// common size, counts[k] of them valid).  Returns m[k][j] = rank k's set
// matched against set j (empty for j == k).
std::vector<std::vector<std::vector<int>>> crossMatch(const std::vector<const void*>& sets,
                                                      const std::vector<int>& counts, int rows,
                                                      const AllGatherFn& gather, const BatchMatchFn& match);

}  // namespace sift_cuda
