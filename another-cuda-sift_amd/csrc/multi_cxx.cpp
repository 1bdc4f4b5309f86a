// sift_cuda::MultiDetector / crossMatch (include/sift_cuda/MultiDetector.hh):
// host threads, one Detector per device, and the C5 exchange over the C ABI
// (include/sift_hip.h).  Plain C++ (g++): no HIP headers, no device code.
#include "sift_cuda/MultiDetector.hh"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <exception>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>

#include "sift_cuda/Detector.hh"
#include "sift_hip.h"

namespace sift_cuda {

namespace {

void check(int rc, const char* what) {
    if (rc != SIFT_HIP_OK) throw std::runtime_error(std::string(what) + ": " + sift_hip_last_error());
}

class HipFrameWorker : public FrameWorker {
public:
    HipFrameWorker(const CudaSiftConfig& config, int device, bool exact) : m_device(device), m_det(config, device) {
        if (exact) m_det.setExactDescriptors(true);  // before the warm-up (captured graphs)
        m_det.gpuWarmUpAndAllocate();
    }
    int device() const override { return m_device; }
    void detect(int frame, const Image8U& image, bool descriptors, FrameResult& out) override {
        m_det.detectAndCompute(image);
        m_det.copyToHost(descriptors);
        out.frame = frame;
        out.device = m_device;
        out.kpts = m_det.final_kpts;
        out.features = m_det.final_features;
        if (descriptors) out.descriptors = m_det.descriptors;
    }

private:
    int m_device;
    Detector m_det;
};

}  // namespace

std::vector<int> shardFrames(int frames, int w, int n) {
    std::vector<int> out;
    for (int i = w; i < frames; i += n) out.push_back(i);
    return out;
}

MultiDetector::MultiDetector(const CudaSiftConfig& config, const std::vector<int>& devices, bool exactDescriptors) {
    for (int d : devices) m_workers.emplace_back(new HipFrameWorker(config, d, exactDescriptors));
}

MultiDetector::MultiDetector(std::vector<std::unique_ptr<FrameWorker>> workers) : m_workers(std::move(workers)) {}

MultiDetector::~MultiDetector() = default;

void MultiDetector::detectAll(const std::vector<Image8U>& frames, bool descriptors,
                              const std::function<void(FrameResult&&)>& sink) {
    const int n = workers();
    std::mutex mu;
    std::vector<std::exception_ptr> errors((size_t)n);
    std::vector<std::thread> threads;
    for (int w = 0; w < n; w++) {
        threads.emplace_back([&, w] {
            try {
                for (int f : shardFrames((int)frames.size(), w, n)) {
                    FrameResult r;
                    m_workers[(size_t)w]->detect(f, frames[(size_t)f], descriptors, r);
                    r.worker = w;
                    std::lock_guard<std::mutex> lock(mu);
                    sink(std::move(r));
                }
            } catch (...) {
                errors[(size_t)w] = std::current_exception();
            }
        });
    }
    for (auto& t : threads) t.join();
    for (auto& e : errors)
        if (e) std::rethrow_exception(e);
}

namespace {

// Receive buffers (one per rank, on that rank's device), grown on demand.
struct GatherBuffers {
    std::vector<int> devices;
    std::vector<void*> recv;
    size_t cap = 0;
    void ensure(size_t bytes) {
        if (bytes <= cap) return;
        for (size_t k = 0; k < recv.size(); k++) {
            check(sift_hip_set_device(devices[k]), "sift_hip_set_device");
            if (recv[k]) sift_hip_free(recv[k]);
            check(sift_hip_malloc(&recv[k], bytes), "sift_hip_malloc");
        }
        cap = bytes;
    }
    ~GatherBuffers() {
        for (size_t k = 0; k < recv.size(); k++)
            if (recv[k]) {
                sift_hip_set_device(devices[k]);
                sift_hip_free(recv[k]);
            }
    }
};

}  // namespace

AllGatherFn copyAllGather(const std::vector<int>& devices) {
    auto buf = std::make_shared<GatherBuffers>();
    buf->devices = devices;
    buf->recv.assign(devices.size(), nullptr);
    return [buf](const std::vector<const void*>& send, size_t bytes) {
        const size_t n = send.size();
        if (n != buf->devices.size()) throw std::invalid_argument("copyAllGather: one block per rank");
        buf->ensure(n * bytes);
        for (size_t k = 0; k < n; k++) {
            check(sift_hip_set_device(buf->devices[k]), "sift_hip_set_device");
            for (size_t r = 0; r < n; r++)
                check(sift_hip_memcpy_d2d((char*)buf->recv[k] + r * bytes, send[r], bytes, nullptr), "all-gather copy");
        }
        return std::vector<const void*>(buf->recv.begin(), buf->recv.end());
    };
}

AllGatherFn rcclAllGather(const std::vector<int>& devices) {
    struct State : GatherBuffers {
        sift_hip_comm_t comm = nullptr;
        ~State() {
            if (comm) sift_hip_comm_destroy(comm);
        }
    };
    auto st = std::make_shared<State>();
    st->devices = devices;
    st->recv.assign(devices.size(), nullptr);
    check(sift_hip_comm_create((int)devices.size(), devices.data(), &st->comm), "sift_hip_comm_create");
    return [st](const std::vector<const void*>& send, size_t bytes) {
        if (send.size() != st->devices.size()) throw std::invalid_argument("rcclAllGather: one block per rank");
        st->ensure(send.size() * bytes);
        check(sift_hip_comm_allgather(st->comm, send.data(), st->recv.data(), bytes, nullptr), "all-gather");
        return std::vector<const void*>(st->recv.begin(), st->recv.end());
    };
}

BatchMatchFn hipBatchMatch(const std::vector<int>& devices, int max_rows, float ratio) {
    struct State {
        std::vector<int> devices;
        std::vector<sift_hip_matcher_t> matchers;
        std::vector<void*> out;  // int32 match per (pair, query), on each rank's device
        int max_rows = 0;
        ~State() {
            for (size_t k = 0; k < matchers.size(); k++) {
                sift_hip_set_device(devices[k]);
                if (matchers[k]) sift_hip_matcher_destroy(matchers[k]);
                if (out[k]) sift_hip_free(out[k]);
            }
        }
    };
    auto st = std::make_shared<State>();
    st->devices = devices;
    st->matchers.assign(devices.size(), nullptr);
    st->out.assign(devices.size(), nullptr);
    st->max_rows = max_rows;
    return [st, ratio](int rank, const void* query, int nq, const std::vector<const void*>& trains,
                       const std::vector<int>& nts) {
        const int P = (int)trains.size();
        std::vector<std::vector<int>> res((size_t)P);
        if (P == 0) return res;
        const int dev = st->devices[(size_t)rank];
        check(sift_hip_set_device(dev), "sift_hip_set_device");
        if (!st->matchers[(size_t)rank]) {
            // One rank matches its set against the other ranks' sets: at most
            // devices - 1 pairs per launch (scratch sized for that, not for the
            // matcher's 64-pair maximum).
            const int maxPairs = std::max(1, std::min((int)st->devices.size() - 1, 64));
            check(sift_hip_matcher_create(dev, st->max_rows, st->max_rows, maxPairs, &st->matchers[(size_t)rank]),
                  "sift_hip_matcher_create");
            check(sift_hip_malloc(&st->out[(size_t)rank], sizeof(int) * (size_t)maxPairs * (size_t)st->max_rows),
                  "sift_hip_malloc");
        }
        if (P > std::max(1, (int)st->devices.size() - 1))
            throw std::invalid_argument("hipBatchMatch: more train sets than peer ranks");
        std::vector<const uint16_t*> q((size_t)P, (const uint16_t*)query), t((size_t)P);
        std::vector<int> nqs((size_t)P, nq);
        for (int p = 0; p < P; p++) t[(size_t)p] = (const uint16_t*)trains[(size_t)p];
        int* match = (int*)st->out[(size_t)rank];
        check(sift_hip_match_batched(st->matchers[(size_t)rank], P, q.data(), nqs.data(), t.data(), nts.data(), ratio,
                                     0, nullptr, nullptr, match, nullptr),
              "sift_hip_match_batched");
        std::vector<int> host((size_t)P * nq);
        check(sift_hip_memcpy_d2h(host.data(), match, sizeof(int) * host.size()), "match copy");
        for (int p = 0; p < P; p++) res[(size_t)p].assign(host.begin() + (size_t)p * nq, host.begin() + (size_t)(p + 1) * nq);
        return res;
    };
}

std::vector<std::vector<std::vector<int>>> crossMatch(const std::vector<const void*>& sets,
                                                      const std::vector<int>& counts, int rows,
                                                      const AllGatherFn& gather, const BatchMatchFn& match) {
    const size_t n = sets.size();
    if (counts.size() != n) throw std::invalid_argument("crossMatch: one count per set");
    const size_t bytes = (size_t)rows * 128 * sizeof(Half);
    const std::vector<const void*> all = gather(sets, bytes);  // all[k]: every set, on rank k's device
    std::vector<std::vector<std::vector<int>>> m(n, std::vector<std::vector<int>>(n));
    for (size_t k = 0; k < n; k++) {
        std::vector<const void*> trains;
        std::vector<int> nts;
        std::vector<size_t> peers;
        for (size_t j = 0; j < n; j++) {
            if (j == k) continue;
            trains.push_back((const char*)all[k] + j * bytes);
            nts.push_back(counts[j]);
            peers.push_back(j);
        }
        auto res = match((int)k, (const char*)all[k] + k * bytes, counts[k], trains, nts);
        for (size_t p = 0; p < peers.size(); p++) m[k][peers[p]] = std::move(res[p]);
    }
    return m;
}

}  // namespace sift_cuda
