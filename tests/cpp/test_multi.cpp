// CPU test of the C++ multi-GPU orchestration (include/sift_cuda/MultiDetector.hh)
// with injected fakes: no device is touched.  Checks the C4 sharding (frame i
// on worker i % n, each worker on its own thread, every frame once, worker
// exceptions propagated) and the C5 exchange wiring (every rank sees every
// set, rank k matches its set against each j != k with set j's count).
#include <atomic>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <stdexcept>
#include <thread>

#include "sift_cuda/MultiDetector.hh"

using namespace sift_cuda;

#define CHECK(c)                                                          \
    do {                                                                  \
        if (!(c)) {                                                       \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s\n", __FILE__, __LINE__, #c); \
            return 1;                                                     \
        }                                                                 \
    } while (0)

struct FakeWorker : FrameWorker {
    int dev;
    std::set<std::thread::id>* threads;
    std::mutex* mu;
    int failAt;
    FakeWorker(int d, std::set<std::thread::id>* t, std::mutex* m, int f = -1) : dev(d), threads(t), mu(m), failAt(f) {}
    int device() const override { return dev; }
    void detect(int frame, const Image8U& image, bool descriptors, FrameResult& out) override {
        if (frame == failAt) throw std::runtime_error("worker failure");
        {
            std::lock_guard<std::mutex> l(*mu);
            threads->insert(std::this_thread::get_id());
        }
        out.frame = frame;
        out.device = dev;
        out.kpts.resize((size_t)image.at(0, 0));  // "keypoints" = first pixel value
        if (descriptors) out.descriptors.resize(out.kpts.size() * 128);
    }
};

int main() {
    // --- C4 sharding -------------------------------------------------------
    const int n = 3, frames = 11;
    std::set<std::thread::id> threads;
    std::mutex mu;
    std::vector<std::unique_ptr<FrameWorker>> ws;
    for (int w = 0; w < n; w++) ws.emplace_back(new FakeWorker(10 + w, &threads, &mu));
    MultiDetector md(std::move(ws));
    CHECK(md.workers() == n);
    std::vector<Image8U> imgs;
    for (int f = 0; f < frames; f++) {
        Image8U im(2, 2);
        im.at(0, 0) = (uint8_t)(f + 1);
        imgs.push_back(im);
    }
    std::map<int, FrameResult> got;
    md.detectAll(imgs, true, [&](FrameResult&& r) { got[r.frame] = std::move(r); });
    CHECK((int)got.size() == frames);
    for (int f = 0; f < frames; f++) {
        CHECK(got[f].worker == f % n);
        CHECK(got[f].device == 10 + f % n);
        CHECK((int)got[f].kpts.size() == f + 1 && got[f].descriptors.size() == (size_t)(f + 1) * 128);
    }
    CHECK((int)threads.size() == n);  // one host thread per worker
    CHECK(shardFrames(256, 3, 8).size() == 32 && shardFrames(256, 3, 8)[1] == 11);

    std::vector<std::unique_ptr<FrameWorker>> bad;
    bad.emplace_back(new FakeWorker(0, &threads, &mu));
    bad.emplace_back(new FakeWorker(1, &threads, &mu, 5));
    MultiDetector mb(std::move(bad));
    bool threw = false;
    try {
        mb.detectAll(imgs, false, [](FrameResult&&) {});
    } catch (const std::runtime_error&) {
        threw = true;
    }
    CHECK(threw);

    // --- C5 exchange wiring --------------------------------------------------
    const int R = 4, rows = 5;
    const size_t bytes = (size_t)rows * 128 * sizeof(uint16_t);
    std::vector<std::vector<uint16_t>> sets((size_t)R, std::vector<uint16_t>((size_t)rows * 128));
    for (int k = 0; k < R; k++)
        for (size_t e = 0; e < sets[(size_t)k].size(); e++) sets[(size_t)k][e] = (uint16_t)(1000 * k + e);
    std::vector<int> counts = {5, 3, 4, 1};
    std::vector<std::vector<uint16_t>> recv((size_t)R);
    int gathers = 0;
    AllGatherFn gather = [&](const std::vector<const void*>& send, size_t b) {
        gathers++;
        std::vector<const void*> out;
        for (int k = 0; k < R; k++) {
            recv[(size_t)k].assign((size_t)R * b / 2, 0);
            for (int r = 0; r < R; r++) std::memcpy((char*)recv[(size_t)k].data() + r * b, send[(size_t)r], b);
            out.push_back(recv[(size_t)k].data());
        }
        return out;
    };
    std::atomic<int> calls{0};
    BatchMatchFn match = [&](int rank, const void* q, int nq, const std::vector<const void*>& trains,
                             const std::vector<int>& nts) {
        calls++;
        std::vector<std::vector<int>> res;
        // the query block is rank's own set inside rank's gathered buffer
        const uint16_t* qq = (const uint16_t*)q;
        if (qq[0] != (uint16_t)(1000 * rank) || nq != counts[(size_t)rank]) throw std::runtime_error("bad query");
        for (size_t p = 0; p < trains.size(); p++) {
            const uint16_t* t = (const uint16_t*)trains[p];
            const int j = t[0] / 1000;  // which set this train block is
            if ((const char*)t < (const char*)recv[(size_t)rank].data() ||
                (const char*)t >= (const char*)recv[(size_t)rank].data() + R * bytes)
                throw std::runtime_error("train block not in the rank's own gathered buffer");
            if (nts[p] != counts[(size_t)j]) throw std::runtime_error("bad train count");
            res.push_back(std::vector<int>((size_t)nq, 100 * rank + j));
        }
        return res;
    };
    std::vector<const void*> sp;
    for (auto& s : sets) sp.push_back(s.data());
    auto m = crossMatch(sp, counts, rows, gather, match);
    CHECK(gathers == 1 && calls == R);
    for (int k = 0; k < R; k++)
        for (int j = 0; j < R; j++) {
            if (j == k) {
                CHECK(m[(size_t)k][(size_t)j].empty());
                continue;
            }
            CHECK((int)m[(size_t)k][(size_t)j].size() == counts[(size_t)k]);
            CHECK(m[(size_t)k][(size_t)j][0] == 100 * k + j);
        }
    std::printf("multi orchestration ok\n");
    return 0;
}
