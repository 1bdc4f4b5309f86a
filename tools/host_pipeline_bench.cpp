// Per-call host costs of the pipelined drop-in loop (no Python): 8-bit
// 1920x1200 frames through sift_cuda::Detector::submit / wait / copyToHost
// with `depth` frames in flight on `lanes` compute lanes (setLanes), as
// bench.py's host_input.pipelined_u8 runs them.  Prints one JSON line:
// ms per frame, and the mean wall time of each call.
//   host_pipeline_bench [lanes] [depth] [frames] [desc 0|1|2|3] [dev 0..5] [micro-batch]
// desc 2: no copyToHost at all; desc 3: hostResults(true) (views of the
// detector's pinned results with descriptors, no copy); dev 1: the frames already in device memory
// (submitDevice) instead of host frames (submit); dev 2: the frames in pinned
// host memory, read by the frame's first kernel over PCIe (submitDevice with
// the mapped pointer: no staging copy on the calling thread); dev 3: the same
// pinned frames moved by DMA (hipMemcpyAsync on a copy stream into a device
// ring of `depth` + 1 slots) and submitted ordered after the copy.  Timing
// diagnostics: dev 4 = device frames ordered after a 4 KiB copy on the copy
// stream (the cross-stream wait alone); dev 5 = dev 3's DMA with the frame
// submitted unordered (the copy's concurrency alone; the frame reads the slot's
// previous contents, a valid older frame).
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "sift_cuda/Detector.hh"
#include "sift_hip.h"

int main(int argc, char** argv) {
    const int lanes = argc > 1 ? std::atoi(argv[1]) : 3, depth = argc > 2 ? std::atoi(argv[2]) : 3;
    const int frames = argc > 3 ? std::atoi(argv[3]) : 200;
    const int descMode = argc > 4 ? std::atoi(argv[4]) : 1;
    const bool desc = descMode == 1, copy = descMode == 0 || descMode == 1, view = descMode == 3;
    const int dev = argc > 5 ? std::atoi(argv[5]) : 0;
    const int mb = argc > 6 ? std::atoi(argv[6]) : 1;  // micro-batch (setMicroBatch)
    const int W = 1920, H = 1200;
    std::vector<Image8U> imgs;
    for (int i = 0; i < 4; i++) {
        std::vector<float> f((size_t)W * H);
        sift_synth_frame(i, W, H, f.data());
        Image8U im(H, W);
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) im.at(y, x) = (unsigned char)f[(size_t)y * W + x];
        imgs.push_back(im);
    }
    CudaSiftConfig cfg;
    cfg.col_width = W;
    cfg.row_width = H;
    cfg.numFeatures = 5000;
    cfg.numOctaves = 3;
    sift_cuda::Detector det(cfg);
    det.setLanes(lanes);
    if (mb > 1) det.setMicroBatch(mb);
    det.gpuWarmUpAndAllocate();
    std::vector<void*> dframes(4, nullptr), pinned(4, nullptr), ring(depth + 1, nullptr);
    hipStream_t cs = nullptr;
    if (dev == 1 || dev == 4)
        for (int i = 0; i < 4; i++) {
            sift_hip_malloc(&dframes[i], (size_t)W * H);
            sift_hip_memcpy_h2d(dframes[i], imgs[i].m_data->data(), (size_t)W * H);
        }
    if (dev == 2 || dev == 3 || dev == 5)
        for (int i = 0; i < 4; i++) {
            if (hipHostMalloc(&pinned[i], (size_t)W * H, hipHostMallocMapped) != hipSuccess) return 1;
            std::memcpy(pinned[i], imgs[i].m_data->data(), (size_t)W * H);
            if (dev == 2 && hipHostGetDevicePointer(&dframes[i], pinned[i], 0) != hipSuccess) return 1;
        }
    void *small = nullptr, *smallDev = nullptr;
    if (dev >= 3) {
        if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) return 1;
        for (auto& r : ring) {
            sift_hip_malloc(&r, (size_t)W * H);
            sift_hip_memcpy_h2d(r, imgs[0].m_data->data(), (size_t)W * H);
        }
        if (hipHostMalloc(&small, 4096, 0) != hipSuccess) return 1;
        sift_hip_malloc(&smallDev, 4096);
    }
    long long nsub = 0;
    auto submit = [&](int s) -> long long {
        if (dev == 0) return det.submit(imgs[s % 4]);
        if (dev == 4) {
            (void)hipMemcpyAsync(smallDev, small, 4096, hipMemcpyHostToDevice, cs);
            return det.submitDevice(dframes[s % 4], W, true, cs);
        }
        if (dev != 3 && dev != 5) return det.submitDevice(dframes[s % 4], W, true);
        // ring slot nsub % (depth + 1) was last read by a frame already waited
        // for (at most `depth` frames in flight)
        void* dst = ring[nsub++ % ring.size()];
        (void)hipMemcpyAsync(dst, pinned[s % 4], (size_t)W * H, hipMemcpyHostToDevice, cs);
        return det.submitDevice(dst, W, true, dev == 3 ? cs : nullptr);
    };
    using clk = std::chrono::steady_clock;
    double tSub = 0, tWait = 0, tCopy = 0;
    volatile float sink = 0;
    std::vector<double> subs;  // per-submit wall times of the timed run (ms)
    auto run = [&](int n, bool timed) {
        std::deque<long long> q;
        auto drain = [&] {
            auto a = clk::now();
            det.wait(q.front());
            q.pop_front();
            auto b = clk::now();
            if (copy) det.copyToHost(desc);
            if (view) {
                const auto r = det.hostResults(true);
                if (r.count > 0) sink += r.kpts[r.count - 1].x + (float)r.descriptors[128 * r.count - 1].bits;
            }
            auto c = clk::now();
            if (timed) {
                tWait += std::chrono::duration<double, std::milli>(b - a).count();
                tCopy += std::chrono::duration<double, std::milli>(c - b).count();
            }
        };
        for (int s = 0; s < n; s++) {
            auto a = clk::now();
            q.push_back(submit(s));
            if (timed) {
                const double ms = std::chrono::duration<double, std::milli>(clk::now() - a).count();
                tSub += ms;
                subs.push_back(ms);
            }
            if ((int)q.size() == depth) drain();
        }
        while (!q.empty()) drain();
    };
    run(3 * depth + 4, false);  // lanes created, graphs warm, prefetch mode set
    const auto t0 = clk::now();
    run(frames, true);
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    std::sort(subs.begin(), subs.end());
    auto pct = [&](double q) { return subs.empty() ? 0.0 : subs[std::min(subs.size() - 1, (size_t)(q * subs.size()))]; };
    std::printf("{\"dev\": %d, \"lanes\": %d, \"depth\": %d, \"micro_batch\": %d, \"desc\": %d, \"ms_per_frame\": %.4f, "
                "\"submit_ms\": %.4f, \"submit_p50_p90_max\": [%.4f, %.4f, %.4f], \"wait_ms\": %.4f, \"copy_ms\": %.4f, "
                "\"keypoints\": %d}\n",
                (int)dev, lanes, depth, mb, descMode, ms / frames, tSub / frames, pct(0.5), pct(0.9), pct(1.0),
                tWait / frames, tCopy / frames, det.total_size);
    return 0;
}
