// Per-call host costs of the pipelined drop-in loop (no Python): 8-bit
// 1920x1200 frames through sift_cuda::Detector::submit / wait / copyToHost
// with `depth` frames in flight on `lanes` compute lanes (setLanes), as
// bench.py's host_input.pipelined_u8 runs them.  Prints one JSON line:
// ms per frame, and the mean wall time of each call.
//   host_pipeline_bench [lanes] [depth] [frames] [desc 0|1|2] [dev 0|1]
// desc 2: no copyToHost at all; dev 1: the frames already in device memory
// (submitDevice) instead of host frames (submit).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <deque>
#include <vector>

#include "sift_cuda/Detector.hh"
#include "sift_hip.h"

int main(int argc, char** argv) {
    const int lanes = argc > 1 ? std::atoi(argv[1]) : 3, depth = argc > 2 ? std::atoi(argv[2]) : 3;
    const int frames = argc > 3 ? std::atoi(argv[3]) : 200;
    const int descMode = argc > 4 ? std::atoi(argv[4]) : 1;
    const bool desc = descMode == 1, copy = descMode != 2;
    const bool dev = argc > 5 && std::atoi(argv[5]) != 0;
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
    det.gpuWarmUpAndAllocate();
    std::vector<void*> dframes(4, nullptr);
    if (dev)
        for (int i = 0; i < 4; i++) {
            sift_hip_malloc(&dframes[i], (size_t)W * H);
            sift_hip_memcpy_h2d(dframes[i], imgs[i].m_data->data(), (size_t)W * H);
        }
    using clk = std::chrono::steady_clock;
    double tSub = 0, tWait = 0, tCopy = 0;
    auto run = [&](int n, bool timed) {
        std::deque<long long> q;
        auto drain = [&] {
            auto a = clk::now();
            det.wait(q.front());
            q.pop_front();
            auto b = clk::now();
            if (copy) det.copyToHost(desc);
            auto c = clk::now();
            if (timed) {
                tWait += std::chrono::duration<double, std::milli>(b - a).count();
                tCopy += std::chrono::duration<double, std::milli>(c - b).count();
            }
        };
        for (int s = 0; s < n; s++) {
            auto a = clk::now();
            q.push_back(dev ? det.submitDevice(dframes[s % 4], W, true) : det.submit(imgs[s % 4]));
            if (timed) tSub += std::chrono::duration<double, std::milli>(clk::now() - a).count();
            if ((int)q.size() == depth) drain();
        }
        while (!q.empty()) drain();
    };
    run(3 * depth + 4, false);  // lanes created, graphs warm, prefetch mode set
    const auto t0 = clk::now();
    run(frames, true);
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    std::printf("{\"dev\": %d, \"lanes\": %d, \"depth\": %d, \"desc\": %d, \"ms_per_frame\": %.4f, \"submit_ms\": %.4f, "
                "\"wait_ms\": %.4f, \"copy_ms\": %.4f, \"keypoints\": %d}\n",
                (int)dev, lanes, depth, descMode, ms / frames, tSub / frames, tWait / frames, tCopy / frames, det.total_size);
    return 0;
}
