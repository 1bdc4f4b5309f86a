// Mirrors /root/reference/tool/extract_and_match_example.cc:38-105: detect on
// consecutive frames and match each frame against the previous one through
// Detector::prev_descriptor + matchBruteForce.  Frames: a synthetic frame and
// copies shifted by (k*dx, k*dy) pixels, so good matches must agree with the shift.
// --pipelined: 8-bit frames through Detector::submit / wait, frame f+1 staged
// and uploaded while frame f computes; prints the same lines as the default
// synchronous Imagef loop.  --exact: Detector::setExactDescriptors(true)
// (OpenCV's descriptor bytes, sift_hip_set_descriptor_mode).  --micro-batch N
// (with --pipelined): Detector::setMicroBatch(N) on 2 lanes, 2N frames
// submitted ahead, so frames run in N-frame launch groups; same lines.
// --ahead N (with --pipelined): N frames submitted past the one waited for
// (default 1, or 2N with --micro-batch); past 2 per lane the default handle
// runs them in automatic launch groups (sift_hip_set_auto_micro_batch).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <string>

#include "sift_cuda/Detector.hh"
#include "sift_hip.h"

int main(int argc, char** argv) {
    int W = 752, H = 480, frames = 4, dx = 3, dy = 2;
    bool pipelined = false, exact = false;
    int micro = 1, ahead_arg = 0;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "--pipelined") pipelined = true;
        else if (a == "--exact") exact = true;
        else if (a == "--width" && i + 1 < argc) W = std::atoi(argv[++i]);
        else if (a == "--height" && i + 1 < argc) H = std::atoi(argv[++i]);
        else if (a == "--frames" && i + 1 < argc) frames = std::atoi(argv[++i]);
        else if (a == "--micro-batch" && i + 1 < argc) micro = std::atoi(argv[++i]);
        else if (a == "--ahead" && i + 1 < argc) ahead_arg = std::atoi(argv[++i]);
    }
    const int PW = W + frames * dx, PH = H + frames * dy;
    std::vector<float> big((size_t)PW * PH);
    sift_synth_frame(7, PW, PH, big.data());

    CudaSiftConfig config;
    config.upscale = false;
    config.numFeatures = 2000;
    config.col_width = W;
    config.row_width = H;
    sift_cuda::Detector detector(config);
    if (exact) detector.setExactDescriptors(true);  // before the warm-up: part of the captured graphs
    if (micro > 1) {
        detector.setLanes(2);
        detector.setMicroBatch(micro);
    }
    detector.gpuWarmUpAndAllocate();
    int prev_size = 0;
    std::vector<sift_cuda::Float3> prev_kpts;
    int failures = 0;
    auto frame = [&](int f, auto& img) {
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) img.at(y, x) = big[(size_t)(y + f * dy) * PW + x + f * dx];
    };
    std::vector<long long> ticket(frames, -1);
    auto submit = [&](int f) {
        Image8U img(H, W);
        frame(f, img);
        ticket[f] = detector.submit(img);
    };
    const int ahead = ahead_arg > 0 ? ahead_arg : (micro > 1 ? 2 * micro : 1);  // frames past the one waited for
    if (pipelined)
        for (int f = 0; f < ahead && f < frames; f++) submit(f);
    for (int f = 0; f < frames; f++) {
        if (pipelined) {
            if (f + ahead < frames) submit(f + ahead);
            detector.wait(ticket[f]);
        } else {
            Imagef img(H, W);
            frame(f, img);
            detector.detectAndCompute(img);
        }
        detector.copyToHost(false);
        const int curr_size = detector.total_size;
        if (f > 0) {
            const auto matches = sift_cuda::matchBruteForce(detector.prev_descriptor, prev_size,
                                                            detector.device_descriptor, curr_size);
            int good = 0, consistent = 0;
            for (int i = 0; i < prev_size; i++) {
                if (matches[i] < 0) continue;
                good++;
                const auto& a = prev_kpts[i];
                const auto& b = detector.final_kpts[matches[i]];
                if (std::fabs((a.x - dx) - b.x) < 1.5f && std::fabs((a.y - dy) - b.y) < 1.5f) consistent++;
            }
            std::printf("frame %d: %d kpts, %d matches, %d consistent with the (%d,%d) shift\n", f, curr_size, good,
                        consistent, -dx, -dy);
            if (good == 0 || consistent * 10 < good * 8) failures++;
        } else {
            std::printf("frame 0: %d kpts\n", curr_size);
        }
        prev_size = curr_size;
        prev_kpts = detector.final_kpts;
    }
    return failures ? 2 : 0;
}
