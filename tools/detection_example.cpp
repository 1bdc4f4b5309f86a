// Mirrors /root/reference/tool/detection_example.cc:16-52: build a Detector for
// one image and run detectAndCompute N times (profile it with rocprofv3).
// Input: a binary PGM (P5, 8-bit) via --pgm, else a synthetic frame.
//   detection_example [--pgm file.pgm] [--width W --height H] [--iters N] [--upscale]
//                     [--octaves N] [--device]
// --device: the frame is uploaded once and detectAndComputeDevice (synchronous,
// HBM-resident input) runs N times; prints the median latency as one JSON
// line -- the drop-in's single-frame latency as a C++ caller sees it.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "sift_cuda/Detector.hh"
#include "sift_hip.h"

static bool readPgm(const std::string& path, Imagef& img) {
    std::ifstream f(path, std::ios::binary);
    std::string magic;
    int w, h, maxv;
    if (!(f >> magic >> w >> h >> maxv) || magic != "P5" || maxv > 255) return false;
    f.get();
    std::vector<unsigned char> buf((size_t)w * h);
    if (!f.read(reinterpret_cast<char*>(buf.data()), (std::streamsize)buf.size())) return false;
    img = Imagef(h, w);
    for (size_t i = 0; i < buf.size(); i++) (*img.m_data)[i] = buf[i];
    return true;
}

int main(int argc, char** argv) {
    std::string pgm;
    int W = 1920, H = 1200, iters = 10, octaves = 0;
    bool upscale = false, device = false;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "--pgm" && i + 1 < argc) pgm = argv[++i];
        else if (a == "--width" && i + 1 < argc) W = std::atoi(argv[++i]);
        else if (a == "--height" && i + 1 < argc) H = std::atoi(argv[++i]);
        else if (a == "--iters" && i + 1 < argc) iters = std::atoi(argv[++i]);
        else if (a == "--upscale") upscale = true;
        else if (a == "--octaves" && i + 1 < argc) octaves = std::atoi(argv[++i]);
        else if (a == "--device") device = true;
    }
    Imagef img;
    if (!pgm.empty()) {
        if (!readPgm(pgm, img)) {
            std::printf("Image DNE\n");
            return 1;
        }
    } else {
        img = Imagef(H, W);
        sift_synth_frame(0, W, H, img.m_data->data());
    }
    CudaSiftConfig config;
    config.upscale = upscale;
    config.col_width = img.cols();
    config.row_width = img.rows();
    config.numOctaves = octaves;
    std::printf("r: %d, c: %d\n", config.row_width, config.col_width);
    sift_cuda::Detector detector(config);
    detector.gpuWarmUpAndAllocate();
    if (device) {
        const size_t bytes = sizeof(float) * img.m_data->size();
        void* dev = nullptr;
        if (sift_hip_malloc(&dev, bytes) != SIFT_HIP_OK) return 1;
        sift_hip_memcpy_h2d(dev, img.m_data->data(), bytes);
        const size_t stride = sizeof(float) * (size_t)img.cols();
        for (int i = 0; i < 10; i++) detector.detectAndComputeDevice(static_cast<const float*>(dev), stride);
        std::vector<double> ms;
        for (int i = 0; i < iters; i++) {
            auto t0 = std::chrono::steady_clock::now();
            detector.detectAndComputeDevice(static_cast<const float*>(dev), stride);
            ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(ms.begin(), ms.end());
        std::printf("{\"width\": %d, \"height\": %d, \"octaves\": %d, \"keypoints\": %d, \"iters\": %d, "
                    "\"sync_ms_median\": %.4f, \"sync_ms_min\": %.4f}\n",
                    config.col_width, config.row_width, detector.numOctaves(), detector.total_size, iters,
                    ms[ms.size() / 2], ms[0]);
        sift_hip_free(dev);
        return 0;
    }
    for (int i = 0; i < iters; i++) {
        auto t0 = std::chrono::steady_clock::now();
        detector.detectAndCompute(img);
        auto t1 = std::chrono::steady_clock::now();
        std::printf("iter %d: %d keypoints, %.3f ms (incl. H2D)\n", i, detector.total_size,
                    std::chrono::duration<double, std::milli>(t1 - t0).count());
    }
    return 0;
}
