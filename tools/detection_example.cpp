// Mirrors /root/reference/tool/detection_example.cc:16-52: build a Detector for
// one image and run detectAndCompute N times (profile it with rocprofv3).
// Input: a binary PGM (P5, 8-bit) via --pgm, else a synthetic frame.
//   detection_example [--pgm file.pgm] [--width W --height H] [--iters N] [--upscale]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>

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
    int W = 1920, H = 1200, iters = 10;
    bool upscale = false;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        if (a == "--pgm" && i + 1 < argc) pgm = argv[++i];
        else if (a == "--width" && i + 1 < argc) W = std::atoi(argv[++i]);
        else if (a == "--height" && i + 1 < argc) H = std::atoi(argv[++i]);
        else if (a == "--iters" && i + 1 < argc) iters = std::atoi(argv[++i]);
        else if (a == "--upscale") upscale = true;
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
    std::printf("r: %d, c: %d\n", config.row_width, config.col_width);
    sift_cuda::Detector detector(config);
    detector.gpuWarmUpAndAllocate();
    for (int i = 0; i < iters; i++) {
        auto t0 = std::chrono::steady_clock::now();
        detector.detectAndCompute(img);
        auto t1 = std::chrono::steady_clock::now();
        std::printf("iter %d: %d keypoints, %.3f ms (incl. H2D)\n", i, detector.total_size,
                    std::chrono::duration<double, std::milli>(t1 - t0).count());
    }
    return 0;
}
