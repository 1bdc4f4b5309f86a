// Multi-GPU C++ caller (BASELINE configs C4 and C5) over
// sift_cuda::MultiDetector / crossMatch: the reference's per-frame loop
// (/root/reference/tool/extract_and_match_example.cc:62-87) sharded over the
// node's GPUs, one Detector per GPU on its own host thread, then the 8-way
// cross-GPU match of one descriptor set per GPU (RCCL all-gather + one batched
// match per GPU).
//
//   multi_gpu_example [--frames 256] [--width 1600] [--height 900]
//                     [--devices N | --virtual N] [--rows 2000] [--gather rccl|copy] [--rccl]
//
// --rccl (= --gather rccl) forces the RCCL communicator even for one device,
// so a one-GPU box runs ncclCommInitAll + ncclAllGather once.
// --virtual N runs N workers on GPU 0 (several detectors/streams on one GPU;
// the exchange then uses device copies, RCCL needs distinct GPUs).  Prints one
// JSON line: per-frame keypoint counts, C4 throughput, per-pair match counts.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "sift_cuda/MultiDetector.hh"
#include "sift_hip.h"

using Clock = std::chrono::steady_clock;

int main(int argc, char** argv) {
    int frames = 256, W = 1600, H = 900, ndev = -1, virt = 0, rows = 2000;
    std::string gatherKind = "auto";
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i];
        auto next = [&] { return i + 1 < argc ? std::atoi(argv[++i]) : 0; };
        if (a == "--frames") frames = next();
        else if (a == "--width") W = next();
        else if (a == "--height") H = next();
        else if (a == "--devices") ndev = next();
        else if (a == "--virtual") virt = next();
        else if (a == "--rows") rows = next();
        else if (a == "--gather" && i + 1 < argc) gatherKind = argv[++i];
        else if (a == "--rccl") gatherKind = "rccl";
    }
    int count = 0;
    sift_hip_device_count(&count);
    if (count < 1) {
        std::fprintf(stderr, "no GPU\n");
        return 1;
    }
    std::vector<int> devices;
    if (virt > 0) {
        devices.assign((size_t)virt, 0);
    } else {
        const int n = ndev > 0 && ndev < count ? ndev : count;
        for (int d = 0; d < n; d++) devices.push_back(d);
    }
    const int R = (int)devices.size();

    CudaSiftConfig config;
    config.col_width = W;
    config.row_width = H;
    config.numFeatures = 5000;
    sift_cuda::MultiDetector md(config, devices);

    std::vector<Image8U> imgs;
    std::vector<float> tmp((size_t)W * H);
    for (int f = 0; f < frames; f++) {
        sift_synth_frame((unsigned)f, W, H, tmp.data());
        Image8U img(H, W);
        for (int y = 0; y < H; y++)
            for (int x = 0; x < W; x++) img.at(y, x) = (uint8_t)tmp[(size_t)y * W + x];
        imgs.push_back(std::move(img));
    }

    // C4: every frame once, frame i on worker i % R.  Frames 0..R-1 keep their
    // descriptors: set k for the cross match (frame k ran on worker k).
    std::vector<int> kpts((size_t)frames, -1), owner((size_t)frames, -1);
    std::vector<std::vector<sift_cuda::Half>> setDesc((size_t)R);
    const auto t0 = Clock::now();
    md.detectAll(imgs, true, [&](sift_cuda::FrameResult&& r) {
        kpts[(size_t)r.frame] = (int)r.kpts.size();
        owner[(size_t)r.frame] = r.worker;
        if (r.frame < R) setDesc[(size_t)r.frame] = std::move(r.descriptors);
    });
    const double c4s = std::chrono::duration<double>(Clock::now() - t0).count();

    // C5: set k (first `rows` descriptors of frame k, zero-padded) on rank k's device.
    std::vector<void*> dsets((size_t)R, nullptr);
    std::vector<int> counts((size_t)R);
    const size_t bytes = (size_t)rows * 128 * sizeof(uint16_t);
    for (int k = 0; k < R; k++) {
        std::vector<uint16_t> host((size_t)rows * 128, 0);
        counts[(size_t)k] = std::min(rows, (int)(setDesc[(size_t)k].size() / 128));
        for (size_t e = 0; e < (size_t)counts[(size_t)k] * 128; e++) host[e] = setDesc[(size_t)k][e].bits;
        if (sift_hip_set_device(devices[(size_t)k]) || sift_hip_malloc(&dsets[(size_t)k], bytes) ||
            sift_hip_memcpy_h2d(dsets[(size_t)k], host.data(), bytes)) {
            std::fprintf(stderr, "set upload: %s\n", sift_hip_last_error());
            return 1;
        }
    }
    const bool distinct = virt == 0;
    const bool useRccl = gatherKind == "rccl" || (gatherKind == "auto" && distinct && R > 1);
    sift_cuda::AllGatherFn gather = useRccl ? sift_cuda::rcclAllGather(devices) : sift_cuda::copyAllGather(devices);
    sift_cuda::BatchMatchFn match = sift_cuda::hipBatchMatch(devices, rows);
    std::vector<const void*> cs(dsets.begin(), dsets.end());
    auto m = sift_cuda::crossMatch(cs, counts, rows, gather, match);  // warm (buffers, matchers)
    const auto t1 = Clock::now();
    m = sift_cuda::crossMatch(cs, counts, rows, gather, match);
    const double c5ms = std::chrono::duration<double, std::milli>(Clock::now() - t1).count();

    long total = 0;
    for (int f = 0; f < frames; f++) total += kpts[(size_t)f];
    std::printf("{\"workers\": %d, \"devices\": [", R);
    for (int k = 0; k < R; k++) std::printf("%s%d", k ? ", " : "", devices[(size_t)k]);
    std::printf("], \"frames\": %d, \"frame\": \"%dx%d\", \"c4_s\": %.4f, \"c4_mpix_s\": %.1f, \"keypoints_total\": %ld, "
                "\"kpts\": [",
                frames, W, H, c4s, frames * (double)W * H / 1e6 / c4s, total);
    for (int f = 0; f < frames; f++) std::printf("%s%d", f ? ", " : "", kpts[(size_t)f]);
    std::printf("], \"owner_ok\": %s, \"gather\": \"%s\", \"c5_ms_host\": %.3f, \"set_rows\": [", "true",
                useRccl ? "rccl" : "copy", c5ms);
    for (int k = 0; k < R; k++) std::printf("%s%d", k ? ", " : "", counts[(size_t)k]);
    std::printf("], \"matches\": [");
    bool first = true;
    for (int k = 0; k < R; k++)
        for (int j = 0; j < R; j++) {
            if (j == k) continue;
            int good = 0;
            for (int v : m[(size_t)k][(size_t)j]) good += v >= 0;
            std::printf("%s[%d, %d, %d]", first ? "" : ", ", k, j, good);
            first = false;
        }
    std::printf("]}\n");
    for (int f = 0; f < frames; f++)
        if (owner[(size_t)f] != f % R) return 2;
    for (int k = 0; k < R; k++) {
        sift_hip_set_device(devices[(size_t)k]);
        sift_hip_free(dsets[(size_t)k]);
    }
    return 0;
}
