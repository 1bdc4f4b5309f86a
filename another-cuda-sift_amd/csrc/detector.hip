// C ABI of libsift_hip.so: Detector state, buffer layout in HBM, the hipGraph
// of the whole fixed-shape pipeline, timing hooks and the matcher handle.
//
// Replaces /root/reference/sift_cuda/interface/Detector.cu (8 stages, 5 CUDA
// graphs with a host sync after each, a mid-pipeline count D2H, a 10-stream
// pool) with ONE graph per descriptor buffer: every data-dependent size lives
// in device counters, every launch has a fixed grid, and the only host sync
// per frame is the final 32-byte counter readback.
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <cmath>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sift_hip.h"
#include "sift_kernels.h"
#include "sift_match.h"

using namespace sift_amd;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                                    \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return fail(SIFT_HIP_ERR_RUNTIME, std::string(#expr) + ": " + hipGetErrorString(e_));      \
    } while (0)

// OpenCV getGaussianKernelBitExact (same arithmetic as oracle gaussianTaps).
Taps gaussian_taps(double sigma) {
    Taps t{};
    int n = (int)lrint(sigma * 4 * 2 + 1) | 1;
    if (n > kMaxTaps) n = kMaxTaps;
    const double scale2X = -0.125 / (sigma * sigma);
    const int n2 = (n - 1) / 2;
    std::vector<double> values(n2 + 1);
    double sum = 0;
    for (int i = 0, x = 1 - n; i < n2; i++, x += 2) {
        const double v = std::exp((double)(x * x) * scale2X);
        values[i] = v;
        sum += v;
    }
    sum *= 2.0;
    sum += 1.0;
    const double mul1 = 1.0 / sum;
    for (int i = 0; i < n2; i++) {
        const float v = (float)(values[i] * mul1);
        t.w[i] = v;
        t.w[n - 1 - i] = v;
    }
    t.w[n2] = (float)(1.0 * mul1);
    t.n = n;
    return t;
}

// Compile-time A/B and instrumentation switches of the kernels (tools/ab_*.sh
// builds pass them through EXTRA_HIPFLAGS, which the Makefile also records as
// SIFT_AB_FLAGS).  Any of them makes this a non-default build:
// sift_hip_version() lists them ("build=ab ..."), and bench.py and
// __graft_entry__.smoke() refuse such a library, so a measured or tested line
// always names the code it ran.
const char* build_flags() {
#ifdef SIFT_AB_FLAGS
    return " " SIFT_AB_FLAGS;
#else
    return "";
#endif
}

// Host copies of large frames split over a few persistent threads (the
// staging copy of a host frame: one thread moves ~10 GB/s, a 1920x1200 f32
// frame is 9.2 MB).  run(parts, fn) calls fn(0..parts-1), part 0 on the
// calling thread, and returns when every part is done.
class CopyPool {
public:
    explicit CopyPool(int workers) {
        for (int i = 0; i < workers; i++) th_.emplace_back([this, i] { loop(i + 1); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> g(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : th_) t.join();
    }
    int parts() const { return (int)th_.size() + 1; }
    void run(const std::function<void(int)>& fn) {
        {
            std::lock_guard<std::mutex> g(m_);
            fn_ = &fn;
            pending_ = (int)th_.size();
            gen_++;
        }
        cv_.notify_all();
        fn(0);
        std::unique_lock<std::mutex> g(m_);
        done_.wait(g, [this] { return pending_ == 0; });
        fn_ = nullptr;
    }

private:
    void loop(int part) {
        unsigned long long seen = 0;
        for (;;) {
            const std::function<void(int)>* fn;
            {
                std::unique_lock<std::mutex> g(m_);
                cv_.wait(g, [&] { return stop_ || gen_ != seen; });
                if (stop_) return;
                seen = gen_;
                fn = fn_;
            }
            (*fn)(part);
            std::lock_guard<std::mutex> g(m_);
            if (--pending_ == 0) done_.notify_one();
        }
    }
    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_, done_;
    const std::function<void(int)>* fn_ = nullptr;
    int pending_ = 0;
    unsigned long long gen_ = 0;
    bool stop_ = false;
};

// Pool threads besides the caller (a copy >= 1 MB runs in kCopyWorkers + 1
// parts).  (Measured alternative: 7 workers, the C++ host loop at 3 lanes
// 0.174-0.176 vs 0.170-0.171 ms/frame, profiles/round5/stage_modes.jsonl.)
constexpr int kCopyWorkers = 3;

// Row copy (dst pitch / src stride in bytes), split over the pool when large.
void copy_rows(CopyPool* pool, char* dst, size_t dpitch, const char* src, size_t sstride, size_t rowB, int rows) {
    auto part = [&](int lo, int hi) {
        if (dpitch == sstride && dpitch == rowB) {
            if (hi > lo) memcpy(dst + dpitch * lo, src + sstride * lo, rowB * (hi - lo));
        } else {
            for (int y = lo; y < hi; y++) memcpy(dst + dpitch * y, src + sstride * y, rowB);
        }
    };
    if (!pool || rowB * rows < (1u << 20)) {
        part(0, rows);
        return;
    }
    const int P = pool->parts();
    pool->run([&](int k) { part((int)((long)rows * k / P), (int)((long)rows * (k + 1) / P)); });
}

struct TimingRec {
    int name;
    hipEvent_t e0, e1;
    double bytes;
    int launches;
};

struct TimingAgg {
    std::string name;
    double ms = 0, bytes = 0;
    int launches = 0;
};

}  // namespace

void sift_amd::set_last_error(const std::string& msg) { g_err = msg; }

namespace {

// Matcher sidecars of the descriptor buffers the detector handles hand out
// (one per results slot and frame of every lane): exact buffer base -> its
// int8 codes and key biases (sift_kernels.h Sidecar).  sift_hip_match_* look
// the query and train pointers up and, when both are detector buffers, match
// their codes directly (k_match_direct) instead of converting the fp16 rows.
struct SidecarReg {
    const uint16_t* desc;
    Sidecar side;
    int cap;
    const void* owner;
};
std::mutex g_side_mu;
std::vector<SidecarReg> g_side;

void register_sidecar(const void* owner, const uint16_t* desc, Sidecar side, int cap) {
    std::lock_guard<std::mutex> g(g_side_mu);
    g_side.push_back(SidecarReg{desc, side, cap, owner});
}
void unregister_sidecars(const void* owner) {
    std::lock_guard<std::mutex> g(g_side_mu);
    g_side.erase(std::remove_if(g_side.begin(), g_side.end(), [&](const SidecarReg& r) { return r.owner == owner; }),
                 g_side.end());
}
bool find_sidecar(const uint16_t* desc, int n, Sidecar* out) {
    std::lock_guard<std::mutex> g(g_side_mu);
    for (const SidecarReg& r : g_side)
        if (r.desc == desc && n <= r.cap) {
            *out = r.side;
            return true;
        }
    return false;
}

}  // namespace

// Results slots per compute lane: frames f-1 .. f+2 of a lane never share one.
constexpr int kResultSlots = 4;
constexpr int kMaxLanes = 4;
constexpr int kFrameRing = 256;  // per-frame (lane, slot, arena) records: > 2 x kMaxLanes x kMaxMicroBatch (frames in flight) + the two readable

// A compute lane: one HIP stream, its B frame arenas (every per-frame buffer of
// the pipeline, sift_kernels.h Frames), the graphs captured on them and a ring
// of kResultSlots results slots.  A lane runs its frames in order; frames on
// different lanes run concurrently ("Frames in flight").
struct Lane {
    hipStream_t stream = nullptr;
    char* arena = nullptr;
    Counters* hCtr = nullptr;     // kResultSlots x B pinned host copies of the counters (written by k_descriptor)
    Counters* hCtrDev = nullptr;  // their device-side address
    hipEvent_t evFrame[kResultSlots] = {};  // recorded after each slot's last frame
    hipGraphExec_t exec[kResultSlots] = {};   // B frames per launch
    hipGraphExec_t exec1[kResultSlots] = {};  // one frame (B > 1 only; exec when B = 1)
    // The same graphs with the f32 head captured in (device input): the head
    // node is re-pointed at each frame's image (hipGraphExecKernelNodeSetParams),
    // so the frame is ONE graph launch -- a separate head launch left ~6 us
    // between the head and the graph's first kernel on every single frame.
    hipGraphExec_t execH[kResultSlots] = {}, execH1[kResultSlots] = {};
    hipGraph_t graphH[kResultSlots] = {}, graphH1[kResultSlots] = {};
    hipGraphNode_t headH[kResultSlots] = {}, headH1[kResultSlots] = {};
    // The input each exec's head node reads now (image, pitch, frame stride;
    // [slot][0]: execH, [1]: execH1): a frame from the same buffer as that
    // exec's last one launches without re-pointing the node.
    struct HeadIn {
        const void* img = nullptr;
        int pitch = 0;
        long sfs = 0;
        bool operator==(const HeadIn& o) const { return img == o.img && pitch == o.pitch && sfs == o.sfs; }
    };
    HeadIn headIn[kResultSlots][2];
    int nfOf[kResultSlots] = {};  // frames of the launch group that wrote each slot
    long long slotFrame[kResultSlots] = {-1, -1, -1, -1};  // the (first) frame whose results each slot holds
    int slotNum[kResultSlots] = {};  // frame numbers in that slot (> 1: a micro-batch, frame slotFrame + i in arena i)
    long long launched = 0;  // launch groups run on this lane; the next takes slot launched % kResultSlots
    long long last = -1;     // the last frame launched here (-1: none since warm-up)
    char* mbIn = nullptr;    // micro-batch input copies: mb frames of f32 rows (created at the first micro-batch)
    // Host-input frames: results written to mapped pinned host memory by the
    // frame's descriptor kernel (HostOut), one region per (slot, arena)
    // (created once a caller reads results back); dHostTab (device, kSlots x
    // B region pointers, null until then) tells the kernel where.
    char* hRes = nullptr;
    char* hResDev = nullptr;
    char** dHostTab = nullptr;
    std::vector<char*> hostTab;  // its host copy (the source of the async upload)
    // Host-input staging of this lane: two pinned host buffers, moved into
    // the lane's device staging by a 64-workgroup copy kernel on the lane's
    // stream ahead of the frame (launch_copy_rows).  Measured alternatives
    // (tools/host_pipeline_bench.cpp, 3 lanes x 6 frames, C2 u8 frames,
    // profiles/round5/): the first blur reading the pinned buffer itself
    // 0.165-0.170 ms/frame against 0.154 (its tiles' workgroups wait out the
    // PCIe transfer and crowd the other lanes); DMA on a separate upload
    // stream 0.169 at HIP's default 4 hardware queues per process (two active
    // streams then share a queue: device frames ordered after a 4 KiB copy on
    // a 4th stream ran at 0.160 instead of 0.112), 0.119-0.126 at
    // GPU_MAX_HW_QUEUES=8 -- but 8 queues slowed the bench process's other
    // legs; DMA on the lane's own stream 0.21-0.23 (the submit waited behind
    // the lane).  Host slot k is rewritten for the lane's frame after next,
    // once evRead[k] (recorded after the copy kernel) has passed; the device
    // slot is stream-ordered.
    static constexpr int kInSlots = 2;
    void* hStage[kInSlots] = {};
    void* dStage[kInSlots] = {};  // device copies (k_stage_to_device), allocated at the lane's first host frame
    hipEvent_t evRead[kInSlots] = {};
    long long uploads = 0;
    // Host results regions: one per (results slot, arena) -- region slot * B + arena.
    static constexpr int kHostRegions = kResultSlots * kMaxBatch;  // B <= kMaxBatch arenas per lane
    long long hostFrame[kHostRegions];  // the frame each host region holds (-1: none; set in add_lane)
    bool hostDesc[kHostRegions] = {};   // ... with its descriptors
};

// Byte offsets of every per-frame buffer inside a frame arena (the same for
// every arena of every lane).
struct ArenaLayout {
    size_t input = 0, up = 0, pyr = 0, cand = 0, ref = 0, ori = 0, slot = 0, order = 0, jobs = 0, range = 0,
           bcount = 0, boff = 0, bitmap = 0, ctr = 0, jord = 0;
    size_t k3[kResultSlots] = {}, f4[kResultSlots] = {}, desc[kResultSlots] = {};
    size_t codes[kResultSlots] = {}, ckeys[kResultSlots] = {};  // matcher sidecar of desc (Sidecar)
    size_t octave[kMaxOctaves] = {};  // float offset of each octave's planes inside the pyramid
};

struct sift_hip_detector {
    sift_hip_config cfg{};
    int device = 0;
    int L = 3, nOct = 0, firstOctave = 0;
    int tailOct = 0;  // first octave of the pyramid-tail launch (nOct: none)
    int baseW = 0, baseH = 0;
    // Frame uploads and result downloads.  Created on first use: a stream
    // holds a hardware queue, and device-input callers (several detectors per
    // GPU, one stream each) need none.
    hipStream_t copyStream = nullptr;
    hipEvent_t evIn = nullptr, evOut = nullptr;
    bool allocated = false;

    // Frames are numbered in submission order.  Frame f runs on lane
    // frec(f).lane and writes that lane's results slot frec(f).slot; `current`
    // is the frame the result accessors expose (its predecessor's descriptors
    // are prev_descriptor).  A frame may take a lane's slot only if the slot
    // holds no frame from current - 1 on, and at most 2 frames per lane may be
    // in flight past `current`.
    static constexpr int kSlots = kResultSlots;
    Lane lanes[kMaxLanes];
    int nLanes = 0;    // lanes created (lane 0 at warm-up, more on demand)
    int maxLanes = 2;  // sift_hip_set_lanes
    int ln = 0;        // the lane the pointer views below are bound to (bind_lane)
    int curLane = 0;   // lane of `current`
    int curIdx = 0;    // arena of `current` in its lane (micro-batches)
    // Micro-batching (sift_hip_set_micro_batch): device frames submitted with
    // sift_hip_submit_device queue here until mb of them run as one launch
    // group on a lane (the B-frame graphs, frame i in arena i), or until a
    // wait / sync / other submit needs them.  Tickets run ahead of `submitted`
    // by the frames pending.
    static constexpr int kMaxMicroBatch = 16;
    int mb = 1;
    struct PendingFrame {
        const void* img;  // device frame, or the device address of a host frame's pinned staging
        size_t stride;
        int fmt;
        bool ordered;  // the lane waits for evPend[i] (the caller's stream)
        int hslot;     // host frames: their staging slot (-1: a device frame)
    };
    // Pinned staging of micro-batched host frames: one block of hstSlots
    // slots (one per frame that can be pending or queued on a lane; a slot is
    // refilled once the copy kernel that read it, event hstRead[i], has run),
    // allocated in one piece at the first such frame (per-slot allocations
    // inside the submits of a running loop stalled it for milliseconds).
    char* hstBlock = nullptr;
    size_t hstSlotBytes = 0;
    int hstSlots = 0;
    std::vector<hipEvent_t> hstRead;
    long long hstNext = 0;
    PendingFrame pend[kMaxMicroBatch] = {};
    hipEvent_t evPend[kMaxMicroBatch] = {};
    int npend = 0;
    struct FrameRec {
        int lane = 0, slot = 0, idx = 0;  // idx: the frame's arena in a micro-batch
    };
    FrameRec frecs[kFrameRing];
    FrameRec& frec(long long f) { return frecs[f & (kFrameRing - 1)]; }
    Lane& lane() { return lanes[ln]; }
    long long submitted = 0, current = -1, firstFrame = 0, uploads = 0;

    // Frame batches: up to B frames per launch (sift_hip_set_batch).  Every
    // per-frame buffer below lives in frame 0's arena of the bound lane; frame
    // f's copy is at + f * afs bytes (Frames, sift_kernels.h).
    int B = 1;
    long afs = 0;
    ArenaLayout lay;

    PyrDesc pyr{};
    Taps initTaps{};
    std::vector<Taps> layerTaps;
    float threshold = 1.f;
    KeypointParams kp{};

    // Views of the bound lane (bind_lane): its stream and frame-0 arena pointers.
    hipStream_t stream = nullptr;
    int inPitch = 0, upPitch = 0;
    float* dInput = nullptr;  // blank warm-up frame; f32 scratch for 8-bit frames at other init radii
    float* dUp = nullptr;
    float* dPyr = nullptr;
    uint2* dCand = nullptr;
    unsigned capCand = 1u << 20;  // sized to the frame in setup_taps
    RefKpt* dRef = nullptr;
    OriKpt* dOri = nullptr;
    int* dSlot = nullptr;
    int* dOrder = nullptr;
    DescJob* dJobs = nullptr;  // per final keypoint, written by k_bucket_rank
    JobOrder* dJord = nullptr;  // descriptor job order (k_order -> k_rank_final)
    unsigned* dRange = nullptr;  // 2 * kRangeSlots pixel-range keys (initial blur -> descriptor)
    unsigned* dBcount = nullptr;
    unsigned* dBoff = nullptr;
    uint32_t* dBitmap = nullptr;
    size_t bitmapWords = 0;
    Counters* dCtr = nullptr;
    Counters* hCtr = nullptr;     // kSlots x B pinned host copies of the counters (written by k_descriptor)
    Counters* hCtrDev = nullptr;  // their device-side address
    float* dKpts3[kSlots] = {};
    float* dFeats4[kSlots] = {};
    uint16_t* dDesc[kSlots] = {};
    Sidecar dSide[kSlots] = {};
    int cur = 0, count = 0, prevCount = 0;  // frec(current).slot and the counts of current, current - 1
    bool countsValid = true;  // count / prevCount / the slot's host counters read after the frame completed

    HeadNode headNode{};
    bool useGraph = true;

    CopyPool* pool = nullptr;  // staging copies of large host frames (created at the first one)
    // The most the caller's sift_hip_copy_to_host / sift_hip_results_host
    // calls took (0 nothing yet, 1 keypoints, 2 keypoints + descriptors):
    // host-input frames have their descriptor kernel write that much to
    // pinned host memory (HostOut; a caller that never reads back pays nothing).
    int hostWant = 0;

    // Stage dumps (sift_hip_set_datagen): directory, and a device copy of the
    // frame's input as float (the caller's buffer may change before the dump).
    std::string dgDir;
    float* dDg = nullptr;

    bool timing = false;
    int blurReps = 1;  // timing mode: each blur launch repeated back to back inside its event pair
    std::vector<TimingRec> trecs;
    std::vector<TimingAgg> tagg;
    std::vector<hipEvent_t> evPool;
    size_t evUsed = 0;

    int name_id(const char* n) {
        for (size_t i = 0; i < tagg.size(); i++)
            if (tagg[i].name == n) return (int)i;
        tagg.push_back(TimingAgg{n});
        return (int)tagg.size() - 1;
    }
    hipEvent_t next_event() {
        if (evUsed == evPool.size()) {
            hipEvent_t e;
            (void)hipEventCreate(&e);
            evPool.push_back(e);
        }
        return evPool[evUsed++];
    }
    template <class F>
    void timed(const char* name, double bytes, F&& fn) {
        if (!timing) {
            fn();
            return;
        }
        // Blur launches are pure (input plane -> output plane; the first blur's
        // counter zeroing and range max are idempotent), so they may be
        // repeated to time them back to back without per-launch event cost.
        const int reps = strncmp(name, "blur_", 5) == 0 ? blurReps : 1;
        TimingRec r{name_id(name), next_event(), next_event(), bytes * reps, reps};
        // A roctx range per stage: rocprofv3
        // --marker-trace shows the stage spans and the kernels launched in them.
        roctxRangePushA(name);
        (void)hipEventRecord(r.e0, stream);
        for (int i = 0; i < reps; i++) fn();
        (void)hipEventRecord(r.e1, stream);
        roctxRangePop();
        trecs.push_back(r);
    }
    void collect_timing() {
        for (auto& r : trecs) {
            float ms = 0;
            (void)hipEventElapsedTime(&ms, r.e0, r.e1);
            tagg[r.name].ms += ms;
            tagg[r.name].bytes += r.bytes;
            tagg[r.name].launches += r.launches;
        }
        trecs.clear();
        evUsed = 0;
    }

    ~sift_hip_detector() {
        unregister_sidecars(this);
        if (allocated) {
            (void)hipSetDevice(device);
            for (int k = 0; k < nLanes; k++) {
                Lane& L = lanes[k];
                if (L.stream) (void)hipStreamSynchronize(L.stream);
                for (int b = 0; b < kSlots; b++) {
                    for (hipGraphExec_t e : {L.exec[b], L.exec1[b], L.execH[b], L.execH1[b]})
                        if (e) (void)hipGraphExecDestroy(e);
                    for (hipGraph_t g : {L.graphH[b], L.graphH1[b]})
                        if (g) (void)hipGraphDestroy(g);
                    if (L.evFrame[b]) (void)hipEventDestroy(L.evFrame[b]);
                }
                if (L.arena) (void)hipFree(L.arena);
                if (L.mbIn) (void)hipFree(L.mbIn);
                if (L.hCtr) (void)hipHostFree(L.hCtr);
                if (L.hRes) (void)hipHostFree(L.hRes);
                if (L.dHostTab) (void)hipFree(L.dHostTab);
                for (int k = 0; k < Lane::kInSlots; k++) {
                    if (L.hStage[k]) (void)hipHostFree(L.hStage[k]);
                    if (L.dStage[k]) (void)hipFree(L.dStage[k]);
                    if (L.evRead[k]) (void)hipEventDestroy(L.evRead[k]);
                }
                if (L.stream) (void)hipStreamDestroy(L.stream);
            }
            if (dDg) (void)hipFree(dDg);
            for (auto e : evPool) (void)hipEventDestroy(e);
            if (hstBlock) (void)hipHostFree(hstBlock);
            for (hipEvent_t e : hstRead) (void)hipEventDestroy(e);
            if (evIn) (void)hipEventDestroy(evIn);
            for (hipEvent_t e : evPend)
                if (e) (void)hipEventDestroy(e);
            if (evOut) (void)hipEventDestroy(evOut);
            if (copyStream) (void)hipStreamDestroy(copyStream);
        }
        delete pool;
    }
};

static_assert(kFrameRing > 2 * kMaxLanes * sift_hip_detector::kMaxMicroBatch + 2 && (kFrameRing & (kFrameRing - 1)) == 0,
              "frame records outlive every frame in flight");

namespace {

int setup_geometry(sift_hip_detector* d) {
    const sift_hip_config& c = d->cfg;
    d->L = c.numOctaveLayers;
    d->firstOctave = c.upscale ? -1 : 0;
    d->baseW = c.upscale ? 2 * c.col_width : c.col_width;
    d->baseH = c.upscale ? 2 * c.row_width : c.row_width;
    int nOct = c.numOctaves;
    if (nOct <= 0)  // [OpenCV 4.x sift.dispatch.cpp] cvRound(log2(min) - 2) - firstOctave
        nOct = (int)lrint(std::log((double)std::min(d->baseW, d->baseH)) / std::log(2.) - 2) - d->firstOctave;
    if (nOct < 1) nOct = 1;
    if (nOct > kMaxOctaves) return fail(SIFT_HIP_ERR_INVALID, "too many octaves");
    d->nOct = nOct;
    int W = d->baseW, H = d->baseH;
    int rowBase = 0;
    long bitBase = 0;
    size_t off = 0;
    for (int o = 0; o < nOct; o++) {
        if (o > 0) {
            W /= 2;
            H /= 2;
        }
        if (W < 1 || H < 1) return fail(SIFT_HIP_ERR_INVALID, "octave smaller than one pixel");
        OctGeom& g = d->pyr.oct[o];
        g.W = W;
        g.H = H;
        g.pitch = (W + 63) / 64 * 64;
        g.planeStride = (long)g.pitch * H;
        g.base = nullptr;  // bound to a lane's arena by bind_lane
        d->lay.octave[o] = off;
        g.rowBase = rowBase;
        g.bitBase = bitBase;
        off += (size_t)g.planeStride * (d->L + 3);
        rowBase += d->L * H;
        bitBase += (long)d->L * H * W;
    }
    d->pyr.nOct = nOct;
    d->pyr.L = d->L;
    d->pyr.firstOctave = d->firstOctave;
    d->kp.numBuckets = rowBase;
    d->bitmapWords = (size_t)(bitBase + 31) / 32;
    return SIFT_HIP_OK;
}

void setup_taps(sift_hip_detector* d) {
    const float sigma = (float)d->cfg.sigma;
    const float sig_diff = d->firstOctave < 0 ? sqrtf(std::max(sigma * sigma - 0.5f * 0.5f * 4, 0.01f))
                                              : sqrtf(std::max(sigma * sigma - 0.5f * 0.5f, 0.01f));
    d->initTaps = gaussian_taps((double)sig_diff);
    const int L = d->L;
    std::vector<double> sig(L + 3);
    sig[0] = d->cfg.sigma;
    const double k = std::pow(2., 1. / L);
    for (int i = 1; i < L + 3; i++) {
        const double sig_prev = std::pow(k, (double)(i - 1)) * d->cfg.sigma;
        const double sig_total = sig_prev * k;
        sig[i] = std::sqrt(sig_total * sig_total - sig_prev * sig_prev);
    }
    d->layerTaps.resize(L + 3);
    for (int i = 0; i < L + 3; i++) d->layerTaps[i] = gaussian_taps(sig[i]);
    // The pyramid tail for the small octaves.  (Measured alternative, round
    // 4: per-plane launches -- 752x480 sync 0.2177 vs 0.2094-0.2107 ms.)
    d->tailOct = L + 3 <= kTailMaxPlanes ? tail_first_octave(d->pyr, d->layerTaps.data(), L) : d->nOct;
    d->threshold = (float)(int)std::floor(0.5 * d->cfg.contrastThreshould / L * 255 * 1.0);
    d->kp.contrastThreshold = (float)d->cfg.contrastThreshould;
    d->kp.edgeThreshold = (float)d->cfg.edgeThreshould;
    d->kp.sigma = (float)d->cfg.sigma;
    d->kp.numFeatures = d->cfg.numFeatures;
    // Capacities sized to the frame (were fixed 1M / 2^18 / 2^19 / 65536, so a
    // small frame held 128 MiB against the reference's 84, readme.md:16).
    // Candidates: 1/8 of the scale-space samples (a 3x3x3 extremum test passes
    // ~7 % of samples of pure noise before the contrast threshold; natural and
    // synthetic frames stay far below); refined <= candidates; oriented: one
    // slot per refined keypoint + as many extra peaks; results: numFeatures
    // (+ a quarter for retainBest's response ties), or 1/32 of the pyramid's
    // pixels without a feature limit (C1 frames keep ~1/3000).  Every stage
    // clamps to its capacity and sets its overflow bit (sift_hip_overflow_flags).
    double sumPx = 0;
    for (int o = 0; o < d->nOct; o++) sumPx += (double)d->pyr.oct[o].W * d->pyr.oct[o].H;
    auto clampu = [](double v, double lo, double hi) { return (unsigned)std::max(lo, std::min(v, hi)); };
    d->capCand = clampu(sumPx * L / 8, 16384, 1u << 20);
    d->kp.capRefined = std::min(d->capCand, 1u << 18);
    d->kp.capOriented = 2 * d->kp.capRefined;
    const int nfeat = d->cfg.numFeatures;
    d->kp.capFinal = d->cfg.maxKeypoints > 0 ? (unsigned)d->cfg.maxKeypoints
                     : nfeat > 0             ? clampu(nfeat + std::max(nfeat / 4, 512), 1024, 65536)
                                             : clampu(sumPx / 32, 4096, 65536);
    // LDS patch bounds: scl_octv = sigma * 2^((layer + xi) / L) <= sigma * 2^((L + 0.5) / L).
    // Larger radii (not reachable from accepted keypoints) fall back to HBM reads.
    const double sclMax = d->cfg.sigma * std::pow(2.0, (L + 0.5) / L);
    d->kp.oriRmax = (int)lrint(4.5 * sclMax) + 1;
    d->kp.descRmax = std::min((int)lrint(3.0 * sclMax * 1.4142135623730951 * 2.5) + 1, 60);
    // Valid descriptor samples lie in a rotated square of side 5 * hist_width.
    const double hw = 3.0 * sclMax;
    d->kp.descNrec = std::min((int)std::ceil((5.0 * hw + 3.0) * (5.0 * hw + 3.0)), 8192);
}

void upload_exp_tab() {
    const double A0 = .9670371139572337719125840413672004409288e-2;
    float tab[64];
    for (int j = 0; j < 64; j++) tab[j] = (float)(std::exp2((double)j / 64.0) * A0);
    upload_exp_table(tab);
    upload_desc_exp_table(tab);
}

template <class T>
int dalloc(T** p, size_t count) {
    if (hipMalloc((void**)p, sizeof(T) * std::max<size_t>(count, 1)) != hipSuccess)
        return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc failed");
    return SIFT_HIP_OK;
}

// Points the handle's buffer views (stream, frame-0 arena pointers, host
// counters) at lane k.  Every entry point binds the lane it works on: the
// submitting lane for a new frame (idx 0: launches address frame 0's arena),
// the current frame's lane and arena for accessors (idx: its arena in a
// micro-batch, which offsets the results views and host counters).
void bind_lane(sift_hip_detector* d, int k, int idx = 0) {
    Lane& L = d->lanes[k];
    const ArenaLayout& a = d->lay;
    char* A = L.arena;
    d->ln = k;
    d->stream = L.stream;
    d->dInput = reinterpret_cast<float*>(A + a.input);
    d->dUp = d->firstOctave < 0 ? reinterpret_cast<float*>(A + a.up) : nullptr;
    d->dPyr = reinterpret_cast<float*>(A + a.pyr);
    for (int o = 0; o < d->nOct; o++) d->pyr.oct[o].base = d->dPyr + a.octave[o];
    d->dCand = reinterpret_cast<uint2*>(A + a.cand);
    d->dRef = reinterpret_cast<RefKpt*>(A + a.ref);
    d->dOri = reinterpret_cast<OriKpt*>(A + a.ori);
    d->dSlot = reinterpret_cast<int*>(A + a.slot);
    d->dOrder = reinterpret_cast<int*>(A + a.order);
    d->dJobs = reinterpret_cast<DescJob*>(A + a.jobs);
    d->dJord = reinterpret_cast<JobOrder*>(A + a.jord);
    d->dRange = reinterpret_cast<unsigned*>(A + a.range);
    d->dBcount = reinterpret_cast<unsigned*>(A + a.bcount);
    d->dBoff = reinterpret_cast<unsigned*>(A + a.boff);
    d->dBitmap = reinterpret_cast<uint32_t*>(A + a.bitmap);
    d->dCtr = reinterpret_cast<Counters*>(A + a.ctr);
    char* R = A + (size_t)idx * d->afs;
    for (int b = 0; b < d->kSlots; b++) {
        d->dKpts3[b] = reinterpret_cast<float*>(R + a.k3[b]);
        d->dFeats4[b] = reinterpret_cast<float*>(R + a.f4[b]);
        d->dDesc[b] = reinterpret_cast<uint16_t*>(R + a.desc[b]);
        d->dSide[b] = Sidecar{reinterpret_cast<int8_t*>(R + a.codes[b]), reinterpret_cast<int*>(R + a.ckeys[b])};
    }
    d->hCtr = L.hCtr + idx;
    d->hCtrDev = L.hCtrDev + idx;
}

// Results of frame f (lane and slot from its record), without binding.
const uint16_t* frame_desc(const sift_hip_detector* d, long long f) {
    const auto& r = d->frecs[f & (kFrameRing - 1)];
    return reinterpret_cast<const uint16_t*>(d->lanes[r.lane].arena + (size_t)r.idx * d->afs + d->lay.desc[r.slot]);
}
const Counters& frame_counters(const sift_hip_detector* d, long long f, int i = 0) {
    const auto& r = d->frecs[f & (kFrameRing - 1)];
    return d->lanes[r.lane].hCtr[(size_t)r.slot * d->B + r.idx + i];
}

// Per-handle allocations shared by the lanes: the upload ring and the frame
// arena layout (the lanes themselves: add_lane).
int allocate(sift_hip_detector* d) {
    HIPCHK(hipSetDevice(d->device));
    d->allocated = true;
    // The pyramid tail is an optimisation: without the LDS it asks for (a
    // device whose opt-in limit is lower, or a refused attribute) the small
    // octaves take the per-plane blur launches instead.
    if (d->tailOct < d->nOct) {
        int optin = 0;
        if (hipDeviceGetAttribute(&optin, hipDeviceAttributeSharedMemPerBlockOptin, d->device) != hipSuccess ||
            optin < (int)(sizeof(float) * kTailLdsFloats) || tail_init() != hipSuccess) {
            (void)hipGetLastError();
            d->tailOct = d->nOct;
        }
    }
    HIPCHK(hipEventCreateWithFlags(&d->evIn, hipEventDisableTiming));
    HIPCHK(hipEventCreateWithFlags(&d->evOut, hipEventDisableTiming));
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    d->inPitch = (W + 63) / 64 * 64;
    if (d->firstOctave < 0) d->upPitch = (2 * W + 63) / 64 * 64;
    size_t pyrFloats = 0;
    for (int o = 0; o < d->nOct; o++) pyrFloats += (size_t)d->pyr.oct[o].planeStride * (d->L + 3);
    const unsigned capO = d->kp.capOriented, capF = d->kp.capFinal;

    // Frame arena: every per-frame buffer at a 256-B aligned offset; B arenas
    // back to back per lane.  Zeroed once at allocation; afterwards the
    // kernels keep the scratch zero for the next frame (first blur: counters,
    // k_order / k_select: range keys, k_bucket_rank: bucket counts,
    // k_orientation: dedupe bits), so the frame graph has no memset node.
    size_t off = 0;
    auto take = [&](size_t bytes) {
        const size_t o = off;
        off += (std::max<size_t>(bytes, 1) + 255) & ~(size_t)255;
        return o;
    };
    ArenaLayout& a = d->lay;
    a.input = take(sizeof(float) * (size_t)d->inPitch * H);  // blank warm-up frame / u8 -> f32 scratch
    a.up = d->firstOctave < 0 ? take(sizeof(float) * (size_t)d->upPitch * 2 * H) : 0;
    a.pyr = take(sizeof(float) * pyrFloats);
    a.cand = take(sizeof(uint2) * d->capCand);
    a.ref = take(sizeof(RefKpt) * d->kp.capRefined);
    a.ori = take(sizeof(OriKpt) * capO);
    a.slot = take(sizeof(int) * capO);
    a.order = take(sizeof(int) * capO);
    a.jobs = take(sizeof(DescJob) * capF);
    a.jord = take(sizeof(JobOrder));
    a.range = take(sizeof(unsigned) * 2 * 2 * kRangeSlots);  // one set per frame parity
    a.bcount = take(sizeof(unsigned) * (size_t)d->kp.numBuckets);
    a.boff = take(sizeof(unsigned) * (size_t)d->kp.numBuckets);
    a.bitmap = take(sizeof(uint32_t) * d->bitmapWords);
    a.ctr = take(sizeof(Counters));
    for (int b = 0; b < d->kSlots; b++) {
        a.k3[b] = take(sizeof(float) * 3 * (size_t)capF);
        a.f4[b] = take(sizeof(float) * 4 * (size_t)capF);
        a.desc[b] = take(sizeof(uint16_t) * 128 * (size_t)capF);
        a.codes[b] = take(128 * (size_t)capF);
        a.ckeys[b] = take(sizeof(int) * (size_t)capF);
    }
    d->afs = (long)off;
    upload_exp_tab();
    return SIFT_HIP_OK;
}

int build_graphs(sift_hip_detector* d);
int ensure_host_res(sift_hip_detector* d, Lane& L);

// A new compute lane: stream, zeroed arenas, host counters, events and the
// captured graphs (bound on return).
int add_lane(sift_hip_detector* d) {
    if (d->nLanes >= kMaxLanes) return fail(SIFT_HIP_ERR_STATE, "no lane left");
    const int k = d->nLanes;
    Lane& L = d->lanes[k];
    d->nLanes++;  // from here the destructor releases what the lane holds
    HIPCHK(hipStreamCreateWithFlags(&L.stream, hipStreamNonBlocking));
    if (hipMalloc((void**)&L.arena, (size_t)d->afs * d->B) != hipSuccess)
        return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the frame arenas failed");
    HIPCHK(hipMemsetAsync(L.arena, 0, (size_t)d->afs * d->B, L.stream));
    const size_t nh = (size_t)d->kSlots * d->B;
    HIPCHK(hipHostMalloc((void**)&L.hCtr, sizeof(Counters) * nh, hipHostMallocMapped | hipHostMallocCoherent));
    memset(L.hCtr, 0, sizeof(Counters) * nh);
    HIPCHK(hipHostGetDevicePointer((void**)&L.hCtrDev, L.hCtr, 0));
    if (hipMalloc((void**)&L.dHostTab, sizeof(char*) * nh) != hipSuccess)
        return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the host results table failed");
    HIPCHK(hipMemsetAsync(L.dHostTab, 0, sizeof(char*) * nh, L.stream));
    for (int b = 0; b < d->kSlots; b++) {
        HIPCHK(hipEventCreateWithFlags(&L.evFrame[b], hipEventDisableTiming));
        HIPCHK(hipEventRecord(L.evFrame[b], L.stream));
    }
    std::fill(std::begin(L.hostFrame), std::end(L.hostFrame), -1LL);
    // The lane's host-input staging, sized for f32 rows of pitch inPitch (an
    // 8-bit frame uses the first quarter with a byte pitch of inPitch); its
    // events start complete.
    const size_t inBytes = sizeof(float) * (size_t)d->inPitch * d->cfg.row_width;
    for (int i = 0; i < Lane::kInSlots; i++) {
        HIPCHK(hipHostMalloc(&L.hStage[i], inBytes, hipHostMallocMapped | hipHostMallocNonCoherent));
        HIPCHK(hipEventCreateWithFlags(&L.evRead[i], hipEventDisableTiming));
        HIPCHK(hipEventRecord(L.evRead[i], L.stream));
    }
    bind_lane(d, k);
    for (int i = 0; i < d->B; i++)
        for (int b = 0; b < d->kSlots; b++)
            register_sidecar(d, fptr(d->dDesc[b], (long)i * d->afs),
                             Sidecar{fptr(d->dSide[b].codes, (long)i * d->afs), fptr(d->dSide[b].keys, (long)i * d->afs)},
                             (int)d->kp.capFinal);
    if (d->hostWant)
        if (int rc = ensure_host_res(d, L)) return rc;
    return build_graphs(d);
}

// The first kernel reads the caller's image (upload ring slot or a device
// pointer); it stays outside the graph so the graph never bakes a user pointer.
// Pixel-range keys by frame parity p (frame f uses p = f & 1; k_select zeroes
// the other set for the next frame).
unsigned* range_keys(sift_hip_detector* d, int p) { return d->dRange + (size_t)p * 2 * kRangeSlots; }

// pitch in elements of the frame's format (bytes for SIFT_HIP_U8); nf frames
// at byte stride sfs.
void enqueue_head(sift_hip_detector* d, const void* img, int pitch, int fmt, int parity, int nf, long sfs) {
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    const bool u8 = fmt == SIFT_HIP_U8;
    const Frames fr{nf, d->afs};
    const double inB = (double)W * H * (u8 ? 1 : 4) * nf;
    // Counters first: the initial blur accumulates the frame's pixel range.
    if (d->firstOctave < 0) {
        d->timed("upsample", inB + (double)W * H * 16 * nf, [&] {
            if (u8)
                launch_upsample2x_u8((const uint8_t*)img, pitch, W, H, d->dUp, d->upPitch, fr, sfs, d->stream);
            else
                launch_upsample2x((const float*)img, pitch, W, H, d->dUp, d->upPitch, fr, sfs, d->stream);
        });
    } else {
        const OctGeom& g = d->pyr.oct[0];
        d->timed("blur_init", inB + (double)W * H * 4 * nf, [&] {
            long s = sfs;
            if (u8) {
                if (launch_blur_u8((const uint8_t*)img, pitch, W, H, g.base, g.pitch, d->initTaps, fr, sfs, d->stream,
                                   range_keys(d, parity), d->dCtr))
                    return;
                launch_u8_to_f32((const uint8_t*)img, pitch, W, H, d->dInput, d->inPitch, fr, sfs, d->stream);
                img = d->dInput;
                pitch = d->inPitch;
                s = d->afs;
            }
            launch_blur((const float*)img, pitch, W, H, g.base, g.pitch, DecOut{}, d->initTaps, fr, s, d->stream,
                        range_keys(d, parity), d->dCtr);
        });
    }
}

// Pyramid tail: octaves d->tailOct.. in one launch (one workgroup per frame,
// planes in LDS), none when every octave is too large for it.
void left_tail(sift_hip_detector* d, int nf, hipStream_t s) {
    if (d->tailOct >= d->nOct) return;
    double bytes = 0;
    for (int o = d->tailOct; o < d->nOct; o++)
        bytes += (double)d->pyr.oct[o].W * d->pyr.oct[o].H * 4 * (o == d->tailOct ? 1 + (d->L + 2) : (d->L + 2)) * nf;
    d->timed("pyr_tail", bytes, [&] { launch_blur_tail(d->pyr, d->layerTaps.data(), d->L, d->tailOct, Frames{nf, d->afs}, s); });
}

// The frame pipeline after the head, as the stages tool/perf.cu replays one
// at a time (sift_hip_replay_stage): pyramid (blur jobs), extrema, refine,
// orientation, order (retainBest + deterministic order + descriptor jobs),
// descriptor.  `parity` = the frame's range-key set (frame parity).
void enqueue_pyramid(sift_hip_detector* d, int nf, int parity) {
    hipStream_t s = d->stream;
    const int L = d->L;
    const Frames fr{nf, d->afs};
    if (d->firstOctave < 0) {
        const OctGeom& g = d->pyr.oct[0];
        d->timed("blur_init", (double)g.W * g.H * 8 * nf, [&] {
            launch_blur(d->dUp, d->upPitch, g.W, g.H, g.base, g.pitch, DecOut{}, d->initTaps, fr, d->afs, s,
                        range_keys(d, parity), d->dCtr);
        });
    }
    static const char* blurNames[kMaxOctaves] = {"blur_o0", "blur_o1", "blur_o2", "blur_o3", "blur_o4", "blur_o5",
                                                 "blur_o6", "blur_o7", "blur_o8", "blur_o9", "blur_o10", "blur_o11",
                                                 "blur_o12", "blur_o13", "blur_o14", "blur_o15"};
    // Blur jobs (o, i): plane i of octave o from plane i-1 (plane 0 of octave
    // o+1 is written by job (o, L) as it stores: the INTER_NEAREST half-size
    // copy of plane L).  List-scheduled in (o, i) order: a job is ready once
    // its input plane's job has been launched (stream order); the two oldest
    // ready jobs share one launch when their radii have a pair kernel -- with
    // L = 3, (o, 4) + (o+1, 1) and (o, 5) + (o+1, 2): 11 launches instead of 15
    // for three octaves.
    struct Job {
        int o, i;
        BlurDesc b;
        double bytes;
    };
    std::vector<Job> jobs;
    // Octaves from d->tailOct on: one pyramid-tail launch after the jobs
    // (launch_blur_tail; their base plane is written by job (tailOct - 1, L)).
    for (int o = 0; o < d->tailOct; o++) {
        const OctGeom& g = d->pyr.oct[o];
        for (int i = 1; i < L + 3; i++) {
            Job j{o, i, {}, 0};
            j.b.src = g.base + (size_t)(i - 1) * g.planeStride;
            j.b.spitch = g.pitch;
            j.b.dst = g.base + (size_t)i * g.planeStride;
            j.b.dpitch = g.pitch;
            j.b.W = g.W;
            j.b.H = g.H;
            j.b.taps = &d->layerTaps[i];
            j.bytes = (double)g.W * g.H * 8 * nf;
            if (i == L && o + 1 < d->nOct) {
                const OctGeom& n = d->pyr.oct[o + 1];
                j.b.dec = DecOut{n.base, n.pitch, n.W, n.H};
                j.bytes += (double)n.W * n.H * 4 * nf;
            }
            jobs.push_back(j);
        }
    }
    auto idx = [&](int o, int i) { return o * (L + 2) + (i - 1); };
    std::vector<bool> done(jobs.size(), false);
    auto ready = [&](size_t k) {
        const Job& j = jobs[k];
        if (done[k]) return false;
        if (j.i >= 2) return (bool)done[idx(j.o, j.i - 1)];
        return j.o == 0 || (bool)done[idx(j.o - 1, L)];
    };
    if (jobs.empty()) left_tail(d, nf, s);
    for (size_t left = jobs.size(); left > 0;) {
        int a = -1, b = -1;
        for (size_t k = 0; k < jobs.size() && b < 0; k++)
            if (ready(k)) (a < 0 ? a : b) = (int)k;
        const Job& ja = jobs[a];
        bool paired = false;
        if (b >= 0) {
            const Job& jb = jobs[b];
            char name[16];
            snprintf(name, sizeof name, "blur_o%d+o%d", ja.o, jb.o);
            d->timed(name, ja.bytes + jb.bytes, [&] { paired = launch_blur_pair(ja.b, jb.b, fr, s); });
            if (paired) {
                done[b] = true;
                left--;
            }
        }
        if (!paired) {
            d->timed(blurNames[ja.o], ja.bytes, [&] {
                launch_blur(ja.b.src, ja.b.spitch, ja.b.W, ja.b.H, ja.b.dst, ja.b.dpitch, ja.b.dec,
                            *ja.b.taps, fr, d->afs, s);
            });
        }
        done[a] = true;
        left--;
    }
    if (!jobs.empty()) left_tail(d, nf, s);
}

void enqueue_extrema(sift_hip_detector* d, int nf) {
    hipStream_t s = d->stream;
    const int L = d->L;
    const Frames fr{nf, d->afs};
    double exBytes = 0;
    for (int o = 0; o < d->nOct; o++) exBytes += (double)d->pyr.oct[o].W * d->pyr.oct[o].H * 4 * (L + 3) * nf;
    d->timed("extrema", exBytes, [&] {
        if (!launch_extrema_all(d->pyr, d->threshold, d->dCand, d->dCtr, d->capCand, fr, s))
            for (int o = 0; o < d->nOct; o++)
                launch_extrema(d->pyr, o, d->threshold, d->dCand, d->dCtr, d->capCand, fr, s);
    });
}

void enqueue_refine(sift_hip_detector* d, int nf) {
    const Frames fr{nf, d->afs};
    d->timed("refine", 0, [&] {
        launch_refine(d->pyr, d->dCand, d->capCand, d->dCtr, d->dBitmap, d->dRef, d->kp, fr, d->stream);
    });
}

void enqueue_orientation(sift_hip_detector* d, int nf) {
    const Frames fr{nf, d->afs};
    d->timed("orientation", 0,
             [&] { launch_orientation(d->pyr, d->dRef, d->dCtr, d->dOri, d->dBitmap, d->kp, fr, d->stream); });
}

void enqueue_order(sift_hip_detector* d, int slot, int nf) {
    hipStream_t s = d->stream;
    const int parity = slot & 1;
    const Frames fr{nf, d->afs};
    if (d->kp.numBuckets <= kOrderMaxBuckets) {
        d->timed("order", 0, [&] {
            launch_order(d->pyr, d->dOri, d->dCtr, range_keys(d, parity ^ 1), d->dBcount, d->dBoff, d->dSlot, d->dOrder,
                         d->dJord, d->kp, fr, s);
        });
    } else {
        d->timed("select", 0, [&] { launch_select(d->dOri, d->dCtr, range_keys(d, parity ^ 1), d->kp, fr, s); });
        d->timed("bucket_count", 0,
                 [&] { launch_bucket_count(d->dOri, d->dCtr, d->dBcount, d->dSlot, d->kp, fr, s); });
        d->timed("bucket_scan", 0, [&] { launch_bucket_scan(d->dBcount, d->dBoff, d->dCtr, d->kp, fr, s); });
        d->timed("bucket_scatter", 0,
                 [&] { launch_bucket_scatter(d->dOri, d->dCtr, d->dBoff, d->dSlot, d->dOrder, d->kp, fr, s); });
    }
    d->timed("bucket_rank", 0, [&] {
        if (d->kp.numBuckets <= kOrderMaxBuckets)
            launch_rank_final(d->pyr, d->dOri, d->dBcount, d->dBoff, d->dOrder, d->dCtr, d->dJord, d->dJobs, d->dKpts3[slot],
                              d->dFeats4[slot], d->kp, fr, s);
        else  // bucket_count needs zeroed counts: the bucket-parallel ranking re-zeroes them
            launch_bucket_rank(d->pyr, d->dOri, d->dBcount, d->dBoff, d->dOrder, d->dCtr, d->dJobs, d->dKpts3[slot],
                               d->dFeats4[slot], d->kp, fr, s);
    });
}

void enqueue_descriptor(sift_hip_detector* d, int slot, int nf) {
    const Frames fr{nf, d->afs};
    d->timed("descriptor", 0, [&] {
        launch_descriptor(d->dJobs, d->dCtr, range_keys(d, slot & 1), d->dDesc[slot], d->dSide[slot],
                          d->hCtrDev + (size_t)slot * d->B,
                          HostOut{d->lanes[d->ln].dHostTab + (size_t)slot * d->B, d->dKpts3[slot], d->dFeats4[slot],
                                  d->kp.capFinal},
                          d->kp, fr, d->stream);
    });
}

void enqueue_body(sift_hip_detector* d, int slot, int nf) {
    enqueue_pyramid(d, nf, slot & 1);  // kSlots is even, so slot parity = frame parity
    enqueue_extrema(d, nf);
    enqueue_refine(d, nf);
    enqueue_orientation(d, nf);
    enqueue_order(d, slot, nf);
    enqueue_descriptor(d, slot, nf);
}

int capture(sift_hip_detector* d, int slot, int nf, hipGraphExec_t* out) {
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
    enqueue_body(d, slot, nf);
    HIPCHK(hipStreamEndCapture(d->stream, &g));
    HIPCHK(hipGraphInstantiate(out, g, nullptr, nullptr, 0));
    HIPCHK(hipGraphDestroy(g));
    return SIFT_HIP_OK;
}

// The head for f32 device input (the frame's first blur, or the 2x upsample)
// as node parameters for image `img` (pitch in floats, nf frames at byte
// stride sfs): what enqueue_head launches.
void head_node(sift_hip_detector* d, HeadNode& h, const float* img, int pitch, int parity, int nf, long sfs) {
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    const Frames fr{nf, d->afs};
    if (d->firstOctave < 0) {
        head_upsample_node(h, img, pitch, W, H, d->dUp, d->upPitch, fr, sfs);
    } else {
        const OctGeom& g = d->pyr.oct[0];
        head_blur_node(h, img, pitch, W, H, g.base, g.pitch, d->initTaps, fr, sfs, range_keys(d, parity), d->dCtr);
    }
}

// head + body captured together; the graph is kept for its head node.
int capture_with_head(sift_hip_detector* d, int slot, int nf, hipGraphExec_t* out, hipGraph_t* graph,
                      hipGraphNode_t* head) {
    HIPCHK(hipStreamBeginCapture(d->stream, hipStreamCaptureModeThreadLocal));
    enqueue_head(d, d->dInput, d->inPitch, SIFT_HIP_F32, slot & 1, nf, d->afs);
    enqueue_body(d, slot, nf);
    HIPCHK(hipStreamEndCapture(d->stream, graph));
    size_t nroot = 0;
    HIPCHK(hipGraphGetRootNodes(*graph, nullptr, &nroot));
    if (nroot != 1) return fail(SIFT_HIP_ERR_RUNTIME, "captured frame graph: expected one root (the head)");
    HIPCHK(hipGraphGetRootNodes(*graph, head, &nroot));
    hipGraphNodeType ty;
    HIPCHK(hipGraphNodeGetType(*head, &ty));
    if (ty != hipGraphNodeTypeKernel) return fail(SIFT_HIP_ERR_RUNTIME, "captured frame graph: the head is not a kernel");
    HIPCHK(hipGraphInstantiate(out, *graph, nullptr, nullptr, 0));
    return SIFT_HIP_OK;
}

int build_graphs(sift_hip_detector* d) {
    Lane& L = d->lane();
    for (int b = 0; b < d->kSlots; b++) {
        if (int rc = capture(d, b, d->B, &L.exec[b])) return rc;
        if (int rc = capture_with_head(d, b, d->B, &L.execH[b], &L.graphH[b], &L.headH[b])) return rc;
        L.headIn[b][0] = Lane::HeadIn{d->dInput, d->inPitch, d->afs};
        if (d->B > 1) {
            if (int rc = capture(d, b, 1, &L.exec1[b])) return rc;
            if (int rc = capture_with_head(d, b, 1, &L.execH1[b], &L.graphH1[b], &L.headH1[b])) return rc;
            L.headIn[b][1] = Lane::HeadIn{d->dInput, d->inPitch, d->afs};
        }
    }
    return SIFT_HIP_OK;
}

int dump_stage_files(sift_hip_detector* d);
void complete_counts(sift_hip_detector* d);

bool event_done(hipEvent_t e) {
    const hipError_t r = hipEventQuery(e);
    if (r == hipSuccess) return true;
    (void)hipGetLastError();  // hipErrorNotReady is not an error of the handle
    return false;
}

// Blank launch groups through every graph of a lane created after warm-up
// (first-launch costs, as sift_hip_warmup's blank frames pay them for lane 0).
// They take no frame numbers; slots 0..kSlots-1 in order keep the lane's
// range-key parity alternating, and the lane's next frame takes slot 0.
int warm_lane(sift_hip_detector* d) {
    Lane& L = d->lane();
    const int nb = d->B > 1 ? 2 : 1;
    for (int r = 0; r < nb; r++)
        for (int b = 0; b < d->kSlots; b++) {
            HIPCHK(hipGraphLaunch(r == 0 ? L.execH[b] : L.execH1[b], L.stream));
            HIPCHK(hipEventRecord(L.evFrame[b], L.stream));
            L.nfOf[b] = r == 0 ? d->B : 1;
        }
    L.launched = (long long)nb * d->kSlots;
    return SIFT_HIP_OK;
}

// The lane for the next frame, bound on return: the first idle lane (its last
// frame complete), else a new lane (up to maxLanes), else the busy lane whose
// last frame is the oldest.  A lane qualifies only if its next results slot
// holds no frame the caller may still read (current - 1 onwards).
int pick_lane(sift_hip_detector* d) {
    auto slot_free = [&](int k) {
        const Lane& L = d->lanes[k];
        const int s = (int)(L.launched % d->kSlots);
        const long long occ = L.slotFrame[s] < 0 ? -1 : L.slotFrame[s] + std::max(L.slotNum[s], 1) - 1;  // its last frame
        return occ < 0 || occ < d->firstFrame || occ < d->current - 1;
    };
    int busy = -1;
    for (int k = 0; k < d->nLanes; k++) {
        if (!slot_free(k)) continue;
        const Lane& L = d->lanes[k];
        if (L.last < 0 || event_done(L.evFrame[(L.launched + d->kSlots - 1) % d->kSlots])) {
            bind_lane(d, k);
            return SIFT_HIP_OK;
        }
        if (busy < 0 || L.last < d->lanes[busy].last) busy = k;
    }
    if (d->nLanes < d->maxLanes) {  // (lane 0 comes from sift_hip_warmup)
        if (int rc = add_lane(d)) return rc;
        return warm_lane(d);
    }
    if (busy < 0)
        return fail(SIFT_HIP_ERR_STATE, "every lane's next results slot is still held: sift_hip_wait first");
    bind_lane(d, busy);
    return SIFT_HIP_OK;
}

// Enqueues launch group d->submitted (nf frames at byte stride sfs) on the
// bound lane (pick_lane); `consumed` (nullable) is recorded once the input has
// been read.  A batch (sift_hip_detect_batch_device) is one frame number; a
// micro-batch (`numbered`) takes nf numbers, frame d->submitted + i in arena i.  With stage dumps on (single frames after warm-up) the frame's
// input is kept as float, the frame is completed synchronously and dumped.
int run_frame(sift_hip_detector* d, const void* img, int pitch, int fmt, hipEvent_t consumed, int nf = 1,
              long sfs = 0, bool numbered = false) {
    const long long f = d->submitted;
    Lane& L = d->lane();
    const int slot = (int)(L.launched % d->kSlots);
    const bool dump = !d->dgDir.empty() && nf == 1 && d->firstFrame > 0;
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    if (dump) {
        if (!d->dDg && hipMalloc((void**)&d->dDg, sizeof(float) * (size_t)W * H) != hipSuccess)
            return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the stage-dump input failed");
        if (fmt == SIFT_HIP_U8)
            launch_u8_to_f32((const uint8_t*)img, pitch, W, H, d->dDg, W, Frames{1, 0}, 0, d->stream);
        else
            HIPCHK(hipMemcpy2DAsync(d->dDg, sizeof(float) * W, img, sizeof(float) * (size_t)pitch, sizeof(float) * W,
                                    H, hipMemcpyDefault, d->stream));
    }
    const bool graphs = d->useGraph && !d->timing;
    hipGraphExec_t gh = !graphs || consumed || fmt != SIFT_HIP_F32 ? nullptr
                        : nf == d->B                                 ? L.execH[slot]
                        : nf == 1                                    ? L.execH1[slot]
                                                                     : nullptr;
    // The head node of execH[slot] is re-pointed only once that exec's last
    // launch (whose completion evFrame[slot] still records) has finished: a
    // queued launch never sees its kernel arguments change.  Otherwise the
    // frame takes the separate head launch and the plain exec.
    if (gh && !event_done(L.evFrame[slot])) gh = nullptr;
    if (gh) {  // device f32 input: one launch for the whole frame, the head re-pointed at img
        const Lane::HeadIn in{img, pitch, sfs};
        Lane::HeadIn& cur = L.headIn[slot][nf == d->B ? 0 : 1];
        if (!(cur == in)) {
            HeadNode& h = d->headNode;
            head_node(d, h, static_cast<const float*>(img), pitch, slot & 1, nf, sfs);
            HIPCHK(hipGraphExecKernelNodeSetParams(gh, nf == d->B ? L.headH[slot] : L.headH1[slot], &h.p));
            cur = in;
        }
        HIPCHK(hipGraphLaunch(gh, d->stream));
    } else {
        enqueue_head(d, img, pitch, fmt, slot & 1, nf, sfs);
        if (consumed) HIPCHK(hipEventRecord(consumed, d->stream));
        hipGraphExec_t g = nf == d->B ? L.exec[slot] : (nf == 1 ? L.exec1[slot] : nullptr);
        if (graphs && g) {
            HIPCHK(hipGraphLaunch(g, d->stream));
        } else {  // timing mode, or a partial batch: the same launches, eagerly
            enqueue_body(d, slot, nf);
        }
    }
    HIPCHK(hipEventRecord(L.evFrame[slot], d->stream));
    const int nums = numbered ? nf : 1;
    L.nfOf[slot] = nf;
    L.slotFrame[slot] = f;
    L.slotNum[slot] = nums;
    L.launched++;
    L.last = f + nums - 1;
    for (int i = 0; i < nums; i++) d->frec(f + i) = sift_hip_detector::FrameRec{d->ln, slot, i};
    d->submitted = f + nums;
    if (dump) {
        HIPCHK(hipStreamSynchronize(d->stream));
        if (d->timing) d->collect_timing();
        d->current = f;
        d->curLane = d->ln;
        d->curIdx = 0;
        d->cur = slot;
        complete_counts(d);
        return dump_stage_files(d);
    }
    return SIFT_HIP_OK;
}

// Exposes frame f through the result accessors (and binds its lane).  Its
// counts are read once the frame is complete (complete_counts).
void make_current(sift_hip_detector* d, long long f) {
    d->current = f;
    d->curLane = d->frec(f).lane;
    d->curIdx = d->frec(f).idx;
    d->cur = d->frec(f).slot;
    d->countsValid = false;
    bind_lane(d, d->curLane, d->curIdx);
}

void complete_counts(sift_hip_detector* d) {
    const long long f = d->current;
    auto n = [&](long long g) {
        return g < d->firstFrame ? 0 : (int)std::min<unsigned>(frame_counters(d, g).final_n, d->kp.capFinal);
    };
    d->count = n(f);
    d->prevCount = n(f - 1);
    d->countsValid = true;
}

// Counts of the current launch group are read from the pinned host copies its
// last kernel writes: an accessor called before sift_hip_sync / sift_hip_wait
// (e.g. straight after sift_hip_detect_device) first waits for that group.  The
// previous frame may run on another lane: its counts are waited for too.
int ensure_counts(sift_hip_detector* d) {
    if (d->countsValid) return SIFT_HIP_OK;
    for (long long g : {d->current - 1, d->current})
        if (g >= d->firstFrame) {
            const auto& r = d->frec(g);
            HIPCHK(hipEventSynchronize(d->lanes[r.lane].evFrame[r.slot]));
        }
    complete_counts(d);
    return SIFT_HIP_OK;
}

int sync_lanes(sift_hip_detector* d) {
    for (int k = 0; k < d->nLanes; k++) HIPCHK(hipStreamSynchronize(d->lanes[k].stream));
    if (d->timing) d->collect_timing();
    return SIFT_HIP_OK;
}

int run_group(sift_hip_detector* d);

int finish_frame(sift_hip_detector* d) {
    if (int rc = run_group(d)) return rc;
    if (int rc = sync_lanes(d)) return rc;
    if (d->submitted > 0) {
        make_current(d, d->submitted - 1);
        complete_counts(d);
    }
    return SIFT_HIP_OK;
}

int copy_stream(sift_hip_detector* d, hipStream_t* s) {
    if (!d->copyStream) HIPCHK(hipStreamCreateWithFlags(&d->copyStream, hipStreamNonBlocking));
    *s = d->copyStream;
    return SIFT_HIP_OK;
}

int format_size(int fmt) { return fmt == SIFT_HIP_U8 ? 1 : (fmt == SIFT_HIP_F32 ? 4 : 0); }

// Frames in flight past `current` (host-input and device submits): at most 2
// per lane the handle may use.
int check_in_flight(sift_hip_detector* d) {
    if (d->submitted + d->npend > d->current + 2LL * d->maxLanes * d->mb)
        return fail(SIFT_HIP_ERR_STATE, "every lane already has two launch groups in flight past the current frame: sift_hip_wait first");
    return SIFT_HIP_OK;
}

// Host results region of a lane slot: kpts3 | feats4 | descriptors at capacity.
size_t host_res_bytes(const sift_hip_detector* d) {
    const size_t c = d->kp.capFinal;
    return ((12 * c + 255) & ~(size_t)255) + 16 * c + 256 * c;
}
void host_res(const sift_hip_detector* d, char* base, int region, float** k3, float** f4, uint16_t** desc) {
    const size_t c = d->kp.capFinal;
    char* p = base + host_res_bytes(d) * region;
    *k3 = reinterpret_cast<float*>(p);
    p += (12 * c + 255) & ~(size_t)255;
    *f4 = reinterpret_cast<float*>(p);
    *desc = reinterpret_cast<uint16_t*>(p + 16 * c);
}

// The lane's pinned results regions (kSlots x B) and the device table that
// points the descriptor kernel at them (HostOut), set up for every lane once a
// caller reads results back (sift_hip_copy_to_host / sift_hip_results_host
// turn hostWant on) and for lanes created after that: a lazy allocation
// inside a submit stalled it for ~14 ms.  The table goes in on the lane's
// stream (after its zeroing; frames launched earlier keep a null table).
int ensure_host_res(sift_hip_detector* d, Lane& L) {
    if (L.hRes) return SIFT_HIP_OK;
    const size_t nr = (size_t)d->kSlots * d->B, rb = host_res_bytes(d);
    HIPCHK(hipHostMalloc((void**)&L.hRes, rb * nr, hipHostMallocMapped | hipHostMallocCoherent));
    HIPCHK(hipHostGetDevicePointer((void**)&L.hResDev, L.hRes, 0));
    L.hostTab.resize(nr);
    for (size_t r = 0; r < nr; r++) L.hostTab[r] = L.hResDev + rb * r;
    HIPCHK(hipMemcpyAsync(L.dHostTab, L.hostTab.data(), sizeof(char*) * nr, hipMemcpyHostToDevice, L.stream));
    return SIFT_HIP_OK;
}

// A host-input frame's results request (the word its staging copy sets:
// arena i's Counters.pad[1], HostOut): null unless a caller reads results back.
unsigned* host_request(sift_hip_detector* d, int i, unsigned* val) {
    *val = (unsigned)d->hostWant << kHostReqShift;
    return d->hostWant ? &fptr(d->dCtr, (long)i * d->afs)->pad[1] : nullptr;
}

// After host-input frame f (arena i of its launch group) was launched with a
// request: its results land in the lane's region slot * B + i.
void mark_host_results(sift_hip_detector* d, long long f) {
    if (!d->hostWant) return;
    const auto& r = d->frec(f);
    Lane& L = d->lanes[r.lane];
    const int region = r.slot * d->B + r.idx;
    L.hostFrame[region] = f;
    L.hostDesc[region] = d->hostWant > 1;
}

int run_group(sift_hip_detector* d);

// A host frame on a micro-batching handle: into the next pinned staging slot
// of the handle's ring (the caller's buffer is free on return), pending until
// its group runs (run_group copies it to the lane's group input).
int queue_host(sift_hip_detector* d, const void* img, size_t stride, int fmt, long long* ticket) {
    const int es = format_size(fmt), H = d->cfg.row_width;
    const size_t rowB = (size_t)es * d->cfg.col_width, pitchB = (size_t)es * d->inPitch;
    if (d->npend && d->pend[0].fmt != fmt)
        if (int rc = run_group(d)) return rc;
    if (d->hstSlotBytes < pitchB * H) {  // first host frame, or a larger format: (re)allocate the block
        if (int rc = run_group(d)) return rc;
        if (int rc = sync_lanes(d)) return rc;  // no copy kernel still reads the old block
        if (d->hstBlock) HIPCHK(hipHostFree(d->hstBlock));
        d->hstBlock = nullptr;
        d->hstSlotBytes = 0;
        d->hstSlots = (2 * d->maxLanes + 1) * d->mb;  // frames pending or queued on the lanes
        if (hipHostMalloc((void**)&d->hstBlock, pitchB * H * d->hstSlots, hipHostMallocMapped | hipHostMallocNonCoherent) !=
            hipSuccess)
            return fail(SIFT_HIP_ERR_NOMEM, "hipHostMalloc of the micro-batch host staging failed");
        d->hstSlotBytes = pitchB * H;
        while ((int)d->hstRead.size() < d->hstSlots) {
            hipEvent_t e;
            HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
            d->hstRead.push_back(e);
        }
    }
    const int hs = (int)(d->hstNext++ % d->hstSlots);
    HIPCHK(hipEventSynchronize(d->hstRead[hs]));  // the copy kernel that last read the slot has run
    char* slot = d->hstBlock + d->hstSlotBytes * hs;
    if (!d->pool && rowB * H >= (1u << 20)) d->pool = new CopyPool(kCopyWorkers);
    copy_rows(d->pool, slot, pitchB, (const char*)img, stride, rowB, H);
    void* dev = nullptr;
    HIPCHK(hipHostGetDevicePointer(&dev, slot, 0));
    const int i = d->npend;
    d->pend[i] = sift_hip_detector::PendingFrame{dev, pitchB, fmt, false, hs};
    d->npend = i + 1;
    if (ticket) *ticket = d->submitted + i;
    return d->npend == d->mb ? run_group(d) : SIFT_HIP_OK;
}

// Host frame -> the lane's pinned staging (the caller's buffer is free on
// return) -> device staging by a small-grid copy kernel on the lane's stream
// -> pipeline on the frame's lane -> results to pinned host memory.  On a
// micro-batching handle the frame joins the pending group (queue_host).
int submit_host(sift_hip_detector* d, const void* img, size_t stride, int fmt, long long* ticket) {
    const int es = format_size(fmt);
    if (!es) return fail(SIFT_HIP_ERR_INVALID, "unknown pixel format");
    if (!img) return fail(SIFT_HIP_ERR_INVALID, "null image");
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    const size_t rowB = (size_t)es * W, pitchB = (size_t)es * d->inPitch;
    if (stride == 0) stride = rowB;
    if (stride < rowB) return fail(SIFT_HIP_ERR_INVALID, "row stride smaller than width");
    if (int rc = check_in_flight(d)) return rc;
    if (d->mb > 1 && d->dgDir.empty() && !d->timing) return queue_host(d, img, stride, fmt, ticket);
    if (int rc = run_group(d)) return rc;  // pending micro-batch frames keep their submission order
    if (int rc = pick_lane(d)) return rc;
    Lane& L = d->lane();
    const int k = (int)(L.uploads & 1);
    HIPCHK(hipEventSynchronize(L.evRead[k]));  // staging slot k no longer being read (the lane's frame before last)
    if (!d->pool && rowB * H >= (1u << 20)) d->pool = new CopyPool(kCopyWorkers);
    copy_rows(d->pool, (char*)L.hStage[k], pitchB, (const char*)img, stride, rowB, H);
    void* src = nullptr;
    HIPCHK(hipHostGetDevicePointer(&src, L.hStage[k], 0));
    const size_t inBytes = sizeof(float) * (size_t)d->inPitch * H;
    if (!L.dStage[k] && hipMalloc(&L.dStage[k], inBytes) != hipSuccess)
        return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the device staging failed");
    unsigned req = 0;
    unsigned* reqAt = d->dgDir.empty() ? host_request(d, 0, &req) : nullptr;
    launch_copy_rows(src, pitchB, L.dStage[k], pitchB, pitchB, H, kStageWg, d->stream, reqAt, req);
    HIPCHK(hipEventRecord(L.evRead[k], d->stream));  // host slot k read; device slot k is stream-ordered
    L.uploads++;
    d->uploads++;
    const long long f = d->submitted;
    if (int rc = run_frame(d, L.dStage[k], d->inPitch, fmt, nullptr)) return rc;
    if (reqAt) mark_host_results(d, f);
    if (ticket) *ticket = f;
    return SIFT_HIP_OK;
}

// The pending micro-batch frames as one launch group on a lane: each frame's
// rows are copied (device to device by launch_copy_rows, on the lane's stream after the caller's
// stream event) into the lane's micro-batch input at a fixed frame stride, and
// the group runs the B-frame graphs (a partial group: the 1-frame graphs, or
// the same launches eagerly), frame d->submitted + i in arena i.
int run_group(sift_hip_detector* d) {
    const int n = d->npend;
    if (!n) return SIFT_HIP_OK;
    if (int rc = pick_lane(d)) return rc;
    Lane& L = d->lane();
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    const size_t fb = sizeof(float) * (size_t)d->inPitch * H;  // one frame of f32 rows (an 8-bit frame uses a quarter)
    if (!L.mbIn && hipMalloc((void**)&L.mbIn, fb * d->mb) != hipSuccess)
        return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the micro-batch input failed");
    const int fmt = d->pend[0].fmt, es = format_size(fmt);
    bool host[sift_hip_detector::kMaxMicroBatch] = {};
    for (int i = 0; i < n; i++) {
        const auto& p = d->pend[i];
        if (p.ordered) HIPCHK(hipStreamWaitEvent(d->stream, d->evPend[i], 0));
        if (p.hslot >= 0) {  // pinned staging: whole pitch rows over PCIe by a small grid
            unsigned req;
            unsigned* reqAt = host_request(d, i, &req);
            launch_copy_rows(p.img, p.stride, L.mbIn + fb * i, p.stride, p.stride, H, kStageWg, d->stream, reqAt, req);
            HIPCHK(hipEventRecord(d->hstRead[p.hslot], d->stream));
            host[i] = reqAt != nullptr;
        } else {
            launch_copy_rows(p.img, p.stride, L.mbIn + fb * i, (size_t)es * d->inPitch, (size_t)es * W, H,
                             kGroupCopyWg, d->stream);
        }
    }
    d->npend = 0;
    const long long f = d->submitted;
    if (int rc = run_frame(d, L.mbIn, d->inPitch, fmt, nullptr, n, (long)fb, true)) return rc;
    for (int i = 0; i < n; i++)
        if (host[i]) mark_host_results(d, f + i);
    return SIFT_HIP_OK;
}

// Device frame (HBM-resident, fp32 or u8) -> the frame's lane; the lane waits
// for `stream` (the caller's producer) before reading it.  `queue`: a single
// frame of sift_hip_submit_device on a micro-batching handle joins the pending
// group instead (one format per group: a frame of the other format flushes it).
int submit_device(sift_hip_detector* d, const void* img, size_t stride, int fmt, void* stream, int nf, size_t fstride,
                  long long* ticket, bool queue = false) {
    hipStream_t ext = (hipStream_t)stream;
    if (queue && d->mb > 1 && nf == 1 && d->dgDir.empty() && !d->timing) {
        if (d->npend && d->pend[0].fmt != fmt)
            if (int rc = run_group(d)) return rc;
        const int i = d->npend;
        if (ext) {
            if (!d->evPend[i]) HIPCHK(hipEventCreateWithFlags(&d->evPend[i], hipEventDisableTiming));
            HIPCHK(hipEventRecord(d->evPend[i], ext));
        }
        d->pend[i] = sift_hip_detector::PendingFrame{img, stride, fmt, ext != nullptr, -1};
        d->npend = i + 1;
        if (ticket) *ticket = d->submitted + i;
        return d->npend == d->mb ? run_group(d) : SIFT_HIP_OK;
    }
    if (int rc = run_group(d)) return rc;  // frames are numbered (and launched) in submission order
    if (int rc = pick_lane(d)) return rc;
    if (ext) {
        HIPCHK(hipEventRecord(d->evIn, ext));
        HIPCHK(hipStreamWaitEvent(d->stream, d->evIn, 0));
    }
    const long long f = d->submitted;
    if (int rc = run_frame(d, img, (int)(stride / format_size(fmt)), fmt, nullptr, nf, (long)fstride)) return rc;
    if (ticket) *ticket = f;
    return SIFT_HIP_OK;
}

int wait_frame(sift_hip_detector* d, long long f) {
    if (f >= d->submitted && f < d->submitted + d->npend)
        if (int rc = run_group(d)) return rc;  // a pending micro-batch frame: launch the partial group now
    if (f < d->firstFrame || f >= d->submitted || f < d->submitted - kFrameRing)
        return fail(SIFT_HIP_ERR_INVALID, "unknown frame ticket");
    const auto& r = d->frec(f);
    Lane& L = d->lanes[r.lane];
    if (L.slotFrame[r.slot] < 0 || f < L.slotFrame[r.slot] || f >= L.slotFrame[r.slot] + std::max(L.slotNum[r.slot], 1))
        return fail(SIFT_HIP_ERR_STATE, "frame results already recycled");
    if (d->timing) {
        if (int rc = sync_lanes(d)) return rc;
    } else {
        HIPCHK(hipEventSynchronize(L.evFrame[r.slot]));
        if (f - 1 >= d->firstFrame) {  // prev_descriptor may come from another lane
            const auto& p = d->frec(f - 1);
            HIPCHK(hipEventSynchronize(d->lanes[p.lane].evFrame[p.slot]));
        }
    }
    make_current(d, f);
    complete_counts(d);
    return SIFT_HIP_OK;
}

// Stage dumps of the current frame (Detector::setDataGen, reference
// Detector.cu:145-229 / PerfData.cuh): raw little-endian row-major files plus a
// meta.json describing them; tests/stage_check.py replays them against the CPU
// oracle (and against this library).
// mkdir -p
bool make_dirs(const std::string& path) {
    for (size_t i = 1; i <= path.size(); i++)
        if (i == path.size() || path[i] == '/') {
            const std::string p = path.substr(0, i);
            if (mkdir(p.c_str(), 0755) != 0 && errno != EEXIST) return false;
        }
    return true;
}

int write_file(const std::string& path, const void* data, size_t bytes) {
    FILE* fp = fopen(path.c_str(), "wb");
    if (!fp) return fail(SIFT_HIP_ERR_INVALID, "cannot write " + path);
    const size_t n = bytes ? fwrite(data, 1, bytes, fp) : 0;
    fclose(fp);
    if (n != bytes) return fail(SIFT_HIP_ERR_INVALID, "short write to " + path);
    return SIFT_HIP_OK;
}

// Portable descriptor jobs: the plane pointer becomes the plane index
// o * (L + 3) + layer (the replaying handle has its own arena).
int job_plane(const sift_hip_detector* d, const float* img) {
    for (int o = 0; o < d->nOct; o++) {
        const OctGeom& g = d->pyr.oct[o];
        for (int l = 0; l < d->L + 3; l++)
            if (img == g.base + (size_t)l * g.planeStride) return o * (d->L + 3) + l;
    }
    return -1;
}

// refined.rec (RefKpt), oriented.rec (OriKpt slots incl. holes), jobs.rec
// (DescJob, plane index in place of the pointer), range.u32 (the frame's
// pixel-range keys), counters.u32 (Counters): frame 0 of the arena, after the
// frame completed (nothing reuses these buffers before the next frame).
int dump_records(sift_hip_detector* d, const std::string& dir) {
    const Counters& c = d->hCtr[(size_t)d->cur * d->B];
    const size_t nRef = std::min<unsigned>(c.refined, d->kp.capRefined);
    const size_t nOri = std::min<size_t>(nRef + c.oriented, d->kp.capOriented);
    const size_t nFin = std::min<unsigned>(c.final_n, d->kp.capFinal);
    std::vector<RefKpt> ref(nRef);
    std::vector<OriKpt> ori(nOri);
    std::vector<DescJob> jobs(nFin);
    std::vector<unsigned> range(2 * kRangeSlots);
    if (nRef) HIPCHK(hipMemcpy(ref.data(), d->dRef, sizeof(RefKpt) * nRef, hipMemcpyDeviceToHost));
    if (nOri) HIPCHK(hipMemcpy(ori.data(), d->dOri, sizeof(OriKpt) * nOri, hipMemcpyDeviceToHost));
    if (nFin) HIPCHK(hipMemcpy(jobs.data(), d->dJobs, sizeof(DescJob) * nFin, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(range.data(), range_keys(d, d->cur & 1), sizeof(unsigned) * range.size(), hipMemcpyDeviceToHost));
    for (DescJob& j : jobs) {
        const long long plane = job_plane(d, j.img);
        std::memcpy(&j.img, &plane, sizeof plane);
    }
    if (int rc = write_file(dir + "/refined.rec", ref.data(), sizeof(RefKpt) * nRef)) return rc;
    if (int rc = write_file(dir + "/oriented.rec", ori.data(), sizeof(OriKpt) * nOri)) return rc;
    if (int rc = write_file(dir + "/jobs.rec", jobs.data(), sizeof(DescJob) * nFin)) return rc;
    if (int rc = write_file(dir + "/range.u32", range.data(), sizeof(unsigned) * range.size())) return rc;
    return write_file(dir + "/counters.u32", &c, sizeof(Counters));
}

int dump_stage_files(sift_hip_detector* d) {
    const std::string& dir = d->dgDir;
    if (!make_dirs(dir)) return fail(SIFT_HIP_ERR_INVALID, "cannot create " + dir);
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    std::vector<float> buf((size_t)W * H);
    HIPCHK(hipMemcpy(buf.data(), d->dDg, sizeof(float) * buf.size(), hipMemcpyDeviceToHost));
    if (int rc = write_file(dir + "/input.f32", buf.data(), sizeof(float) * buf.size())) return rc;
    std::string octs;
    for (int o = 0; o < d->nOct; o++) {
        const OctGeom& g = d->pyr.oct[o];
        std::vector<float> plane((size_t)g.W * g.H);
        for (int l = 0; l < d->L + 3; l++) {
            HIPCHK(hipMemcpy2D(plane.data(), sizeof(float) * g.W, g.base + (size_t)l * g.planeStride,
                               sizeof(float) * g.pitch, sizeof(float) * g.W, g.H, hipMemcpyDeviceToHost));
            char name[64];
            snprintf(name, sizeof name, "/gauss_o%d_l%d.f32", o, l);
            if (int rc = write_file(dir + name, plane.data(), sizeof(float) * plane.size())) return rc;
        }
        char e[64];
        snprintf(e, sizeof e, "%s[%d, %d]", o ? ", " : "", g.W, g.H);
        octs += e;
    }
    const Counters& c = d->hCtr[(size_t)d->cur * d->B];
    const int nc = (int)std::min<unsigned>(c.cand, d->capCand);
    std::vector<uint2> cand(nc);
    std::vector<int> quads(4 * (size_t)nc);
    if (nc) HIPCHK(hipMemcpy(cand.data(), d->dCand, sizeof(uint2) * nc, hipMemcpyDeviceToHost));
    for (int i = 0; i < nc; i++) {
        quads[4 * i] = (int)(cand[i].x >> 8);
        quads[4 * i + 1] = (int)(cand[i].x & 255);
        quads[4 * i + 2] = (int)(cand[i].y >> 16);
        quads[4 * i + 3] = (int)(cand[i].y & 0xffff);
    }
    if (int rc = write_file(dir + "/candidates.i32", quads.data(), sizeof(int) * quads.size())) return rc;
    const int n = d->count;
    std::vector<float> k3(3 * (size_t)n), f4(4 * (size_t)n);
    std::vector<uint16_t> desc(128 * (size_t)n);
    if (n) {
        HIPCHK(hipMemcpy(k3.data(), d->dKpts3[d->cur], sizeof(float) * k3.size(), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(f4.data(), d->dFeats4[d->cur], sizeof(float) * f4.size(), hipMemcpyDeviceToHost));
        HIPCHK(hipMemcpy(desc.data(), d->dDesc[d->cur], sizeof(uint16_t) * desc.size(), hipMemcpyDeviceToHost));
    }
    if (int rc = write_file(dir + "/kpts3.f32", k3.data(), sizeof(float) * k3.size())) return rc;
    if (int rc = write_file(dir + "/feats4.f32", f4.data(), sizeof(float) * f4.size())) return rc;
    if (int rc = write_file(dir + "/desc.f16", desc.data(), sizeof(uint16_t) * desc.size())) return rc;
    // The keypoint stages' own device records (inputs of sift_hip_replay_stage).
    if (int rc = dump_records(d, dir)) return rc;
    const sift_hip_config& g = d->cfg;
    char meta[4096];
    snprintf(meta, sizeof meta,
             "{\n \"format\": \"sift_hip stage dump 2\",\n \"frame\": %lld,\n \"width\": %d,\n \"height\": %d,\n"
             " \"config\": {\"numFeatures\": %d, \"numOctaveLayers\": %d, \"contrastThreshould\": %.17g,"
             " \"edgeThreshould\": %.17g, \"sigma\": %.17g, \"upscale\": %d, \"numOctaves\": %d},\n"
             " \"octaves\": [%s],\n \"planes_per_octave\": %d,\n \"candidates\": %d,\n \"keypoints\": %d,\n"
             " \"overflow\": %u,\n"
             " \"files\": {\"input.f32\": \"float32 [height][width], the frame as the pipeline read it\",\n"
             "  \"gauss_o<o>_l<l>.f32\": \"float32 [h_o][w_o], Gaussian plane l of octave o\",\n"
             "  \"candidates.i32\": \"int32 [candidates][4] (octave, layer, row, col) of the 3x3x3 extrema, unordered\",\n"
             "  \"kpts3.f32\": \"float32 [keypoints][3] {x, y, layer}\",\n"
             "  \"feats4.f32\": \"float32 [keypoints][4] {packed octave, size, response, angle}\",\n"
             "  \"desc.f16\": \"float16 [keypoints][128], integers 0..255\",\n"
             "  \"refined.rec\": \"RefKpt [refined] {f32 x, y, size, response; i32 octave, o, layer, r << 16 | c}\",\n"
             "  \"oriented.rec\": \"OriKpt [slots] {f32 x, y, size, angle, response; i32 octave, bucket, sub}; "
             "bucket 0xffffffff = hole\",\n"
             "  \"jobs.rec\": \"DescJob [keypoints] 64 B {i64 plane o*(L+3)+layer; f32 cos_t, sin_t, angle, hist_width; "
             "i32 ptx, pty, rows, cols, pitch, radius, out (the output row), pad[3]}; exact mode: largest windows first\",\n"
             "  \"range.u32\": \"u32 [2][%d] pixel-range keys of the frame\",\n"
             "  \"counters.u32\": \"u32 [8] {cand, refined, oriented, final, overflow, retainBest threshold bits, "
             "order entries, 0}\"}\n}\n",
             d->current - d->firstFrame, g.col_width, g.row_width, g.numFeatures, g.numOctaveLayers,
             g.contrastThreshould, g.edgeThreshould, g.sigma, g.upscale, d->nOct, octs.c_str(), d->L + 3, nc, n,
             c.overflow, kRangeSlots);
    return write_file(dir + "/meta.json", meta, strlen(meta));
}

// ---------------------------------------------------------------------------
// Per-stage replay (sift_hip_replay_stage): one stage of the pipeline on a
// dump's recorded input, as the reference's tool/perf.cu:43-100 runs each
// HostInterface.hh:11-69 stage on a snapshot.  Runs on frame 0's arena.
// ---------------------------------------------------------------------------
template <class T>
int read_vec(const std::string& path, std::vector<T>& v) {
    FILE* fp = fopen(path.c_str(), "rb");
    if (!fp) return fail(SIFT_HIP_ERR_INVALID, "cannot read " + path);
    fseek(fp, 0, SEEK_END);
    const long bytes = ftell(fp);
    fseek(fp, 0, SEEK_SET);
    if (bytes < 0 || bytes % (long)sizeof(T)) {
        fclose(fp);
        return fail(SIFT_HIP_ERR_INVALID, path + ": size is not a whole number of records");
    }
    v.resize((size_t)bytes / sizeof(T));
    const size_t got = bytes ? fread(v.data(), 1, (size_t)bytes, fp) : 0;
    fclose(fp);
    if (got != (size_t)bytes) return fail(SIFT_HIP_ERR_INVALID, "short read of " + path);
    return SIFT_HIP_OK;
}

int upload_planes(sift_hip_detector* d, const std::string& dir) {
    for (int o = 0; o < d->nOct; o++) {
        const OctGeom& g = d->pyr.oct[o];
        for (int l = 0; l < d->L + 3; l++) {
            char name[64];
            snprintf(name, sizeof name, "/gauss_o%d_l%d.f32", o, l);
            std::vector<float> p;
            if (int rc = read_vec(dir + name, p)) return rc;
            if (p.size() != (size_t)g.W * g.H)
                return fail(SIFT_HIP_ERR_INVALID, dir + name + ": plane size differs from this handle's octave geometry");
            HIPCHK(hipMemcpy2D(g.base + (size_t)l * g.planeStride, sizeof(float) * g.pitch, p.data(), sizeof(float) * g.W,
                               sizeof(float) * g.W, g.H, hipMemcpyHostToDevice));
        }
    }
    return SIFT_HIP_OK;
}

int write_planes(sift_hip_detector* d, const std::string& dir) {
    for (int o = 0; o < d->nOct; o++) {
        const OctGeom& g = d->pyr.oct[o];
        std::vector<float> plane((size_t)g.W * g.H);
        for (int l = 0; l < d->L + 3; l++) {
            HIPCHK(hipMemcpy2D(plane.data(), sizeof(float) * g.W, g.base + (size_t)l * g.planeStride,
                               sizeof(float) * g.pitch, sizeof(float) * g.W, g.H, hipMemcpyDeviceToHost));
            char name[64];
            snprintf(name, sizeof name, "/gauss_o%d_l%d.f32", o, l);
            if (int rc = write_file(dir + name, plane.data(), sizeof(float) * plane.size())) return rc;
        }
    }
    return SIFT_HIP_OK;
}

// Returns the handle to its post-warm-up state: every scratch invariant the
// kernels keep (zeroed counters, range keys, dedupe bitmap) restored by one
// memset of the arenas; the handle has no current frame afterwards.
int replay_reset(sift_hip_detector* d) {
    bind_lane(d, 0);
    HIPCHK(hipMemsetAsync(d->lanes[0].arena, 0, (size_t)d->afs * d->B, d->stream));
    if (int rc = sync_lanes(d)) return rc;
    d->firstFrame = d->submitted;
    d->current = d->submitted - 1;
    d->curLane = 0;
    d->curIdx = 0;
    d->cur = 0;
    d->count = d->prevCount = 0;
    d->countsValid = true;
    return SIFT_HIP_OK;
}

// The stage itself (replay_stage below owns the handle's state around it:
// every return from here, error or not, is followed by the restore).
int replay_stage_body(sift_hip_detector* d, const std::string& in, const std::string& stage, const std::string& out) {
    std::vector<Counters> dumped;  // the frame's final counters
    if (stage != "pyramid" && stage != "extrema") {
        if (int rc = read_vec(in + "/counters.u32", dumped)) return rc;
        if (dumped.size() != 1) return fail(SIFT_HIP_ERR_INVALID, "counters.u32: expected one Counters record");
    }
    Counters c{};
    int rc = SIFT_HIP_OK;
    hipStream_t s = d->stream;
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    if (stage == "pyramid") {
        std::vector<float> img;
        if ((rc = read_vec(in + "/input.f32", img))) return rc;
        if (img.size() != (size_t)W * H) return fail(SIFT_HIP_ERR_INVALID, "input.f32: size differs from the config");
        HIPCHK(hipMemcpy2D(d->dInput, sizeof(float) * d->inPitch, img.data(), sizeof(float) * W, sizeof(float) * W, H,
                           hipMemcpyHostToDevice));
        enqueue_head(d, d->dInput, d->inPitch, SIFT_HIP_F32, 0, 1, d->afs);
        enqueue_pyramid(d, 1, 0);
        HIPCHK(hipStreamSynchronize(s));
        rc = write_planes(d, out);
    } else if ((rc = upload_planes(d, in))) {
        return rc;
    } else if (stage == "extrema") {
        enqueue_extrema(d, 1);
        HIPCHK(hipMemcpyAsync(&c, d->dCtr, sizeof c, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const int nc = (int)std::min<unsigned>(c.cand, d->capCand);
        std::vector<uint2> cand(nc);
        std::vector<int> quads(4 * (size_t)nc);
        if (nc) HIPCHK(hipMemcpy(cand.data(), d->dCand, sizeof(uint2) * nc, hipMemcpyDeviceToHost));
        for (int i = 0; i < nc; i++) {
            quads[4 * i] = (int)(cand[i].x >> 8);
            quads[4 * i + 1] = (int)(cand[i].x & 255);
            quads[4 * i + 2] = (int)(cand[i].y >> 16);
            quads[4 * i + 3] = (int)(cand[i].y & 0xffff);
        }
        rc = write_file(out + "/candidates.i32", quads.data(), sizeof(int) * quads.size());
    } else if (stage == "refine") {
        std::vector<int> quads;
        if ((rc = read_vec(in + "/candidates.i32", quads))) return rc;
        const size_t nc = quads.size() / 4;
        if (nc > d->capCand) return fail(SIFT_HIP_ERR_INVALID, "candidates.i32: more candidates than the capacity");
        std::vector<uint2> cand(nc);
        for (size_t i = 0; i < nc; i++)
            cand[i] = make_uint2((unsigned)(quads[4 * i] << 8 | quads[4 * i + 1]),
                                 (unsigned)(quads[4 * i + 2] << 16 | quads[4 * i + 3]));
        if (nc) HIPCHK(hipMemcpy(d->dCand, cand.data(), sizeof(uint2) * nc, hipMemcpyHostToDevice));
        c.cand = (unsigned)nc;
        HIPCHK(hipMemcpy(d->dCtr, &c, sizeof c, hipMemcpyHostToDevice));
        enqueue_refine(d, 1);
        HIPCHK(hipMemcpyAsync(&c, d->dCtr, sizeof c, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const size_t n = std::min<unsigned>(c.refined, d->kp.capRefined);
        std::vector<RefKpt> ref(n);
        if (n) HIPCHK(hipMemcpy(ref.data(), d->dRef, sizeof(RefKpt) * n, hipMemcpyDeviceToHost));
        rc = write_file(out + "/refined.rec", ref.data(), sizeof(RefKpt) * n);
    } else if (stage == "orientation") {
        std::vector<RefKpt> ref;
        if ((rc = read_vec(in + "/refined.rec", ref))) return rc;
        if (ref.size() > d->kp.capRefined) return fail(SIFT_HIP_ERR_INVALID, "refined.rec: above the capacity");
        if (!ref.empty()) HIPCHK(hipMemcpy(d->dRef, ref.data(), sizeof(RefKpt) * ref.size(), hipMemcpyHostToDevice));
        c.cand = dumped[0].cand;
        c.refined = (unsigned)ref.size();
        HIPCHK(hipMemcpy(d->dCtr, &c, sizeof c, hipMemcpyHostToDevice));
        enqueue_orientation(d, 1);
        HIPCHK(hipMemcpyAsync(&c, d->dCtr, sizeof c, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const size_t n = std::min<size_t>(ref.size() + c.oriented, d->kp.capOriented);
        std::vector<OriKpt> ori(n);
        if (n) HIPCHK(hipMemcpy(ori.data(), d->dOri, sizeof(OriKpt) * n, hipMemcpyDeviceToHost));
        rc = write_file(out + "/oriented.rec", ori.data(), sizeof(OriKpt) * n);
    } else if (stage == "order") {
        std::vector<OriKpt> ori;
        if ((rc = read_vec(in + "/oriented.rec", ori))) return rc;
        if (ori.size() > d->kp.capOriented) return fail(SIFT_HIP_ERR_INVALID, "oriented.rec: above the capacity");
        if (!ori.empty()) HIPCHK(hipMemcpy(d->dOri, ori.data(), sizeof(OriKpt) * ori.size(), hipMemcpyHostToDevice));
        c.cand = dumped[0].cand;
        c.refined = dumped[0].refined;
        c.oriented = dumped[0].oriented;
        HIPCHK(hipMemcpy(d->dCtr, &c, sizeof c, hipMemcpyHostToDevice));
        enqueue_order(d, 0, 1);
        HIPCHK(hipMemcpyAsync(&c, d->dCtr, sizeof c, hipMemcpyDeviceToHost, s));
        HIPCHK(hipStreamSynchronize(s));
        const size_t n = std::min<unsigned>(c.final_n, d->kp.capFinal);
        std::vector<float> k3(3 * n), f4(4 * n);
        std::vector<DescJob> jobs(n);
        if (n) {
            HIPCHK(hipMemcpy(k3.data(), d->dKpts3[0], sizeof(float) * k3.size(), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(f4.data(), d->dFeats4[0], sizeof(float) * f4.size(), hipMemcpyDeviceToHost));
            HIPCHK(hipMemcpy(jobs.data(), d->dJobs, sizeof(DescJob) * n, hipMemcpyDeviceToHost));
        }
        for (DescJob& j : jobs) {
            const long long plane = job_plane(d, j.img);
            std::memcpy(&j.img, &plane, sizeof plane);
        }
        if (!(rc = write_file(out + "/kpts3.f32", k3.data(), sizeof(float) * k3.size())) &&
            !(rc = write_file(out + "/feats4.f32", f4.data(), sizeof(float) * f4.size())))
            rc = write_file(out + "/jobs.rec", jobs.data(), sizeof(DescJob) * n);
    } else {  // descriptor
        std::vector<DescJob> jobs;
        std::vector<unsigned> range;
        if ((rc = read_vec(in + "/jobs.rec", jobs)) || (rc = read_vec(in + "/range.u32", range))) return rc;
        if (jobs.size() > d->kp.capFinal) return fail(SIFT_HIP_ERR_INVALID, "jobs.rec: above the capacity");
        if (range.size() != 2 * (size_t)kRangeSlots) return fail(SIFT_HIP_ERR_INVALID, "range.u32: wrong size");
        for (DescJob& j : jobs) {
            long long plane;
            std::memcpy(&plane, &j.img, sizeof plane);
            if (plane < 0 || plane >= (long long)d->nOct * (d->L + 3))
                return fail(SIFT_HIP_ERR_INVALID, "jobs.rec: plane index out of range");
            const OctGeom& g = d->pyr.oct[plane / (d->L + 3)];
            j.img = g.base + (size_t)(plane % (d->L + 3)) * g.planeStride;
        }
        if (!jobs.empty()) HIPCHK(hipMemcpy(d->dJobs, jobs.data(), sizeof(DescJob) * jobs.size(), hipMemcpyHostToDevice));
        HIPCHK(hipMemcpy(range_keys(d, 0), range.data(), sizeof(unsigned) * range.size(), hipMemcpyHostToDevice));
        c = dumped[0];
        c.final_n = (unsigned)jobs.size();
        c.pad[1] = 0;  // no host results request (HostOut)
        HIPCHK(hipMemcpy(d->dCtr, &c, sizeof c, hipMemcpyHostToDevice));
        enqueue_descriptor(d, 0, 1);
        HIPCHK(hipStreamSynchronize(s));
        std::vector<uint16_t> desc(128 * jobs.size());
        if (!jobs.empty()) HIPCHK(hipMemcpy(desc.data(), d->dDesc[0], sizeof(uint16_t) * desc.size(), hipMemcpyDeviceToHost));
        rc = write_file(out + "/desc.f16", desc.data(), sizeof(uint16_t) * desc.size());
    }
    return rc;
}

// One cleanup path: once the arenas may have been touched (uploads, kernels),
// the handle's timing mode and its post-warm-up scratch state (counters, the
// dedupe bitmap, range keys) are restored on every exit, including a failed
// read, capacity check, HIP call or output write, so the next frame starts
// clean.  The first error is the one returned (and kept in last_error).
int replay_stage(sift_hip_detector* d, const std::string& in, const std::string& stage, const std::string& out) {
    static const char* kStages[] = {"pyramid", "extrema", "refine", "orientation", "order", "descriptor"};
    bool known = false;
    for (const char* k : kStages) known |= stage == k;
    if (!known) return fail(SIFT_HIP_ERR_INVALID, "unknown stage '" + stage + "'");
    if (!make_dirs(out)) return fail(SIFT_HIP_ERR_INVALID, "cannot create " + out);
    HIPCHK(hipStreamSynchronize(d->stream));
    const bool timing = d->timing;
    d->timing = false;
    int rc = replay_reset(d);
    if (!rc) rc = replay_stage_body(d, in, stage, out);
    d->timing = timing;
    const int rc_reset = replay_reset(d);
    return rc ? rc : rc_reset;
}

// Every entry point starts bound to the current frame's lane (the accessors
// address it); submitting entry points re-bind to the lane they pick.
#define CHECK_HANDLE(h)                                                                       \
    do {                                                                                      \
        if (!(h)) return fail(SIFT_HIP_ERR_INVALID, "null handle");                          \
        if (!(h)->allocated || !(h)->nLanes)                                                  \
            return fail(SIFT_HIP_ERR_STATE, "sift_hip_warmup not called");                    \
        HIPCHK(hipSetDevice((h)->device));                                                    \
        bind_lane((h), (h)->curLane, (h)->curIdx);                                            \
    } while (0)

}  // namespace

extern "C" {

void sift_hip_default_config(sift_hip_config* c, int w, int h) {
    c->col_width = w;
    c->row_width = h;
    c->numFeatures = 5000;
    c->numOctaveLayers = 3;
    c->contrastThreshould = 0.04;
    c->edgeThreshould = 10;
    c->sigma = 1.6;
    c->upscale = 0;
    c->numOctaves = 0;
    c->maxKeypoints = 0;
}

const char* sift_hip_version(void) {
    static char buf[512];
    int rt = 0;
    (void)hipRuntimeGetVersion(&rt);
    const char* ab = build_flags();
    snprintf(buf, sizeof buf, "abi=%d arch=gfx950 hip=%d build=%s%s", SIFT_HIP_ABI_VERSION, rt, ab[0] ? "ab" : "default",
             ab);
    return buf;
}

const char* sift_hip_last_error(void) { return g_err.c_str(); }

int sift_hip_create(const sift_hip_config* cfg, int device, sift_hip_t* out) {
    if (!cfg || !out) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *out = nullptr;
    if (cfg->col_width <= 0 || cfg->row_width <= 0) return fail(SIFT_HIP_ERR_INVALID, "image width or height not set");
    if (cfg->col_width >= 65536 || cfg->row_width >= 65536)
        return fail(SIFT_HIP_ERR_INVALID, "image dimension >= 65536 unsupported");
    if (cfg->numOctaveLayers < 1 || cfg->numOctaveLayers > 32)
        return fail(SIFT_HIP_ERR_INVALID, "numOctaveLayers out of range");
    if (!(cfg->sigma > 0)) return fail(SIFT_HIP_ERR_INVALID, "sigma must be > 0");
    auto* d = new sift_hip_detector();
    d->cfg = *cfg;
    if (device < 0) {
        if (hipGetDevice(&d->device) != hipSuccess) d->device = 0;
    } else {
        d->device = device;
    }
    int rc = setup_geometry(d);
    if (rc) {
        delete d;
        return rc;
    }
    setup_taps(d);
    *out = d;
    return SIFT_HIP_OK;
}

int sift_hip_destroy(sift_hip_t h) {
    delete h;
    return SIFT_HIP_OK;
}

int sift_hip_warmup(sift_hip_t d) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (d->allocated) return d->nLanes ? SIFT_HIP_OK : fail(SIFT_HIP_ERR_STATE, "an earlier warm-up failed");
    if (d->mb > 1) {  // a micro-batch runs the lane's B-frame graphs
        if (d->B > 1 && d->B != d->mb)
            return fail(SIFT_HIP_ERR_INVALID, "micro-batch and batch size differ (set one, or both equal)");
        d->B = d->mb;
    }
    int rc = allocate(d);
    if (rc) return rc;
    rc = add_lane(d);  // lane 0; more lanes on demand (pick_lane)
    if (rc) return rc;
    // One blank frame (batch) through each graph: first-touch, code-object load.
    for (int i = 0; i < d->kSlots * (d->B > 1 ? 2 : 1); i++) {
        const int nf = i < d->kSlots ? d->B : 1;
        if ((rc = run_frame(d, d->dInput, d->inPitch, SIFT_HIP_F32, nullptr, nf, d->afs))) return rc;
        if ((rc = finish_frame(d))) return rc;
    }
    d->firstFrame = d->submitted;
    d->count = d->prevCount = 0;
    return SIFT_HIP_OK;
}

int sift_hip_num_octaves(sift_hip_t h, int* n) {
    if (!h || !n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *n = h->nOct;
    return SIFT_HIP_OK;
}

int sift_hip_octave_dims(sift_hip_t h, int o, int* w, int* hh, int* pitch) {
    if (!h || o < 0 || o >= h->nOct) return fail(SIFT_HIP_ERR_INVALID, "bad octave");
    if (w) *w = h->pyr.oct[o].W;
    if (hh) *hh = h->pyr.oct[o].H;
    if (pitch) *pitch = h->pyr.oct[o].pitch;
    return SIFT_HIP_OK;
}

int sift_hip_detect(sift_hip_t d, const float* img, size_t stride) {
    CHECK_HANDLE(d);
    long long f = 0;
    int rc = submit_host(d, img, stride, SIFT_HIP_F32, &f);
    return rc ? rc : wait_frame(d, f);
}

int sift_hip_detect_u8(sift_hip_t d, const uint8_t* img, size_t stride) {
    CHECK_HANDLE(d);
    long long f = 0;
    int rc = submit_host(d, img, stride, SIFT_HIP_U8, &f);
    return rc ? rc : wait_frame(d, f);
}

int sift_hip_submit(sift_hip_t d, const void* img, size_t stride, int format, long long* ticket) {
    CHECK_HANDLE(d);
    return submit_host(d, img, stride, format, ticket);
}

int sift_hip_wait(sift_hip_t d, long long ticket) {
    CHECK_HANDLE(d);
    return wait_frame(d, ticket);
}

int sift_hip_detect_device_fmt(sift_hip_t d, const void* img, size_t stride, int format, void* stream) {
    CHECK_HANDLE(d);
    if (!img) return fail(SIFT_HIP_ERR_INVALID, "null image");
    const int es = format_size(format);
    if (!es) return fail(SIFT_HIP_ERR_INVALID, "unknown pixel format");
    const int W = d->cfg.col_width;
    if (stride == 0) stride = (size_t)es * W;
    if (stride % es || stride < (size_t)es * W)
        return fail(SIFT_HIP_ERR_INVALID, "row stride must be a multiple of the pixel size and >= width");
    if (int rc = check_in_flight(d)) return rc;
    long long f = 0;
    if (int rc = submit_device(d, img, stride, format, stream, 1, 0, &f)) return rc;
    // Device-ordered consumers see this frame's buffers at once; counts
    // follow at sift_hip_sync / sift_hip_wait.
    make_current(d, f);
    if (stream) {
        HIPCHK(hipEventRecord(d->evOut, d->stream));
        HIPCHK(hipStreamWaitEvent((hipStream_t)stream, d->evOut, 0));
    }
    return SIFT_HIP_OK;
}

int sift_hip_submit_device(sift_hip_t d, const void* img, size_t stride, int format, void* stream, long long* ticket) {
    CHECK_HANDLE(d);
    if (!img) return fail(SIFT_HIP_ERR_INVALID, "null image");
    const int es = format_size(format);
    if (!es) return fail(SIFT_HIP_ERR_INVALID, "unknown pixel format");
    const int W = d->cfg.col_width;
    if (stride == 0) stride = (size_t)es * W;
    if (stride % es || stride < (size_t)es * W)
        return fail(SIFT_HIP_ERR_INVALID, "row stride must be a multiple of the pixel size and >= width");
    if (int rc = check_in_flight(d)) return rc;
    return submit_device(d, img, stride, format, stream, 1, 0, ticket, true);
}

int sift_hip_detect_device(sift_hip_t d, const float* img, size_t stride, void* stream) {
    return sift_hip_detect_device_fmt(d, img, stride, SIFT_HIP_F32, stream);
}

int sift_hip_set_batch(sift_hip_t d, int frames) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (frames < 1 || frames > kMaxBatch) return fail(SIFT_HIP_ERR_INVALID, "batch size out of range (1..64)");
    if (d->allocated) return fail(SIFT_HIP_ERR_STATE, "sift_hip_set_batch after sift_hip_warmup");
    d->B = frames;
    return SIFT_HIP_OK;
}

int sift_hip_set_lanes(sift_hip_t d, int lanes) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (lanes < 1 || lanes > kMaxLanes) return fail(SIFT_HIP_ERR_INVALID, "lanes out of range (1..4)");
    if (d->allocated) return fail(SIFT_HIP_ERR_STATE, "sift_hip_set_lanes after sift_hip_warmup");
    d->maxLanes = lanes;
    return SIFT_HIP_OK;
}

int sift_hip_set_micro_batch(sift_hip_t d, int frames) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (frames < 1 || frames > sift_hip_detector::kMaxMicroBatch)
        return fail(SIFT_HIP_ERR_INVALID, "micro-batch out of range (1..16)");
    if (d->allocated) return fail(SIFT_HIP_ERR_STATE, "sift_hip_set_micro_batch after sift_hip_warmup");
    d->mb = frames;
    return SIFT_HIP_OK;
}

int sift_hip_micro_batch(sift_hip_t d, int* frames) {
    if (!d || !frames) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *frames = d->mb;
    return SIFT_HIP_OK;
}

int sift_hip_lanes(sift_hip_t d, int* max_lanes, int* created) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (max_lanes) *max_lanes = d->maxLanes;
    if (created) *created = d->nLanes;
    return SIFT_HIP_OK;
}

int sift_hip_set_descriptor_mode(sift_hip_t d, int mode) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (mode != SIFT_HIP_DESC_FAST && mode != SIFT_HIP_DESC_EXACT) return fail(SIFT_HIP_ERR_INVALID, "unknown descriptor mode");
    if (d->allocated) return fail(SIFT_HIP_ERR_STATE, "sift_hip_set_descriptor_mode after sift_hip_warmup");
    d->kp.descExact = mode == SIFT_HIP_DESC_EXACT;
    return SIFT_HIP_OK;
}

int sift_hip_descriptor_mode(sift_hip_t d, int* mode) {
    if (!d || !mode) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *mode = d->kp.descExact ? SIFT_HIP_DESC_EXACT : SIFT_HIP_DESC_FAST;
    return SIFT_HIP_OK;
}

int sift_hip_batch_capacity(sift_hip_t d, int* frames) {
    if (!d || !frames) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *frames = d->B;
    return SIFT_HIP_OK;
}

int sift_hip_detect_batch_device(sift_hip_t d, const void* frames, int n, size_t stride, size_t frame_stride,
                                 int format, void* stream) {
    CHECK_HANDLE(d);
    if (!frames) return fail(SIFT_HIP_ERR_INVALID, "null frames");
    if (n < 1 || n > d->B) return fail(SIFT_HIP_ERR_INVALID, "frame count outside 1..batch capacity");
    const int es = format_size(format);
    if (!es) return fail(SIFT_HIP_ERR_INVALID, "unknown pixel format");
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    if (stride == 0) stride = (size_t)es * W;
    if (stride % es || stride < (size_t)es * W)
        return fail(SIFT_HIP_ERR_INVALID, "row stride must be a multiple of the pixel size and >= width");
    if (frame_stride == 0) frame_stride = stride * H;
    if (n > 1 && frame_stride < stride * (H - 1) + (size_t)es * W)
        return fail(SIFT_HIP_ERR_INVALID, "frame stride smaller than one frame");
    if (int rc = check_in_flight(d)) return rc;
    long long f = 0;
    if (int rc = submit_device(d, frames, stride, format, stream, n, frame_stride, &f)) return rc;
    make_current(d, f);
    if (stream) {
        HIPCHK(hipEventRecord(d->evOut, d->stream));
        HIPCHK(hipStreamWaitEvent((hipStream_t)stream, d->evOut, 0));
    }
    return SIFT_HIP_OK;
}

int sift_hip_batch_frames(sift_hip_t d, int* n) {
    CHECK_HANDLE(d);
    if (!n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *n = d->current < d->firstFrame ? 0 : d->lane().nfOf[d->cur];
    return SIFT_HIP_OK;
}

int sift_hip_batch_results_device(sift_hip_t d, int i, int* count, int* overflow, const float** k3,
                                  const float** f4, const uint16_t** desc) {
    CHECK_HANDLE(d);
    if (d->current < d->firstFrame || i < 0 || i >= d->lane().nfOf[d->cur])
        return fail(SIFT_HIP_ERR_INVALID, "no such frame in the current batch");
    if (count || overflow)
        if (int rc = ensure_counts(d)) return rc;
    const Counters& c = d->hCtr[(size_t)d->cur * d->B + i];
    const long o = (long)i * d->afs;
    if (count) *count = (int)std::min<unsigned>(c.final_n, d->kp.capFinal);
    if (overflow) *overflow = (int)c.overflow;
    if (k3) *k3 = fptr(d->dKpts3[d->cur], o);
    if (f4) *f4 = fptr(d->dFeats4[d->cur], o);
    if (desc) *desc = fptr(d->dDesc[d->cur], o);
    return SIFT_HIP_OK;
}

int sift_hip_batch_copy_to_host(sift_hip_t d, int i, float* k3, float* f4, uint16_t* desc, int cap, int* count) {
    int n = 0;
    const float *dk = nullptr, *df = nullptr;
    const uint16_t* dd = nullptr;
    if (int rc = sift_hip_batch_results_device(d, i, &n, nullptr, &dk, &df, &dd)) return rc;
    n = std::min(n, cap);
    if (count) *count = n;
    hipStream_t s;
    if (int rc = copy_stream(d, &s)) return rc;
    HIPCHK(hipStreamWaitEvent(s, d->lane().evFrame[d->cur], 0));
    if (n > 0) {
        if (k3) HIPCHK(hipMemcpyAsync(k3, dk, sizeof(float) * 3 * n, hipMemcpyDeviceToHost, s));
        if (f4) HIPCHK(hipMemcpyAsync(f4, df, sizeof(float) * 4 * n, hipMemcpyDeviceToHost, s));
        if (desc) HIPCHK(hipMemcpyAsync(desc, dd, sizeof(uint16_t) * 128 * n, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    return SIFT_HIP_OK;
}

int sift_hip_sync(sift_hip_t d) {
    CHECK_HANDLE(d);
    return finish_frame(d);
}

int sift_hip_num_keypoints(sift_hip_t d, int* n) {
    if (!d || !n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    if (d->allocated && d->nLanes) {
        HIPCHK(hipSetDevice(d->device));
        bind_lane(d, d->curLane, d->curIdx);
        if (int rc = ensure_counts(d)) return rc;
    }
    *n = d->count;
    return SIFT_HIP_OK;
}

int sift_hip_overflow_flags(sift_hip_t d, int* flags) {
    if (!d || !flags) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    if (d->allocated && d->nLanes) {
        HIPCHK(hipSetDevice(d->device));
        bind_lane(d, d->curLane, d->curIdx);
        if (int rc = ensure_counts(d)) return rc;
    }
    *flags = d->hCtr ? (int)d->hCtr[(size_t)d->cur * d->B].overflow : 0;
    return SIFT_HIP_OK;
}

int sift_hip_capacities(sift_hip_t d, int* cand, int* refined, int* oriented, int* results) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    if (cand) *cand = (int)d->capCand;
    if (refined) *refined = (int)d->kp.capRefined;
    if (oriented) *oriented = (int)d->kp.capOriented;
    if (results) *results = (int)d->kp.capFinal;
    return SIFT_HIP_OK;
}

int sift_hip_results_device(sift_hip_t d, const float** k3, const float** f4, const uint16_t** desc,
                            const uint16_t** prev, int* prevCount, int* capacity) {
    CHECK_HANDLE(d);
    if (prevCount)
        if (int rc = ensure_counts(d)) return rc;
    if (k3) *k3 = d->dKpts3[d->cur];
    if (f4) *f4 = d->dFeats4[d->cur];
    if (desc) *desc = d->dDesc[d->cur];
    if (prev) *prev = d->current - 1 >= d->firstFrame ? frame_desc(d, d->current - 1) : d->dDesc[(d->cur + d->kSlots - 1) % d->kSlots];
    if (prevCount) *prevCount = d->prevCount;
    if (capacity) *capacity = (int)d->kp.capFinal;
    return SIFT_HIP_OK;
}

int sift_hip_copy_to_host(sift_hip_t d, float* k3, float* f4, uint16_t* desc, int cap) {
    CHECK_HANDLE(d);
    if (int rc = ensure_counts(d)) return rc;
    const int n = std::min(d->count, cap);
    Lane& L = d->lane();
    if (!d->hostWant)
        for (int k = 0; k < d->nLanes; k++)
            if (int rc = ensure_host_res(d, d->lanes[k])) return rc;
    d->hostWant = std::max(d->hostWant, desc ? 2 : 1);
    const int region = d->cur * d->B + d->curIdx;
    if (L.hRes && L.hostFrame[region] == d->current && d->current >= d->firstFrame && (!desc || L.hostDesc[region])) {
        // A host-input frame: its descriptor kernel wrote them to pinned host memory.
        HIPCHK(hipEventSynchronize(L.evFrame[d->cur]));
        float *hk3, *hf4;
        uint16_t* hdesc;
        host_res(d, L.hRes, region, &hk3, &hf4, &hdesc);
        if (n > 0) {
            if (k3) memcpy(k3, hk3, sizeof(float) * 3 * n);
            if (f4) memcpy(f4, hf4, sizeof(float) * 4 * n);
            if (desc) {  // 2.2 MB at C2: split over the copy pool (one thread: 0.100 -> 0.047 ms, C++ loop)
                if (!d->pool && 256u * n >= (1u << 20)) d->pool = new CopyPool(kCopyWorkers);
                copy_rows(d->pool, (char*)desc, 256, (const char*)hdesc, 256, 256, n);
            }
        }
        return SIFT_HIP_OK;
    }
    // On the copy stream, ordered after the current frame only: frames
    // submitted after it keep running.
    hipStream_t s;
    if (int rc = copy_stream(d, &s)) return rc;
    HIPCHK(hipStreamWaitEvent(s, d->lane().evFrame[d->cur], 0));
    if (n > 0) {
        if (k3) HIPCHK(hipMemcpyAsync(k3, d->dKpts3[d->cur], sizeof(float) * 3 * n, hipMemcpyDeviceToHost, s));
        if (f4) HIPCHK(hipMemcpyAsync(f4, d->dFeats4[d->cur], sizeof(float) * 4 * n, hipMemcpyDeviceToHost, s));
        if (desc)
            HIPCHK(hipMemcpyAsync(desc, d->dDesc[d->cur], sizeof(uint16_t) * 128 * n, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    return SIFT_HIP_OK;
}

// The current frame's results in the handle's pinned host region (the lane's
// region slot * B + idx): a host-input frame's were written there by its
// descriptor kernel (HostOut), any other frame's are copied there now over the
// copy stream.  No copy into caller memory.
int sift_hip_results_host(sift_hip_t d, const float** k3, const float** f4, const uint16_t** desc, int* count) {
    CHECK_HANDLE(d);
    if (int rc = ensure_counts(d)) return rc;
    const int n = std::min(d->count, (int)d->kp.capFinal);
    Lane& L = d->lane();
    if (!d->hostWant)
        for (int k = 0; k < d->nLanes; k++)
            if (int rc = ensure_host_res(d, d->lanes[k])) return rc;
    d->hostWant = std::max(d->hostWant, desc ? 2 : 1);
    const int region = d->cur * d->B + d->curIdx;
    float *hk3, *hf4;
    uint16_t* hdesc;
    host_res(d, L.hRes, region, &hk3, &hf4, &hdesc);
    if (L.hostFrame[region] == d->current && d->current >= d->firstFrame && (!desc || L.hostDesc[region])) {
        HIPCHK(hipEventSynchronize(L.evFrame[d->cur]));
    } else {
        hipStream_t s;
        if (int rc = copy_stream(d, &s)) return rc;
        HIPCHK(hipStreamWaitEvent(s, L.evFrame[d->cur], 0));
        if (n > 0) {
            HIPCHK(hipMemcpyAsync(hk3, d->dKpts3[d->cur], sizeof(float) * 3 * n, hipMemcpyDeviceToHost, s));
            HIPCHK(hipMemcpyAsync(hf4, d->dFeats4[d->cur], sizeof(float) * 4 * n, hipMemcpyDeviceToHost, s));
            if (desc)
                HIPCHK(hipMemcpyAsync(hdesc, d->dDesc[d->cur], sizeof(uint16_t) * 128 * n, hipMemcpyDeviceToHost, s));
        }
        HIPCHK(hipStreamSynchronize(s));
        L.hostFrame[region] = d->current;
        L.hostDesc[region] = desc != nullptr;
    }
    if (k3) *k3 = hk3;
    if (f4) *f4 = hf4;
    if (desc) *desc = hdesc;
    if (count) *count = n;
    return SIFT_HIP_OK;
}

int sift_hip_copy_descriptors_device(sift_hip_t d, uint16_t* dst, int cap, void* stream) {
    CHECK_HANDLE(d);
    if (int rc = ensure_counts(d)) return rc;
    const int n = std::min(d->count, cap);
    hipStream_t s = stream ? (hipStream_t)stream : d->stream;
    if (s != d->stream) HIPCHK(hipStreamWaitEvent(s, d->lane().evFrame[d->cur], 0));
    if (n > 0) HIPCHK(hipMemcpyAsync(dst, d->dDesc[d->cur], sizeof(uint16_t) * 128 * n, hipMemcpyDeviceToDevice, s));
    if (!stream) HIPCHK(hipStreamSynchronize(s));
    return SIFT_HIP_OK;
}

int sift_hip_set_datagen(sift_hip_t d, const char* dir) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    d->dgDir = dir ? dir : "";
    return SIFT_HIP_OK;
}

int sift_hip_replay_stage(sift_hip_t d, const char* dump_dir, const char* stage, const char* out_dir) {
    CHECK_HANDLE(d);
    if (!dump_dir || !stage || !out_dir) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    return replay_stage(d, dump_dir, stage, out_dir);
}

int sift_hip_set_timing(sift_hip_t d, int enable) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    d->timing = enable != 0;
    d->blurReps = enable > 1 ? enable : 1;
    return SIFT_HIP_OK;
}

int sift_hip_timing_count(sift_hip_t d, int* n) {
    if (!d || !n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    *n = (int)d->tagg.size();
    return SIFT_HIP_OK;
}

int sift_hip_timing_entry(sift_hip_t d, int i, const char** name, double* ms, int* launches, double* bytes) {
    if (!d || i < 0 || i >= (int)d->tagg.size()) return fail(SIFT_HIP_ERR_INVALID, "bad timing index");
    if (name) *name = d->tagg[i].name.c_str();
    if (ms) *ms = d->tagg[i].ms;
    if (launches) *launches = d->tagg[i].launches;
    if (bytes) *bytes = d->tagg[i].bytes;
    return SIFT_HIP_OK;
}

int sift_hip_timing_reset(sift_hip_t d) {
    if (!d) return fail(SIFT_HIP_ERR_INVALID, "null handle");
    for (auto& a : d->tagg) a.ms = a.bytes = 0, a.launches = 0;
    return SIFT_HIP_OK;
}

int sift_hip_debug_gaussian(sift_hip_t d, int o, int layer, float* out) {
    CHECK_HANDLE(d);
    if (o < 0 || o >= d->nOct || layer < 0 || layer >= d->L + 3 || !out)
        return fail(SIFT_HIP_ERR_INVALID, "bad plane");
    const OctGeom& g = d->pyr.oct[o];
    HIPCHK(hipMemcpy2D(out, sizeof(float) * g.W, g.base + (size_t)layer * g.planeStride, sizeof(float) * g.pitch,
                       sizeof(float) * g.W, g.H, hipMemcpyDeviceToHost));
    return SIFT_HIP_OK;
}

int sift_hip_debug_candidates(sift_hip_t d, int* quads, int cap, int* count) {
    CHECK_HANDLE(d);
    if (int rc = ensure_counts(d)) return rc;
    const Counters& c = d->hCtr[(size_t)d->cur * d->B];
    const int n = (int)std::min<unsigned>(c.cand, d->capCand);
    if (count) *count = (int)c.cand;
    const int m = std::min(n, cap);
    if (m > 0 && quads) {
        std::vector<uint2> tmp(m);
        HIPCHK(hipMemcpy(tmp.data(), d->dCand, sizeof(uint2) * m, hipMemcpyDeviceToHost));
        for (int i = 0; i < m; i++) {
            quads[4 * i] = (int)(tmp[i].x >> 8);
            quads[4 * i + 1] = (int)(tmp[i].x & 255);
            quads[4 * i + 2] = (int)(tmp[i].y >> 16);
            quads[4 * i + 3] = (int)(tmp[i].y & 0xffff);
        }
    }
    return SIFT_HIP_OK;
}

// ----------------------------------------------------------------------------
// Matcher
// ----------------------------------------------------------------------------
}  // extern "C"

struct sift_hip_matcher {
    int device = 0;
    int maxQ = 0, maxT = 0, maxP = 0;
    unsigned long long* dKeys = nullptr;  // running top-2 keys per (pair, query), all ones between calls
    unsigned* dDone = nullptr;            // finished splits per (pair, 256-query block), zero between calls
    int* dMatch = nullptr;
    int8_t* dCodes = nullptr;             // int8 codes of a call's distinct sets (k_match_prep)
    int* dRowKeys = nullptr;              // key bias per code row; row codeRows: the zero/padding sentinel
    unsigned* dFlags = nullptr;           // per set slot: == epoch if the set is not all integers 0..255
    long codeRows = 0;
    unsigned epoch = 0;
    bool sidecars = true;  // single pairs of detector buffers: match their sidecar codes (k_match_direct)
    ~sift_hip_matcher() {
        (void)hipSetDevice(device);
        for (void* p : {(void*)dKeys, (void*)dDone, (void*)dMatch, (void*)dCodes, (void*)dRowKeys, (void*)dFlags})
            if (p) (void)hipFree(p);
    }
};

extern "C" {

int sift_hip_matcher_create(int device, int max_query, int max_train, int max_pairs, sift_hip_matcher_t* out) {
    if (!out || max_query <= 0 || max_train <= 0 || max_pairs <= 0 || max_pairs > kMaxMatchPairs)
        return fail(SIFT_HIP_ERR_INVALID, "bad matcher limits");
    *out = nullptr;
    auto* m = new sift_hip_matcher();
    if (device < 0) {
        if (hipGetDevice(&m->device) != hipSuccess) m->device = 0;
    } else {
        m->device = device;
    }
    m->maxQ = max_query;
    m->maxT = max_train;
    m->maxP = max_pairs;
    // Distinct sets of a call: at most 2 per pair, each at most max(maxQ, maxT) rows.
    m->codeRows = 2L * max_pairs * std::max(max_query, max_train);
    const size_t nkeys = 2 * (size_t)max_pairs * max_query;
    const size_t nblk = (size_t)max_pairs * ((max_query + kMatchQB - 1) / kMatchQB);
    if (hipSetDevice(m->device) != hipSuccess ||
        hipMalloc((void**)&m->dKeys, sizeof(unsigned long long) * nkeys) != hipSuccess ||
        hipMalloc((void**)&m->dDone, sizeof(unsigned) * nblk) != hipSuccess ||
        hipMalloc((void**)&m->dMatch, sizeof(int) * (size_t)max_pairs * max_query) != hipSuccess ||
        hipMalloc((void**)&m->dCodes, (size_t)(m->codeRows + 1) * 128) != hipSuccess ||
        hipMalloc((void**)&m->dRowKeys, sizeof(int) * (size_t)(m->codeRows + 1)) != hipSuccess ||
        hipMemset(m->dCodes + (size_t)m->codeRows * 128, 0, 128) != hipSuccess ||
        hipMemcpy(m->dRowKeys + m->codeRows, &kMatchPadKey, sizeof(int), hipMemcpyHostToDevice) != hipSuccess ||
        hipMalloc((void**)&m->dFlags, sizeof(unsigned) * 2 * kMaxMatchPairs) != hipSuccess ||
        hipMemset(m->dKeys, 0xff, sizeof(unsigned long long) * nkeys) != hipSuccess ||
        hipMemset(m->dDone, 0, sizeof(unsigned) * nblk) != hipSuccess ||
        hipMemset(m->dFlags, 0, sizeof(unsigned) * 2 * kMaxMatchPairs) != hipSuccess ||
        hipDeviceSynchronize() != hipSuccess) {
        delete m;
        return fail(SIFT_HIP_ERR_NOMEM, "matcher allocation failed");
    }
    *out = m;
    return SIFT_HIP_OK;
}

int sift_hip_matcher_set_sidecars(sift_hip_matcher_t m, int enable) {
    if (!m) return fail(SIFT_HIP_ERR_INVALID, "null matcher");
    m->sidecars = enable != 0;
    return SIFT_HIP_OK;
}

int sift_hip_matcher_destroy(sift_hip_matcher_t m) {
    delete m;
    return SIFT_HIP_OK;
}

int sift_hip_match_batched(sift_hip_matcher_t m, int P, const uint16_t* const* q, const int* nq,
                           const uint16_t* const* t, const int* nt, float ratio, int ratio_on_squared, int* idx2,
                           float* d2, int* match, void* stream) {
    if (!m || P <= 0 || P > m->maxP || !q || !nq || !t || !nt) return fail(SIFT_HIP_ERR_INVALID, "bad batch");
    Sidecar sq{}, st{};
    if (P == 1 && m->sidecars && nq[0] > 0 && nt[0] > 0 && nq[0] <= m->maxQ && nt[0] <= m->maxT &&
        find_sidecar(q[0], nq[0], &sq) && find_sidecar(t[0], nt[0], &st)) {
        // Both sets are detector buffers: their codes are ready (no conversion).
        HIPCHK(hipSetDevice(m->device));
        const MatchPair pr{q[0], t[0], nq[0], nt[0], 0, 0, 0, 0, 0, 0};
        launch_match_direct(pr, sq.codes, sq.keys, st.codes, st.keys, m->dCodes + (size_t)m->codeRows * 128,
                            m->dRowKeys + m->codeRows, m->dKeys, m->dDone, ratio, ratio_on_squared, idx2, d2, match,
                            (hipStream_t)stream);
        HIPCHK(hipGetLastError());
        return SIFT_HIP_OK;
    }
    MatchBatch b{};
    MatchSets sets{};
    b.P = P;
    // Distinct sets by pointer (a set used by several pairs is prepared once).
    auto set_of = [&](const uint16_t* ptr, int n) {
        for (int k = 0; k < sets.nsets; k++)
            if (sets.set[k].src == ptr) {
                sets.set[k].n = std::max(sets.set[k].n, n);
                return k;
            }
        sets.set[sets.nsets] = MatchSet{ptr, n, 0};
        return sets.nsets++;
    };
    int off = 0, maxq = 1, maxt = 1;
    for (int p = 0; p < P; p++) {
        if (nq[p] < 0 || nt[p] < 0 || nq[p] > m->maxQ || nt[p] > m->maxT)
            return fail(SIFT_HIP_ERR_INVALID, "pair size exceeds matcher limits");
        if ((nq[p] && !q[p]) || (nt[p] && !t[p])) return fail(SIFT_HIP_ERR_INVALID, "null descriptor pointer");
        const int qs = set_of(q[p], nq[p]), ts = set_of(t[p], nt[p]);
        b.pair[p] = MatchPair{q[p], t[p], nq[p], nt[p], off, qs, ts, 0, 0, 0};
        off += nq[p];
        maxq = std::max(maxq, nq[p]);
        maxt = std::max(maxt, nt[p]);
    }
    long row = 0;
    for (int k = 0; k < sets.nsets; k++) {
        sets.set[k].row0 = (int)row;
        row += sets.set[k].n;
        sets.maxn = std::max(sets.maxn, sets.set[k].n);
    }
    if (row > m->codeRows) return fail(SIFT_HIP_ERR_INVALID, "descriptor sets exceed the matcher's code buffer");
    for (int p = 0; p < P; p++) {
        b.pair[p].qrow0 = sets.set[b.pair[p].qset].row0;
        b.pair[p].trow0 = sets.set[b.pair[p].tset].row0;
    }
    m->epoch = m->epoch + 1 == 0 ? 1 : m->epoch + 1;  // flags from earlier calls never equal it
    HIPCHK(hipSetDevice(m->device));
    const MatchPlan plan = match_plan(maxq, maxt, P);
    launch_match(sets, b, plan, m->maxQ, m->dCodes, m->dRowKeys, (int)m->codeRows, m->dFlags, m->epoch, m->dKeys, m->dDone, ratio,
                 ratio_on_squared, idx2, d2, match, (hipStream_t)stream);
    HIPCHK(hipGetLastError());
    return SIFT_HIP_OK;
}

int sift_hip_match_device(sift_hip_matcher_t m, const uint16_t* q, int nq, const uint16_t* t, int nt, float ratio,
                          int ratio_on_squared, int* idx2, float* d2, int* match, void* stream) {
    return sift_hip_match_batched(m, 1, &q, &nq, &t, &nt, ratio, ratio_on_squared, idx2, d2, match, stream);
}

int sift_hip_match_plan(int max_query, int max_train, int pairs, int* splits, int* waves) {
    if (max_query < 0 || max_train < 0 || pairs < 1 || !splits) return fail(SIFT_HIP_ERR_INVALID, "bad match shape");
    const MatchPlan pl = match_plan(max_query, max_train, pairs);
    *splits = pl.S;
    if (waves) *waves = pl.nw;
    return SIFT_HIP_OK;
}

int sift_hip_match_host(sift_hip_matcher_t m, const uint16_t* q, int nq, const uint16_t* t, int nt, float ratio,
                        int ratio_on_squared, int* out) {
    if (!m || !out) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    if (nq <= 0) return SIFT_HIP_OK;
    int rc = sift_hip_match_device(m, q, nq, t, nt, ratio, ratio_on_squared, nullptr, nullptr, m->dMatch, nullptr);
    if (rc) return rc;
    HIPCHK(hipMemcpy(out, m->dMatch, sizeof(int) * nq, hipMemcpyDeviceToHost));
    return SIFT_HIP_OK;
}

int sift_hip_device_count(int* n) {
    if (!n) return fail(SIFT_HIP_ERR_INVALID, "null argument");
    if (hipGetDeviceCount(n) != hipSuccess) *n = 0;
    return SIFT_HIP_OK;
}
int sift_hip_malloc(void** p, size_t bytes) {
    HIPCHK(hipMalloc(p, bytes));
    return SIFT_HIP_OK;
}
int sift_hip_free(void* p) {
    HIPCHK(hipFree(p));
    return SIFT_HIP_OK;
}
int sift_hip_memcpy_h2d(void* dst, const void* src, size_t bytes) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyHostToDevice));
    return SIFT_HIP_OK;
}
int sift_hip_memcpy_d2h(void* dst, const void* src, size_t bytes) {
    HIPCHK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    return SIFT_HIP_OK;
}
int sift_hip_device_sync(void) {
    HIPCHK(hipDeviceSynchronize());
    return SIFT_HIP_OK;
}

}  // extern "C"
