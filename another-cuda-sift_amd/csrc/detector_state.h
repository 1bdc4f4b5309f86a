// Host-side state of a detector handle (struct sift_hip_detector, the opaque
// type of include/sift_hip.h) and the orchestration shared by the C-ABI
// translation units of libsift_hip.so:
//   detector.hip     geometry, frame arenas, graph capture, frame launch, the
//                    detector entry points
//   lanes.hip        compute lanes, micro-batching, host staging, submit/wait
//   datagen.hip      stage dumps and per-stage replay (sift_hip_replay_stage)
//   matcher_api.hip  the matcher handle and the descriptor sidecar registry
// Internal (not installed), host code only; no torch types.  Included by those
// four files alone, which is why it opens its namespaces (as detector.hip did).
#pragma once
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "sift_hip.h"
#include "sift_kernels.h"

namespace sift_amd {
namespace det {

extern thread_local std::string g_err;  // sift_hip_last_error
int fail(int code, const std::string& msg);

#define HIPCHK(expr)                                                                                    \
    do {                                                                                                \
        hipError_t e_ = (expr);                                                                         \
        if (e_ != hipSuccess)                                                                           \
            return ::sift_amd::det::fail(SIFT_HIP_ERR_RUNTIME, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

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
void copy_rows(CopyPool* pool, char* dst, size_t dpitch, const char* src, size_t sstride, size_t rowB, int rows);

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

// Matcher sidecars of the descriptor buffers the detector handles hand out
// (matcher_api.hip): exact buffer base -> its int8 codes and key biases.
void register_sidecar(const void* owner, const uint16_t* desc, Sidecar side, int cap);
void unregister_sidecars(const void* owner);
bool find_sidecar(const uint16_t* desc, int n, Sidecar* out);
bool sidecar_written(const uint16_t* desc);     // the caller wrote the rows: drop the sidecar
void sidecar_refreshed(const uint16_t* desc);   // a frame is launched into the buffer: valid again

// Results slots per compute lane (Lane::nslots): 4 -- frames f-1 .. f+2 of a
// lane never share one -- and 8 on the lanes of automatic launch groups, whose
// launch groups vary in size (a lane's slots then hold at least 8 launches'
// frames before one is reused).  The arena layout holds kResultSlots.
constexpr int kResultSlots = 8;
constexpr int kLaneSlots = 4;
constexpr int kMaxLanes = 4;
constexpr int kFrameRing = 256;  // per-frame (lane, slot, arena) records: > 2 x kMaxLanes x kMaxMicroBatch (frames in flight) + the two readable

// A compute lane: one HIP stream, its B frame arenas (every per-frame buffer of
// the pipeline, sift_kernels.h Frames), the graphs captured on them and a ring
// of kResultSlots results slots.  A lane runs its frames in order; frames on
// different lanes run concurrently ("Frames in flight").
struct Lane {
    hipStream_t stream = nullptr;
    // Frame arenas of this lane (launch groups of up to B frames): the handle's
    // batch size, or its automatic group size for the lanes created after lane
    // 0 (sift_hip_set_auto_micro_batch).
    int B = 1;
    int nslots = kLaneSlots;  // results slots in use (even: slot parity = launch parity)
    // Set once add_lane completed (stream, arenas, host counters, graphs): a
    // lane whose creation failed part-way is never picked, synchronised or
    // handed host regions (its partial allocations wait for the destructor).
    bool ready = false;
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
    long long slotFrame[kResultSlots] = {-1, -1, -1, -1, -1, -1, -1, -1};  // the (first) frame whose results each slot holds
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

}  // namespace det
}  // namespace sift_amd

using namespace sift_amd;
using namespace sift_amd::det;

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
    int nLanes = 0;    // lanes created (lane 0 at warm-up, more on demand; see Lane::ready)
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
    // Automatic launch groups (sift_hip_set_auto_micro_batch, default 8) on a
    // handle with neither a batch nor a micro-batch set: a submitted frame runs
    // at once while a lane is free; once every lane is busy, frames queue and
    // the queue runs as one launch group when a lane frees or when it holds
    // autoMb frames.  Lane 0 keeps one arena (the synchronous path's memory);
    // lanes created later hold autoMb.
    int autoMb = 8;
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

namespace sift_amd {
namespace det {

// ---- detector.hip ----
int setup_geometry(sift_hip_detector* d);
void setup_taps(sift_hip_detector* d);
int allocate(sift_hip_detector* d);
// Points the handle's buffer views at lane k (idx: the arena of a micro-batch frame).
void bind_lane(sift_hip_detector* d, int k, int idx = 0);
const uint16_t* frame_desc(const sift_hip_detector* d, long long f);
const Counters& frame_counters(const sift_hip_detector* d, long long f, int i = 0);
int add_lane(sift_hip_detector* d, int B, int nslots = kLaneSlots);
int warm_lane(sift_hip_detector* d);
unsigned* range_keys(sift_hip_detector* d, int p);
void enqueue_head(sift_hip_detector* d, const void* img, int pitch, int fmt, int parity, int nf, long sfs);
void enqueue_pyramid(sift_hip_detector* d, int nf, int parity);
void enqueue_extrema(sift_hip_detector* d, int nf);
void enqueue_refine(sift_hip_detector* d, int nf);
void enqueue_orientation(sift_hip_detector* d, int nf);
void enqueue_order(sift_hip_detector* d, int slot, int nf);
void enqueue_descriptor(sift_hip_detector* d, int slot, int nf);
bool event_done(hipEvent_t e);
int run_frame(sift_hip_detector* d, const void* img, int pitch, int fmt, hipEvent_t consumed, int nf = 1, long sfs = 0,
              bool numbered = false);
void make_current(sift_hip_detector* d, long long f);
void complete_counts(sift_hip_detector* d);
int ensure_counts(sift_hip_detector* d);
int sync_lanes(sift_hip_detector* d);
int finish_frame(sift_hip_detector* d);

// ---- lanes.hip ----
int group_cap(const sift_hip_detector* d);
bool auto_groups(const sift_hip_detector* d);
bool lane_available(sift_hip_detector* d, int nf);
int pick_lane(sift_hip_detector* d, int nf = 1);
int copy_stream(sift_hip_detector* d, hipStream_t* s);
int format_size(int fmt);
int check_in_flight(sift_hip_detector* d);
size_t host_res_bytes(const sift_hip_detector* d);
void host_res(const sift_hip_detector* d, char* base, int region, float** k3, float** f4, uint16_t** desc);
int ensure_host_res(sift_hip_detector* d, Lane& L);
int submit_host(sift_hip_detector* d, const void* img, size_t stride, int fmt, long long* ticket);
int run_group(sift_hip_detector* d);
int submit_device(sift_hip_detector* d, const void* img, size_t stride, int fmt, void* stream, int nf, size_t fstride,
                  long long* ticket, bool queue = false);
int wait_frame(sift_hip_detector* d, long long f);

// ---- datagen.hip ----
int dump_stage_files(sift_hip_detector* d);
int replay_stage(sift_hip_detector* d, const std::string& in, const std::string& stage, const std::string& out);

}  // namespace det
}  // namespace sift_amd
