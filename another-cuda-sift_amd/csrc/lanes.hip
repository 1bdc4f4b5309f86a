// Compute lanes, micro-batching, host-frame staging and the submit / wait
// path of libsift_hip.so ("Compute lanes" and
// "Micro-batching"): which lane a frame runs on, how host frames reach the
// device, how queued device frames form launch groups, and when a frame's
// results become current.  Replaces the reference's synchronous
// detectAndCompute upload (/root/reference/sift_cuda/interface/Detector.cu:133-145)
// and its per-call result download (utils/CudaMemcpyUtils.cu).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "detector_state.h"

namespace sift_amd {
namespace det {

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

// Launch-group size of a submitted frame's queue: the micro-batch, else the
// automatic group size (a handle without a batch, with a second lane to run
// groups on), else 1 (no queue).
bool auto_groups(const sift_hip_detector* d) { return d->mb == 1 && d->B == 1 && d->autoMb > 1 && d->maxLanes > 1; }
int group_cap(const sift_hip_detector* d) { return d->mb > 1 ? d->mb : (auto_groups(d) ? d->autoMb : 1); }

namespace {
// Automatic groups: frames past the current one (queued ones included).  Up
// to 2 per lane run as single frames (the unbatched regime); past that, a
// queue launches early only with at least half a group, so every results slot
// of a group lane holds >= that many frames and the frames the caller may
// still read fit in the slots (in_flight_limit).
long long past_current(const sift_hip_detector* d) {
    return d->submitted + d->npend - 1 - std::max(d->current, d->firstFrame - 1);
}
int auto_min_group(const sift_hip_detector* d) { return std::max(2, d->autoMb / 2); }
long long in_flight_limit(const sift_hip_detector* d) {
    if (!auto_groups(d)) return 2LL * d->maxLanes * group_cap(d);
    return std::max(2LL * d->maxLanes, (long long)(d->maxLanes - 1) * 3 * auto_min_group(d));
}

// A lane qualifies for a launch group of nf frames if it has the arenas and
// its next results slot holds no frame the caller may still read (current - 1
// onwards); it is idle once its last launch group completed.
bool lane_fits(const sift_hip_detector* d, int k, int nf) {
    const Lane& L = d->lanes[k];
    if (!L.ready || L.B < nf) return false;
    const int s = (int)(L.launched % L.nslots);
    const long long occ = L.slotFrame[s] < 0 ? -1 : L.slotFrame[s] + std::max(L.slotNum[s], 1) - 1;  // its last frame
    return occ < 0 || occ < d->firstFrame || occ < d->current - 1;
}
bool lane_idle(const sift_hip_detector* d, int k) {
    const Lane& L = d->lanes[k];
    return L.last < 0 || event_done(L.evFrame[(L.launched + L.nslots - 1) % L.nslots]);
}
// Arenas of a lane created now: the handle's batch, or the automatic group size.
int new_lane_frames(const sift_hip_detector* d) { return auto_groups(d) ? d->autoMb : d->B; }
}  // namespace

// Whether a launch group of nf frames would start at once: an idle lane that
// fits it, or a lane still to be created.
bool lane_available(sift_hip_detector* d, int nf) {
    for (int k = 0; k < d->nLanes; k++)
        if (lane_fits(d, k, nf) && lane_idle(d, k)) return true;
    return d->nLanes < d->maxLanes && new_lane_frames(d) >= nf;
}

// The lane for the next launch group (nf frames), bound on return: the first
// idle lane that fits it, else a new lane (up to maxLanes), else the busy lane
// that fits it whose last frame is the oldest.
int pick_lane(sift_hip_detector* d, int nf) {
    int busy = -1;
    for (int k = 0; k < d->nLanes; k++) {
        if (!lane_fits(d, k, nf)) continue;
        if (lane_idle(d, k)) {
            bind_lane(d, k);
            return SIFT_HIP_OK;
        }
        if (busy < 0 || d->lanes[k].last < d->lanes[busy].last) busy = k;
    }
    if (d->nLanes < d->maxLanes && new_lane_frames(d) >= nf) {  // (lane 0 comes from sift_hip_warmup)
        if (int rc = add_lane(d, new_lane_frames(d), auto_groups(d) ? kResultSlots : kLaneSlots)) return rc;
        return warm_lane(d);
    }
    if (busy < 0)
        return fail(SIFT_HIP_ERR_STATE, "every lane's next results slot is still held: sift_hip_wait first");
    bind_lane(d, busy);
    return SIFT_HIP_OK;
}

int copy_stream(sift_hip_detector* d, hipStream_t* s) {
    if (!d->copyStream) HIPCHK(hipStreamCreateWithFlags(&d->copyStream, hipStreamNonBlocking));
    *s = d->copyStream;
    return SIFT_HIP_OK;
}

int format_size(int fmt) { return fmt == SIFT_HIP_U8 ? 1 : (fmt == SIFT_HIP_F32 ? 4 : 0); }

// Frames in flight past `current` (host-input and device submits, queued ones
// included): at most in_flight_limit -- 2 per lane unbatched, 2 groups per
// lane with a micro-batch, max(2 x lanes, (lanes - 1) x 3 x frames / 2) with
// automatic groups.
int check_in_flight(sift_hip_detector* d) {
    if (d->submitted + d->npend > d->current + in_flight_limit(d))
        return fail(SIFT_HIP_ERR_STATE, "the frames in flight past the current frame reach the handle's limit: sift_hip_wait first");
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

// The lane's pinned results regions (nslots x B) and the device table that
// points the descriptor kernel at them (HostOut), set up for every lane once a
// caller reads results back (sift_hip_copy_to_host / sift_hip_results_host
// turn hostWant on) and for lanes created after that: a lazy allocation
// inside a submit stalled it for ~14 ms.  The table goes in on the lane's
// stream (after its zeroing; frames launched earlier keep a null table).
int ensure_host_res(sift_hip_detector* d, Lane& L) {
    if (L.hRes) return SIFT_HIP_OK;
    const size_t nr = (size_t)L.nslots * L.B, rb = host_res_bytes(d);
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
    const int region = r.slot * L.B + r.idx;
    L.hostFrame[region] = f;
    L.hostDesc[region] = d->hostWant > 1;
}

// Whether a submitted frame joins the pending queue: always with a micro-batch;
// with automatic groups once frames are pending or the frame would be the
// third in flight per lane (up to that it is launched at once, on a busy lane
// if none is free, as without groups: its stream starts it as soon as the
// lane frees, where a queue waits for the next call).  Stage dumps and the
// timing mode run frames one at a time.
bool queue_frame(sift_hip_detector* d) {
    if (!d->dgDir.empty() || d->timing) return false;
    if (d->mb > 1) return true;
    return auto_groups(d) && (d->npend > 0 || past_current(d) + 1 > 2LL * d->maxLanes);
}
// Whether the pending queue runs now: it holds a full group, or (automatic
// groups) a lane that fits it has become free and the queue holds half a
// group (any count while the frames in flight stay within 2 per lane).
bool launch_now(sift_hip_detector* d) {
    if (d->npend >= group_cap(d)) return true;
    if (d->mb > 1) return false;
    const bool shallow = past_current(d) <= 2LL * d->maxLanes;
    return (shallow || d->npend >= auto_min_group(d)) && lane_available(d, d->npend);
}

// A host frame on a micro-batching handle: into the next pinned staging slot
// of the handle's ring (the caller's buffer is free on return), pending until
// its group runs (run_group copies it to the lane's group input).
int queue_host(sift_hip_detector* d, const void* img, size_t stride, int fmt, long long* ticket) {
    const int es = format_size(fmt), H = d->cfg.row_width;
    const size_t rowB = (size_t)es * d->cfg.col_width, pitchB = (size_t)es * d->inPitch;
    if (d->hstSlotBytes < pitchB * H) {  // first host frame, or a larger format: (re)allocate the block
        if (int rc = run_group(d)) return rc;
        if (int rc = sync_lanes(d)) return rc;  // no copy kernel still reads the old block
        if (d->hstBlock) HIPCHK(hipHostFree(d->hstBlock));
        d->hstBlock = nullptr;
        d->hstSlotBytes = 0;
        d->hstSlots = (2 * d->maxLanes + 1) * group_cap(d);  // frames pending or queued on the lanes
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
    if (!launch_now(d)) return SIFT_HIP_OK;
    const int rc = run_group(d);
    if (rc && d->npend == i + 1) {  // the group did not launch: this call's frame is not queued either
        d->npend = i;
        d->hstNext--;  // (its staging slot is free again)
    }
    return rc;
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
    if (queue_frame(d)) return queue_host(d, img, stride, fmt, ticket);
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
    if (int rc = pick_lane(d, n)) return rc;
    Lane& L = d->lane();
    const int W = d->cfg.col_width, H = d->cfg.row_width;
    if (n == 1 && d->pend[0].hslot < 0) {  // one device frame: straight from the caller's buffer
        const auto& p = d->pend[0];
        if (p.ordered) HIPCHK(hipStreamWaitEvent(d->stream, d->evPend[0], 0));
        d->npend = 0;
        return run_frame(d, p.img, (int)(p.stride / format_size(p.fmt)), p.fmt, nullptr);
    }
    // One format per launch group: the frames' own, or f32 when they mix (an
    // 8-bit frame converted exactly, as the 8-bit head does).
    int fmt = d->pend[0].fmt;
    for (int i = 1; i < n; i++)
        if (d->pend[i].fmt != fmt) fmt = SIFT_HIP_F32;
    const int es = format_size(fmt);
    const size_t fb = sizeof(float) * (size_t)d->inPitch * H;  // one frame of f32 rows (an 8-bit frame uses a quarter)
    if (!L.mbIn && hipMalloc((void**)&L.mbIn, fb * L.B) != hipSuccess)
        return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the micro-batch input failed");
    bool host[sift_hip_detector::kMaxMicroBatch] = {};
    for (int i = 0; i < n; i++) {
        const auto& p = d->pend[i];
        if (p.ordered) HIPCHK(hipStreamWaitEvent(d->stream, d->evPend[i], 0));
        char* dst = L.mbIn + fb * i;
        const bool convert = p.fmt != fmt;  // an 8-bit frame in an f32 group
        if (p.hslot >= 0) {  // pinned staging: whole pitch rows over PCIe by a small grid
            unsigned req;
            unsigned* reqAt = host_request(d, i, &req);
            if (convert && !L.dStage[0] && hipMalloc(&L.dStage[0], fb) != hipSuccess)
                return fail(SIFT_HIP_ERR_NOMEM, "hipMalloc of the device staging failed");
            // (the lane's host staging slot 0 as scratch: stream-ordered with its other users)
            char* to = convert ? static_cast<char*>(L.dStage[0]) : dst;
            launch_copy_rows(p.img, p.stride, to, p.stride, p.stride, H, kStageWg, d->stream, reqAt, req);
            HIPCHK(hipEventRecord(d->hstRead[p.hslot], d->stream));
            if (convert)
                launch_u8_to_f32((const uint8_t*)to, (int)p.stride, W, H, (float*)dst, d->inPitch, Frames{1, 0}, 0,
                                 d->stream);
            host[i] = reqAt != nullptr;
        } else if (convert) {
            launch_u8_to_f32((const uint8_t*)p.img, (int)p.stride, W, H, (float*)dst, d->inPitch, Frames{1, 0}, 0,
                             d->stream);
        } else {
            launch_copy_rows(p.img, p.stride, dst, (size_t)es * d->inPitch, (size_t)es * W, H, kGroupCopyWg, d->stream);
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
// group instead.
int submit_device(sift_hip_detector* d, const void* img, size_t stride, int fmt, void* stream, int nf, size_t fstride,
                  long long* ticket, bool queue) {
    hipStream_t ext = (hipStream_t)stream;
    if (queue && nf == 1 && queue_frame(d)) {
        const int i = d->npend;
        if (ext) {
            if (!d->evPend[i]) HIPCHK(hipEventCreateWithFlags(&d->evPend[i], hipEventDisableTiming));
            HIPCHK(hipEventRecord(d->evPend[i], ext));
        }
        d->pend[i] = sift_hip_detector::PendingFrame{img, stride, fmt, ext != nullptr, -1};
        d->npend = i + 1;
        if (ticket) *ticket = d->submitted + i;
        if (!launch_now(d)) return SIFT_HIP_OK;
        const int rc = run_group(d);
        if (rc && d->npend == i + 1) d->npend = i;  // the group did not launch: this call's frame is not queued
        return rc;
    }
    if (int rc = run_group(d)) return rc;  // frames are numbered (and launched) in submission order
    if (int rc = pick_lane(d, nf)) return rc;
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

}  // namespace det
}  // namespace sift_amd
