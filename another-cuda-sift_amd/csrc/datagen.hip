// Stage dumps (sift_hip_set_datagen) and per-stage replay
// (sift_hip_replay_stage) of libsift_hip.so: the reference's setDataGen /
// tool/perf.cu snapshots (/root/reference/sift_cuda/interface/Detector.cu:145-229,
// PerfData.cuh) restated for this pipeline's own stages.
#include <hip/hip_runtime.h>
#include <sys/stat.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>

#include "detector_state.h"

namespace sift_amd {
namespace det {

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
    const Counters& c = d->hCtr[(size_t)d->cur * d->lane().B];
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
    const Counters& c = d->hCtr[(size_t)d->cur * d->lane().B];
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
    HIPCHK(hipMemsetAsync(d->lanes[0].arena, 0, (size_t)d->afs * d->lanes[0].B, d->stream));
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

}  // namespace det
}  // namespace sift_amd
