/*
 * sift_hip.h -- C ABI of the MI355X SIFT hot path (libsift_hip.so).
 *
 * Plain C types only: no HIP, torch or C++ types cross this boundary.  Device
 * memory is owned by the handle; device pointers handed out are valid until the
 * next sift_hip_detect* call on the same handle (the reference's contract for
 * Detector::device_* members, /root/reference/sift_cuda/interface/Detector.hh:54-57).
 * Streams are passed as `void*` (a hipStream_t; NULL = the handle's own stream).
 * Every function returns 0 (SIFT_HIP_OK) or a negative error; the message of the
 * last error on the calling thread is in sift_hip_last_error().
 *
 * Each entry point names the reference interface it replaces.  The C++ surface
 * sift_cuda::Detector / CudaSiftConfig / matchBruteForce in include/sift_cuda/ is
 * a thin wrapper over this ABI.
 */
#ifndef SIFT_HIP_H
#define SIFT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SIFT_HIP_OK 0
#define SIFT_HIP_ERR_INVALID (-1)   /* bad argument / size mismatch        */
#define SIFT_HIP_ERR_RUNTIME (-2)   /* HIP runtime error                   */
#define SIFT_HIP_ERR_STATE   (-3)   /* call out of order (e.g. no warmup)  */
#define SIFT_HIP_ERR_NOMEM   (-4)   /* device allocation failed            */

#define SIFT_HIP_ABI_VERSION 1

typedef struct sift_hip_detector* sift_hip_t;
typedef struct sift_hip_matcher* sift_hip_matcher_t;

/* Mirrors CudaSiftConfig (/root/reference/sift_cuda/types/CudaSiftConfig.hh:3-14),
 * field for field including the reference's spellings, plus defaulted extras. */
typedef struct {
    int    col_width;           /* image width  (CudaSiftConfig.hh:4)            */
    int    row_width;           /* image height (CudaSiftConfig.hh:5)            */
    int    numFeatures;         /* retainBest count, 0 = keep all (.hh:6)        */
    int    numOctaveLayers;     /* (.hh:7)                                      */
    double contrastThreshould;  /* (.hh:8)                                      */
    double edgeThreshould;      /* (.hh:9)                                      */
    double sigma;               /* (.hh:10)                                     */
    int    upscale;             /* 1 = double the base image = OpenCV default   */
                                /* firstOctave -1 (.hh:12, broken there)        */
    int    numOctaves;          /* extra: 0 = auto (OpenCV formula)             */
    int    maxKeypoints;        /* extra: result capacity; 0 = numFeatures + 25 % (or pyramid pixels / 32 when numFeatures = 0), at most 65536 */
} sift_hip_config;

/* Fills the reference defaults (CudaSiftConfig.hh:6-12) for a w x h image. */
void sift_hip_default_config(sift_hip_config* cfg, int w, int h);

/* Library / build info: "abi=<n> arch=gfx950 hip=<ver>". */
const char* sift_hip_version(void);
const char* sift_hip_last_error(void);

/* --- Detector (replaces sift_cuda::Detector, Detector.hh:24-96) ------------ */

/* Detector::Detector(const CudaSiftConfig&) (Detector.hh:26-29).  device < 0
 * binds to the calling thread's current HIP device like the reference. */
int sift_hip_create(const sift_hip_config* cfg, int device, sift_hip_t* out);
int sift_hip_destroy(sift_hip_t h);

/* Detector::gpuWarmUpAndAllocate() (Detector.cu:17-39): allocate every buffer,
 * build the hipGraph of the whole pipeline and run it once on a blank frame. */
int sift_hip_warmup(sift_hip_t h);

/* Octave count and per-octave geometry chosen for this configuration. */
int sift_hip_num_octaves(sift_hip_t h, int* n);
int sift_hip_octave_dims(sift_hip_t h, int octave, int* w, int* hgt, int* pitch_floats);

/* Detector::detectAndCompute(const Imagef&) (Detector.cu:133-233): uploads the
 * fp32 host image (row stride in bytes, 0 = packed) and runs the pipeline;
 * returns when results are ready.  Keypoint count via sift_hip_num_keypoints. */
int sift_hip_detect(sift_hip_t h, const float* host_img, size_t row_stride_bytes);

/* Pixel formats of a caller's frame.  OpenCV converts CV_8U input to float
 * exactly (createInitialImage), so an 8-bit frame gives the results of the
 * float frame holding the same values; it crosses PCIe in a quarter of the
 * bytes and is converted inside the first GPU kernel. */
#define SIFT_HIP_F32 0  /* float, 0..255 (Imagef, HostImage.hh:188)        */
#define SIFT_HIP_U8  1  /* uint8 (Image8U, HostImage.hh:187; cv::Mat CV_8U) */

/* Detector::detectAndCompute for an 8-bit host frame (the reference converts
 * cv::Mat to Imagef first, cvUtils/ConversionImpl.hpp:8-31).  Synchronous. */
int sift_hip_detect_u8(sift_hip_t h, const uint8_t* host_img, size_t row_stride_bytes);

/* Same, for an image already in device memory (HBM-resident input); enqueued on
 * `stream` (NULL = internal) and NOT synchronised: call sift_hip_sync.  The
 * result accessors address this frame at once (device-ordered use); counts
 * are valid after sift_hip_sync. */
int sift_hip_detect_device(sift_hip_t h, const float* dev_img, size_t row_stride_bytes, void* stream);
int sift_hip_detect_device_fmt(sift_hip_t h, const void* dev_img, size_t row_stride_bytes, int format,
                               void* stream);
int sift_hip_sync(sift_hip_t h);

/* Frame batches (C4: many frames per GPU).  sift_hip_set_batch(h, B), called
 * before sift_hip_warmup, gives the handle B frame arenas (pyramid, keypoint
 * lists, counters and result slots per frame) and a pipeline graph whose every
 * launch processes all B frames: B x the workgroups per launch and 1/B of the
 * dispatches per frame.  Results per frame are those of the single-frame call
 * on the same frame, bit for bit.  B = 1 (default) is the single-frame handle;
 * every single-frame entry point keeps working on a batch handle (frame 0's
 * arena, a one-frame graph).  Replaces the per-frame loop of
 * /root/reference/tool/extract_and_match_example.cc:69-101 over
 * Detector::detectAndCompute (Detector.cu:133-233). */
int sift_hip_set_batch(sift_hip_t h, int frames);
int sift_hip_batch_capacity(sift_hip_t h, int* frames);

/* Descriptor histogram summation, called before sift_hip_warmup (the mode is
 * part of the captured graphs).  The reference sums each bin with float
 * shared-memory atomics in scheduling order (SiftOps.cu:587-600); OpenCV sums
 * it sequentially in raster order (sift.simd.hpp calcSIFTDescriptor).
 *   SIFT_HIP_DESC_FAST  (default) fixed-point integer histogram: deterministic,
 *                       the exact sum of the rounded contributions; a byte can
 *                       differ from OpenCV's by +-1 (float summation order).
 *   SIFT_HIP_DESC_EXACT OpenCV's sequential float sum and correctly rounded
 *                       sample math: descriptors bit-identical to the oracle,
 *                       at a higher descriptor cost.
 * Keypoints are identical in both modes. */
#define SIFT_HIP_DESC_FAST  0
#define SIFT_HIP_DESC_EXACT 1
int sift_hip_set_descriptor_mode(sift_hip_t h, int mode);
int sift_hip_descriptor_mode(sift_hip_t h, int* mode);

/* n (1..B) device frames, frame i at dev_frames + i * frame_stride_bytes (0 =
 * row_stride * height), enqueued on `stream` (NULL = internal), NOT
 * synchronised (sift_hip_sync).  The batch becomes the current launch group. */
int sift_hip_detect_batch_device(sift_hip_t h, const void* dev_frames, int n, size_t row_stride_bytes,
                                 size_t frame_stride_bytes, int format, void* stream);
/* Frames in the current launch group (1 after a single-frame call). */
int sift_hip_batch_frames(sift_hip_t h, int* n);
/* Frame i of the current group: count / overflow flags (valid after
 * sift_hip_sync) and its device result arrays (layouts as
 * sift_hip_results_device). */
int sift_hip_batch_results_device(sift_hip_t h, int i, int* count, int* overflow, const float** kpts3,
                                  const float** feats4, const uint16_t** desc);
/* Copies min(count, cap) results of frame i to host memory (desc nullable). */
int sift_hip_batch_copy_to_host(sift_hip_t h, int i, float* kpts3, float* feats4, uint16_t* desc, int cap,
                                int* count);

/* Pipelined host input (replaces the synchronous upload of CudaImage.cu:97-105
 * and the per-frame loop of extract_and_match_example.cc:69-101).
 * sift_hip_submit copies the frame into one of its lane's two mapped pinned
 * staging buffers (the caller's buffer is free again on return), enqueues a
 * small copy kernel (staging -> device, over PCIe) and the pipeline on the
 * lane's stream and returns a ticket without waiting.
 * sift_hip_wait(ticket) blocks until that frame is complete and makes it the
 * frame the result accessors address (prev_desc = frame ticket-1).  At most
 * 2 x lanes frames may be in flight past the last waited one
 * (SIFT_HIP_ERR_STATE otherwise); sift_hip_detect / sift_hip_detect_u8 =
 * submit + wait.
 *
 * Frames in flight compute concurrently: a handle has up to `lanes` compute
 * lanes (a HIP stream with its own frame arenas, graphs and results ring
 * each).  A frame goes to the first idle lane; when every lane is busy and
 * fewer than `lanes` exist, a new one is created (its arenas and graphs, once:
 * a synchronous caller never pays for a second lane).  Results are identical
 * on every lane.  sift_hip_set_lanes(h, n), n = 1..4 (default 2), before
 * sift_hip_warmup; n = 1 runs every frame of the handle in submission order
 * on one stream.  sift_hip_lanes reports the limit and the lanes created. */
int sift_hip_submit(sift_hip_t h, const void* host_img, size_t row_stride_bytes, int format,
                    long long* ticket);
int sift_hip_wait(sift_hip_t h, long long ticket);
int sift_hip_set_lanes(sift_hip_t h, int lanes);
int sift_hip_lanes(sift_hip_t h, int* max_lanes, int* created);

/* Pipelined device input: like sift_hip_submit for a frame already in device
 * memory (f32 or u8, row stride in bytes), read on the frame's lane after
 * `stream` (NULL: no ordering) reaches this call; the buffer must stay
 * unchanged until sift_hip_wait(ticket) returns.  The results follow at
 * sift_hip_wait, as for host frames. */
int sift_hip_submit_device(sift_hip_t h, const void* dev_img, size_t row_stride_bytes, int format, void* stream,
                           long long* ticket);

/* Micro-batching of pipelined frames: with frames = M > 1 (before
 * sift_hip_warmup; the handle's batch size becomes M), frames submitted by
 * sift_hip_submit_device or sift_hip_submit queue until M of them run as ONE
 * launch group on a lane (each frame's rows copied into the lane's group
 * input -- device frames after their `stream` event, host frames from the
 * pinned staging block they were copied into at submit; one launch per
 * pipeline stage for the group, as sift_hip_detect_batch_device).  Tickets, results and prev_descriptor are per
 * frame and identical to unbatched submission.  A frame still queued is
 * launched (with the frames before it, as a partial group) by sift_hip_wait
 * on it, sift_hip_sync, or any other detect / submit call; its `dev_img` must
 * stay unchanged until then.  At most 2 x lanes x M frames may be in flight
 * past the last waited one.  Default 1 (every frame launched at submit). */
int sift_hip_set_micro_batch(sift_hip_t h, int frames);
int sift_hip_micro_batch(sift_hip_t h, int* frames);

/* Automatic launch groups (the default, frames = 8; before sift_hip_warmup;
 * 0 or 1 turns them off) on a handle without a batch or micro-batch and with
 * more than one lane.  Frames of sift_hip_submit / sift_hip_submit_device run
 * as single frames while at most 2 per lane are in flight past the last
 * waited one (exactly as without groups); past that they queue, and the queue
 * runs as ONE launch group (as with a micro-batch) when it holds `frames`
 * frames, or -- checked at each submit -- when a lane that can take it is
 * free and it holds frames / 2, or at a wait on a queued frame /
 * sift_hip_sync / any other detect.  So a caller keeping many frames in
 * flight gets micro-batched launches with no extra call, and a synchronous or
 * shallow caller runs unchanged.  Lane 0 keeps one frame arena; lanes created
 * later hold `frames` arenas and 8 results slots.  Each results slot of a
 * group lane then holds at least frames / 2 frames, which bounds the frames in flight past the last
 * waited one at max(2 x lanes, (lanes - 1) x 3 x frames / 2) (24 for 3 lanes
 * and the default 8).  A group of 8-bit and f32 frames runs as f32 (8-bit
 * frames converted exactly).  Queued host frames go through a pinned staging
 * block of (2 x lanes + 1) x frames frame slots, allocated at the first one
 * (1920x1200 8-bit frames, 2 lanes: 92 MB; f32: 369 MB) -- a caller that
 * never keeps more than 2 frames per lane in flight never allocates it.
 * Results, tickets and prev_descriptor are per frame and identical to
 * unbatched submission. */
int sift_hip_set_auto_micro_batch(sift_hip_t h, int frames);
int sift_hip_auto_micro_batch(sift_hip_t h, int* frames);

/* Detector::total_size (Detector.hh:62, Detector.cu:584-604). */
int sift_hip_num_keypoints(sift_hip_t h, int* n);
/* Capacities of the handle's per-frame buffers (host-only, valid right after
 * sift_hip_create): 3x3x3 candidates, refined keypoints, oriented slots and
 * results.  Sized from the octave geometry and numFeatures (maxKeypoints
 * overrides the result capacity); NULL arguments are skipped. */
int sift_hip_capacities(sift_hip_t h, int* candidates, int* refined, int* oriented, int* results);

/* Non-zero when a capacity (candidates / keypoints / results) overflowed. */
int sift_hip_overflow_flags(sift_hip_t h, int* flags);

/* Device result arrays (Detector.hh:54-57): kpts = float3 {x, y, layer}
 * per keypoint, features = float4 {octave packed as float, size, response,
 * angle}, descriptors = 128 x IEEE half (values 0..255) per keypoint.
 * prev_desc = the previous frame's descriptors (Detector.cu:136-141).  Blocks
 * the host until the current frame's counts are final (they come from the
 * device), as the reference's own count read-back does (Detector.cu:542-548). */
int sift_hip_results_device(sift_hip_t h, const float** kpts3, const float** feats4,
                            const uint16_t** desc, const uint16_t** prev_desc,
                            int* prev_count, int* capacity);

/* Detector::copyToHost(bool descriptor) (Detector.cu:606-634).  Copies
 * min(count, cap) results; desc may be NULL. */
int sift_hip_copy_to_host(sift_hip_t h, float* kpts3, float* feats4, uint16_t* desc, int cap);

/* The same results without a copy into caller memory: the reference's
 * detector-owned host vectors final_kpts / final_features / descriptors
 * (Detector.hh:58-60, filled by copyToHost).  Returns pointers into the
 * handle's pinned results region of the current frame (*count rows; desc may
 * be NULL).  A frame submitted from host memory already had its results
 * written there by its last kernel; any other frame's are copied there by
 * this call.  The rows stay valid while the frame is the current or the
 * previous one (the lifetime of prev_descriptor): until a second later frame
 * has been made current by wait / detect.  Read-only for the caller. */
int sift_hip_results_host(sift_hip_t h, const float** kpts3, const float** feats4, const uint16_t** desc,
                          int* count);

/* Device-to-device copy of this frame's descriptors (e.g. into a torch tensor
 * for an RCCL all-gather).  Copies min(count, cap) rows, pads nothing.  The
 * row count is needed on the host, so this call (like sift_hip_results_device
 * and sift_hip_num_keypoints after an unsynchronised detect) first blocks the
 * host until the frame's counts are final; the copy itself is then enqueued on
 * `stream`. */
int sift_hip_copy_descriptors_device(sift_hip_t h, uint16_t* dst, int cap, void* stream);

/* The current frame's matcher sidecar (device pointers, valid as its
 * descriptor rows): int8 codes v - 128 (128 B per keypoint row) and per row
 * the key bias -(256 |c|^2 + (row & 255)), written by the descriptor kernel
 * beside the fp16 rows.  The C5 exchange all-gathers these (132 B per row
 * instead of 256) and matches them with sift_hip_match_codes_batched.  No
 * reference counterpart (the reference gathers nothing, Match.cu:8-33). */
int sift_hip_results_sidecar(sift_hip_t h, const int8_t** codes, const int** keys);

/* Detector::setDataGen(path) (Detector.hh:48-51; the reference dumps each
 * stage's octave-0 inputs/outputs as msgpack+zlib, Detector.cu:145-229,
 * PerfData.cuh:12-155).  With a non-empty dir every following single-frame
 * detect completes synchronously and writes this build's stage dumps of the
 * frame into dir (overwritten per frame; dir is created): meta.json (config,
 * octave geometry, counts, file layouts), input.f32, gauss_o<o>_l<l>.f32 (every
 * Gaussian plane), candidates.i32, kpts3.f32, feats4.f32, desc.f16, and the
 * keypoint stages' device records refined.rec, oriented.rec, jobs.rec,
 * range.u32, counters.u32 -- raw little-endian arrays.  tests/stage_check.py replays a dump against
 * the CPU oracle and this library.  NULL or "" switches the dumps off. */
int sift_hip_set_datagen(sift_hip_t h, const char* dir);

/* Per-stage replay (the reference's tool/perf.cu:43-100, which runs each
 * HostInterface.hh:11-69 stage -- runFilter ... runDescriptor -- alone on a
 * setDataGen snapshot): runs ONE stage of the pipeline on the inputs recorded
 * in a sift_hip_set_datagen dump directory and writes that stage's outputs,
 * with the dump's file names and formats, into out_dir.  Stages and files:
 *   "pyramid"     input.f32                          -> gauss_o<o>_l<l>.f32
 *   "extrema"     gauss planes                       -> candidates.i32
 *   "refine"      planes, candidates.i32             -> refined.rec
 *   "orientation" planes, refined.rec                -> oriented.rec
 *   "order"       planes, oriented.rec, counters.u32 -> kpts3.f32, feats4.f32, jobs.rec
 *   "descriptor"  planes, jobs.rec, range.u32        -> desc.f16
 * The dump must come from a handle of the same configuration.  Synchronous;
 * the handle's current results are discarded (it is left as after warm-up). */
int sift_hip_replay_stage(sift_hip_t h, const char* dump_dir, const char* stage, const char* out_dir);

/* Stage timing for roofline reporting: when enabled, the next detect calls run
 * un-graphed with HIP events around every kernel; names are stable strings.
 * enable >= 2 also repeats each (pure) blur launch `enable` times back to back
 * inside its event pair, so the per-launch figure carries one event pair per
 * `enable` launches instead of one per launch. */
int sift_hip_set_timing(sift_hip_t h, int enable);
int sift_hip_timing_count(sift_hip_t h, int* n);
int sift_hip_timing_entry(sift_hip_t h, int i, const char** name, double* total_ms,
                          int* launches, double* algo_bytes);
int sift_hip_timing_reset(sift_hip_t h);

/* Debug/parity accessors (tests): Gaussian plane (octave, layer) as w*h floats;
 * pre-refinement candidates as (octave, layer, r, c) int quadruples. */
int sift_hip_debug_gaussian(sift_hip_t h, int octave, int layer, float* out);
int sift_hip_debug_candidates(sift_hip_t h, int* quads, int cap, int* count);

/* --- Brute-force matcher (replaces sift_cuda::matchBruteForce, Match.cuh:9-25) */

/* Scratch for up to max_query x max_train per pair and max_pairs pairs.  One
 * launch per match call: the split workgroups merge their top-2 through
 * device-scope atomics in this scratch, so calls on ONE matcher must be
 * ordered (same stream, or synchronised); use one matcher per stream for
 * concurrent matching. */
int sift_hip_matcher_create(int device, int max_query, int max_train, int max_pairs,
                            sift_hip_matcher_t* out);
int sift_hip_matcher_destroy(sift_hip_matcher_t m);

/* Top-2 L2 neighbours of each query row in train, 128-D half descriptors in
 * device memory.  Outputs (device, may be NULL): idx2[2*i+{0,1}] (-1 if none),
 * d2[2*i+{0,1}] squared L2 distance (exact for integer descriptors).
 * match[i] = idx2[2i] if d2[2i] < ratio^2 * d2[2i+1] (ratio on distances,
 * ratio_on_squared = 0) or d2[2i] < ratio * d2[2i+1] (ratio_on_squared = 1, the
 * reference's Match.cu:172 convention), else -1; a query with one train row
 * matches it.  Enqueued on `stream`. */
int sift_hip_match_device(sift_hip_matcher_t m, const uint16_t* query, int nq,
                          const uint16_t* train, int nt, float ratio, int ratio_on_squared,
                          int* idx2, float* d2, int* match, void* stream);

/* P independent (query_p, train_p) pairs in ONE launch (8-way cross-GPU match).
 * Arrays of P device pointers / counts live in host memory; outputs are packed
 * per pair at offset sum_{q<p} nq[q]. */
int sift_hip_match_batched(sift_hip_matcher_t m, int P, const uint16_t* const* query,
                           const int* nq, const uint16_t* const* train, const int* nt,
                           float ratio, int ratio_on_squared, int* idx2, float* d2,
                           int* match, void* stream);

/* Descriptor buffers handed out by a detector handle (sift_hip_results_device
 * and the batch accessors: the base of a results slot) carry a matcher
 * sidecar written by the same kernel -- int8 codes v - 128 and a per-row key
 * bias.  A single-pair call whose query and train pointers are both such
 * bases (e.g. matchBruteForce(prev_descriptor, n0, device_descriptor, n1))
 * matches those codes directly: no fp16 conversion, no prep launch (results
 * identical).  Treat detector buffers as read-only.  enable = 0 turns the
 * lookup off for matcher m (every call converts the fp16 rows). */
int sift_hip_matcher_set_sidecars(sift_hip_matcher_t m, int enable);

/* The caller wrote into a detector descriptor buffer (a results-slot base as
 * handed out above; C++: DeviceBuffer::mutable_data, Python:
 * DeviceBuffer.mutable_data): its sidecar no longer describes the rows, so
 * matches on that buffer convert the fp16 rows, as for a foreign buffer, until
 * the detector launches a frame into it again.  Unknown pointers: no-op. */
int sift_hip_descriptors_written(const uint16_t* desc);

/* Pairs of code sets already in device memory (e.g. every rank's sidecar
 * all-gathered, C5): int8 codes (128 B rows) and int32 key biases as
 * sift_hip_results_sidecar lays them out (biases computed with set-local row
 * indices).  Pair p matches the nq[p] query rows starting at code row qrow0[p]
 * (their biases from key index qkey0[p]) against the nt[p] train rows starting
 * at code row trow0[p] (biases from tkey0[p]), all pairs in ONE batched launch
 * with no conversion (no k_match_prep).  Outputs and the ratio test as
 * sift_hip_match_batched (packed per pair).  Host arrays of P ints. */
int sift_hip_match_codes_batched(sift_hip_matcher_t m, const int8_t* codes, const int* keys, int P,
                                 const int* qrow0, const int* qkey0, const int* nq, const int* trow0,
                                 const int* tkey0, const int* nt, float ratio, int ratio_on_squared, int* idx2,
                                 float* d2, int* match, void* stream);

/* matchBruteForce(des, num_des, src, num_src) (Match.cu:8-33): synchronous,
 * result to host memory out[nq]. */
int sift_hip_match_host(sift_hip_matcher_t m, const uint16_t* query, int nq,
                        const uint16_t* train, int nt, float ratio, int ratio_on_squared,
                        int* out);

/* The launch plan a match call of this shape gets: train splits S per query
 * block (S > 1: split workgroups merge their top-2 through the scratch's
 * atomics) and waves per workgroup.  Host-only (no GPU call beyond reading the
 * CU count; 256 without a device), for tests and tools. */
int sift_hip_match_plan(int max_query, int max_train, int pairs, int* splits, int* waves);

/* --- Multi-GPU (the reference binds one Detector to the current
 * device, Detector.hh:26-29, and has no multi-GPU path) ----------------------- */

/* Binds the calling host thread to `device` (a thread per GPU drives its own
 * Detector; sift_hip_malloc & co. then allocate there). */
int sift_hip_set_device(int device);
/* Any-to-any device copy (peer or same device) on `stream` (NULL: synchronous). */
int sift_hip_memcpy_d2d(void* dst, const void* src, size_t bytes, void* stream);

/* Node-local communicator over RCCL (xGMI): one rank per entry of `devices`
 * (distinct GPUs), created with ncclCommInitAll.  RCCL is loaded with dlopen on
 * first use (no link-time dependency). */
typedef struct sift_hip_comm* sift_hip_comm_t;
int sift_hip_comm_create(int ndev, const int* devices, sift_hip_comm_t* out);
int sift_hip_comm_destroy(sift_hip_comm_t c);
int sift_hip_comm_size(sift_hip_comm_t c, int* n);
/* All-gather: recv[k] (device k) receives ndev * bytes, rank r's send[r] at
 * offset r * bytes (the C5 exchange of descriptor sets).  One ncclAllGather per
 * rank inside an ncclGroupStart/End; streams[k] may be NULL for the
 * communicator's own stream, and with streams == NULL the call returns after
 * every rank's copy has completed.  Ordering: the gather runs on streams[k]
 * (or the communicator's non-blocking stream), which is NOT ordered after the
 * stream that produced send[k] -- pass the producer's stream in streams[k], or
 * make send[k] complete (stream/device synchronise) before the call. */
int sift_hip_comm_allgather(sift_hip_comm_t c, const void* const* send, void* const* recv, size_t bytes,
                            void* const* streams);

/* --- Utilities -------------------------------------------------------------- */

/* Deterministic synthetic frame, fp32 0..255 integers. */
int sift_synth_frame(unsigned frame_index, int w, int h, float* out);

/* Device helpers for callers without a HIP toolchain (ctypes tests/bench). */
int sift_hip_device_count(int* n);
int sift_hip_malloc(void** p, size_t bytes);
int sift_hip_free(void* p);
int sift_hip_memcpy_h2d(void* dst, const void* src, size_t bytes);
int sift_hip_memcpy_d2h(void* dst, const void* src, size_t bytes);
int sift_hip_device_sync(void);

#ifdef __cplusplus
}
#endif
#endif
