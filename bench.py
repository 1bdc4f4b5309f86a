#!/usr/bin/env python3
"""Benchmark of the SIFT hot path (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
        --master-addr 127.0.0.1 --master-port P bench.py --gpus N --steps K --warmup W

Workload (BASELINE.json configs[1], "C2"): synthetic 1920x1200 frames,
detectAndCompute with numOctaveLayers=3 (5 DoG scales per octave), 3 octaves,
upscale=false, numFeatures=5000; frames are resident in HBM when the timed
region starts (H2D excluded, like the reference's readme.md:11).  A step is one
batch of --batch frames (default 16) through a frame-batch detector: every
pipeline launch processes the whole batch (sift_hip_set_batch), and steps
rotate over --streams detectors (default 2, each its own HIP stream + graphs)
so consecutive batches overlap.  Every frame is fully processed (results are
those of the single-frame pipeline, bit for bit: tests/test_gpu_batch.py).
Frames shard per image across ranks with no data-path collective ("weak").
value = all frames' pixels / max-over-ranks wall time, in Mpix/s; the strictly
serial one-frame-at-a-time rate and the synchronous per-frame latency are
reported beside it.

Side measurements in the same JSON line: 2000x2000x128 brute-force match (C3),
the 8-way all-gather + pairwise match (C5) when N > 1, the per-kernel roofline of
the dominant kernel (HIP events on the stream the kernels run on) and the CPU
oracle on the host's cores (bounded sample).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "another-cuda-sift_amd"), os.path.join(ROOT, "tests")]

# One HIP runtime per process: torch (bundled libamdhip64) must load first.
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402
import numpy as np  # noqa: E402

import sift_amd as sift  # noqa: E402
from sift_amd import multi  # noqa: E402

METRIC = "detectAndCompute Mpix/s + 2kx2k 128-D match ms at 1/2/4/8 MI355X"
W, H = 1920, 1200
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
I8_MFMA_PEAK_TOPS = 5000.0  # dense int8 MFMA (MI355X_MICROARCH.md: 2x the 2.5 PF bf16 rate); the matcher's dtype


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL) on the 8-GPU node; gloo to rehearse N > 1 on one GPU")
    ap.add_argument("--streams", type=int, default=2, help="detectors (HIP streams) steps rotate over")
    ap.add_argument("--batch", type=int, default=16,
                    help="frames per step: one launch per pipeline stage processes the whole batch "
                         "(sift_hip_set_batch); 1 = single-frame graphs")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="bounded CPU-oracle sample length")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--roofline-only", action="store_true",
                    help="only the eager per-kernel timing pass (every launch event-bracketed): the command whose "
                         "rocprofv3 --kernel-trace --stats summary is committed beside the roofline numbers")
    ap.add_argument("--traffic-summary", default=os.path.join(ROOT, "profiles", "round6", "pmc_summary.json"),
                    help="PMC summary (tools/pmc_summary.py) with FETCH_SIZE/WRITE_SIZE of this code")
    ap.add_argument("--cv-traffic-summary",
                    default=os.path.join(ROOT, "profiles", "round6", "pmc_summary_cvdefault.json"),
                    help="PMC summary of the OpenCV-default leg (tools/pmc.sh ... --upscale --octaves 0 --features 0)")
    ap.add_argument("--no-cv-default", action="store_true", help="skip the OpenCV-default configuration leg")
    ap.add_argument("--exact-descriptors", action="store_true",
                    help="run the C2 steps in the exact descriptor mode (SIFT_HIP_DESC_EXACT) instead of the default")
    ap.add_argument("--allow-ab-build", action="store_true",
                    help="run on a library built with A/B or instrumentation macros (never for reported numbers)")
    ap.add_argument("--launcher-selftest", action="store_true",
                    help="CPU test of the N-rank launcher: the ranks join a gloo group and report; no GPU work")
    return ap.parse_args()


def _free_port():
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """`python bench.py --gpus N` without a torchrun parent: start N rank
    processes (LOCAL_RANK = RANK = r, one per GPU) with the torch.distributed
    environment and wait for them.  This process only parses arguments -- it
    never touches the GPU -- so the ranks are plain fresh child processes.
    Rank 0 inherits stdout and prints the JSON line; if a rank fails the
    others are terminated (by PID) and the exit code is non-zero."""
    import subprocess

    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    rc, live = 0, list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks", file=sys.stderr)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    return rc


def launcher_selftest(world, rank):
    """The N > 1 plumbing without a GPU: gloo group, barrier, max over ranks."""
    if world > 1:
        dist.init_process_group("gloo")
    t = torch.tensor([float(rank + 1)])
    if world > 1:
        dist.barrier()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "n_gpus": world, "selftest": True, "max_rank_plus_1": t.item()}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def make_config(**kw):
    cfg = dict(col_width=W, row_width=H, numFeatures=5000, numOctaveLayers=3, upscale=False, numOctaves=3)
    cfg.update(kw)
    return sift.CudaSiftConfig(**cfg)


def timed_rows(summ, kernel_names):
    """The PMC rows of the profiled batch launches only.  tools/profile_frames.py
    --batch B --frames F runs the handle's warm-up first: kSlots (4) replays of
    each batch graph and 4 of each single-frame graph, then F batches.  A
    (kernel, grid) row of a batch launch therefore has a multiple of 4 + F
    dispatches and a single-frame warm-up row a multiple of 4; only the former
    have the bench's grid (the verdict's round-3 finding: mixing them averaged
    extrema's 16-frame rows with its single-frame ones)."""
    rows = [k for k in summ.get("kernels", []) if k["kernel"].split("<")[0].split("::")[-1] in kernel_names]
    if summ.get("profiled_only"):  # tools/pmc_summary.py already dropped the warm-up dispatches
        return rows
    unit = 4 + 5  # older summaries: kSlots warm-up replays + tools/pmc.sh's 5 profiled batches
    return [k for k in rows if k.get("dispatches", 0) >= unit and k["dispatches"] % unit == 0]


def pmc_traffic(summary_path, kernel_names):
    """HBM bytes per launch of a kernel family from a committed PMC summary
    (tools/pmc.sh + tools/pmc_summary.py over tools/profile_frames.py, i.e.
    the bench's C2 frame, on the same code): total over every dispatch of the
    named kernels / their dispatch count, so it averages over the frame's
    launches exactly like `achieved`.

    MI355X_MICROARCH.md HBM section + our calibration (tools/hbm_calib.hip, in
    the summary): FETCH_SIZE counts 1/2 of the bytes read, WRITE_SIZE is exact;
    both in KiB."""
    try:
        with open(summary_path) as f:
            summ = json.load(f)
    except (OSError, ValueError):
        return None
    cal = summ.get("calibration_counter_over_true_bytes", {})
    fetch_scale = 1.0 / cal.get("copy4:FETCH_SIZE", 0.5)
    write_scale = 1.0 / cal.get("copy4:WRITE_SIZE", 1.0)
    rows = [k for k in timed_rows(summ, kernel_names) if "FETCH_SIZE" in k and "WRITE_SIZE" in k]
    tot, n = 0.0, 0
    for k in rows:
        tot += (k["FETCH_SIZE"] * fetch_scale + k["WRITE_SIZE"] * write_scale) * 1024 * k["dispatches"]
        n += k["dispatches"]
    return {"bytes_per_launch": round(tot / n), "launches": n, "source": os.path.relpath(summary_path, ROOT)} if n else None


BLUR_REPS = 10
C4_PASSES = 7  # timed repetitions of the 256-frame C4 pass


def stage_table(timing, nt):
    """Per-frame microseconds per stage (blur stages were repeated BLUR_REPS times)."""
    per = {k: v["ms"] / nt * 1e3 / (BLUR_REPS if k.startswith("blur_") else 1) for k, v in timing.items()}
    return {k: round(v, 2) for k, v in sorted(per.items(), key=lambda kv: -kv[1])}


def measure_roofline(det, frames, stride, traffic_summary, nt=20, warm=3, batch=None):
    """k_blur, the kernel with the largest share of frame time (all its launches):
    algorithmic bytes per launch / average launch duration, by HIP events on the
    detector's own stream (eager timing mode).  Each blur launch of the frame is
    repeated BLUR_REPS times back to back inside its event pair (blurs are
    pure), so the average carries the stream's inter-kernel gap but not one
    event pair per launch."""
    det.set_timing(True, blur_reps=BLUR_REPS)

    def run(s):
        if batch is not None:  # (tensor of B frames): every launch carries the B frames
            det.detectBatchDevice(batch.data_ptr(), batch.shape[0], stride, batch[0].numel() * batch.element_size())
        else:
            det.detectAndComputeDevice(frames[s % len(frames)].data_ptr(), stride, sync=True)

    for s in range(warm):
        run(s)
    det.timing_reset()
    for s in range(nt):
        run(s)
    timing = det.timing()
    det.set_timing(False)
    blurs = [v for k, v in timing.items() if k.startswith("blur_")]
    blur_launches = sum(v["launches"] for v in blurs)
    per_launch_bytes = sum(v["bytes"] for v in blurs) / blur_launches
    per_launch_s = sum(v["ms"] for v in blurs) / blur_launches / 1e3
    achieved = per_launch_bytes / per_launch_s / 1e9
    traffic = pmc_traffic(traffic_summary, ("k_blur", "k_blur2"))
    per = "step" if batch is not None else "frame"
    fr = f", {batch.shape[0]} frames per launch" if batch is not None else ""
    roof = {
        "kernel": f"k_blur / k_blur2 (all {blur_launches // nt // BLUR_REPS} blur launches/{per}{fr}, each "
                  f"x{BLUR_REPS} back to back between HIP events, eager)",
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic["bytes_per_launch"] if traffic else None,
        "traffic_source": traffic,
        "algo_bytes_per_launch": per_launch_bytes,
        "avg_launch_us": round(per_launch_s * 1e6, 3),
    }
    return {"roofline": roof, "timing": timing, "frames": nt}


def cpu_threads():
    """Threads for the CPU legs: OMP_NUM_THREADS when set (the GPU box sets it to
    this job's CPU share), else every CPU in this process's affinity mask."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    env = os.environ.get("OMP_NUM_THREADS", "")
    return (int(env) if env.isdigit() and int(env) > 0 else aff), aff, env or None


def _median_ms(fn, reps, warm=1):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts) * 1e3)


def cpu_baseline(a, cfg, c3_sets):
    """The CPU oracle (oracle/sift_oracle.cpp, OpenMP; a restatement of OpenCV
    4.x SIFT + BFMatcher knn-2, test infrastructure) on this host's cores, on
    bounded samples: C2 (the headline workload) for ~a.cpu_seconds, C1 (the
    reference's CPU plumbing, tool/extract_and_match_example.cc:62-100: detect
    two 752x480 frames with OpenCV defaults, knn-2 + ratio 0.8) and the C3
    knn-2 on the GPU bench's 2000 x 2000 sets."""
    import oracle_binding as oracle

    threads, aff, env = cpu_threads()
    p = oracle.from_config(cfg)
    imgs = [sift.synth_frame(i, W, H) for i in range(4)]
    oracle.detect_and_compute(imgs[0], p, threads=threads)  # warm
    n, t = 0, time.perf_counter()
    while True:
        oracle.detect_and_compute(imgs[n % 4], p, threads=threads)
        n += 1
        if time.perf_counter() - t > a.cpu_seconds and n >= 3:
            break
    dt = time.perf_counter() - t
    cpu = {"value": round(n * W * H / 1e6 / dt, 2), "unit": "Mpix/s", "cores": threads, "kind": "port",
           "sample": f"{n} frames of the C2 workload (1920x1200, 3 octaves, numFeatures 5000) in {dt:.1f}s, "
                     f"oracle/sift_oracle.cpp OpenMP {threads} threads",
           "cpu_model": cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": aff, "omp_num_threads": env}
    cpu["value_per_thread"] = round(cpu["value"] / threads, 3)
    cpu["stage_ms_per_frame"] = {str(threads): oracle.stage_ms()}
    # Thread scaling on the same workload, measured (1, 4 and the job's CPU
    # share; the box's OMP_NUM_THREADS is that share, and its rules cap worker
    # pools at it, so no figure is given for the host's other CPUs), with the
    # per-stage wall times that say where the threads stop helping.
    curve = {str(threads): cpu["value"]}
    for th in (1, 4):
        if th >= threads:
            continue
        oracle.detect_and_compute(imgs[1], p, threads=th)
        m, t = 0, time.perf_counter()
        while True:
            oracle.detect_and_compute(imgs[m % 4], p, threads=th)
            m += 1
            if time.perf_counter() - t > a.cpu_seconds / 4 and m >= 2:
                break
        curve[str(th)] = round(m * W * H / 1e6 / (time.perf_counter() - t), 3)
        cpu["stage_ms_per_frame"][str(th)] = oracle.stage_ms()
    cpu["scaling_curve_mpix_s"] = dict(sorted(curve.items(), key=lambda kv: int(kv[0])))
    if "1" in curve:
        cpu["value_1_thread"] = curve["1"]
        cpu["scaling_1_to_%d_threads" % threads] = round(cpu["value"] / curve["1"], 2)
    # C1: 752x480, cv::SIFT defaults (firstOctave -1, nfeatures 0), frames 0 and 1, knn-2 + ratio 0.8.
    p1 = oracle.params(nfeatures=0, firstOctave=-1)
    f0, f1 = sift.synth_frame(0, 752, 480), sift.synth_frame(1, 752, 480)
    res = {}

    def c1():
        _, d0 = oracle.detect_and_compute(f0, p1, threads=threads)
        _, d1 = oracle.detect_and_compute(f1, p1, threads=threads)
        idx, dist = oracle.knn2(d0, d1, threads=threads)
        res.update(k0=len(d0), k1=len(d1), matches=int((dist[:, 0] < 0.8 * dist[:, 1]).sum()))

    c1_ms = _median_ms(c1, 5)
    cpu["c1_752x480_detect2_match_ms"] = round(c1_ms, 2)
    cpu["c1"] = {"keypoints": [res["k0"], res["k1"]], "matches": res["matches"],
                 "note": "two detectAndCompute calls (OpenCV defaults) + knn-2 + ratio 0.8 on distances, per frame pair"}
    q, tr = (np.ascontiguousarray(x, np.float32) for x in c3_sets)
    cpu["c3_knn2_2000x2000_ms"] = round(_median_ms(lambda: oracle.knn2(q, tr, threads=threads), 5), 2)
    try:  # OpenCV itself, when the box has it (secondary)
        import cv2

        cv2.setNumThreads(threads)
        sift_cv = cv2.SIFT_create(nfeatures=5000, nOctaveLayers=3)
        u8 = imgs[0].astype(np.uint8)
        sift_cv.detectAndCompute(u8, None)
        m, t = 0, time.perf_counter()
        while time.perf_counter() - t < 5.0 or m < 3:
            sift_cv.detectAndCompute(imgs[m % 4].astype(np.uint8), None)
            m += 1
        cpu["opencv"] = {"version": cv2.__version__, "value": round(m * W * H / 1e6 / (time.perf_counter() - t), 2),
                         "note": "cv2.SIFT_create defaults (firstOctave -1), not the C2 octave count"}
    except ImportError:
        cpu["opencv"] = "cv2 not importable on this box"
    return cpu


def run_c1_gpu(local):
    """C1's pipeline on the GPU for comparison: two synchronous 752x480 frames
    through one Detector (OpenCV defaults), then matchBruteForce of the
    previous frame's descriptors against the current (ratio 0.8 on distances),
    host frames in, match indices out -- the reference tool's per-frame loop."""
    cfg1 = sift.CudaSiftConfig(col_width=752, row_width=480, numFeatures=0, upscale=True)
    det = sift.Detector(cfg1, device=local)
    det.gpuWarmUpAndAllocate()
    f = [sift.synth_frame(0, 752, 480), sift.synth_frame(1, 752, 480)]
    m = sift.Matcher(8192, 8192, device=local)
    out = {}

    def once():
        det.detectAndCompute(f[0])
        det.detectAndCompute(f[1])
        r = m.match_host(det.prev_descriptor.data(), det.prev_size, det.device_descriptor.data(), det.total_size,
                         0.8, False)
        out["matches"] = int((r >= 0).sum())
        out["k"] = [det.prev_size, det.total_size]

    ms = _median_ms(once, 20, warm=3)
    return {"ms": round(ms, 4), "keypoints": out["k"], "matches": out["matches"],
            "note": "host f32 frames, synchronous detectAndCompute x2 + matchBruteForce (prev vs current), median of 20"}



def run_ref_configs(local, dev, reps=40):
    """The reference's published configuration beside C2 (readme.md:11-16): one
    synchronous detectAndCompute per frame at the tool default -- auto octaves
    (Detector.hh:27), upscale=false, numFeatures=5000 -- on 752x480, 1920x1200
    and 1600x900 frames resident in HBM (the readme excludes transfers), median
    of `reps`; and the device memory one Detector holds (hipMemGetInfo free
    bytes before creation minus after warm-up), the readme's 84/298/214 MiB
    column.  Single-frame handles, as the reference's Detector."""
    out = {}
    for (w, h, ref_ms, ref_mib) in ((752, 480, 0.95, 84), (1920, 1200, 3.1, 298), (1600, 900, 2.5, 214)):
        torch.cuda.synchronize()
        free0 = torch.cuda.mem_get_info(local)[0]
        d = sift.Detector(sift.CudaSiftConfig(col_width=w, row_width=h, numFeatures=5000, upscale=False, numOctaves=0),
                          device=local)
        d.gpuWarmUpAndAllocate()
        torch.cuda.synchronize()
        used = free0 - torch.cuda.mem_get_info(local)[0]
        img = torch.from_numpy(sift.synth_frame(0, w, h)).to(dev)
        torch.cuda.synchronize()
        for _ in range(5):
            d.detectAndComputeDevice(img.data_ptr(), w * 4, sync=True)
        lat = []
        for _ in range(reps):
            t = time.perf_counter()
            d.detectAndComputeDevice(img.data_ptr(), w * 4, sync=True)
            lat.append(time.perf_counter() - t)
        ms = float(np.median(lat) * 1e3)
        out[f"{w}x{h}"] = {"octaves": d.nOctaves, "sync_ms_per_frame": round(ms, 4),
                           "mpix_s": round(w * h / 1e3 / ms, 1), "keypoints": d.total_size,
                           "device_mib": round(used / 2**20, 1), "ref_ms_rtx4070s": ref_ms, "ref_mib": ref_mib}
        del d, img
    out["note"] = ("reference tool default (auto octaves, upscale=false, numFeatures=5000), synchronous single frame "
                   "from HBM, median of %d; device_mib = hipMemGetInfo delta of one Detector (create + warm-up)" % reps)
    return out


def pmc_kernel(summary_path, kernel_names):
    """Per-dispatch means of a kernel family's counters in a committed PMC
    summary (the profiled batch launches only, timed_rows): corrected HBM
    bytes and the VALU busy fraction (2 cycles per wave64 VALU instruction on
    a SIMD32, over the dispatch's wall cycles x 1024 SIMDs; GRBM_GUI_ACTIVE
    sums the 8 XCDs)."""
    try:
        with open(summary_path) as f:
            summ = json.load(f)
    except (OSError, ValueError):
        return None
    cal = summ.get("calibration_counter_over_true_bytes", {})
    fetch_scale = 1.0 / cal.get("copy4:FETCH_SIZE", 0.5)
    write_scale = 1.0 / cal.get("copy4:WRITE_SIZE", 1.0)
    rows = timed_rows(summ, kernel_names)
    if not rows:
        return None
    n = sum(k["dispatches"] for k in rows)

    def mean(c):
        v = [(k[c], k["dispatches"]) for k in rows if c in k]
        return sum(x * d for x, d in v) / sum(d for _, d in v) if v else None

    out = {"dispatches": n, "source": os.path.relpath(summary_path, ROOT)}
    fs, ws = mean("FETCH_SIZE"), mean("WRITE_SIZE")
    if fs is not None and ws is not None:
        out["hbm_bytes"] = round((fs * fetch_scale + ws * write_scale) * 1024)
    valu, gui = mean("SQ_INSTS_VALU"), mean("GRBM_GUI_ACTIVE")
    if valu and gui:
        out["valu_busy_frac"] = round(2.0 * valu / (gui / 8.0 * 1024), 4)
    conf, lds = mean("SQ_LDS_BANK_CONFLICT"), mean("SQ_ACTIVE_INST_LDS")
    if conf is not None and lds:
        out["lds_bank_conflict_over_active_lds"] = round(conf / lds, 4)
    return out


def window_bytes(kpts3, feats4, first_octave=0):
    """Algorithmic (unique input) bytes of the keypoint kernels for one frame's
    final keypoints (SURVEY.md 8d keypoint term): orientation reads the
    (2r+3)^2 pixels of its r = round(4.5 scl) window plus gradient neighbours,
    once per refined keypoint (= distinct (x, y, size, octave)); the
    descriptor reads the (5 hist_width + 3)^2 pixels of its rotated 4x4-cell
    square (at most the (2r+1)^2 window, r = round(hist_width * sqrt2 * 2.5))
    and writes 256 B of descriptor + reads its 64-B job."""
    oct_ = feats4[:, 0].astype(np.int64) & 255
    oct_ = np.where(oct_ >= 128, oct_ - 256, oct_)
    size_o = feats4[:, 1] / np.exp2(oct_.astype(np.float64))  # size in its octave's pixels
    hw = 1.5 * size_o
    r_desc = np.round(hw * np.sqrt(2.0) * 2.5)
    desc = 4.0 * np.minimum((2 * r_desc + 1) ** 2, (5 * hw + 3) ** 2) + 256 + 64
    uniq = np.unique(np.stack([kpts3[:, 0], kpts3[:, 1], feats4[:, 1], feats4[:, 0]], 1), axis=0)
    o_u = uniq[:, 3].astype(np.int64) & 255
    o_u = np.where(o_u >= 128, o_u - 256, o_u) - first_octave
    r_ori = np.round(4.5 * uniq[:, 2] * 0.5 / np.exp2(o_u.astype(np.float64) + first_octave))
    ori = 4.0 * (2 * r_ori + 3) ** 2 + 32 + 32
    return float(ori.sum()), float(desc.sum()), len(uniq)


def kernel_rooflines(det, timing, steps, B, pmc_path, first_octave=0):
    """Per-kernel roofline entries of the C2 step (eager timing pass, HIP
    events on the detector's stream): algorithmic bytes per launch / average
    launch time against the 8 TB/s HBM peak, with the committed PMC summary's
    measured HBM bytes and VALU busy fraction beside it."""
    per_frame = [det.batch_copy_to_host(i, descriptor=False) for i in range(B)]
    ori_b = desc_b = 0.0
    refined = 0
    for k3, f4, _ in per_frame:
        o, d, n = window_bytes(k3, f4, first_octave)
        ori_b += o
        desc_b += d
        refined += n
    out = {}

    def entry(names, bytes_per_launch, pmc_names, note):
        ms = sum(timing[n]["ms"] for n in names if n in timing)
        launches = sum(timing[n]["launches"] for n in names if n in timing)
        if not launches:
            return None
        us = ms / launches * 1e3
        achieved = bytes_per_launch / (us * 1e-6) / 1e9
        e = {"bound": "hbm", "algo_bytes_per_launch": round(bytes_per_launch), "avg_launch_us": round(us, 3),
             "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
             "frac": round(achieved / HBM_PEAK_GBS, 4), "note": note}
        p = pmc_kernel(pmc_path, pmc_names)
        if p:
            e["pmc"] = p
            if "hbm_bytes" in p:
                e["traffic"] = p["hbm_bytes"]
                e["traffic_over_algo"] = round(p["hbm_bytes"] / bytes_per_launch, 3)
        return e

    blurs = [k for k in timing if k.startswith("blur_")]
    bl = sum(timing[k]["launches"] for k in blurs)
    out["blur"] = entry(blurs, sum(timing[k]["bytes"] for k in blurs) / bl, ("k_blur", "k_blur2"),
                        "all blur launches of a step, each x10 back to back between events; read + write of "
                        "every plane (+ the decimated base copy)")
    out["extrema"] = entry(["extrema"], timing["extrema"]["bytes"] / timing["extrema"]["launches"],
                           ("k_extrema_all",), "reads the L+3 Gaussian planes of every octave once (24 B/px)")
    out["orientation"] = entry(["orientation"], ori_b, ("k_orientation",),
                               f"window model over {refined} refined keypoints of the {B}-frame step "
                               "(L2-served windows: latency/VALU-bound, frac vs HBM is not its limit)")
    out["descriptor"] = entry(["descriptor"], desc_b, ("k_descriptor",),
                              "rotated-square window model + 256 B out + 64 B job per keypoint "
                              "(L2-served windows: latency/VALU-bound)")
    return {k: v for k, v in out.items() if v}

def main():
    a = parse()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        sys.exit(launch_ranks(a.gpus))  # before any GPU call in this process
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        print(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    if a.launcher_selftest:
        launcher_selftest(world, rank)
        return
    if not sift.is_default_build() and not a.allow_ab_build:
        print(f"bench.py: {sift.LIB_PATH} is a non-default build ({sift.version()}); rebuild with `make`",
              file=sys.stderr)
        sys.exit(3)
    local = local % max(torch.cuda.device_count(), 1)  # one rank per GPU on the driver's node
    torch.cuda.set_device(local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:  # gloo: exercises the N > 1 logic where RCCL cannot run (several ranks on one GPU)
            dist.init_process_group("gloo")
    dev = torch.device("cuda", local)
    cdev = dev if a.dist_backend == "nccl" else torch.device("cpu")  # collectives' tensors

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=cdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # ---- C2: detectAndCompute on HBM-resident frames -------------------------
    cfg = make_config()
    # a.streams detectors (one HIP stream + graph pair each) take consecutive
    # frames round-robin, so independent frames overlap on the GPU; every step
    # is still one complete frame.
    B = max(a.batch, 1)
    nstreams = 1 if a.roofline_only else a.streams
    dets = [sift.Detector(cfg, device=local, batch=B, exact_descriptors=a.exact_descriptors, lanes=1)
            for _ in range(nstreams)]
    for d in dets:
        d.gpuWarmUpAndAllocate()
    det = dets[0]
    nframes = 4
    frames = [torch.from_numpy(sift.synth_frame(1000 * rank + i, W, H)).to(dev) for i in range(nframes)]
    stride = W * 4
    # A step's batch: B distinct frames, contiguous (frame stride W*H*4 bytes).
    fb = torch.from_numpy(np.stack([sift.synth_frame(1000 * rank + i, W, H) for i in range(B)])).to(dev)
    torch.cuda.synchronize()

    def step(s):
        d = dets[s % len(dets)]
        if B == 1:
            d.detectAndComputeDevice(frames[s % nframes].data_ptr(), stride, sync=False)
        else:
            d.detectBatchDevice(fb.data_ptr(), B, stride, W * H * 4, sync=False)

    if a.roofline_only:
        rl = measure_roofline(det, frames, stride, a.traffic_summary, nt=a.steps, batch=fb if B > 1 else None)
        if rank == 0:
            nt = rl["frames"] * B
            print(json.dumps({"roofline": rl["roofline"], "frames": nt, "frames_per_launch": B,
                              "stage_us_per_frame_eager": stage_table(rl["timing"], nt)}),
                  flush=True)
        return
    for s in range(a.warmup):
        step(s)
    for d in dets:
        d.sync()
    kcount = det.total_size
    sum_px = sum(det.octave_dims(o)[0] * det.octave_dims(o)[1] for o in range(det.nOctaves))
    barrier()
    t0 = time.perf_counter()
    for s in range(a.steps):
        step(s)
    for d in dets:
        d.sync()
    t1 = time.perf_counter()
    barrier()
    elapsed = max_over_ranks(t1 - t0)
    ms_per_step = elapsed / a.steps * 1e3
    value = world * a.steps * B * W * H / 1e6 / elapsed
    ms_per_frame = elapsed / (a.steps * B) * 1e3
    detb = dets[0]  # kept for the roofline pass (same frames per launch as the timed steps)
    del dets

    # The same frames one at a time through ONE single-frame detector (frames
    # strictly serialised): latency-side reference numbers.
    det = sift.Detector(cfg, device=local, lanes=1)
    det.gpuWarmUpAndAllocate()
    n1 = max(a.steps // 2, 1)
    barrier()
    t = time.perf_counter()
    for s in range(n1):
        det.detectAndComputeDevice(frames[s % nframes].data_ptr(), stride, sync=False)
    det.sync()
    single = max_over_ranks(time.perf_counter() - t)
    single_value = world * n1 * W * H / 1e6 / single

    # The C2 step with the exact descriptor mode (SIFT_HIP_DESC_EXACT: OpenCV's
    # sequential float histogram, descriptors bit-identical to the oracle):
    # its cost next to the default fixed-point mode (value above).
    detx = [sift.Detector(cfg, device=local, batch=B, exact_descriptors=True, lanes=1) for _ in range(nstreams)]
    for d in detx:
        d.gpuWarmUpAndAllocate()

    def stepx(s):
        d = detx[s % len(detx)]
        if B == 1:
            d.detectAndComputeDevice(frames[s % nframes].data_ptr(), stride, sync=False)
        else:
            d.detectBatchDevice(fb.data_ptr(), B, stride, W * H * 4, sync=False)

    nx = max(a.steps // 4, 1)
    for s in range(2 * len(detx)):
        stepx(s)
    for d in detx:
        d.sync()
    barrier()
    t = time.perf_counter()
    for s in range(nx):
        stepx(s)
    for d in detx:
        d.sync()
    exact_t = max_over_ranks(time.perf_counter() - t)
    exact_leg = {"value": round(world * nx * B * W * H / 1e6 / exact_t, 2), "unit": "Mpix/s",
                 "ms_per_frame": round(exact_t / (nx * B) * 1e3, 4), "steps": nx,
                 "note": "same C2 steps with sift_hip_set_descriptor_mode(SIFT_HIP_DESC_EXACT): descriptors "
                         "bit-identical to the oracle (tests/test_gpu_parity.py::test_exact_descriptors_bitexact)"}
    del detx

    # ---- C2 at OpenCV's defaults: upscale (firstOctave -1), numFeatures 0 ----
    # (SURVEY 8d's secondary C2 row; the configuration the parity bar is defined
    # on, reference Detector.cu:235-252 / CudaSiftConfig.hh:12-13.)  Same frames,
    # batches and streams as C2; its own eager stage table and per-kernel
    # rooflines (a 4x base plane, ~4x the keypoints of the 5000-feature cap).
    def cv_default_leg():
        cfgd = make_config(upscale=True, numFeatures=0, numOctaves=0)
        detd = [sift.Detector(cfgd, device=local, batch=B, lanes=1) for _ in range(nstreams)]
        for d in detd:
            d.gpuWarmUpAndAllocate()

        def stepd(s):
            detd[s % len(detd)].detectBatchDevice(fb.data_ptr(), B, stride, W * H * 4, sync=False)

        for s in range(2 * len(detd)):
            stepd(s)
        for d in detd:
            d.sync()
        nd = max(a.steps // 4, 1)
        barrier()
        t = time.perf_counter()
        for s in range(nd):
            stepd(s)
        for d in detd:
            d.sync()
        td = max_over_ranks(time.perf_counter() - t)
        kpf = detd[0].total_size
        octs = detd[0].nOctaves
        rld = measure_roofline(detd[0], frames, stride, a.cv_traffic_summary, nt=6, batch=fb)
        nt_d = rld["frames"] * B
        stages_d = stage_table(rld["timing"], nt_d)
        rk_d = kernel_rooflines(detd[0], rld["timing"], rld["frames"], B, a.cv_traffic_summary, first_octave=-1)
        return {"value": round(world * nd * B * W * H / 1e6 / td, 2), "unit": "Mpix/s",
                "ms_per_frame": round(td / (nd * B) * 1e3, 4), "steps": nd, "frames_per_launch": B,
                "streams": len(detd), "octaves": octs, "keypoints_per_frame": kpf,
                "stage_us_per_frame_eager": stages_d, "stage_sum_us_eager": round(sum(stages_d.values()), 1),
                "dominant_stage": next(iter(stages_d)), "roofline_kernels": rk_d,
                "note": "1920x1200 frames (the C2 batch) with OpenCV's cv::SIFT defaults: upscale=true (2x INTER_LINEAR "
                        "base, firstOctave -1), numFeatures=0 (keep all), auto octaves; fixed-point descriptors"}

    cv_default = None
    if not a.no_cv_default:
        try:
            cv_default = cv_default_leg()
        except Exception as e:  # noqa: BLE001 -- side leg: keep the C2 line
            cv_default = {"error": repr(e)[:300]}

    # ---- C4: 256 synthetic 1600x900 frames sharded per image over the ranks -------
    W4, H4, N4 = 1600, 900, 256
    mine4 = multi.frame_shard(N4, rank, world)
    dets4 = [sift.Detector(make_config(col_width=W4, row_width=H4, numOctaves=0), device=local, batch=B, lanes=1)
             for _ in range(a.streams)]
    for d in dets4:
        d.gpuWarmUpAndAllocate()
    nd4 = max(min(len(mine4), 4 if B == 1 else B), 1)  # distinct frames resident per rank
    fb4 = torch.from_numpy(np.stack([sift.synth_frame(i, W4, H4) for i in (mine4 or [0])[:nd4]])).to(dev)
    groups = [mine4[k:k + B] for k in range(0, len(mine4), B)]  # the last one may be a partial batch

    def step4(s, n):
        d = dets4[s % a.streams]
        if B == 1:
            d.detectAndComputeDevice(fb4[s % nd4].data_ptr(), W4 * 4, sync=False)
        else:
            d.detectBatchDevice(fb4.data_ptr(), n, W4 * 4, W4 * H4 * 4, sync=False)

    for s in range(2 * a.streams):
        step4(s, min(B, nd4))
    for d in dets4:
        d.sync()
    # The 256-frame pass is repeated (at N = 8 one pass is 2 batches per rank,
    # ~2 ms: a single sample would carry launch jitter); median and spread.
    passes4 = []
    for _ in range(C4_PASSES):
        barrier()
        t = time.perf_counter()
        for s, g in enumerate(groups):
            step4(s, len(g))
        for d in dets4:
            d.sync()
        passes4.append(max_over_ranks(time.perf_counter() - t))
    t4 = float(np.median(passes4))
    c4 = {"frames": N4, "frame": f"{W4}x{H4}", "octaves": "auto", "value": round(N4 * W4 * H4 / 1e6 / t4, 2),
          "unit": "Mpix/s", "ms_total": round(t4 * 1e3, 3), "passes": len(passes4),
          "median_ms": round(t4 * 1e3, 3), "min_ms": round(min(passes4) * 1e3, 3),
          "max_ms": round(max(passes4) * 1e3, 3),
          "spread": round((max(passes4) - min(passes4)) / t4, 4),
          "frames_per_rank": len(mine4), "frames_per_launch": B,
          "note": f"frame i on rank i mod N (no collective); {nd4} distinct synthetic frames per rank, "
                  f"{B} frames per launch, batches rotating over {a.streams} streams; value from the median of "
                  f"{len(passes4)} passes (max over ranks per pass), spread = (max - min) / median"}
    del dets4, fb4

    # Synchronous per-frame latency (reference semantics: detectAndCompute blocks).
    lat = []
    for s in range(min(a.steps, 50)):
        t = time.perf_counter()
        det.detectAndComputeDevice(frames[s % nframes].data_ptr(), stride, sync=True)
        lat.append(time.perf_counter() - t)
    sync_ms = float(np.median(lat) * 1e3)

    def pipelined_legs():
        # ---- Host input path, PCIe-inclusive (reported beside `value`, never as it) ----
        # Host frame in -> keypoints, features and descriptors back in host memory,
        # one detector.  (a) the reference's sequence: synchronous fp32 upload,
        # detectAndCompute, copyToHost(true); (b) 8-bit frames through submit/wait
        # with the next frame staged and uploaded while the current one computes.
        host_f32 = [sift.synth_frame(1000 * rank + i, W, H) for i in range(nframes)]
        host_u8 = [f.astype(np.uint8) for f in host_f32]
        nh = max(min(a.steps, 60), 4)
        for s in range(3):
            det.detectAndCompute(host_f32[s % nframes])
            det.copyToHost(True)
        t = time.perf_counter()
        for s in range(nh):
            det.detectAndCompute(host_f32[s % nframes])
            det.copyToHost(True)
        t_sync = max_over_ranks(time.perf_counter() - t)
        # Frames in flight at the drop-in API: submit/wait with `depth` frames
        # outstanding on a detector with that many compute lanes (one stream,
        # frame arenas and graphs per lane; consecutive frames overlap).
        PIPE_LANES, PIPE_DEPTH = 3, 6  # (3 x 3: 0.118-0.122 ms/frame for device frames, 3 x 6: 0.114-0.117)
        detp = sift.Detector(cfg, device=local, lanes=PIPE_LANES)
        detp.gpuWarmUpAndAllocate()

        def copy_out():
            detp.copyToHost(True)

        def view_out():  # the detector's pinned host rows, no copy (sift_hip_results_host)
            k3, _, d = detp.results_host(True)
            if len(k3):
                float(k3[-1, 0]) + float(d[-1, -1])

        def pipelined(submit, fetch):
            # The first `warm` frames (the same loop) create and warm the lanes,
            # their staging and results regions; then npipe frames are timed
            # (at least 8 x the frames in flight, so the pipeline's fill and
            # drain stay a small part of the run).  Returns the time of nh
            # frames at the measured rate (the legs below divide by nh).
            tickets, warm = [], max(3 * PIPE_DEPTH, 24)
            npipe = max(nh, 8 * PIPE_DEPTH)
            for s in range(npipe + warm):
                if s == warm:
                    while tickets:
                        detp.wait(tickets.pop(0))
                        if fetch:
                            fetch()
                    t = time.perf_counter()
                tickets.append(submit(s))
                if len(tickets) == PIPE_DEPTH:
                    detp.wait(tickets.pop(0))
                    if fetch:
                        fetch()
            while tickets:
                detp.wait(tickets.pop(0))
                if fetch:
                    fetch()
            return max_over_ranks(time.perf_counter() - t) * nh / npipe

        t_pipe = pipelined(lambda s: detp.submit(host_u8[s % nframes]), copy_out)
        dev_u8 = [torch.from_numpy(f).to(dev) for f in host_u8]
        torch.cuda.synchronize()
        t_dev = pipelined(lambda s: detp.submitDevice(frames[s % nframes].data_ptr(), stride), None)
        t_dev8 = pipelined(lambda s: detp.submitDevice(dev_u8[s % nframes].data_ptr(), W, u8=True), None)
        shallow_u8 = {"value": round(world * nh * W * H / 1e6 / t_pipe, 2), "ms_per_frame": round(t_pipe / nh * 1e3, 4),
                      "lanes": PIPE_LANES, "in_flight": PIPE_DEPTH,
                      "note": f"the same loop with {PIPE_DEPTH} frames in flight (2 per lane: every frame launched alone)"}
        # The same default handle (no micro-batch call) with AUTO_DEPTH frames in
        # flight: past 2 frames per lane the submitted frames queue and run as
        # automatic launch groups of up to 8 (sift_hip_set_auto_micro_batch).
        AUTO_DEPTH = 24
        PIPE_DEPTH_SAVED, PIPE_DEPTH = PIPE_DEPTH, AUTO_DEPTH
        t_ah = pipelined(lambda s: detp.submit(host_u8[s % nframes]), copy_out)
        t_av = pipelined(lambda s: detp.submit(host_u8[s % nframes]), view_out)
        t_ad = pipelined(lambda s: detp.submitDevice(frames[s % nframes].data_ptr(), stride), None)
        t_ad8 = pipelined(lambda s: detp.submitDevice(dev_u8[s % nframes].data_ptr(), W, u8=True), None)
        PIPE_DEPTH = PIPE_DEPTH_SAVED
        auto_note = (f"default handle ({PIPE_LANES} lanes, no micro-batch call), {AUTO_DEPTH} frames in flight: past 2 "
                     f"per lane they run as automatic launch groups of up to {detp.auto_micro_batch()} frames")
        host_input = {
            "sync_f32": {"value": round(world * nh * W * H / 1e6 / t_sync, 2), "ms_per_frame": round(t_sync / nh * 1e3, 4)},
            "pipelined_u8": {"value": round(world * nh * W * H / 1e6 / t_ah, 2), "ms_per_frame": round(t_ah / nh * 1e3, 4),
                             "lanes": PIPE_LANES, "in_flight": AUTO_DEPTH, "lanes_created": detp.lanes()[1]},
            "pipelined_u8_views": {"value": round(world * nh * W * H / 1e6 / t_av, 2),
                                   "ms_per_frame": round(t_av / nh * 1e3, 4), "lanes": PIPE_LANES, "in_flight": AUTO_DEPTH,
                                   "note": "results_host(True) after every wait instead of copyToHost(True)"},
            "pipelined_u8_in_flight_6": shallow_u8,
            "unit": "Mpix/s",
            "note": "PCIe-inclusive, host frame -> results in host memory (copyToHost with descriptors), one detector; "
                    f"pipelined: submit/wait on a {auto_note}",
        }
        shallow_dev = {
            "f32": {"value": round(world * nh * W * H / 1e6 / t_dev, 2), "ms_per_frame": round(t_dev / nh * 1e3, 4)},
            "u8": {"value": round(world * nh * W * H / 1e6 / t_dev8, 2), "ms_per_frame": round(t_dev8 / nh * 1e3, 4)},
            "lanes": PIPE_LANES, "in_flight": PIPE_DEPTH,
            "note": f"the same loop with {PIPE_DEPTH} frames in flight (2 per lane: every frame launched alone)"}
        del detp
        # The same loop on a micro-batching handle (sift_hip_set_micro_batch):
        # submitted frames run MB at a time as one launch group per lane.
        # (device frames: 2 lanes x 8 in flight 0.0998 ms/frame, 3 x 12 in 4-frame groups 0.0942, 2-frame
        # groups 0.110; host frames read back with views, C++ loop: 4-frame groups x 12 in flight 0.129-0.143,
        # 8-frame groups x 24 0.112-0.119, 12-frame 0.126-0.129, 16-frame x 48 0.113, 4 lanes x 16 0.140;
        # profiles/round5/host_mb8.jsonl, host_mb16.jsonl)
        MB_LANES, MB, MB_DEPTH = 3, 8, 24
        detp = sift.Detector(cfg, device=local, lanes=MB_LANES, micro_batch=MB)
        detp.gpuWarmUpAndAllocate()
        PIPE_DEPTH_SAVED, PIPE_DEPTH = PIPE_DEPTH, MB_DEPTH
        t_mbh = pipelined(lambda s: detp.submit(host_u8[s % nframes]), copy_out)
        host_input["pipelined_u8_micro_batch"] = {
            "value": round(world * nh * W * H / 1e6 / t_mbh, 2), "ms_per_frame": round(t_mbh / nh * 1e3, 4),
            "lanes": MB_LANES, "frames_per_group": MB, "in_flight": MB_DEPTH}
        # The same, reading the results where the frame's last kernel put them
        # (results_host: views of the detector's pinned rows, as the
        # reference's final_kpts / descriptors host vectors) instead of copying
        # them into new arrays.
        t_mbv = pipelined(lambda s: detp.submit(host_u8[s % nframes]), view_out)
        host_input["pipelined_u8_micro_batch_views"] = {
            "value": round(world * nh * W * H / 1e6 / t_mbv, 2), "ms_per_frame": round(t_mbv / nh * 1e3, 4),
            "lanes": MB_LANES, "frames_per_group": MB, "in_flight": MB_DEPTH,
            "note": "results_host(True) after every wait instead of copyToHost(True)"}
        t_mb = pipelined(lambda s: detp.submitDevice(frames[s % nframes].data_ptr(), stride), None)
        t_mb8 = pipelined(lambda s: detp.submitDevice(dev_u8[s % nframes].data_ptr(), W, u8=True), None)
        PIPE_DEPTH = PIPE_DEPTH_SAVED
        device_submit = {
            "f32": {"value": round(world * nh * W * H / 1e6 / t_ad, 2), "ms_per_frame": round(t_ad / nh * 1e3, 4)},
            "u8": {"value": round(world * nh * W * H / 1e6 / t_ad8, 2), "ms_per_frame": round(t_ad8 / nh * 1e3, 4)},
            "unit": "Mpix/s", "lanes": PIPE_LANES, "in_flight": AUTO_DEPTH,
            "note": "HBM-resident single frames through submitDevice/wait (sift_hip_submit_device) on a "
                    f"{auto_note}; results stay on the device",
            "in_flight_6": shallow_dev,
            "micro_batch": {
                "f32": {"value": round(world * nh * W * H / 1e6 / t_mb, 2), "ms_per_frame": round(t_mb / nh * 1e3, 4)},
                "u8": {"value": round(world * nh * W * H / 1e6 / t_mb8, 2), "ms_per_frame": round(t_mb8 / nh * 1e3, 4)},
                "lanes": MB_LANES, "frames_per_group": MB, "in_flight": MB_DEPTH,
                "note": f"the same submitDevice/wait loop on a handle with sift_hip_set_micro_batch({MB}): frames run as "
                        f"{MB}-frame launch groups (per-frame results identical, tests/test_gpu_lanes.py)"},
        }
        del detp, dev_u8
        return host_input, device_submit

    # Side legs: a failure here keeps the C2 line (recorded as an error).
    try:
        host_input, device_submit = pipelined_legs()
    except Exception as e:  # noqa: BLE001
        host_input = device_submit = {"error": repr(e)[:300]}

    # ---- per-kernel roofline: HIP events on the detector's own stream --------
    rl = measure_roofline(detb, frames, stride, a.traffic_summary, batch=fb if B > 1 else None)
    timing, nt = rl["timing"], rl["frames"] * B
    try:
        rk = kernel_rooflines(detb, timing, rl["frames"], B, a.traffic_summary) if B > 1 else {}
    except Exception as e:  # keep the line if a model input is missing
        rk = {"error": repr(e)[:300]}
    del detb
    stages = stage_table(timing, nt)
    total_ms = sum(stages.values()) * nt / 1e3
    dom = next(iter(stages))

    # ---- C3: 2000 x 2000 x 128 match -----------------------------------------
    det2 = sift.Detector(make_config(numOctaves=0), device=local)
    det2.gpuWarmUpAndAllocate()
    sets, sets_codes = [], []
    # C3 uses sets 0 and 1; C5 uses set k on rank k (world > 1), or all 8 on
    # one GPU (world == 1 rehearsal).  Each set also keeps the detector's
    # matcher sidecar rows (int8 codes + key biases: what C5 exchanges).
    for i in range(8 if world == 1 else max(2, world)):
        det2.detectAndCompute(sift.synth_frame(77 + i, W, H))
        det2.copyToHost(True)
        nsc = min(det2.total_size, 2000)
        cp, kp = det2.results_sidecar()
        sc = torch.empty((2000, 128), dtype=torch.int8, device=dev)
        sk = torch.empty(2000, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        if nsc:
            sift._check(sift.lib().sift_hip_memcpy_d2d(sc.data_ptr(), cp, nsc * 128, None), "sidecar codes")
            sift._check(sift.lib().sift_hip_memcpy_d2d(sk.data_ptr(), kp, nsc * 4, None), "sidecar keys")
        d = det2.descriptors[:2000]
        if len(d) < 2000:  # pad with seeded SIFT-like rows (normalised, clipped, x512, rounded)
            rng = np.random.default_rng(i)
            v = rng.random((2000 - len(d), 128)) ** 3
            v /= np.linalg.norm(v, axis=1, keepdims=True)
            v = np.minimum(v, 0.2)
            v = np.round(np.clip(v / np.linalg.norm(v, axis=1, keepdims=True) * 512, 0, 255))
            d = np.concatenate([d.astype(np.float32), v.astype(np.float32)]).astype(np.float16)
        sets.append(torch.from_numpy(np.ascontiguousarray(d).view(np.int16)).to(dev))
        if nsc < 2000:  # padding rows: their codes as the sidecar defines them
            pc, pk = multi.codes_from_rows(sets[-1])  # (set-local row indices in the key biases)
            sc[nsc:], sk[nsc:] = pc[nsc:], pk[nsc:]
        sets_codes.append((sc, sk))
    torch.cuda.synchronize()
    nq = 2000
    matcher = sift.Matcher(nq, nq, max_pairs=8, device=local)
    out_idx = torch.empty((nq, 2), dtype=torch.int32, device=dev)
    out_d2 = torch.empty((nq, 2), dtype=torch.float32, device=dev)
    out_m = torch.empty(nq, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream().cuda_stream

    def one_match():
        matcher.match_device(sets[0].data_ptr(), nq, sets[1].data_ptr(), nq, 0.8, False,
                             out_idx.data_ptr(), out_d2.data_ptr(), out_m.data_ptr(), stream)

    for _ in range(20):
        one_match()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = 200
    e0.record()
    for _ in range(reps):
        one_match()
    e1.record()
    torch.cuda.synchronize()
    match_ms = e0.elapsed_time(e1) / reps
    match_ms = max_over_ranks(match_ms)
    t = time.perf_counter()
    for _ in range(20):
        one_match()
        torch.cuda.synchronize()
    match_sync_ms = (time.perf_counter() - t) / 20 * 1e3
    flops = 2.0 * nq * nq * 128
    n_matches = int((out_m >= 0).sum().item())

    # The reference's own pairing (tool/extract_and_match_example.cc:87):
    # matchBruteForce(prev_descriptor, n0, device_descriptor, n1) on the
    # detector's last two results, 2000 rows each; detector buffers carry
    # their int8 codes (matcher sidecar), so no conversion runs.
    n0d, n1d = min(det2.prev_size, nq), min(det2.total_size, nq)
    qd, td = det2.prev_descriptor.data(), det2.device_descriptor.data()

    def det_match():
        matcher.match_device(qd, n0d, td, n1d, 0.8, False, out_idx.data_ptr(), out_d2.data_ptr(), out_m.data_ptr(),
                             stream)

    for _ in range(20):
        det_match()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(reps):
        det_match()
    e1.record()
    torch.cuda.synchronize()
    match_det_ms = max_over_ranks(e0.elapsed_time(e1) / reps)
    t = time.perf_counter()
    for _ in range(20):
        det_match()
        torch.cuda.synchronize()
    match_det_sync_ms = (time.perf_counter() - t) / 20 * 1e3
    match_det = {"ms": round(match_det_ms, 4), "ms_sync_host": round(match_det_sync_ms, 4), "rows": [n0d, n1d],
                 "tops": round(2.0 * n0d * n1d * 128 / (match_det_ms * 1e-3) / 1e12, 2),
                 "path": "detector buffers (prev_descriptor x device_descriptor): sidecar int8 codes, k_match_direct",
                 "matches": int((out_m[:n0d] >= 0).sum().item())}

    # ---- C5: 8-way (world-way) all-gather + pairwise match -------------------
    def time_ms(fn, reps):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        m0, m1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        m0.record()
        for _ in range(reps):
            fn()
        m1.record()
        torch.cuda.synchronize()
        return m0.elapsed_time(m1) / reps

    def c5_codes_matcher(buf, pairs, P):
        bm = sift.Matcher(nq, nq, max_pairs=P, device=local)
        bi = torch.empty((P * nq, 2), dtype=torch.int32, device=dev)
        return lambda: bm.match_codes_batched(buf.data_ptr(), buf.data_ptr(), pairs, idx2_ptr=bi.data_ptr(),
                                              stream=torch.cuda.current_stream().cuda_stream)

    def run_c5_single_gpu(K=8):
        """world == 1: the 8 sets are already on this GPU (no exchange).  The
        56 ordered pairs of the 8-way match in ONE batched launch (fp16 rows,
        converted by k_match_prep, and the exchanged codes), and rank 0's share
        at N = 8 -- its set against the 7 others -- which is what one GPU runs
        per exchange on the 8-GPU node: the per-GPU C5 figure."""
        pairs = [(i, j) for i in range(K) for j in range(K) if i != j]
        P = len(pairs)
        bm = sift.Matcher(nq, nq, max_pairs=P, device=local)
        bi = torch.empty((P * nq, 2), dtype=torch.int32, device=dev)

        def batched(pp):
            bm.match_batched([sets[i].data_ptr() for i, _ in pp], [nq] * len(pp), [sets[j].data_ptr() for _, j in pp],
                             [nq] * len(pp), idx2_ptr=bi.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)

        ms56 = time_ms(lambda: batched(pairs), 20)
        mine7 = [(0, j) for j in range(1, K)]
        ms7_f16 = time_ms(lambda: batched(mine7), 50)
        # The gathered codes buffer as multi.all_gather_codes lays it out (K blocks).
        n_pad = multi.code_block_rows(nq)
        buf = torch.cat([multi.pack_codes(c, k, n_pad) for c, k in sets_codes[:K]])
        counts = [nq] * K
        code56 = [p for r in range(K) for p in multi.code_pairs(counts, r, K, n_pad)]
        ms56_codes = time_ms(c5_codes_matcher(buf, code56, P), 20)
        ms7 = time_ms(c5_codes_matcher(buf, multi.code_pairs(counts, 0, K, n_pad), K - 1), 50)
        fl, fl7 = 2.0 * nq * nq * 128 * P, 2.0 * nq * nq * 128 * (K - 1)
        return {"virtual_ranks": K, "pairs_per_gpu": K - 1, "allgather_us": None,
                "pairs7_ms": round(ms7, 4), "pairs7_tops": round(fl7 / ms7 / 1e9, 2),
                "pairs7_frac": round(fl7 / ms7 / 1e9 / I8_MFMA_PEAK_TOPS, 4), "pairs7_fp16_prep_ms": round(ms7_f16, 4),
                "pairs56_ms": round(ms56_codes, 4), "pairs56_frac": round(fl / ms56_codes / 1e9 / I8_MFMA_PEAK_TOPS, 4),
                "pairs56_fp16_prep_ms": round(ms56, 4),
                "batched_match_ms": round(ms7, 4), "tops": round(fl7 / ms7 / 1e9, 2),
                "mfma_frac": round(fl7 / ms7 / 1e9 / I8_MFMA_PEAK_TOPS, 4),
                "exchange": "int8 codes + key biases (132 B/row, detector sidecars, multi.all_gather_codes layout)",
                "note": "one-GPU rehearsal of C5: pairs7 = one GPU's share at N = 8 (its set x the 7 gathered ones, "
                        "sift_hip_match_codes_batched, no conversion), the per-GPU C5 figure; pairs56 = all 56 "
                        "ordered pairs in one launch; *_fp16_prep = the same pairs from fp16 rows (k_match_prep + "
                        "k_match_batch)"}

    def run_c5():
        """world > 1: every rank all-gathers the detector's matcher codes (one
        RCCL all_gather_into_tensor of a 2016 x 132 B block per rank, 266 KB
        instead of 512 KB of fp16 rows) and matches its set against the
        world - 1 gathered ones in one launch, no conversion."""
        mine_c, mine_k = sets_codes[rank]
        counts = multi.all_gather_counts(nq, world, cdev)  # once; the exchange itself is the block

        def gather():
            return multi.all_gather_codes(mine_c.to(cdev), mine_k.to(cdev), world)

        for _ in range(5):
            buf, n_pad = gather()
        torch.cuda.synchronize()
        barrier()
        ag0, ag1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ag0.record()
        for _ in range(20):
            buf, n_pad = gather()
        ag1.record()
        torch.cuda.synchronize()
        ag_us = max_over_ranks(ag0.elapsed_time(ag1) / 20 * 1e3)
        assert counts == [nq] * world
        buf = buf.to(dev)
        pairs = multi.code_pairs(counts, rank, world, n_pad)
        P = len(pairs)
        bms = max_over_ranks(time_ms(c5_codes_matcher(buf, pairs, P), 50))
        fl = 2.0 * nq * nq * 128 * P
        return {"allgather_us": round(ag_us, 2), "allgather_bytes_per_rank": n_pad * 132, "pairs_per_gpu": P,
                "batched_match_ms": round(bms, 4), "tops_per_gpu": round(fl / bms / 1e9, 2),
                "mfma_frac": round(fl / bms / 1e9 / I8_MFMA_PEAK_TOPS, 4),
                "exchange": "int8 codes + key biases (132 B/row, detector sidecars)",
                "collective": f"all_gather ({a.dist_backend}; nccl = RCCL all_gather_into_tensor), "
                              "sift_amd/multi.py all_gather_codes"}

    try:
        c5 = run_c5() if world > 1 else run_c5_single_gpu()
    except Exception as e:  # keep the C2 line even if the C5 side measurement fails
        c5 = {"error": repr(e)[:300]}
    if isinstance(rk, dict) and "batched_match_ms" in c5:
        ops = 2.0 * nq * nq * 128 * c5["pairs_per_gpu"]
        rk["matcher"] = {"bound": "mfma",
                         "kernel": "k_match_batch on exchanged codes: one GPU's C5 share (its set x the world - 1 "
                                   "others, 7 pairs at N = 8), no conversion launch",
                         "algo_ops_per_launch": ops, "avg_launch_us": round(c5["batched_match_ms"] * 1e3, 3),
                         "achieved": round(ops / c5["batched_match_ms"] / 1e9, 1), "peak": I8_MFMA_PEAK_TOPS,
                         "unit": "TOPS", "frac": round(ops / c5["batched_match_ms"] / 1e9 / I8_MFMA_PEAK_TOPS, 4),
                         "pairs56_frac": c5.get("pairs56_frac"),
                         "c3_single_pair_frac": round(flops / match_ms / 1e9 / I8_MFMA_PEAK_TOPS, 5)}

    # ---- CPU baseline: the oracle on the host cores (rank 0, N=1 only) -------
    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(a, cfg, [s.cpu().view(torch.float16).float().numpy() for s in sets[:2]])
    c1_gpu = run_c1_gpu(local) if rank == 0 else None
    try:
        ref_cfg = run_ref_configs(local, dev) if rank == 0 else None
    except Exception as e:  # side measurement: keep the line
        ref_cfg = {"error": repr(e)[:300]}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic",
            "library": sift.version(),
            "config": {
                "workload": f"C2: detectAndCompute on 1920x1200 frames, {B} per step per GPU (one launch per stage "
                            "for the batch), numOctaveLayers=3 (5 DoG scales/octave), numOctaves=3, upscale=false, "
                            "numFeatures=5000; frames HBM-resident",
                "frames_per_step_per_gpu": B,
                "frames_per_launch": B,
                "streams_per_gpu": a.streams,
                "parallelism": f"frame-sharded x{world}, no data-path collective",
                "descriptor_mode": "exact" if a.exact_descriptors else "fixed-point (default)",
                "keypoints_per_frame": kcount,
            },
            "roofline": rl["roofline"],
            "roofline_kernels": rk,
            "cpu_baseline": cpu,
            "ms_per_frame": round(ms_per_frame, 4),
            "pipeline_hbm_frac": round(88.0 * sum_px / (ms_per_frame / 1e3) / 1e9 / HBM_PEAK_GBS, 4),
            "sync_ms_per_frame": round(sync_ms, 4),
            "single_stream": {"value": round(single_value, 2), "ms_per_frame": round(single / n1 * 1e3, 4)},
            "exact_descriptors": exact_leg,
            "opencv_default_1920x1200": cv_default,
            "host_input": host_input,
            "device_submit": device_submit,
            "stage_us_per_frame_eager": stages,
            "stage_sum_us_eager": round(total_ms / nt * 1e3, 1),
            "dominant_stage": dom,
            "match_2k": {"ms": round(match_ms, 4), "ms_sync_host": round(match_sync_ms, 4),
                         "tops": round(flops / match_ms / 1e9, 2), "mfma_frac": round(flops / match_ms / 1e9 / I8_MFMA_PEAK_TOPS, 5),
                         "dtype": "int8 codes (v - 128) on v_mfma_i32_32x32x32_i8, exact int32 d^2",
                         "matches": n_matches, "ratio": 0.8,
                         "path": "foreign fp16 buffers (converted in the kernel, k_match_single)"},
            "match_2k_detector": match_det,
            "c4_256_frames_1600x900": c4,
            "c5_allgather_match": c5,
            "c1_gpu": c1_gpu,
            "ref_config_sync": ref_cfg,
            "ref_published": {"detect_1920x1200_ms": 3.1, "match_2k_ms": "just under 1", "hardware": "RTX 4070 Super",
                              "note": "reference readme.md:11-15; config not stated (tool default upscale=false, auto octaves)"},
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
