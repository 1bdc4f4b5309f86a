"""Matcher workload for MFMA counters (rocprofv3 --pmc): 2000x2000x128 single
calls (C3) and a 56-pair batched call (C5 rehearsal on one GPU); an optional
argument multiplies the repetitions (the kernel-trace-only run for the
unprofiled durations).
    rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
        --kernel-trace -d gpurun_out/mfma -o run --output-format csv -- python3 tools/match_pmc.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import numpy as np  # noqa: E402
import sift_amd as sift  # noqa: E402

n, K = 2000, 8
REPS = int(sys.argv[1]) if len(sys.argv) > 1 else 1
rng = np.random.default_rng(3)
sets = [sift.DeviceArray.from_numpy(np.ascontiguousarray(rng.integers(0, 256, (n, 128)).astype(np.float16)))
        for _ in range(K)]
idx2 = sift.DeviceArray(K * (K - 1) * n * 8)
m = sift.Matcher(n, n, max_pairs=K * (K - 1))
for _ in range(10 * REPS):
    m.match_device(sets[0].value, n, sets[1].value, n, 0.8, False, idx2.value, 0, 0)
# C3 on detector buffers (the reference's prev_descriptor x device_descriptor
# call): the sidecar path, k_match_direct.
W, H = 1920, 1200
det = sift.Detector(sift.CudaSiftConfig(col_width=W, row_width=H, numOctaves=3, numFeatures=5000), device=0)
det.gpuWarmUpAndAllocate()
det.detectAndCompute(sift.synth_frame(77, W, H))
det.detectAndCompute(sift.synth_frame(78, W, H))
for _ in range(10 * REPS):
    m.match_device(det.prev_descriptor.data(), n, det.device_descriptor.data(), n, 0.8, False, idx2.value, 0, 0)
pairs = [(i, j) for i in range(K) for j in range(K) if i != j]
for _ in range(5 * REPS):
    m.match_batched([sets[i].value for i, _ in pairs], [n] * len(pairs), [sets[j].value for _, j in pairs],
                    [n] * len(pairs), idx2_ptr=idx2.value)
print("done")
