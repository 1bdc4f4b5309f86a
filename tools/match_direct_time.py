"""Single 2000 x 2000 pair on detector buffers (k_match_direct, the matcher
sidecar path): 200 back-to-back calls between HIP events, for A/B builds
(SIFT_HIP_LIB).  Also the same pair with the sidecar lookup off (the
converting k_match_single path) and the results compared."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import torch  # noqa: E402
import sift_amd as sift  # noqa: E402

W, H = 1920, 1200
det = sift.Detector(sift.CudaSiftConfig(col_width=W, row_width=H, numOctaves=3, numFeatures=5000), device=0)
det.gpuWarmUpAndAllocate()
det.detectAndCompute(sift.synth_frame(77, W, H))
det.detectAndCompute(sift.synth_frame(78, W, H))
n0, n1 = min(det.prev_size, 2000), min(det.total_size, 2000)
q, t = det.prev_descriptor.data(), det.device_descriptor.data()
out = {}
for name, side in (("direct", True), ("converted", False)):
    m = sift.Matcher(2000, 2000, device=0)
    m.set_sidecars(side)
    oi = torch.empty((n0, 2), dtype=torch.int32, device="cuda")
    od = torch.empty((n0, 2), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream

    def one():
        m.match_device(q, n0, t, n1, 0.8, False, oi.data_ptr(), od.data_ptr(), 0, st)

    for _ in range(20):
        one()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        one()
    e1.record()
    torch.cuda.synchronize()
    out[name] = {"ms": round(e0.elapsed_time(e1) / 200, 5)}
    out[name + "_res"] = (oi.clone(), od.clone())
same = torch.equal(out["direct_res"][0], out["converted_res"][0]) and torch.equal(out["direct_res"][1], out["converted_res"][1])
print(json.dumps({"lib": os.environ.get("SIFT_HIP_LIB", "default"), "rows": [n0, n1], "direct": out["direct"],
                  "converted": out["converted"], "identical": same}), flush=True)
