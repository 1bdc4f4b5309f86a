"""In-kernel shader clock while the batched matcher runs (C5 rehearsal: 8 sets
of 2000 x 128, all 56 ordered pairs per call, back to back), and with the GPU
otherwise idle.  tools/libclock_probe.so (tools/clock_probe.hip) stamps
s_memtime / s_memrealtime in 64 one-wave workgroups on a stream of their own
(MI355X_MICROARCH.md, DVFS item 6).  The MFMA-busy fraction of
profiles/roundN/mfma_counters.json is priced at 2.4 GHz; tools/mfma_summary.py
--clock-json prices it at this measured clock as well.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/libclock_probe.so tools/clock_probe.hip
    python3 tools/match_clock.py > gpurun_out/match_clock.json
"""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import torch  # noqa: E402
import numpy as np  # noqa: E402
import sift_amd as sift  # noqa: E402

probe = ctypes.CDLL(os.path.join(ROOT, "tools", "libclock_probe.so"))
probe.probe_start.argtypes = [ctypes.c_double]
probe.probe_finish.argtypes = [ctypes.POINTER(ctypes.c_double), ctypes.c_int]

nq, K = 2000, 8
rng = np.random.default_rng(1)
sets = [torch.from_numpy(rng.integers(0, 256, (nq, 128)).astype(np.float16).view(np.int16)).cuda() for _ in range(K)]
pairs = [(i, j) for i in range(K) for j in range(K) if i != j]
P = len(pairs)
m = sift.Matcher(nq, nq, max_pairs=P, device=0)
oi = torch.empty((P * nq, 2), dtype=torch.int32, device="cuda")
od = torch.empty((P * nq, 2), dtype=torch.float32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
qp, tp = [sets[i].data_ptr() for i, _ in pairs], [sets[j].data_ptr() for _, j in pairs]


def batched():
    m.match_batched(qp, [nq] * P, tp, [nq] * P, idx2_ptr=oi.data_ptr(), d2_ptr=od.data_ptr(), stream=st)


def clock(seconds, load):
    """Median probe clock (GHz) over the 64 workgroups; `load` runs meanwhile."""
    if probe.probe_start(seconds) != 0:
        raise RuntimeError("probe_start failed")
    calls = 0
    if load:
        t_end = time.time() + seconds + 0.2
        while time.time() < t_end:
            for _ in range(20):
                batched()
            calls += 20
            torch.cuda.synchronize()
    buf = (ctypes.c_double * 128)()
    n = probe.probe_finish(buf, 64)
    if n <= 0:
        raise RuntimeError("probe_finish failed")
    ghz = [buf[2 * i] / buf[2 * i + 1] * 0.1 for i in range(n) if buf[2 * i + 1] > 0]
    return {"ghz_median": round(statistics.median(ghz), 4), "ghz_min": round(min(ghz), 4),
            "ghz_max": round(max(ghz), 4), "workgroups": len(ghz), "matcher_calls": calls}


# warm-up: 2 s of back-to-back calls (the clock settles under sustained load)
t_end = time.time() + 2.0
while time.time() < t_end:
    for _ in range(20):
        batched()
    torch.cuda.synchronize()
busy = clock(1.0, True)
idle = clock(0.5, False)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(50):
    batched()
e1.record()
torch.cuda.synchronize()
print(json.dumps({"workload": "batched matcher, 8 sets x 2000 x 128, 56 ordered pairs per call, back to back",
                  "clock_under_matcher": busy, "clock_idle": idle,
                  "c5_call_us": round(e0.elapsed_time(e1) / 50 * 1e3, 2),
                  "method": "delta s_memtime / delta s_memrealtime x 100 MHz in 64 one-wave probe workgroups "
                            "(tools/clock_probe.hip) running beside the workload"}, indent=1))
