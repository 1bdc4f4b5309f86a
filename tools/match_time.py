"""2000 x 2000 x 128 match latency (bench.py's match_2k timing: 200 back-to-back
calls between HIP events) for A/B of library builds (SIFT_HIP_LIB)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
import torch  # noqa: E402
import numpy as np  # noqa: E402
import sift_amd as sift  # noqa: E402

nq = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
rng = np.random.default_rng(1)
sets = [torch.from_numpy(rng.integers(0, 256, (nq, 128)).astype(np.float16).view(np.int16)).cuda() for _ in range(2)]
m = sift.Matcher(nq, nq, max_pairs=8, device=0)
oi = torch.empty((nq, 2), dtype=torch.int32, device="cuda")
od = torch.empty((nq, 2), dtype=torch.float32, device="cuda")
om = torch.empty(nq, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def one():
    m.match_device(sets[0].data_ptr(), nq, sets[1].data_ptr(), nq, 0.8, False, oi.data_ptr(), od.data_ptr(),
                   om.data_ptr(), st)


for _ in range(20):
    one()
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(200):
    one()
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 200
# check against torch fp32 (exact for integer descriptors)
q, t = sets[0].view(torch.float16).float(), sets[1].view(torch.float16).float()
d2 = (q * q).sum(1, keepdim=True) + (t * t).sum(1)[None] - 2 * q @ t.T
ref = torch.topk(d2, 2, dim=1, largest=False)
ok = bool((oi[:, 0].long() == ref.indices[:, 0]).float().mean() > 0.999)
print(json.dumps({"lib": os.environ.get("SIFT_HIP_LIB", "default"), "nq": nq, "ms": round(ms, 4), "top1_ok": ok}))
