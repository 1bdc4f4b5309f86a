"""Matcher timings for A/B of library builds (SIFT_HIP_LIB): the C3 single
2000 x 2000 x 128 pair (bench.py's match_2k: 200 back-to-back calls between HIP
events) and the C5 rehearsal (8 sets, all 56 ordered pairs in one batched
call), each checked against torch fp32 (exact for integer descriptors)."""
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
K = 8
sets = [torch.from_numpy(rng.integers(0, 256, (nq, 128)).astype(np.float16).view(np.int16)).cuda() for _ in range(K)]
pairs = [(i, j) for i in range(K) for j in range(K) if i != j]
P = len(pairs)
m = sift.Matcher(nq, nq, max_pairs=P, device=0)
oi = torch.empty((P * nq, 2), dtype=torch.int32, device="cuda")
od = torch.empty((P * nq, 2), dtype=torch.float32, device="cuda")
om = torch.empty(P * nq, dtype=torch.int32, device="cuda")
st = torch.cuda.current_stream().cuda_stream


def one():
    m.match_device(sets[0].data_ptr(), nq, sets[1].data_ptr(), nq, 0.8, False, oi.data_ptr(), od.data_ptr(),
                   om.data_ptr(), st)


def batched():
    m.match_batched([sets[i].data_ptr() for i, _ in pairs], [nq] * P, [sets[j].data_ptr() for _, j in pairs], [nq] * P,
                    idx2_ptr=oi.data_ptr(), d2_ptr=od.data_ptr(), stream=st)


def timed(fn, reps):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def ref_top2(q, t):
    q, t = q.view(torch.float16).float(), t.view(torch.float16).float()
    d2 = (q * q).sum(1, keepdim=True) + (t * t).sum(1)[None] - 2 * q @ t.T
    return torch.topk(d2, 2, dim=1, largest=False)


ms1 = timed(one, 200)
r = ref_top2(sets[0], sets[1])
ok1 = bool((oi[:nq, 0].long() == r.indices[:, 0]).float().mean() > 0.999)
ms56 = timed(batched, 50)
ok56 = True
for p in (0, 17, 55):
    i, j = pairs[p]
    r = ref_top2(sets[i], sets[j])
    ok56 &= bool((oi[p * nq:(p + 1) * nq, 0].long() == r.indices[:, 0]).float().mean() > 0.999)
fl1, fl56 = 2.0 * nq * nq * 128, 2.0 * nq * nq * 128 * P
print(json.dumps({"lib": os.environ.get("SIFT_HIP_LIB", "default"), "nq": nq, "ms": round(ms1, 4),
                  "top1_ok": ok1, "c5_56_pairs_ms": round(ms56, 4), "c5_top1_ok": ok56,
                  "c5_tops": round(fl56 / ms56 / 1e9, 1), "c3_tops": round(fl1 / ms1 / 1e9, 1)}))
