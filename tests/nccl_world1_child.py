"""Child process of tests/test_gpu_rccl.py (not a test module): the C5
exchange of sift_amd.multi over torch.distributed "nccl" (= RCCL) at world
size 1 on the one-GPU box, followed by the batched HIP matcher, checked
against the oracle's knn-2.  Run in a fresh process so the process group is
created before anything else touches the GPU.  Prints one JSON line.

Test infrastructure: the oracle is the checker, never the thing measured.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "another-cuda-sift_amd"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda:0"))
    import oracle_binding as oracle
    import sift_amd
    from sift_amd import multi

    rng = np.random.default_rng(71)
    n, m = 700, 900
    q = rng.integers(0, 256, (n, 128)).astype(np.float16)
    t = rng.integers(0, 256, (m, 128)).astype(np.float16)
    t[17] = t[5]  # tie: lower index first
    local = torch.from_numpy(q).to("cuda:0")
    gathered, counts = multi.all_gather_sets(local, n, 1)  # all_gather_into_tensor on RCCL (int32 view)
    torch.cuda.synchronize()
    assert gathered.shape == (1, n, 128) and counts == [n]
    assert torch.equal(gathered[0].view(torch.int16).cpu(), local.view(torch.int16).cpu()), "gather changed bytes"
    dt = torch.from_numpy(t).to("cuda:0")
    idx2 = torch.empty((2, n, 2), dtype=torch.int32, device="cuda:0")
    mt = sift_amd.Matcher(n, m, max_pairs=2)
    g = gathered[0].contiguous()
    mt.match_batched([g.data_ptr(), g.data_ptr()], [n, n], [dt.data_ptr(), dt[:400].data_ptr()], [m, 400],
                     idx2_ptr=idx2.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = idx2.cpu().numpy()
    oi, _ = oracle.knn2(q.astype(np.float32), t.astype(np.float32))
    oi2, _ = oracle.knn2(q.astype(np.float32), t[:400].astype(np.float32))
    ok = bool(np.array_equal(got[0], oi) and np.array_equal(got[1], oi2))
    # The codes exchange (multi.all_gather_codes: the packed int8 codes + key
    # biases block, one RCCL all_gather_into_tensor), then the batched matcher
    # on the gathered buffer (no conversion): q against t and t[:400].
    qc, qk = multi.codes_from_rows(local.view(torch.int16))
    buf, n_pad = multi.all_gather_codes(qc, qk, 1)
    assert buf.numel() == n_pad * 132
    tc, tk = multi.codes_from_rows(dt.view(torch.int16))
    tpad = multi.code_block_rows(m)
    both = torch.cat([buf, multi.pack_codes(tc, tk, tpad)])
    t0, tk0 = multi.code_set(0, tpad)  # the train block starts after the gathered one
    t0 += n_pad * 132 // 128
    tk0 += n_pad * 132 // 4
    q0, qk0 = multi.code_set(0, n_pad)
    idx2c = torch.empty((2, n, 2), dtype=torch.int32, device="cuda:0")
    mt.match_codes_batched(both.data_ptr(), both.data_ptr(), [(q0, qk0, n, t0, tk0, m), (q0, qk0, n, t0, tk0, 400)],
                           idx2_ptr=idx2c.data_ptr(), stream=torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    gc = idx2c.cpu().numpy()
    ok_codes = bool(np.array_equal(gc[0], oi) and np.array_equal(gc[1], oi2))
    dist.destroy_process_group()
    print(json.dumps({"backend": "nccl", "world": 1, "rows": n, "match_exact": ok, "codes_match_exact": ok_codes}))
    return 0 if ok and ok_codes else 1


if __name__ == "__main__":
    sys.exit(main())
