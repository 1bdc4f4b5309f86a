"""The RCCL exchange paths run once on the one-GPU box, so
the first 8-GPU run does not also debug dlopen / ncclCommInitAll:

  * C ABI: sift_hip_comm_create(1, {0}) + sift_hip_comm_allgather moves the
    bytes (RCCL loaded with dlopen inside libsift_hip.so).
  * Python: torch.distributed "nccl" (= RCCL) at world size 1 through
    sift_amd.multi.all_gather_sets -> Matcher.match_batched, and the codes
    exchange multi.all_gather_codes -> Matcher.match_codes_batched, both exact
    vs the oracle (fresh child process: tests/nccl_world1_child.py).
  * C++: tools/multi_gpu_example --rccl (sift_cuda::rcclAllGather) on one GPU.
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_comm_allgather_one_rank(sift):
    L = sift.lib()
    comm = ctypes.c_void_p()
    devs = (ctypes.c_int * 1)(0)
    sift._check(L.sift_hip_comm_create(1, devs, ctypes.byref(comm)), "comm_create")
    try:
        n = ctypes.c_int()
        sift._check(L.sift_hip_comm_size(comm, ctypes.byref(n)), "comm_size")
        assert n.value == 1
        nbytes = 2000 * 128 * 2  # one C5 descriptor set (2000 x 128 fp16)
        src = np.random.default_rng(3).integers(0, 65536, nbytes // 2).astype(np.uint16)
        send = sift.DeviceArray.from_numpy(src)
        recv = sift.DeviceArray(nbytes)
        for rep in range(2):  # communicator and its stream reused
            sp = (ctypes.c_void_p * 1)(send.value)
            rp = (ctypes.c_void_p * 1)(recv.value)
            sift._check(L.sift_hip_comm_allgather(comm, sp, rp, nbytes, None), "comm_allgather")
            assert np.array_equal(recv.to_numpy(np.uint16, src.shape), src), rep
    finally:
        L.sift_hip_comm_destroy(comm)


def test_torch_nccl_world1_exchange_and_match():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29533")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "nccl_world1_child.py")], capture_output=True,
                       text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["backend"] == "nccl" and out["match_exact"] and out["codes_match_exact"]


def test_multi_gpu_example_rccl_one_gpu():
    exe = os.path.join(ROOT, "another-cuda-sift_amd", "lib", "multi_gpu_example")
    r = subprocess.run([exe, "--rccl", "--devices", "1", "--frames", "4", "--width", "640", "--height", "360",
                        "--rows", "500"], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert out["gather"] == "rccl" and out["workers"] == 1 and out["devices"] == [0]
    assert all(k > 20 for k in out["kpts"])
