"""Per-workgroup timeline of the batched matcher (diagnostic builds only).

build: patch a temporary copy of csrc/match.hip so every k_match_batch
       workgroup stamps s_memrealtime (100 MHz, one clock for the whole chip)
       and s_memtime at entry, after its split's compute and at exit into a
       __device__ array of its own (no output element is touched), export
       sift_hip_debug_wg_stamps() to read it, and build ab/NAME.so.
run:   (on the GPU, SIFT_HIP_LIB=ab/NAME.so) C5 rehearsal calls back to back,
       then the stamps of the last call: spread of workgroup starts, compute
       and merge phases, and the time from the last start to the last exit.

    python3 tools/match_wgstamps.py build wgs
    SIFT_HIP_LIB=ab/wgs.so python3 tools/match_wgstamps.py run
"""
import json
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def build(name):
    tmp = tempfile.mkdtemp()
    shutil.copy(os.path.join(ROOT, "Makefile"), tmp)
    shutil.copytree(os.path.join(ROOT, "include"), os.path.join(tmp, "include"))
    shutil.copytree(os.path.join(ROOT, "another-cuda-sift_amd", "csrc"), os.path.join(tmp, "another-cuda-sift_amd", "csrc"))
    path = os.path.join(tmp, "another-cuda-sift_amd", "csrc", "match.hip")
    s = open(path).read()
    anchor_ns = "namespace sift_amd {\n"
    s = s.replace(anchor_ns, anchor_ns + """
__device__ unsigned long long g_wg_stamps[16384][6];
__device__ __forceinline__ void wg_stamp(int slot) {
    if (threadIdx.x == 0) {
        const unsigned b = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        if (b < 16384) {
            g_wg_stamps[b][2 * slot] = __builtin_amdgcn_s_memrealtime();
            g_wg_stamps[b][2 * slot + 1] = __builtin_amdgcn_s_memtime();
        }
    }
}
""", 1)
    a1 = "    const int q0w = q0 + 64 * w;\n    Top2 res[2];\n    if (flags[pr.qset] != epoch"
    assert s.count(a1) == 1
    s = s.replace(a1, "    wg_stamp(0);\n" + a1)
    a2 = "        res[0] = match_f16_block(pr, q0w, tb, te, col, h);\n        res[1] = match_f16_block(pr, q0w + 32, tb, te, col, h);\n    }\n"
    assert s.count(a2) == 1
    s = s.replace(a2, a2 + "    wg_stamp(1);\n")
    a3 = "    merge_contribution(s_res, &s_last, keys + 2 * ((size_t)p * nq_stride + q0)"
    assert s.count(a3) == 1
    i3 = s.index(a3)
    e3 = s.index(";\n}\n", i3)
    s = s[:e3] + ";\n    wg_stamp(2);\n}\n" + s[e3 + 4:]
    a4 = "        if (qv) write_top2(s_res[tid], o, ratio, ratio_on_squared, idx2, d2out, match);\n        return;\n"
    i4 = s.rindex(a4, 0, i3)  # the S == 1 exit of k_match_batch
    s = s[:i4] + a4.replace("        return;\n", "        wg_stamp(2);\n        return;\n") + s[i4 + len(a4):]
    s += """
extern "C" int sift_hip_debug_wg_stamps(void* dst, size_t bytes) {
    return (int)hipMemcpyFromSymbol(dst, HIP_SYMBOL(sift_amd::g_wg_stamps), bytes, 0, hipMemcpyDeviceToHost);
}
"""
    open(path, "w").write(s)
    r = subprocess.run(["make", "-C", tmp, "-j8", "another-cuda-sift_amd/lib/libsift_hip.so"], capture_output=True,
                       text=True)
    if r.returncode:
        print(r.stdout[-3000:], r.stderr[-3000:])
        sys.exit(1)
    os.makedirs(os.path.join(ROOT, "ab"), exist_ok=True)
    shutil.copy(os.path.join(tmp, "another-cuda-sift_amd", "lib", "libsift_hip.so"), os.path.join(ROOT, "ab", name + ".so"))
    shutil.rmtree(tmp)
    print(f"ab/{name}.so <- stamped match.hip")


def run():
    import ctypes
    import statistics
    sys.path.insert(0, os.path.join(ROOT, "another-cuda-sift_amd"))
    import torch
    import numpy as np
    import sift_amd as sift
    nq, K = 2000, 8
    rng = np.random.default_rng(1)
    sets = [torch.from_numpy(rng.integers(0, 256, (nq, 128)).astype(np.float16).view(np.int16)).cuda()
            for _ in range(K)]
    pairs = [(i, j) for i in range(K) for j in range(K) if i != j]
    P = len(pairs)
    m = sift.Matcher(nq, nq, max_pairs=P, device=0)
    oi = torch.empty((P * nq, 2), dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    qp, tp = [sets[i].data_ptr() for i, _ in pairs], [sets[j].data_ptr() for _, j in pairs]
    for _ in range(2000):
        m.match_batched(qp, [nq] * P, tp, [nq] * P, idx2_ptr=oi.data_ptr(), stream=st)
    torch.cuda.synchronize()
    lib = sift.lib()
    lib.sift_hip_debug_wg_stamps.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    buf = (ctypes.c_ulonglong * (16384 * 6))()
    if lib.sift_hip_debug_wg_stamps(ctypes.addressof(buf), ctypes.sizeof(buf)) != 0:
        raise RuntimeError("stamp copy failed")
    wgs = [(buf[6 * b], buf[6 * b + 1], buf[6 * b + 2], buf[6 * b + 3], buf[6 * b + 4], buf[6 * b + 5])
           for b in range(16384) if buf[6 * b] and buf[6 * b + 4]]
    r0 = min(w[0] for w in wgs)
    us = lambda t: (t - r0) / 100.0  # noqa: E731  realtime ticks (10 ns) -> us
    starts = sorted(us(w[0]) for w in wgs)
    comp = [(w[2] - w[0]) / 100.0 for w in wgs]
    merge = [(w[4] - w[2]) / 100.0 for w in wgs]
    ends = sorted(us(w[4]) for w in wgs)
    clk = [(w[5] - w[1]) / max(1, w[4] - w[0]) * 0.1 for w in wgs]
    q = lambda xs, f: sorted(xs)[min(len(xs) - 1, int(f * len(xs)))]  # noqa: E731
    print(json.dumps({
        "workgroups": len(wgs),
        "start_us": {"first": starts[0], "p50": q(starts, 0.5), "p90": q(starts, 0.9), "last": starts[-1]},
        "compute_us": {"min": min(comp), "p50": q(comp, 0.5), "p90": q(comp, 0.9), "max": max(comp)},
        "merge_us": {"min": min(merge), "p50": q(merge, 0.5), "p90": q(merge, 0.9), "max": max(merge)},
        "end_us": {"first": ends[0], "p50": q(ends, 0.5), "last": ends[-1]},
        "in_kernel_clock_ghz_median": round(statistics.median(clk), 3),
        "note": "one C5 call (8 sets x 2000, 56 pairs) after 2000 back-to-back calls; times from the first "
                "workgroup's entry (s_memrealtime); diagnostic build only",
    }, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "build":
        build(sys.argv[2])
    else:
        run()
