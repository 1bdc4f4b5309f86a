"""bench.py's multi-GPU launch contract on CPU (no GPU work):

* `python bench.py --gpus N` with no torchrun parent starts N rank processes
  itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set before any GPU call)
  and rank 0 prints the line with n_gpus = N;
* a torchrun-style launch whose WORLD_SIZE disagrees with --gpus is refused.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _run(args, env=None, timeout=240):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, BENCH] + args, capture_output=True, text=True, timeout=timeout, env=e)


def test_gpus_flag_spawns_ranks():
    r = _run(["--gpus", "2", "--launcher-selftest"])
    assert r.returncode == 0, r.stdout + r.stderr
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # only rank 0 prints
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["max_rank_plus_1"] == 2.0


def test_single_rank_default():
    r = _run(["--launcher-selftest"])
    assert r.returncode == 0, r.stdout + r.stderr
    assert json.loads(r.stdout.strip().splitlines()[-1])["n_gpus"] == 1


def test_world_size_mismatch_refused():
    r = _run(["--gpus", "1", "--launcher-selftest"],
             env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0", "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": "1"})
    assert r.returncode == 2
    assert "WORLD_SIZE" in r.stderr
