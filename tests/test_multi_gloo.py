"""The N > 1 path on CPU: two gloo ranks run the multi-GPU orchestration
(sift_amd/multi.py) with the CPU oracle in place of the HIP detector/matcher.

Checks the frame sharding (C4: frame i -> rank i mod world, no collective) and
the C5 exchange (all-gather of every rank's descriptor set, each rank matching
its own set against every peer) against a single-process computation -- both
exchange formats: fp16 rows, and the matcher codes + key biases (one packed
block per rank, multi.all_gather_codes) that the GPU ranks send.
"""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W, H, NSET = 200, 150, 96


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _desc_set(frame):
    """Descriptor set of one synthetic frame (oracle), fp16 bits padded to NSET rows."""
    import oracle_binding as oracle
    import sift_amd

    img = sift_amd.synth_frame(frame, W, H)
    _, d = oracle.detect_and_compute(img, oracle.params(nfeatures=NSET), threads=2)
    d = d[:NSET]
    out = np.zeros((NSET, 128), np.float16)
    out[: len(d)] = d
    return out.view(np.int16), len(d)


def _ratio_match(q, nq, t, nt):
    import oracle_binding as oracle

    qf = q[:nq].view(np.float16).astype(np.float32)
    tf = t[:nt].view(np.float16).astype(np.float32)
    idx, dist = oracle.knn2(qf, tf, threads=2)
    return np.where(dist[:, 0] < 0.8 * dist[:, 1], idx[:, 0], -1).astype(np.int32)


def _worker(rank, world, port, n_frames, q):
    sys.path[:0] = [os.path.join(ROOT, "another-cuda-sift_amd"), os.path.join(ROOT, "tests")]
    import torch
    import torch.distributed as dist

    from sift_amd import multi

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        _run(rank, world, n_frames, q, torch, dist, multi)
    except Exception as e:  # surface worker failures instead of a queue timeout
        q.put(repr(e))
        raise
    finally:
        dist.destroy_process_group()


def _run(rank, world, n_frames, q, torch, dist, multi):
    frames = multi.frame_shard(n_frames, rank, world)
    own, cnt = _desc_set(frames[0])
    gathered, counts = multi.all_gather_sets(torch.from_numpy(own), cnt, world)

    def match_batched(qs, nqs, ts, nts):
        return [torch.from_numpy(_ratio_match(a.numpy(), x, b.numpy(), y)) for a, x, b, y in zip(qs, nqs, ts, nts)]

    res = multi.cross_match(gathered, counts, rank, world, match_batched)
    # The codes exchange: one packed block per rank, then this rank's pairs
    # over the gathered buffer (a CPU matcher on the decoded codes v = c + 128).
    codes, keys = multi.codes_from_rows(torch.from_numpy(own))
    buf, n_pad = multi.all_gather_codes(codes, keys, world)
    got = {}
    for (q0, qk, nq, t0, tk, nt) in multi.code_pairs(counts, rank, world, n_pad):
        j = [jj for jj in range(world) if multi.code_set(jj, n_pad)[0] == t0][0]
        qc = buf[q0 * 128: (q0 + nq) * 128].view(torch.int8).reshape(nq, 128).to(torch.int32) + 128
        tc = buf[t0 * 128: (t0 + nt) * 128].view(torch.int8).reshape(nt, 128).to(torch.int32) + 128
        assert torch.equal(buf[4 * qk: 4 * (qk + nq)].view(torch.int32), keys[:nq])
        got[j] = _ratio_match(qc.to(torch.float16).numpy().view(np.int16), nq, tc.to(torch.float16).numpy().view(np.int16), nt)
    codes_sets = [tuple(x.numpy() for x in multi.unpack_codes(buf, j, NSET, n_pad)) for j in range(world)]
    out = [None] * world
    dist.all_gather_object(out, {"frames": frames, "counts": counts, "codes_sets": codes_sets, "code_matches": got,
                                 "gathered": gathered.numpy(), "matches": {j: r.numpy() for j, r in res.items()}})
    if rank == 0:
        q.put(out)


@pytest.mark.timeout(300)
def test_two_rank_shard_gather_match():
    import multiprocessing as mp

    world, n_frames = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_frames, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    assert not isinstance(out, str), out
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    # Sharding: every frame exactly once, frame i on rank i mod world.
    assert out[0]["frames"] == [0, 2, 4] and out[1]["frames"] == [1, 3]
    # Expected, single process.
    sets = [_desc_set(f) for f in (0, 1)]
    for r in range(world):
        assert out[r]["counts"] == [c for _, c in sets]
        for j in range(world):
            assert np.array_equal(out[r]["gathered"][j], sets[j][0])
        peers = [j for j in range(world) if j != r]
        assert sorted(out[r]["matches"]) == peers
        for j in peers:
            exp = _ratio_match(sets[r][0], sets[r][1], sets[j][0], sets[j][1])
            assert np.array_equal(out[r]["matches"][j], exp)
            assert np.array_equal(out[r]["code_matches"][j], exp)
        for j in range(world):  # every rank received every rank's codes and key biases
            v = sets[j][0].view(np.float16).astype(np.int32)
            c = v - 128
            assert np.array_equal(out[r]["codes_sets"][j][0], c.astype(np.int8))
            assert np.array_equal(out[r]["codes_sets"][j][1], -(256 * (c * c).sum(1) + (np.arange(NSET) & 255)))
    assert sets[0][1] > 20


def test_single_rank_helpers():
    sys.path[:0] = [os.path.join(ROOT, "another-cuda-sift_amd")]
    import torch

    from sift_amd import multi

    assert multi.frame_shard(7, 0, 1) == list(range(7))
    assert multi.frame_shard(256, 3, 8)[:3] == [3, 11, 19] and len(multi.frame_shard(256, 3, 8)) == 32
    assert multi.peer_pairs(2, 4) == [(2, 0), (2, 1), (2, 3)]
    t = torch.zeros((4, 128), dtype=torch.int16)
    g, c = multi.all_gather_sets(t, 3, 1)
    assert g.shape == (1, 4, 128) and c == [3]
    assert multi.cross_match(g, c, 0, 1, None) == {}
    # Packed code blocks: whole 128-B code rows per rank, keys after the codes.
    assert multi.code_block_rows(2000) == 2016 and multi.code_set(1, 2016) == (2079, 66528 + 64512)
    rows = torch.from_numpy(np.arange(3 * 128, dtype=np.float16).reshape(3, 128) % 256).view(torch.int16)
    codes, keys = multi.codes_from_rows(rows)
    buf, n_pad = multi.all_gather_codes(codes, keys, 1)
    assert n_pad == 32 and buf.numel() == 32 * 132
    c2, k2 = multi.unpack_codes(buf, 0, 3, n_pad)
    assert torch.equal(c2, codes) and torch.equal(k2, keys)
    assert multi.code_pairs([3], 0, 1, n_pad) == []
