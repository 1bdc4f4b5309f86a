"""Multi-GPU orchestration: one process per GPU, torch.distributed.

* Detect (C2/C4) shards per frame: frame i -> rank i mod world.  Frames are
  independent, so the data path has no collective ("weak" scaling).
* Cross-GPU matching (C5) has one real exchange: every rank's descriptor set
  (n x 128 fp16 bits, padded to a common n) is all-gathered, then each rank
  matches its own set against every peer's (world - 1 ordered pairs) in one
  batched launch.  On MI355X the backend is "nccl" (= RCCL over xGMI) and the
  gather is one all_gather_into_tensor; the CPU tests run the same code over
  "gloo" with a CPU matcher.

The reference has no multi-GPU path; this replaces nothing in
it.  The matcher itself is pluggable so that the exchange logic is testable
without a GPU.
"""
from __future__ import annotations

from typing import Callable, Dict, List, Sequence, Tuple

import torch
import torch.distributed as dist


def frame_shard(n_frames: int, rank: int, world: int) -> List[int]:
    """Frames this rank detects (C4): i = rank, rank + world, ..."""
    return list(range(rank, n_frames, world))


def peer_pairs(rank: int, world: int) -> List[Tuple[int, int]]:
    """Ordered (query set, train set) pairs this rank matches in C5."""
    return [(rank, j) for j in range(world) if j != rank]


def all_gather_rows(local: torch.Tensor, world: int, group=None) -> torch.Tensor:
    """All-gather every rank's (n, 128) descriptor rows (same n on all ranks):
    (world, n, 128).  16-bit descriptor bits travel as int32 (RCCL and gloo
    have no int16); on "nccl" (= RCCL over xGMI) one all_gather_into_tensor."""
    if world == 1 and not dist.is_initialized():
        return local.unsqueeze(0)
    local = local.contiguous()
    wide = local.view(torch.int32) if local.dtype in (torch.int16, torch.float16) else local
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world,) + tuple(wide.shape), dtype=wide.dtype, device=wide.device)
        dist.all_gather_into_tensor(out, wide, group=group)
    else:  # gloo (CPU tests)
        parts = [torch.empty_like(wide) for _ in range(world)]
        dist.all_gather(parts, wide, group=group)
        out = torch.stack(parts)
    return out.view(local.dtype)


def all_gather_counts(count: int, world: int, device, group=None) -> List[int]:
    """Every rank's valid row count (once per set size change, not per exchange)."""
    if world == 1:
        return [count]
    cnt = torch.tensor([count], dtype=torch.int64, device=device)
    counts = [torch.empty_like(cnt) for _ in range(world)]
    dist.all_gather(counts, cnt, group=group)
    return [int(c.item()) for c in counts]


def all_gather_sets(local: torch.Tensor, count: int, world: int, group=None) -> Tuple[torch.Tensor, List[int]]:
    """All-gather every rank's (n, 128) descriptor set (same n on all ranks) and
    its valid row count.  Returns (world, n, 128) and the per-rank counts."""
    counts = all_gather_counts(count, world, local.device, group)
    return all_gather_rows(local, world, group), counts


# ---- C5 exchange of matcher codes instead of fp16 rows ---------------------
# Every detector frame's descriptor kernel also writes the matcher's int8 code
# row c = v - 128 (128 B) and key bias -(256 |c|^2 + (row & 255)) (4 B) beside
# the fp16 row (Detector.results_sidecar): 132 B per row instead of 256, and
# the receivers match them as they arrive (Matcher.match_codes_batched: no
# conversion launch).  One collective per exchange: each rank sends one packed
# block [n_pad code rows | n_pad keys], n_pad = n rounded up to CODE_ROWS so
# the block is whole 128-B code rows (32 x 132 B = 33 x 128 B).
CODE_ROWS = 32


def codes_from_rows(rows: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(codes int8 (n, 128), keys int32 (n,)) of fp16 descriptor rows holding
    integers 0..255 -- the sidecar's definition, for rows no detector wrote
    (padding, foreign sets)."""
    v = rows.view(torch.float16).to(torch.int32)
    c = v - 128
    r = torch.arange(rows.shape[0], dtype=torch.int32, device=rows.device)
    keys = -(256 * (c * c).sum(dim=1, dtype=torch.int32) + (r & 255))
    return c.to(torch.int8), keys.to(torch.int32)


def code_block_rows(n: int) -> int:
    return (n + CODE_ROWS - 1) // CODE_ROWS * CODE_ROWS


def pack_codes(codes: torch.Tensor, keys: torch.Tensor, n_pad: int) -> torch.Tensor:
    """One rank's send block: uint8 [n_pad * 132] = n_pad code rows, then n_pad keys."""
    n = codes.shape[0]
    blk = torch.zeros(n_pad * 132, dtype=torch.uint8, device=codes.device)
    blk[: n * 128] = codes.contiguous().view(torch.uint8).reshape(-1)
    blk[n_pad * 128: n_pad * 128 + n * 4] = keys.contiguous().view(torch.uint8).reshape(-1)
    return blk


def code_set(r: int, n_pad: int) -> Tuple[int, int]:
    """(first code row, first key index) of rank r's set in a gathered buffer."""
    return r * n_pad * 132 // 128, (r * n_pad * 132 + n_pad * 128) // 4


def all_gather_codes(codes: torch.Tensor, keys: torch.Tensor, world: int, group=None) -> Tuple[torch.Tensor, int]:
    """All-gather every rank's (n, 128) int8 codes and (n,) int32 keys (same n
    on all ranks) as ONE collective: returns (the gathered uint8 buffer of
    world blocks, n_pad); set r's codes start at code row code_set(r)[0] and its
    keys at key index code_set(r)[1] of that buffer."""
    n_pad = code_block_rows(codes.shape[0])
    blk = pack_codes(codes, keys, n_pad)
    if world == 1 and not dist.is_initialized():
        return blk, n_pad
    if dist.get_backend(group) == "nccl":
        out = torch.empty(world * blk.numel(), dtype=torch.uint8, device=blk.device)
        dist.all_gather_into_tensor(out, blk, group=group)
    else:  # gloo (CPU tests)
        parts = [torch.empty_like(blk) for _ in range(world)]
        dist.all_gather(parts, blk, group=group)
        out = torch.cat(parts)
    return out, n_pad


def unpack_codes(buf: torch.Tensor, r: int, n: int, n_pad: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Rank r's (codes, keys) back from a gathered buffer (tests, CPU matchers)."""
    base = r * n_pad * 132
    codes = buf[base: base + n * 128].view(torch.int8).reshape(n, 128)
    keys = buf[base + n_pad * 128: base + n_pad * 128 + n * 4].view(torch.int32)
    return codes, keys


def code_pairs(counts: Sequence[int], rank: int, world: int, n_pad: int) -> List[Tuple[int, int, int, int, int, int]]:
    """This rank's C5 pairs over a gathered code buffer, as
    Matcher.match_codes_batched takes them: (qrow0, qkey0, nq, trow0, tkey0, nt)."""
    q0, qk = code_set(rank, n_pad)
    out = []
    for _, j in peer_pairs(rank, world):
        t0, tk = code_set(j, n_pad)
        out.append((q0, qk, counts[rank], t0, tk, counts[j]))
    return out


MatchFn = Callable[[Sequence[torch.Tensor], Sequence[int], Sequence[torch.Tensor], Sequence[int]], List[torch.Tensor]]


def cross_match(gathered: torch.Tensor, counts: Sequence[int], rank: int, world: int,
                match_batched: MatchFn) -> Dict[int, torch.Tensor]:
    """Match this rank's set against every peer's in one batched call.

    match_batched(queries, nqs, trains, nts) -> per-pair int32 match index
    arrays (-1 = no match); on the GPU this is sift_amd.Matcher.match_batched
    (one launch for all pairs)."""
    pairs = peer_pairs(rank, world)
    if not pairs:
        return {}
    q = [gathered[rank]] * len(pairs)
    t = [gathered[j] for _, j in pairs]
    res = match_batched(q, [counts[rank]] * len(pairs), t, [counts[j] for _, j in pairs])
    return {j: r for (_, j), r in zip(pairs, res)}
