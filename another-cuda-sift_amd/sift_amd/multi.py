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
