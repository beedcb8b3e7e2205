"""Multi-GPU: one process per GPU, clips sharded contiguously across ranks, and ONE collective —
an all-gather of the generated token ids (+ lengths) to every rank for scoring.

The caption path has no cross-clip state (predict_prompt.py:129-148 iterates clips
independently), so ranks never exchange activations; ``torch.distributed`` with backend "nccl"
is RCCL over xGMI on ROCm (gloo on CPU for the tests).
"""
from __future__ import annotations

from typing import List, Sequence, Tuple

import torch


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, count-balanced slice [lo, hi) of n clips for `rank` (first n % world ranks
    take one extra clip)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def gather_token_ids(ids: torch.Tensor, lengths: torch.Tensor, n_per_rank: Sequence[int],
                     group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-gather ``ids`` [n_local, T] int32 and ``lengths`` [n_local] from every rank into
    [sum(n_per_rank), T] / [sum] in rank order.  Ranks pad to max(n_per_rank) rows so the
    collective is a single fixed-size all_gather_into_tensor (RCCL) or all_gather (gloo)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    nmax = max(n_per_rank)
    T = ids.shape[1]
    pad_ids = torch.zeros(nmax, T, dtype=ids.dtype, device=ids.device)
    pad_len = torch.zeros(nmax, dtype=lengths.dtype, device=lengths.device)
    pad_ids[:ids.shape[0]] = ids
    pad_len[:lengths.shape[0]] = lengths
    if dist.get_backend(group) == "nccl":
        all_ids = torch.empty(world * nmax, T, dtype=ids.dtype, device=ids.device)
        all_len = torch.empty(world * nmax, dtype=lengths.dtype, device=lengths.device)
        dist.all_gather_into_tensor(all_ids, pad_ids, group=group)
        dist.all_gather_into_tensor(all_len, pad_len, group=group)
    else:
        li = [torch.empty_like(pad_ids) for _ in range(world)]
        ll = [torch.empty_like(pad_len) for _ in range(world)]
        dist.all_gather(li, pad_ids, group=group)
        dist.all_gather(ll, pad_len, group=group)
        all_ids, all_len = torch.cat(li), torch.cat(ll)
    keep: List[int] = []
    for r, n in enumerate(n_per_rank):
        keep.extend(range(r * nmax, r * nmax + n))
    idx = torch.tensor(keep, device=ids.device)
    return all_ids.index_select(0, idx), all_len.index_select(0, idx)
