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


def shard_counts(n: int, world: int) -> List[int]:
    """Clips per rank under shard_range."""
    return [shard_range(n, r, world)[1] - shard_range(n, r, world)[0] for r in range(world)]


def gather_rows(t: torch.Tensor, n_per_rank: Sequence[int], group=None) -> torch.Tensor:
    """All-gather the leading-dimension rows ``t`` [n_local, ...] of every rank into
    [sum(n_per_rank), ...] in rank order.  Ranks pad to max(n_per_rank) rows so the collective is
    ONE fixed-size all_gather_into_tensor (RCCL over xGMI) or all_gather (gloo)."""
    import torch.distributed as dist
    world = dist.get_world_size(group)
    nmax = max(n_per_rank)
    pad = torch.zeros((nmax,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    pad[:t.shape[0]] = t
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * nmax,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        dist.all_gather_into_tensor(out, pad, group=group)
    else:
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        out = torch.cat(parts)
    keep: List[int] = []
    for r, n in enumerate(n_per_rank):
        keep.extend(range(r * nmax, r * nmax + n))
    return out.index_select(0, torch.tensor(keep, device=t.device))


def gather_token_ids(ids: torch.Tensor, lengths: torch.Tensor, n_per_rank: Sequence[int],
                     group=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """All-gather ``ids`` [n_local, T] int32 and ``lengths`` [n_local] from every rank into
    [sum(n_per_rank), T] / [sum] in rank order (the one collective of the caption path).  The
    lengths travel as an extra column of the id rows: one all-gather, not two."""
    T = ids.shape[1]
    both = torch.cat([ids.to(torch.int32), lengths.to(torch.int32).view(-1, 1)], 1)
    out = gather_rows(both, n_per_rank, group)
    return out[:, :T].to(ids.dtype), out[:, T].to(lengths.dtype)


def collect_captions(results, n_per_rank: Sequence[int], group=None):
    """The bench / predict N>1 collective: the local CaptionBatch results (in clip order; greedy
    ids [b, T] + lengths [b], or beam [b, beam, T] + seq_len / scores [b, beam] of which the best
    beam is gathered) -> every rank's clips' token ids and lengths, in global clip order."""
    ids, ln = [], []
    for r in results:
        if r.ids.dim() == 2:
            ids.append(r.ids)
            ln.append(r.lengths.int())
        else:      # beam: the best beam (scores / seq_len, first on ties as a stable sort)
            best = (r.scores / r.lengths).argmax(1)
            ar = torch.arange(best.numel(), device=best.device)
            ids.append(r.ids[ar, best])
            ln.append(r.lengths[ar, best].int())
    return gather_token_ids(torch.cat(ids), torch.cat(ln), n_per_rank, group)
