"""Multi-GPU layout of the channel-parallel workloads (BASELINE configs[2]).

One process per GPU (torch.distributed over RCCL/xGMI).  Independent channels
are block-partitioned over ranks -- rank r owns channels [r*C, (r+1)*C) -- and
every rank generates its own channels' input on its own device, so the data
path has no collective at all (weak scaling).  The only exchange is the
optional gather of the decimated outputs to rank 0 (RCCL gather over xGMI,
timed separately from the hot path).
"""
from __future__ import annotations


def channels_for_rank(total_channels: int, world: int, rank: int) -> range:
    """Contiguous block partition; the first total % world ranks get one extra."""
    if not (0 <= rank < world) or total_channels < 0:
        raise ValueError("bad rank/world/channels")
    q, r = divmod(total_channels, world)
    lo = rank * q + min(rank, r)
    return range(lo, lo + q + (1 if rank < r else 0))


def gather_to_root(t, world: int, rank: int):
    """Gather equal-shaped tensors from every rank to rank 0 (None elsewhere).
    Over the "nccl" backend this is RCCL over xGMI; over "gloo" (tests) the
    same call runs on CPU tensors."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return [t]
    cplx = t.is_complex()
    src = torch.view_as_real(t) if cplx else t  # collectives move complex data as real pairs
    bufs = [torch.empty_like(src) for _ in range(world)] if rank == 0 else None
    dist.gather(src, bufs, dst=0)
    if bufs is not None and cplx:
        bufs = [torch.view_as_complex(b) for b in bufs]
    return bufs


def max_over_ranks(x: float, world: int, device=None) -> float:
    """MAX of a host scalar over ranks (the bench's per-rank wall times)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
