"""Multi-GPU layouts.  One process per GPU (torch.distributed
over RCCL/xGMI).

* Channels (BASELINE configs[2]): independent channels are block-partitioned
  over ranks -- rank r owns channels [r*C, (r+1)*C) -- and every rank generates
  its own channels' input on its own device, so the data path has no
  collective at all (weak scaling).  The only exchange is the optional gather
  of the decimated outputs to rank 0 (RCCL gather over xGMI, timed separately
  from the hot path).
* One long buffer, split in time: rank r owns samples [s_r, e_r) (aligned to
  the decimation M) and seeds its operator state from the halo just before
  s_r -- the decimator by stepping ceil((N-1)/M)*M halo samples (outputs
  dropped), the mixer by setting its phase to the closed form (mixers.h:177),
  the correlator with prime() over its N*S+2 halo samples.  Each rank's
  outputs are then bit-identical to the same outputs of the unsplit call.
  The correlator's answer is the FIRST detection over all ranks: one MIN
  all-reduce of the rank-local first index (the only data-path collective).
"""
from __future__ import annotations


def _single(world: int) -> bool:
    """world 1 and no process group: nothing to exchange (with a one-rank
    group -- bench.py's SRCDSP_BENCH_PG rehearsal -- the collectives run)"""
    if world != 1:
        return False
    import torch.distributed as dist
    return not (dist.is_available() and dist.is_initialized())


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
    if _single(world):
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
    if _single(world):
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def time_segment(total: int, world: int, rank: int, align: int = 1) -> tuple[int, int]:
    """[start, end) of rank's contiguous share of `total` samples, boundaries
    multiples of `align` (the decimation factor), earlier ranks larger."""
    if not (0 <= rank < world) or total < 0 or align < 1 or total % align:
        raise ValueError("bad rank/world/total/align")
    units = channels_for_rank(total // align, world, rank)
    return units.start * align, units.stop * align


def decim_halo(ntaps: int, M: int) -> int:
    """Halo samples that rebuild a decimator's N-1 history with whole output
    groups: ceil((N-1)/M)*M."""
    return -(-(ntaps - 1) // M) * M


def corr_halo(N: int, S: int) -> int:
    """Halo that rebuilds the correlator's history (N*S-1 samples) and its
    three corr/energy registers: N*S + 2 samples."""
    return N * S + 2


NO_DETECTION = 2**62


def first_detection(local_index, world: int, device=None) -> int:
    """Global first detection index: MIN over ranks of each rank's first local
    detection (already in global sample coordinates; NO_DETECTION if none)."""
    import torch
    import torch.distributed as dist
    v = NO_DETECTION if local_index is None else int(local_index)
    if _single(world):
        return v
    t = torch.tensor([v], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def corr_segment_search(corr, x_halo, x_seg, start: int):
    """Run one rank's share of a split correlator call: prime with the halo
    (the samples just before `start`, at most corr_halo() of them), step the
    segment.  Returns the global corrIndex of the first local detection, or
    None.  `corr` is any object with prime()/step() (the product operator, or
    an oracle in CPU tests)."""
    if x_halo is not None and len(x_halo):
        corr.prime(x_halo)
    found, idx = corr.step(x_seg)
    return start + idx if found else None
