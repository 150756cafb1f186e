"""The N>1 path on CPU: two gloo ranks run bench.py's channel sharding and the
result gather to rank 0; the gathered outputs must equal a single-process run
over all channels (outputs bit-identical to 1 GPU).  The decimator
compute is stood in by the oracle here (no GPU); the sharding and collective
code is the product's (srcdsp_amd.dist)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from srcdsp_amd.dist import channels_for_rank, gather_to_root, max_over_ranks

TOTAL_CH, L = 6, 4096


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pyoracle
    from srcdsp_amd.design import hamming_sinc
    o = pyoracle.Oracle(1)
    c = hamming_sinc(127)
    mine = channels_for_rank(TOTAL_CH, world, rank)
    assert len(mine) == TOTAL_CH // world
    ys = np.stack([o.decim(0, 4, c).step(o.gen_cf32(0x5EED, ch, 0, L)) for ch in mine])
    got = gather_to_root(torch.from_numpy(ys), world, rank)
    t = max_over_ranks(float(rank + 1), world)
    if rank == 0:
        q.put((np.concatenate([g.numpy() for g in got]), t))
    dist.barrier()
    dist.destroy_process_group()


def test_partition_is_a_block_cover():
    for total in (1, 7, 8, 64):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                seen += list(channels_for_rank(total, world, r))
            assert seen == list(range(total))


def test_two_rank_shard_and_gather_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:  # read before join: a child blocks at exit until its queued result is consumed
        gathered, tmax = q.get(timeout=120)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs), "a gloo rank failed"
    import pyoracle
    from srcdsp_amd.design import hamming_sinc
    o = pyoracle.Oracle(1)
    ref = np.stack([o.decim(0, 4, hamming_sinc(127)).step(o.gen_cf32(0x5EED, ch, 0, L))
                    for ch in range(TOTAL_CH)])
    assert np.array_equal(gathered, ref)
    assert tmax == 2.0


# ---------------------------------------------------------------- time split
def _time_worker(rank, world, port, q, case):
    """One long buffer split in time: the decimator seeded by its
    halo, the correlator primed by its halo, first detection = MIN all-reduce."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import pyoracle
    from srcdsp_amd import dist as D
    from srcdsp_amd.design import hamming_sinc, qpsk_pattern
    o = pyoracle.Oracle(0)
    # decimator: halo + segment, outputs of the halo dropped
    c = hamming_sinc(127)
    x = o.gen_cf32(0x5EED, 0, 0, 40000)
    s0, s1 = D.time_segment(len(x), world, rank, align=4)
    h = min(s0, D.decim_halo(127, 4))
    d = o.decim(0, 4, c)
    y = d.step(x[s0 - h:s1])[h // 4:]
    ys = gather_to_root(torch.from_numpy(np.ascontiguousarray(y)), world, rank)
    # correlator: pattern placed per case
    p = qpsk_pattern(32, 500, seed=2)
    rng = np.random.default_rng(0)
    xc = rng.integers(-125, 126, size=(20000, 2))
    if case is not None:
        xc[case:case + 32] += 2 * p
    xc = xc.astype(np.int16)
    s0, s1 = D.time_segment(len(xc), world, rank)
    g = o.corr(32, 1)
    g.set_pattern(p)
    hc = min(s0, D.corr_halo(32, 1))
    local = D.corr_segment_search(g, xc[s0 - hc:s0], xc[s0:s1], s0)
    first = D.first_detection(local, world)
    if rank == 0:
        q.put((np.concatenate([t.numpy() for t in ys]), first))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case", [None, 3000, 9984, 9990, 15000])
def test_two_rank_time_split_matches_single_call(case):
    """case = where the pattern starts: rank 0's share, straddling the rank
    boundary (10000) or inside rank 1's share, or no pattern at all."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_time_worker, args=(r, 2, port, q, case)) for r in range(2)]
    for p in procs:
        p.start()
    try:  # read before join: a child blocks at exit until its queued result is consumed
        ys, first = q.get(timeout=120)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs), "a gloo rank failed"
    import pyoracle
    from srcdsp_amd import dist as D
    from srcdsp_amd.design import hamming_sinc, qpsk_pattern
    o = pyoracle.Oracle(0)
    assert np.array_equal(ys, o.decim(0, 4, hamming_sinc(127)).step(o.gen_cf32(0x5EED, 0, 0, 40000)))
    p = qpsk_pattern(32, 500, seed=2)
    rng = np.random.default_rng(0)
    xc = rng.integers(-125, 126, size=(20000, 2))
    if case is not None:
        xc[case:case + 32] += 2 * p
    g = o.corr(32, 1)
    g.set_pattern(p)
    found, idx = g.step(xc.astype(np.int16))
    assert first == (idx if found else D.NO_DETECTION)
    assert found == (case is not None)


def test_time_segments_cover_and_align():
    from srcdsp_amd.dist import time_segment
    for total, align in ((400, 4), (1 << 20, 4), (12, 1), (0, 4)):
        for world in (1, 2, 3, 8):
            segs = [time_segment(total, world, r, align) for r in range(world)]
            assert segs[0][0] == 0 and segs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(segs, segs[1:]))
            assert all(s % align == 0 for seg in segs for s in seg)
