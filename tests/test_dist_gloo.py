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
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0, "a gloo rank failed"
    gathered, tmax = q.get(timeout=10)
    import pyoracle
    from srcdsp_amd.design import hamming_sinc
    o = pyoracle.Oracle(1)
    ref = np.stack([o.decim(0, 4, hamming_sinc(127)).step(o.gen_cf32(0x5EED, ch, 0, L))
                    for ch in range(TOTAL_CH)])
    assert np.array_equal(gathered, ref)
    assert tmax == 2.0
