"""One rank of the 2-rank GPU rehearsal of the N > 1 path (tests/test_gpu_dist.py).

Started as a child process (RANK / WORLD_SIZE / MASTER_* in the environment)
before it touches the GPU; every rank shares cuda:0 and runs the PRODUCT
kernels, the collectives go over gloo (two ranks on one GPU cannot form an
RCCL communicator: "Duplicate GPU detected").

  channels:  rank r owns dist.channels_for_rank(C, 2, r), steps them with one
             batched launch (S.decim_step_batched), then dist.gather_to_root;
  time split: one long buffer, rank r primes the correlator with the N*S+2
             samples before its share, scans its share, first detection by
             dist.first_detection (MIN all-reduce); the decimator is seeded by
             its halo the same way.
Rank 0 writes the gathered / reduced results to OUT (.npz) for the test to
compare with a single-process run and the oracle."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CH, L = 5, 1 << 20          # channels (uneven over 2 ranks: 3 + 2), samples per channel
LC, NC, SC = 1 << 20, 1024, 1  # correlator: samples, pattern length, bitSamples


def corr_input(pat_at):
    from srcdsp_amd.design import qpsk_pattern
    p = qpsk_pattern(NC, 500, seed=2)
    rng = np.random.default_rng(0)
    x = rng.integers(-125, 126, size=(LC, 2)).astype(np.int32)
    if pat_at is not None:
        x[pat_at:pat_at + NC] += 2 * p
    return p, np.clip(x, -32768, 32767).astype(np.int16)


def main():
    import torch
    import torch.distributed as dist
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    out_path = os.environ["OUT"]
    pat_at = int(os.environ["PAT_AT"]) if os.environ.get("PAT_AT") else None
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import srcdsp_amd as S
    from srcdsp_amd import dist as D
    from srcdsp_amd.design import hamming_sinc
    S.lib()  # the HIP library, loudly
    c = hamming_sinc(127)

    # ---- channels: batched product launch on this rank's share, gather to rank 0
    mine = D.channels_for_rank(CH, world, rank)
    x = torch.empty((len(mine), L), dtype=torch.complex64, device="cuda")
    for i, ch in enumerate(mine):
        S.fill_synthetic(x[i], "cf32", seed=0x5EED, channel=ch)
    y = torch.empty((len(mine), L // 4), dtype=torch.complex64, device="cuda")
    fs = [S.FilterDnsamplingFir(c, 4) for _ in mine]
    S.decim_step_batched(fs, x, y)
    torch.cuda.synchronize()
    # gather needs equal shapes: pad the short rank with empty rows, drop them at the root
    rows = max(len(D.channels_for_rank(CH, world, r)) for r in range(world))
    yp = torch.zeros((rows, L // 4), dtype=torch.complex64)
    yp[:len(mine)] = y.cpu()
    got = D.gather_to_root(yp, world, rank)

    # ---- one long buffer split in time: decimator halo + correlator prime + MIN all-reduce
    s0, s1 = D.time_segment(L, world, rank, align=4)
    xs = torch.empty(L, dtype=torch.complex64, device="cuda")
    S.fill_synthetic(xs, "cf32", seed=0x5EED, channel=11)
    h = min(s0, D.decim_halo(127, 4))
    d = S.FilterDnsamplingFir(c, 4)
    ys = d.step(xs[s0 - h:s1])[h // 4:].cpu()
    seg = [D.time_segment(L, world, r, align=4) for r in range(world)]
    ysp = torch.zeros(max(b - a for a, b in seg) // 4, dtype=torch.complex64)  # gather needs equal shapes
    ysp[:len(ys)] = ys
    ys_all = D.gather_to_root(ysp, world, rank)
    p, xc = corr_input(pat_at)
    c0, c1 = D.time_segment(LC, world, rank)
    hc = min(c0, D.corr_halo(NC, SC))
    g = S.FixedPatternCorrelator(NC, SC)
    g.setPattern(p)
    halo = torch.from_numpy(xc[c0 - hc:c0]).cuda() if hc else None
    local = D.corr_segment_search(g, halo, torch.from_numpy(xc[c0:c1]).cuda(), c0)
    first = D.first_detection(local, world)

    if rank == 0:
        sizes = [len(D.channels_for_rank(CH, world, r)) for r in range(world)]
        chans = np.concatenate([got[r].numpy()[:sizes[r]] for r in range(world)])
        split = np.concatenate([ys_all[r].numpy()[:(b - a) // 4] for r, (a, b) in enumerate(seg)])
        np.savez(out_path, chans=chans, split=split, first=np.int64(first))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
