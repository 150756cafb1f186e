"""The N > 1 code path with the real kernels: two ranks,
child processes started before they touch the GPU, share cuda:0 and run the
product's batched decimator on their channels_for_rank share + gather_to_root,
and the time-split decimator / correlator + first_detection's MIN all-reduce
(tests/dist_ranks.py; collectives over gloo: two ranks on one GPU cannot form
an RCCL communicator).  Rank 0's gathered results must equal a
single-process GPU run byte for byte, and the oracle."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("pat_at", [None, 300000, (1 << 19) - 500, 700000],
                         ids=["no-hit", "hit-rank0", "hit-straddles", "hit-rank1"])
def test_two_ranks_on_gpu_match_single_process(tmp_path, pat_at):
    import torch
    if torch.cuda.device_count() < 1:  # counts devices without initialising the GPU here
        pytest.skip("no GPU")
    out = str(tmp_path / "rank0.npz")
    port = _free_port()
    env = dict(os.environ, WORLD_SIZE="2", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OUT=out,
               PAT_AT="" if pat_at is None else str(pat_at))
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "dist_ranks.py")],
                              env=dict(env, RANK=str(r), LOCAL_RANK="0")) for r in range(2)]
    try:
        rcs = [p.wait(timeout=180) for p in procs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert rcs == [0, 0], f"rank exit codes {rcs}"
    got = np.load(out)

    sys.path.insert(0, HERE)
    import dist_ranks as R
    import pyoracle
    import srcdsp_amd as S
    from srcdsp_amd.design import hamming_sinc
    c = hamming_sinc(127)
    # single process, every channel in one batched launch
    x = torch.empty((R.CH, R.L), dtype=torch.complex64, device="cuda")
    for ch in range(R.CH):
        S.fill_synthetic(x[ch], "cf32", seed=0x5EED, channel=ch)
    y = torch.empty((R.CH, R.L // 4), dtype=torch.complex64, device="cuda")
    S.decim_step_batched([S.FilterDnsamplingFir(c, 4) for _ in range(R.CH)], x, y)
    one = y.cpu().numpy()
    assert np.array_equal(got["chans"].view(np.uint32), one.view(np.uint32))
    o = pyoracle.Oracle(1)
    for ch in (0, R.CH - 1):  # and the oracle on the first and last channel
        ref = o.decim(0, 4, c).step(o.gen_cf32(0x5EED, ch, 0, R.L))
        assert np.array_equal(one[ch].view(np.uint32), ref.view(np.uint32))
    # one long buffer, split in time
    xs = torch.empty(R.L, dtype=torch.complex64, device="cuda")
    S.fill_synthetic(xs, "cf32", seed=0x5EED, channel=11)
    whole = S.FilterDnsamplingFir(c, 4).step(xs).cpu().numpy()
    assert np.array_equal(got["split"].view(np.uint32), whole.view(np.uint32))
    p, xc = R.corr_input(pat_at)
    g = S.FixedPatternCorrelator(R.NC, R.SC)
    g.setPattern(p)
    found, idx = g.step(torch.from_numpy(xc).cuda())
    from srcdsp_amd import dist as D
    assert int(got["first"]) == (idx if found else D.NO_DETECTION)
    assert found == (pat_at is not None)
    go = o.corr(R.NC, R.SC)
    go.set_pattern(p)
    ofound, oidx = go.step(xc)
    assert ofound == found and (not found or oidx == idx)


def test_bench_two_rank_rehearsal_default_layout():
    """`bench.py --gpus 2` as the driver runs it, both ranks on cuda:0
    (collectives rehearsed over gloo: two ranks on one device cannot form an
    RCCL communicator): the main series is one 2^28 channel per rank (the
    N = 1 line's work per GPU, weak scaling); `configs2_share` beside it runs
    8 channels per rank, labelled as configs[2]'s per-GPU layout (16 of 64),
    and its timed gather moves all 16 channels' outputs (8 GiB) to rank 0;
    both report 0 mismatches against the channel digests."""
    import json
    import torch
    if torch.cuda.device_count() < 1:
        pytest.skip("no GPU")
    root = os.path.dirname(HERE)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["SRCDSP_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--no-cpu-baseline", "--no-pcie"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["world_size_reported"] == 2 and line["backend"] == "gloo"
    cfg = line["config"]
    assert cfg["channels_per_gpu"] == 1 and cfg["channels_total"] == 2
    assert cfg["baseline_config"] == "configs[1] on each of 2 GPUs (2 independent channels)"
    assert cfg["samples_per_channel"] == 1 << 28
    assert line["roofline"]["per_gpu"] and line["roofline"]["channels_per_launch"] == 1
    assert line["roofline"]["algorithmic_bytes_per_launch"] == (1 << 28) * 10
    sh = line["configs2_share"]
    assert sh["baseline_config"] == "configs[2] per-GPU layout (16 of 64 channels)"
    assert sh["channels_per_gpu"] == 8 and sh["channels_total"] == 16 and sh["value"] > 0
    assert sh["gather_bytes"] == 16 * (1 << 26) * 8 and sh["gather_ms"] > 0
    assert sh["roofline"]["channels_per_launch"] == 8
    assert sh["roofline"]["algorithmic_bytes_per_launch"] == 8 * (1 << 28) * 10
    # cross-rank parity: every rank's channels and what the gather
    # delivered equal the oracle/reference digests (tests/golden/channel_digests.json)
    p = line["parity"]
    assert (p["channels_checked"], p["mismatches"], p["missing"]) == (2, 0, 0), p
    assert (sh["parity"]["channels_checked"], sh["parity"]["mismatches"]) == (16, 0), sh["parity"]
    assert (sh["gather_parity"]["channels_checked"], sh["gather_parity"]["mismatches"]) == (16, 0)
