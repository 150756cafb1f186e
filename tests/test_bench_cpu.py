"""bench.py's CPU-side legs (no GPU): the reference CPU baselines it prints
beside the GPU numbers.  Only the checker (oracle/_ref) runs here."""
import os
import sys
import types

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

REF = os.path.join(ROOT, "oracle", "_ref", "strict", "libref_decim_old.so")


@pytest.mark.skipif(not os.path.exists(REF), reason="reference build (oracle/_ref) not present")
def test_cpu_baseline_single_and_allcores_shape():
    a = types.SimpleNamespace(workload="decim", cpu_sample=1 << 18, samples=1 << 28)
    one = bench.cpu_baseline(a)
    assert one["kind"] == "reference" and one["cores"] == 1 and one["value"] > 0
    many = bench.cpu_baseline_allcores(a, threads=2)
    assert many["kind"] == "reference" and many["cores"] == 2 and many["value"] > 0
    assert "2 threads" in many["sample"]


def test_allcores_only_for_the_headline():
    a = types.SimpleNamespace(workload="fir", cpu_sample=1 << 18, samples=1 << 28)
    assert bench.cpu_baseline_allcores(a, threads=2) is None


def test_gpus_flag_starts_that_many_ranks():
    """`bench.py --gpus 2` with no launcher starts 2 ranks itself (a child
    torch.distributed.run, no exec); --dry-run makes every rank rendezvous over
    gloo, report its world and exit before any GPU call."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(l["rank"] for l in lines) == [0, 1]
    assert all(l["world"] == 2 and l["world_seen"] == 2 and l["gpus"] == 2 for l in lines)


def test_world_mismatch_fails_loudly():
    """A rank whose launcher world differs from --gpus refuses to run."""
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "--gpus 2" in (r.stderr + r.stdout)


def test_host_cores_reports_share():
    n, note = bench.host_cores()
    assert n >= 1 and "machine nproc" in note


def test_channel_layout_matches_baseline_configs():
    """The main series holds the same per-GPU work at every N: one 2^28
    channel per GPU (configs[1] at N = 1), so SCALE's 1/2/4/8 values are weak
    scaling on one layout.  configs[2]'s share (8 x 2^28 per GPU, 64 over 8
    GPUs, 32 GiB gather at N = 8) is measured beside it at N > 1 (N = 1 with
    --share), and only N = 8 is labelled configs[2] (VERDICT r4 item 6,
    ADVICE r4)."""
    a = types.SimpleNamespace(workload="decim", samples=None, channels_per_gpu=None, no_share=False, share=False)
    one = bench.channel_layout(a, 1)
    assert one == {"channels_per_gpu": 1, "channels_total": 1, "samples_per_channel": 1 << 28,
                   "baseline_config": "configs[1]"}
    for n in (2, 4, 8):
        lay = bench.channel_layout(a, n)
        assert lay["channels_per_gpu"] == 1 and lay["channels_total"] == n
        assert lay["baseline_config"] == f"configs[1] on each of {n} GPUs ({n} independent channels)"
    labels = {1: "configs[2] per-GPU layout (8 of 64 channels)", 2: "configs[2] per-GPU layout (16 of 64 channels)",
              4: "configs[2] per-GPU layout (32 of 64 channels)", 8: "configs[2]"}
    assert bench.share_layout(a, 1) is None  # N = 1: the headline's launches alone unless --share
    for n, want in labels.items():
        a.share = n == 1
        sh = bench.share_layout(a, n)
        assert sh["channels_per_gpu"] == 8 and sh["channels_total"] == 8 * n and sh["baseline_config"] == want
        assert sh["gather_bytes"] == (8 * n * (1 << 26) * 8 if n > 1 else 0)
    assert bench.share_layout(a, 8)["gather_bytes"] == 32 << 30
    a.channels_per_gpu = 8  # an explicit layout becomes the main series, no share beside it
    assert bench.channel_layout(a, 8)["baseline_config"] == "configs[2]"
    assert bench.channel_layout(a, 4)["baseline_config"] == "configs[2] per-GPU layout (32 of 64 channels)"
    assert bench.share_layout(a, 8) is None
    a.channels_per_gpu = 3
    assert bench.channel_layout(a, 2)["baseline_config"] == "custom"
    c = types.SimpleNamespace(workload="corr", samples=1 << 26, channels_per_gpu=None, no_share=False, share=True)
    assert bench.channel_layout(c, 8)["channels_per_gpu"] == 1 and bench.channel_layout(c, 8)["baseline_config"] is None
    assert bench.share_layout(c, 8) is None


@pytest.mark.parametrize("n", [2, 4, 8])
def test_gpus_n_dry_run_world_and_labels(n):
    """`bench.py --gpus N --dry-run`, the driver's N-GPU command with no GPU
    touched: N ranks assemble one gloo world; every rank holds the main
    series' layout (one 2^28 channel per GPU) and configs[2]'s share, labelled
    configs[2] only at N = 8."""
    import json
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert sorted(l["rank"] for l in lines) == list(range(n))
    for l in lines:
        assert l["world"] == n and l["world_seen"] == n
        assert l["layout"] == {"channels_per_gpu": 1, "channels_total": n, "samples_per_channel": 1 << 28,
                               "baseline_config": f"configs[1] on each of {n} GPUs ({n} independent channels)"}
        sh = l["share_layout"]
        assert sh["channels_per_gpu"] == 8 and sh["channels_total"] == 8 * n
        assert sh["gather_bytes"] == 8 * n * (1 << 26) * 8
        assert sh["baseline_config"] == ("configs[2]" if n == 8 else
                                         f"configs[2] per-GPU layout ({8 * n} of 64 channels)")


def _host_ranks(n, extra_env=None, args=()):
    """Run tests/bench_host_rank.py as n gloo ranks (the driver's `bench.py
    --gpus n` path with host stand-ins for the operators and the device) and
    return rank 0's JSON line."""
    import json
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(n), OMP_NUM_THREADS="1",
               **(extra_env or {}))
    cmd = [sys.executable, os.path.join(ROOT, "tests", "bench_host_rank.py"), "--gpus", str(n),
           "--samples", str(1 << 20), "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-pcie", *args]
    procs = [subprocess.Popen(cmd, env=dict(env, RANK=str(r), LOCAL_RANK=str(r)), stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True) for r in range(n)]
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-3000:]
    lines = [l for l in outs[0][0].splitlines() if l.startswith("{")]
    assert len(lines) == 1 and not any(l.startswith("{") for o, _ in outs[1:] for l in o.splitlines())
    return json.loads(lines[0])


DIGESTS = os.path.join(ROOT, "tests", "golden", "channel_digests.json")


@pytest.mark.skipif(not os.path.exists(DIGESTS), reason="tests/golden/channel_digests.json not generated")
def test_bench_main_two_ranks_end_to_end_on_host():
    """bench.main() past timed_steps at --gpus 2 (gloo,
    host stand-ins): the line is assembled, the main series' parity covers
    channels 0 and 1, configs[2]'s share covers channels 0..15 on the ranks
    and again after the gather at rank 0, all with 0 mismatches against the
    committed digests."""
    line = _host_ranks(2)
    assert line["n_gpus"] == 2 and line["world_size_reported"] == 2 and line["backend"] == "gloo"
    assert line["value"] > 0 and line["ms_per_step"] > 0 and line["steps"] == 2
    assert line["config"]["channels_total"] == 2 and line["config"]["samples_per_channel"] == 1 << 20
    p = line["parity"]
    assert (p["channels_checked"], p["mismatches"], p["missing"]) == (2, 0, 0), p
    sh = line["configs2_share"]
    assert sh["channels_total"] == 16 and sh["gather_bytes"] == 16 * (1 << 18) * 8
    assert (sh["parity"]["channels_checked"], sh["parity"]["mismatches"]) == (16, 0), sh["parity"]
    assert (sh["gather_parity"]["channels_checked"], sh["gather_parity"]["mismatches"]) == (16, 0)


@pytest.mark.skipif(not os.path.exists(DIGESTS), reason="tests/golden/channel_digests.json not generated")
def test_bench_main_eight_ranks_end_to_end_on_host():
    """The driver's N = 8 command on the CPU (8 gloo ranks, host stand-ins):
    configs[2] itself (64 channels, 8 per rank) with every rank's digests and
    all 64 gathered at rank 0 clean, the main series one channel per rank."""
    line = _host_ranks(8)
    assert line["n_gpus"] == 8 and line["world_size_reported"] == 8
    assert (line["parity"]["channels_checked"], line["parity"]["mismatches"]) == (8, 0)
    sh = line["configs2_share"]
    assert sh["channels_total"] == 64 and sh["baseline_config"] == "configs[2]"
    assert (sh["parity"]["channels_checked"], sh["parity"]["mismatches"]) == (64, 0)
    assert (sh["gather_parity"]["channels_checked"], sh["gather_parity"]["mismatches"]) == (64, 0)


@pytest.mark.skipif(not os.path.exists(DIGESTS), reason="tests/golden/channel_digests.json not generated")
def test_bench_parity_reports_a_corrupted_channel():
    """One flipped input sample on channel 9 (rank 1's share, not rank 0's):
    the summed counts over ranks and the gathered check both show exactly one
    mismatching channel; the main series (channels 0, 1) stays clean."""
    line = _host_ranks(2, {"STUB_CORRUPT_CHANNEL": "9"})
    assert line["parity"]["mismatches"] == 0
    assert line["configs2_share"]["parity"]["mismatches"] == 1
    assert line["configs2_share"]["gather_parity"]["mismatches"] == 1


@pytest.mark.skipif(not os.path.exists(DIGESTS), reason="tests/golden/channel_digests.json not generated")
def test_bench_main_one_rank_with_share_on_host():
    """The N = 1 path (no process group) with --share: one channel in the main
    series, 8 in the share, no gather."""
    line = _host_ranks(1, args=("--share",))
    assert line["n_gpus"] == 1 and line["backend"] is None
    assert line["parity"]["channels_checked"] == 1 and line["parity"]["mismatches"] == 0
    sh = line["configs2_share"]
    assert sh["parity"]["channels_checked"] == 8 and "gather_ms" not in sh


@pytest.mark.skipif(not os.path.exists(DIGESTS), reason="tests/golden/channel_digests.json not generated")
def test_bench_main_one_rank_process_group_rehearsal():
    """SRCDSP_BENCH_PG=1 at one rank: the process group and every N > 1
    collective (barriers, MAX, parity SUMs, the share's gather, rank 0's
    gathered digests) run at world 1 -- what the GPU box's one-rank RCCL
    rehearsal (scripts/gpu_session.sh pg1) executes on the real backend."""
    line = _host_ranks(1, {"SRCDSP_BENCH_PG": "1"}, args=("--share",))
    assert line["n_gpus"] == 1 and line["backend"] == "gloo" and line["world_size_reported"] == 1
    assert line["parity"]["channels_checked"] == 1 and line["parity"]["mismatches"] == 0
    sh = line["configs2_share"]
    assert sh["gather_bytes"] == 8 * (1 << 18) * 8 and sh["gather_ms"] > 0
    assert (sh["gather_parity"]["channels_checked"], sh["gather_parity"]["mismatches"]) == (8, 0)


def test_host_leg_reports_a_failure_instead_of_raising():
    def boom(args):
        raise OSError("affinity refused")
    assert bench.host_leg(boom, None) == {"error": "OSError: affinity refused"}
    assert bench.host_leg(lambda a, b=1: a + b, 1, b=2) == 3


def test_cpu_topology_and_quota():
    cpus, phys = bench.cpu_topology()
    assert cpus and phys and set(phys) <= set(cpus) and len(phys) <= len(cpus)
    assert "cgroup CPU quota" in bench.cpu_quota() or "no cgroup CPU quota" in bench.cpu_quota()


@pytest.mark.skipif(not os.path.exists(REF), reason="reference build (oracle/_ref) not present")
def test_cpu_baseline_allcores_all_threads_physical_and_share():
    """The default all-cores leg: every CPU of the affinity mask (pinned), one
    per physical core, the job's share, and the cgroup quota note."""
    a = types.SimpleNamespace(workload="decim", cpu_sample=1 << 18, samples=1 << 16)
    r = bench.cpu_baseline_allcores(a)
    cpus, phys = bench.cpu_topology()
    assert r["cores"] == len(cpus) and r["value"] > 0 and "every hardware thread" in r["sample"]
    assert r["physical_cores"]["cores"] == len(phys) and r["physical_cores"]["value"] > 0
    assert r["job_share"]["cores"] == min(len(cpus), bench.host_cores()[0]) and "cpu_quota" in r
