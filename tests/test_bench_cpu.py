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
