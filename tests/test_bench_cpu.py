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
