"""CPU: the correlator tie-point fixtures (tests/golden/corr_ties.*, made
from the reference build by tests/golden/gen_corr_ties.py) force the
threshold test's tie branch, and the C restatement replays them bit-exactly
(detections, indices, bitSamples and the 3-tap registers at every step)."""
import numpy as np
import pytest

import corr_ties as T

MAN, ARR = T.load()


@pytest.mark.parametrize("case", MAN["cases"], ids=lambda c: c["key"])
def test_fixture_forces_the_tie_band(case):
    """Every stream holds local peaks inside the GPU fast test's 1e-9 band
    that the reference detects AND ones it rejects (rule: a rare branch needs
    an input that forces it), at exactly the crafted events."""
    x = ARR[case["key"] + "_x"]
    at, verdict = T.band_peaks(x, case)
    assert verdict.any() and (~verdict).any()
    assert len(at) == case["band_peaks"] >= 8
    assert int(verdict.sum()) == case["band_detected"]
    evs = {e["peak"]: e for e in case["events"]}
    for i, v in zip(at, verdict):
        assert evs[int(i)]["band"] and evs[int(i)]["ref_hit"] == bool(v)
    # exact ties c * 100 == 729 * e among them, both verdicts
    ties = [e for e in case["events"] if e["c"] * 100 == 729 * e["e"]]
    assert any(e["detected"] for e in ties) and any(not e["detected"] for e in ties)


@pytest.mark.parametrize("fp", [0, 1])
@pytest.mark.parametrize("case", MAN["cases"], ids=lambda c: c["key"])
def test_oracle_replays_tie_fixture(case, fp):
    import pyoracle
    o = pyoracle.Oracle(fp).corr(case["N"], case["S"])
    assert T.replay(case, ARR, o) == []


def test_host_threshold_expression_at_ties():
    """The host evaluation the GPU tests compare against: IEEE double sqrt and
    multiply, as the reference's `corr > energy * 2.7 && energy > 300`.
    Perfect-square ties are never detected; general ties split."""
    k = np.arange(31, 600, dtype=np.float64)
    assert not (np.sqrt(729 * k * k) > np.sqrt(100 * k * k) * 2.7).any()
    m = np.arange(901, 20000, dtype=np.float64)
    v = np.sqrt(729 * m) > np.sqrt(100 * m) * 2.7
    assert v[912 - 901] and not v[0] and 0 < v.sum() < len(m)
