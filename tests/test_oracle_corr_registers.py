"""The oracle's per-sample correlator registers (orc_corr_registers, test
infrastructure for the integer matrix-core probe scripts/tune/corr_mfma.py):
every sample's corrValue[0] and energyValue[0] (correlators.h:244-250) must
equal the registers the reference itself holds after stepping that sample
(one-sample step() calls on the real build, oracle/_ref, read through its
getStatus), and the oracle's own step + status, on streams without a
detection (a detection's `break` leaves `top` unadvanced, correlators.h:291)."""
import os

import numpy as np
import pytest

import pyoracle

HAVE_REF = pyoracle.reference_available("strict")


def _stream(N, S, n, seed):
    rng = np.random.default_rng(seed)
    amp = min(3000, int((1073217600 / (2 * N)) ** 0.5))  # setPattern's energy assert (correlators.h:185)
    p = rng.integers(-amp, amp, (N, 2)).astype(np.int32)
    x = rng.integers(-200, 200, (n, 2)).astype(np.int16)  # noise: the peak/threshold test never passes
    return p, x


@pytest.mark.parametrize("N,S", [(16, 1), (128, 1), (32, 4), (64, 2), (1024, 1)])  # the reference build's shapes
def test_registers_equal_stepwise_status(N, S):
    o = pyoracle.Oracle(0)
    n = 3000 if N < 1024 else 2500
    p, x = _stream(N, S, n, N + S)
    c = o.corr(N, S)
    c.set_pattern(p)
    corr, energy = c.registers(x)
    refs = [o.corr(N, S)] + ([pyoracle.Reference("strict").corr(N, S)] if HAVE_REF else [])
    for r in refs:
        r.set_pattern(p)
        for i in range(n):
            found, _ = r.step(x[i:i + 1])
            assert not found
            st = r.status()
            assert (st["corr"][0], st["energy"][0]) == (int(corr[i]), int(energy[i])), (type(r).__name__, i)


def test_registers_continue_the_stream():
    """Two calls equal one call (the history ring carries over)."""
    o = pyoracle.Oracle(0)
    p, x = _stream(128, 1, 5000, 3)
    a = o.corr(128, 1)
    a.set_pattern(p)
    c1, e1 = a.registers(x)
    b = o.corr(128, 1)
    b.set_pattern(p)
    c2a, e2a = b.registers(x[:1777])
    c2b, e2b = b.registers(x[1777:])
    assert np.array_equal(c1, np.concatenate([c2a, c2b])) and np.array_equal(e1, np.concatenate([e2a, e2b]))
