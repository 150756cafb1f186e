"""Filter-design and synthetic-signal helpers (host side, numpy only).

These produce the coefficient sets and pattern the benchmark configurations of
BASELINE.json use; they are ordinary product utilities, not part
of the oracle.
"""
from __future__ import annotations

import numpy as np


def hamming_sinc(ntaps: int = 127, cutoff: float = 0.125) -> np.ndarray:
    """Hamming-windowed sinc low-pass, cutoff in cycles/sample, computed in
    double and cast to float32 (127 taps at fs/8: sum|c| = 1.9288, so the
    reference's coeffScaling is 0 under both abs() bindings)."""
    n = np.arange(ntaps, dtype=np.float64)
    m = n - (ntaps - 1) / 2.0
    h = 2.0 * cutoff * np.sinc(2.0 * cutoff * m)
    w = 0.54 - 0.46 * np.cos(2.0 * np.pi * n / (ntaps - 1))
    return (h * w).astype(np.float32)


def q14(c: np.ndarray) -> np.ndarray:
    """Q14 fixed-point version of float coefficients (lround(c * 16384))."""
    return np.array([int(np.round(float(v) * 16384.0)) for v in c], dtype=np.int32)


def qpsk_pattern(n: int, amplitude: int = 500, seed: int = 0x5EED) -> np.ndarray:
    """+-amplitude QPSK pattern as complex<int32_t> pairs, shape [n, 2]."""
    rng = np.random.default_rng(seed)
    bits = rng.integers(0, 2, size=(n, 2))
    return np.where(bits == 1, amplitude, -amplitude).astype(np.int32)
