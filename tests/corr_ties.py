"""Loader and replay of tests/golden/corr_ties.* (the correlator's threshold
tie points, generated from the reference by tests/golden/gen_corr_ties.py).

A replay target is any object with the oracle's correlator face:
set_pattern(p), step(x) -> (found, index), bit_samples(), status()."""
from __future__ import annotations

import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
GOLDEN = os.path.join(HERE, "golden")


def load():
    with open(os.path.join(GOLDEN, "corr_ties.json")) as f:
        man = json.load(f)
    arr = np.load(os.path.join(GOLDEN, "corr_ties.npz"))
    return man, arr


def pattern(case) -> np.ndarray:
    p = np.zeros((case["N"], 2), np.int32)
    p[0, 0] = case["pattern_tap0"]
    return p


def registers(x: np.ndarray, case):
    """corr and (scaled) energy of every output for the fixture's one-tap
    pattern (correlators.h:233-250 with coeffScaling 12): the correlation is a
    function of the window's oldest sample alone."""
    N, S, P = case["N"], case["S"], case["pattern_tap0"]
    xr, xi = x[:, 0].astype(np.int64), x[:, 1].astype(np.int64)
    n = len(x)
    j = np.arange(n)
    old = j - (N - 1) * S
    ok = old >= 0
    corr = np.zeros(n, np.int64)
    corr[ok] = ((P * xr[old[ok]] >> 12) >> 2) ** 2 + ((P * xi[old[ok]] >> 12) >> 2) ** 2
    p = xr * xr + xi * xi
    en = np.zeros(n, np.int64)
    for k in range(N):
        idx = j - k * S
        m = idx >= 0
        en[m] += p[idx[m]]
    return corr, en >> 6


def band_peaks(x: np.ndarray, case):
    """Local peaks with energy above 300^2 whose registers lie inside the GPU
    test's 1e-9 relative band around corr = 7.29 energy, and the reference's
    verdict on each (sqrt in double, correlators.h:265-268)."""
    corr, en = registers(x, case)
    c1, c2, c0, e1 = corr[1:-1], corr[:-2], corr[2:], en[1:-1]
    peak = (c1 > c2) & (c1 > c0) & (e1 > 90000)
    band = np.abs(c1 - 7.29 * e1) <= 1e-9 * c1
    sel = np.nonzero(peak & band)[0]
    cs, es = c1[sel].astype(np.float64), e1[sel].astype(np.float64)
    verdict = np.sqrt(cs) > np.sqrt(es) * 2.7
    return sel + 1, verdict


def replay(case, arr, obj) -> list[str]:
    """Step `obj` through the case's script; return mismatch strings."""
    fails = []
    key = case["key"]
    x = arr[key + "_x"]
    obj.set_pattern(pattern(case))
    for i, st in enumerate(case["steps"]):
        xs = x[st["pos"]:st["pos"] + st["len"]]
        found, idx = obj.step(xs)
        if (bool(found), idx if found else -1) != (st["found"], st["index"]):
            fails.append(f"{key} step {i}: ({found}, {idx}) != ({st['found']}, {st['index']})")
            break
        s = obj.status()
        if list(s["energy"]) != st["energy"] or list(s["corr"]) != st["corr"]:
            fails.append(f"{key} step {i}: registers {s['energy']} {s['corr']} != {st['energy']} {st['corr']}")
        if found and not np.array_equal(np.asarray(obj.bit_samples()).reshape(-1, 2), arr[f"{key}_bits{i}"]):
            fails.append(f"{key} step {i}: bitSamples differ")
    return fails
