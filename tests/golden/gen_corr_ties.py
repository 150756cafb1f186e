#!/usr/bin/env python3
"""Correlator streams whose local peaks land ON the threshold's tie points.

The reference's detection test (correlators.h:262-268) is
    sqrt((double)corr) > sqrt((double)energy) * 2.7  &&  sqrt(energy) > 300
For integer registers it is decided by double rounding exactly at the ties
corr * 100 == 729 * energy (sqrt(corr) == 2.7 sqrt(energy) in exact
arithmetic): e.g. corr = 729 m, energy = 100 m is detected for m = 912 and
not for m = 901, and never for perfect squares m = k^2.  The GPU kernels
decide by the sign of corr - 7.29 energy and take correctly rounded square
roots only inside a 1e-9 relative band around the tie (srcdsp_amd/csrc/
corr_hit.h), so these streams force that band.

Construction (pattern p[0] = (8000, 0), every other tap 0, so coeffScaling
= 12 and the energy shift is 6): the correlation of output j is the function
f(x) = ((8000 x.re >> 12) >> 2)^2 + (...im...)^2 of the window's OLDEST sample
a = x[j - (N-1) S] alone, and the energy is the sum of |x|^2 over the N
window samples >> 6.  Each event writes `a` with f(a) = corr, then a tail of
non-increasing |x| (stride samples chosen greedily so the window energy lands
in [64 energy, 64 energy + 63]), then zeros: f(stream) -- hence the
correlation sequence -- has a strict local maximum only at `a`, so each event
is one peak with exactly the crafted (corr, energy).

Events per stream, in order: ties that the reference rejects (perfect-square
and general), the largest representable c < 7.29 e just below a tie, energy
90000 with a clear correlation (rejected: sqrt(e) > 300 fails), a tie the
reference detects; then (the caller resumes two samples after each detection,
as the tests do) c just above a tie, energy 90001, large-value ties, and a
final clear detection.  Streams at the shapes the reference build
instantiates (oracle/refbuild/ref_ops.cpp): (N, S) = (16, 1), (128, 1) and
(1024, 1, config 5's) on the fused scan corr_scan_s1; (32, 4) on corr_eval +
corr_detect; (64, 2) on corr_eval_dot2 + corr_detect.

Expected outputs come from the REAL reference (oracle/_ref, both flavours,
which must agree), cross-checked against the C restatement; every event's
peak registers are recomputed here and the number of peaks inside the 1e-9
band recorded.  Run in the build container: python tests/golden/gen_corr_ties.py
"""
from __future__ import annotations

import json
import math
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle as P  # noqa: E402

PEAK_TAP = 8000          # p[0]; coeffScaling = floor(log2(8000)) = 12
CS, ESH = 12, 6


def f_corr(re: int, im: int) -> int:
    return ((PEAK_TAP * re >> CS) >> 2) ** 2 + ((PEAK_TAP * im >> CS) >> 2) ** 2


def ref_hit(c: int, e: int) -> bool:
    return math.sqrt(c) > math.sqrt(e) * 2.7 and math.sqrt(e) > 300


def in_band(c: int, e: int) -> bool:
    return abs(c - 7.29 * e) <= 1e-9 * c


def two_squares(c: int):
    """(qr, qi), qr >= qi >= 0, qr^2 + qi^2 == c, or None."""
    q = math.isqrt(c)
    while q * q * 2 >= c:
        r = c - q * q
        s = math.isqrt(r)
        if s * s == r:
            return q, s
        q -= 1
    return None


def sample_for(q: int) -> int:
    """Smallest x >= 0 with (8000 x >> 12) >> 2 == q."""
    x = -(-16384 * q // 8000)
    assert (PEAK_TAP * x >> CS) >> 2 == q
    return x


def event_samples(c: int, e: int, N: int, S: int):
    """Samples from `a` on (positions a, a+1, ..., a+(N-1)S) for a peak with
    correlation c and energy e, or None when not constructible."""
    qs = two_squares(c)
    if qs is None:
        return None
    a = (sample_for(qs[0]), sample_for(qs[1]))
    if max(a) > 32767:
        return None
    lo = 64 * e - (a[0] ** 2 + a[1] ** 2)
    if lo < 0:
        return None
    cap = int(0.9 * math.hypot(*a))
    v, rem, prev = [], lo, cap
    for _ in range(N - 2):  # greedy, non-increasing stride samples
        x = min(prev, math.isqrt(rem))
        v.append((x, 0))
        rem -= x * x
        prev = x
    # last stride sample (u, w): u^2 + w^2 in [rem, rem + 63], no larger than prev
    last = None
    for u in range(math.isqrt(rem // 2), math.isqrt(rem + 63) + 1):
        w2lo = max(0, rem - u * u)
        w = math.isqrt(w2lo)
        if w * w < w2lo:
            w += 1
        if u * u + w * w <= rem + 63 and w <= u:
            last = (u, w)
            break
    if last is None or (N > 2 and math.hypot(*last) > prev):
        return None
    v.append(last)
    # positions a+1 .. a+(N-1)S: stride sample k at k*S, the positions before it
    # (after the previous stride sample) repeat it, so |x| never increases
    out = [a]
    for k in range(1, N):
        out += [v[k - 1]] * S
    # re-check the crafted registers
    E = sum(x * x + y * y for x, y in out[::S][:N])
    assert 64 * e <= E <= 64 * e + 63 and f_corr(*a) == c, (c, e)
    fs = [f_corr(*s) for s in out]
    assert all(fs[i + 1] <= fs[i] for i in range(len(fs) - 1)) and fs[1] < fs[0], (c, e)
    return out


def tie_ms(want: bool, lo: int, hi: int, square: bool = False):
    """m in [lo, hi) with c = 729 m, e = 100 m a tie the reference decides `want`."""
    if square:
        for k in range(math.isqrt(lo) + 1, math.isqrt(hi)):
            yield k * k
        return
    for m in range(lo, hi):
        if ref_hit(729 * m, 100 * m) == want and two_squares(729 * m) is not None:
            yield m


def near(e: int, above: bool):
    """The representable c closest to 7.29 e strictly above or below it."""
    c, step = ((729 * e) // 100 + 1, 1) if above else ((729 * e - 1) // 100, -1)
    while two_squares(c) is None:
        c += step
    assert (c * 100 > 729 * e) == above
    return c


def at_least(c: int):
    while two_squares(c) is None:
        c += 1
    return c


def events_for(N: int, S: int):
    """(c, e, note) in stream order; the reference's verdicts are recorded, not assumed."""
    m_false = list(tie_ms(False, 901, 4000))
    m_true = list(tie_ms(True, 901, 20000))
    m_true_big = list(tie_ms(True, 250000, 262000))
    m_false_big = list(tie_ms(False, 250000, 250100))
    ev = [
        (729 * 1600, 100 * 1600, "tie k=40 square (rejected)"),
        (729 * 961 * 4, 100 * 961 * 4, "tie k=62 square (rejected)"),
        (729 * m_false[0], 100 * m_false[0], "tie general (rejected)"),
        (729 * m_false[5], 100 * m_false[5], "tie general (rejected)"),
        (near(100 * 3001, False), 100 * 3001, "just below a tie"),
        (at_least(8 * 90000), 90000, "energy 90000, c = 8 e (rejected)"),
        (729 * m_false_big[0], 100 * m_false_big[0], "large tie (rejected)"),
        (729 * m_true[0], 100 * m_true[0], "tie general (DETECTED)"),
        (near(100 * 5003, True), 100 * 5003, "just above a tie (DETECTED)"),
        (at_least(8 * 90001), 90001, "energy 90001, c = 8 e (DETECTED)"),
        (729 * m_true[3], 100 * m_true[3], "tie general (DETECTED)"),
        (729 * m_true_big[0], 100 * m_true_big[0], "large tie (DETECTED)"),
        (729 * 2500, 100 * 2500, "tie k=50 square (rejected)"),
        (near(100 * 7007, False), 100 * 7007, "just below a tie"),
        (729 * m_true[7], 100 * m_true[7], "tie general (DETECTED)"),
        (10 * 200000, 200000, "clear detection"),
    ]
    return ev


def build_stream(N: int, S: int):
    gap = N * S + 37
    xs = [np.zeros((gap, 2), np.int32)]
    meta = []
    pos = gap
    for c, e, note in events_for(N, S):
        s = event_samples(c, e, N, S)
        if s is None:
            raise RuntimeError(f"event not constructible: {note} c={c} e={e} N={N} S={S}")
        arr = np.array(s, np.int32)
        meta.append({"a": pos, "peak": pos + (N - 1) * S, "c": c, "e": e, "note": note,
                     "ref_hit": ref_hit(c, e), "band": in_band(c, e)})
        xs += [arr, np.zeros((gap, 2), np.int32)]
        pos += len(arr) + gap
    x = np.concatenate(xs)
    assert np.abs(x).max() <= 32767
    return x.astype(np.int16), meta


def registers(x: np.ndarray, N: int, S: int):
    """corr and energy of every output, restated for this one-tap pattern."""
    xr, xi = x[:, 0].astype(np.int64), x[:, 1].astype(np.int64)
    n = len(x)
    corr = np.zeros(n, np.int64)
    en = np.zeros(n, np.int64)
    j = np.arange(n)
    old = j - (N - 1) * S
    ok = old >= 0
    corr[ok] = ((PEAK_TAP * xr[old[ok]] >> CS) >> 2) ** 2 + ((PEAK_TAP * xi[old[ok]] >> CS) >> 2) ** 2
    p = xr * xr + xi * xi
    for k in range(N):
        idx = j - k * S
        m = idx >= 0
        en[m] += p[idx[m]]
    return corr, en >> ESH


def run(obj, x, chunks):
    """Step in chunks, resuming two samples after each detection (the tests' protocol)."""
    steps, pos, ci = [], 0, 0
    while pos < len(x):
        k = chunks[ci % len(chunks)]
        ci += 1
        xs = x[pos:pos + k]
        found, idx = obj.step(xs)
        st = obj.status()
        steps.append({"pos": pos, "len": int(len(xs)), "found": bool(found), "index": int(idx) if found else -1,
                      "bits": obj.bit_samples().copy(), "energy": st["energy"], "corr": st["corr"]})
        pos += (idx + 2) if found else len(xs)
    return steps


def main():
    pattern = lambda N: np.array([[PEAK_TAP, 0]] + [[0, 0]] * (N - 1), np.int32)  # noqa: E731
    ref = {f: P.Reference(f) for f in ("strict", "fma")}
    orc = P.Oracle(1)
    arrays, cases = {}, []
    for N, S, chunks in ((16, 1, [3001, 777, 5000]), (128, 1, [4096, 1500]), (32, 4, [2500, 6000]),
                         (64, 2, [9000, 1234]), (1024, 1, [20000, 3333])):
        x, meta = build_stream(N, S)
        corr, en = registers(x, N, S)
        # every crafted peak carries exactly its registers, and is the only
        # strict local maximum of the correlation sequence
        pk = np.nonzero((corr[1:-1] > corr[:-2]) & (corr[1:-1] > corr[2:]))[0] + 1
        assert sorted(pk.tolist()) == [m["peak"] for m in meta], (N, S)
        for m in meta:
            assert (corr[m["peak"]], en[m["peak"]]) == (m["c"], m["e"]), m
        runs = {}
        for name, o in (("strict", ref["strict"]), ("fma", ref["fma"]), ("oracle", orc)):
            cr = o.corr(N, S)
            cr.set_pattern(pattern(N))
            runs[name] = run(cr, x, chunks)
        for name in ("fma", "oracle"):
            a, b = runs["strict"], runs[name]
            assert len(a) == len(b), name
            for sa, sb in zip(a, b):
                assert all(np.array_equal(sa[k], sb[k]) if k == "bits" else sa[k] == sb[k] for k in sa), name
        steps = runs["strict"]
        key = f"n{N}_s{S}"
        arrays[key + "_x"] = x
        for i, st in enumerate(steps):
            if st["found"]:
                arrays[f"{key}_bits{i}"] = st["bits"]
        detected = {st["pos"] + st["index"] for st in steps if st["found"]}
        for m in meta:
            m["detected"] = m["peak"] in detected
            # detections follow the reference's own verdict on the crafted registers
            assert m["detected"] == m["ref_hit"], m
        cases.append({"key": key, "N": N, "S": S, "chunks": chunks, "pattern_tap0": PEAK_TAP,
                      "steps": [{k: v for k, v in st.items() if k != "bits"} for st in steps],
                      "events": meta,
                      "band_peaks": int(sum(m["band"] for m in meta)),
                      "band_detected": int(sum(m["band"] and m["detected"] for m in meta)),
                      "band_rejected": int(sum(m["band"] and not m["detected"] for m in meta))})
        print(f"{key}: {len(x)} samples, {len(steps)} steps, {len(detected)} detections, "
              f"{cases[-1]['band_peaks']} band peaks ({cases[-1]['band_detected']} detected)")
    np.savez_compressed(os.path.join(HERE, "corr_ties.npz"), **arrays)
    with open(os.path.join(HERE, "corr_ties.json"), "w") as fh:
        json.dump({"generator": "tests/golden/gen_corr_ties.py",
                   "source": "oracle/_ref (reference headers, strict and fma builds, identical)",
                   "reference": "correlators.h:209-303", "cases": cases}, fh, indent=1)


if __name__ == "__main__":
    main()
