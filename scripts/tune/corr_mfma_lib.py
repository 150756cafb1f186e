#!/usr/bin/env python3
"""Parity of the corrmfma tuning library (scripts/tune/corr_mfma_scan.h behind
the product's C ABI; never shipped) against the oracle, on the cases its
tiling adds to the product's own tests:

* detections on the tile seams (the peak at tile outputs 0 and 1, which
  corr_mfma_seams tests, and at 2, the first one the tile tests itself), also
  on the seam of a continued call (outputs 0 / 1 of a call take the registers
  of the one before);
* a stream continued over many calls (the history words before each call);
* both pattern-limb forms: config 5's +-500 QPSK (= 500 x int8, one limb) and
  a full int16-range pattern (two limbs);
* every call counted: srcdsp_tune_corr_mfma_launches() must grow by the calls
  that qualify (N = 1024, S = 1, length % 4 == 0, 16-B aligned input).

  SRCDSP_HIP_LIB=scripts/tune/ab/libsrcdsp_hip_corrmfma.so python scripts/tune/corr_mfma_lib.py"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import pyoracle  # noqa: E402

TILE = 8192


def stream(p, n, outs, amp, seed):
    """noise +-125 with amp x pattern copies whose peak (the copy's last
    sample) is tested at output e of `outs` (the 3-point test fires one
    sample after the peak: corrIndex = e - 1)"""
    rng = np.random.default_rng(seed)
    x = rng.integers(-125, 126, size=(n, 2)).astype(np.int64)
    for e in outs:
        x[e - 1024:e] += amp * p
    return np.clip(x, -32768, 32767).astype(np.int16)


def run(S, torch, p, x, calls):
    """step the library and the oracle through x in calls of the given
    lengths (stepping on after every detection); returns mismatch notes and
    how many library calls were eligible"""
    g, r = S.FixedPatternCorrelator(1024, 1), pyoracle.Oracle(1).corr(1024, 1)
    g.setPattern(p)
    r.set_pattern(p)
    bad, eligible, pos, k, hits = [], 0, 0, 0, []
    while pos < len(x) and len(bad) < 5:
        ln = calls[k % len(calls)]
        k += 1
        xs = x[pos:pos + ln]
        eligible += len(xs) % 4 == 0
        fg, ig = g.step(torch.from_numpy(np.ascontiguousarray(xs)).cuda())
        fr, ir = r.step(xs)
        if (fg, fg and ig) != (fr, fr and ir):
            bad.append(f"call at {pos}: gpu {fg, ig} oracle {fr, ir}")
            break
        if not np.array_equal(g.getRefBitSamples(), r.bit_samples()):
            bad.append(f"bitSamples after call at {pos}")
        st, sr = g.getStatus(), r.status()
        if any(st[q] != sr[q] for q in ("energy", "corr")):
            bad.append(f"registers after call at {pos}: {st['corr']} {sr['corr']}")
        if fr:
            hits.append(pos + ir + 1)  # the output the test fired at
        pos += (ir + 2) if fr else len(xs)
    return bad, eligible, hits


def main():
    import torch
    import srcdsp_amd as S
    from srcdsp_amd.design import qpsk_pattern
    lib = S.lib()
    count = lib.srcdsp_tune_corr_mfma_launches
    count.restype = __import__("ctypes").c_long
    rng = np.random.default_rng(5)
    pats = {"qpsk500_1limb": qpsk_pattern(1024, 500, seed=2),
            "rand_2limb": rng.integers(-1000, 1000, size=(1024, 2)).astype(np.int64)}  # energy ~6.8e8: under
    # setPattern's assert (correlators.h:185), components past one limb, gcd 1
    res = {"cases": {}}
    ok = True
    for pn, p in pats.items():
        amp = 2 if pn.startswith("qpsk") else 1
        noise_seed = 11 if pn.startswith("qpsk") else 12
        cases = {
            # detections on tile seams of one call: outputs 0, 1, 2 of 8192-output tiles (one
            # row block per wave) and of 16384-output tiles (two: 4 TILE, 6 TILE + 1, 8 TILE + 2)
            "seams_one_call": (stream(p, 10 * TILE, [TILE, 2 * TILE + 1, 3 * TILE + 2, 4 * TILE, 5 * TILE + 1,
                                                     6 * TILE + 1, 8 * TILE + 2], amp, noise_seed),
                               [10 * TILE]),
            # peaks at outputs 0 and 1 of a continued call (the seam on the registers of the call before)
            "seam_call_start": (stream(p, 8 * TILE, [3 * TILE, 5 * TILE + 1], amp, noise_seed + 1),
                                [3 * TILE, 2 * TILE, 3 * TILE]),
            # a stream over many short calls (history words before each call), unaligned lengths mixed in
            "many_calls": (stream(p, 1 << 18, [40000, 90001, 150002, 200003], amp, noise_seed + 2),
                           [20000, 4096, 12, 16384, 30001, 8192]),
        }
        for cn, (x, calls) in cases.items():
            before = count()
            bad, eligible, hits = run(S, torch, p, x, calls)
            launched = count() - before
            key = f"{pn}/{cn}"
            res["cases"][key] = {"mismatches": bad, "hits": hits, "eligible_calls": eligible, "mfma_calls": launched}
            ok &= not bad and launched == eligible and len(hits) > 0
            print(key, json.dumps(res["cases"][key]), flush=True)
    res["ok"] = bool(ok)
    print(json.dumps({"ok": res["ok"]}))
    out = os.path.join(ROOT, "gpurun_out", "corr_mfma_lib.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
