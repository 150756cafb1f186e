#!/usr/bin/env python3
"""Parity of the mixmfma tuning library (scripts/tune/mixdecim_mfma_step.h:
config 4's mixer -> decimator chain with its tap loop on the i8 matrix cores,
behind the product's srcdsp_mixdecim_step; never shipped) against the oracle's
Mixer and FilterDnsamplingFir stepped the same way, on the cases the tiling
adds to the product's own tests:

* a stream continued over calls of many lengths (4 samples up to several
  tiles, tails off the 8192-sample tile): the decimator's history and the
  mixer's phase across calls;
* tap counts 1 (no history), 31, 100, 127 (config 4), 128 (the most the
  three 64-sample chunks cover), with their own shifts (coeffScaling);
* mixer tables of 4096, 1024 and 64 entries, positive and negative frequency;
* taps past two int8 limbs (|c| >= 32640) and a 256-tap filter: not eligible,
  the product path serves them (the launch counter must not move);
* srcdsp_tune_mixdecim_mfma_launches() grows by exactly the eligible calls;
* the plain decimator (row a2, srcdsp_decim_step) through the same kernel
  without the mixer: the same streams at 1, 31, 127 and 128 taps
  (srcdsp_tune_decim_mfma_launches()).

  SRCDSP_HIP_LIB=scripts/tune/ab/libsrcdsp_hip_mixmfma.so python scripts/tune/mixdecim_mfma_lib.py"""
import ctypes as C
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)

import pyoracle  # noqa: E402

TYPES = ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")


def taps(n, amp, seed):
    from srcdsp_amd.design import hamming_sinc, q14
    if amp is None:
        return q14(hamming_sinc(n))
    return np.random.default_rng(seed).integers(-amp, amp + 1, n).astype(np.int32)


def run_case(S, torch, c, N, f, calls, seed, limbs_ok):
    o = pyoracle.Oracle(0)
    om, od = o.mixer(N), o.decim(1, 4, c)
    om.reset(f)
    m = S.Mixer(N)
    m.reset(f)
    d = S.FilterDnsamplingFir(c, 4, *TYPES)
    chain = S.MixerDecimatorChain(m, d)
    x = o.gen_ci16(seed, 0, 0, sum(calls), -32768, 32767)
    bad, eligible, pos = [], 0, 0
    for k, ln in enumerate(calls):
        xs = x[pos:pos + ln]
        pos += ln
        want = od.step(om.step(xs))
        y = torch.empty((ln // 4, 2), dtype=torch.int16, device="cuda")
        chain.step(torch.from_numpy(np.ascontiguousarray(xs)).cuda(), y)
        got = y.cpu().numpy()
        eligible += limbs_ok
        if not np.array_equal(got, want):
            i = int(np.nonzero((got != want).any(axis=1))[0][0])
            bad.append(f"call {k} (len {ln}): first differing output {i}: {got[i].tolist()} vs {want[i].tolist()}")
            break
    return bad, eligible


def run_plain(S, torch, c, calls, seed):
    """the plain decimator (row a2) stepped through calls, against the oracle's"""
    o = pyoracle.Oracle(0)
    od = o.decim(1, 4, c)
    d = S.FilterDnsamplingFir(c, 4, *TYPES)
    x = o.gen_ci16(seed, 0, 0, sum(calls), -32768, 32767)
    bad, pos = [], 0
    for k, ln in enumerate(calls):
        xs = x[pos:pos + ln]
        pos += ln
        want = od.step(xs)
        y = torch.empty((ln // 4, 2), dtype=torch.int16, device="cuda")
        d.step(torch.from_numpy(np.ascontiguousarray(xs)).cuda(), y)
        got = y.cpu().numpy()
        if not np.array_equal(got, want):
            i = int(np.nonzero((got != want).any(axis=1))[0][0])
            bad.append(f"call {k} (len {ln}): first differing output {i}")
            break
    return bad


def main():
    import torch
    import srcdsp_amd as S
    lib = S.lib()
    count = lib.srcdsp_tune_mixdecim_mfma_launches
    count.restype = C.c_long
    T = 8192
    calls = [T, 4, 12, 3 * T + 4, 1000, T - 4, 65536, 4 * T + 1020]
    cases = {
        "config4_127q14_N4096": (taps(127, None, 0), 4096, 0.1, calls, True),
        "128taps_N4096_negf": (taps(128, 20000, 1), 4096, -0.37, calls, True),
        "31taps_N1024": (taps(31, 9000, 2), 1024, 0.21, calls, True),
        "100taps_N64": (taps(100, 32000, 3), 64, 0.3, calls, True),
        "1tap_N4096": (np.array([16384], np.int32), 4096, 0.05, calls, True),
        "127taps_past_limbs": (np.concatenate([taps(126, 1000, 4), [40000]]).astype(np.int32), 4096, 0.1,
                               calls[:4], False),
    }
    res, ok = {"cases": {}}, True
    for name, (c, N, f, cl, elig) in cases.items():
        before = count()
        bad, eligible = run_case(S, torch, c, N, f, cl, 7 + len(res["cases"]), elig)
        launched = count() - before
        res["cases"][name] = {"mismatches": bad, "calls": len(cl), "eligible_calls": eligible, "mfma_calls": launched}
        ok &= not bad and launched == eligible
        print(name, json.dumps(res["cases"][name]), flush=True)
    # a 256-tap filter is past the three 64-sample chunks: the product's path
    before = count()
    bad, _ = run_case(S, torch, taps(256, 3000, 5), 4096, 0.1, calls[:3], 30, False)
    res["cases"]["256taps_product_path"] = {"mismatches": bad, "mfma_calls": count() - before}
    ok &= not bad and count() == before
    # the plain decimator (row a2: srcdsp_decim_step without a mixer) through the same kernel
    pcount = lib.srcdsp_tune_decim_mfma_launches
    pcount.restype = C.c_long
    for name, c in (("plain_127q14", taps(127, None, 0)), ("plain_128taps", taps(128, 20000, 1)),
                    ("plain_31taps", taps(31, 9000, 2)), ("plain_1tap", np.array([16384], np.int32))):
        before = pcount()
        bad = run_plain(S, torch, c, calls, 40 + len(res["cases"]))
        launched = pcount() - before
        res["cases"][name] = {"mismatches": bad, "calls": len(calls), "mfma_calls": launched}
        ok &= not bad and launched == len(calls)
        print(name, json.dumps(res["cases"][name]), flush=True)
    res["ok"] = bool(ok)
    print(json.dumps({"ok": res["ok"]}))
    out = os.path.join(ROOT, "gpurun_out", "mixdecim_mfma_lib.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
