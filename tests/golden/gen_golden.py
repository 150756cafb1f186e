#!/usr/bin/env python3
"""Generate the golden fixtures from the REAL reference (oracle/_ref).

Run in the build container (needs /root/reference, compiled by
``make -C oracle``):  ``python tests/golden/gen_golden.py``.
Writes ``tests/golden/golden.npz`` (inputs + reference outputs, both float
flavours) and ``tests/golden/manifest.json`` (the operation scripts).

Each case is a script of operations replayed identically by the tests against
the C oracle and, on the GPU box, against the HIP path:
  ["step", in_key, {"strict": out_key, "fma": out_key}]      decim / fir / mixer
  ["step_up", in_key, flush, iterator, {...}]                 upsampler
  ["corr_step", in_key, found, index, bits_key, status]       correlator
  ["reset"], ["set_left_shift", v], ["set_coeffs", key],
  ["mixer_reset", f], ["mixer_set_frequency", f], ["mixer_adjust", f]
Integer cases store one output (flavour independent, asserted here).
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)

import pyoracle as P  # noqa: E402
from srcdsp_amd.design import hamming_sinc, q14, qpsk_pattern  # noqa: E402

ARR: dict[str, np.ndarray] = {}
CASES: list[dict] = []
REF = {"strict": P.Reference("strict"), "fma": P.Reference("fma")}
RNG = np.random.default_rng(0x5EED)


def put(name: str, a: np.ndarray) -> str:
    assert name not in ARR, name
    ARR[name] = np.ascontiguousarray(a)
    return name


def cf32(n, lo=-2048, hi=2047, integer=True):
    if integer:
        v = RNG.integers(lo, hi + 1, size=(n, 2)).astype(np.float32)
    else:
        v = RNG.uniform(lo, hi, size=(n, 2)).astype(np.float32)
    return v.view(np.complex64).reshape(n)


def ci(n, lo, hi, dtype=np.int16):
    return RNG.integers(lo, hi + 1, size=(n, 2)).astype(dtype)


def same(a, b):
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a).view(np.uint8),
                                                 np.ascontiguousarray(b).view(np.uint8))


# ------------------------------------------------------------------ decimator
def decim_case(name, variant, M, coeffs, chunks, header="old", ops_between=None, integer=None):
    """Run the same script on both reference flavours and record."""
    kin, kout, kc = P.DECIM_VARIANTS[variant]
    coeffs = P.coeff_array(coeffs, kc)
    objs = {f: REF[f].decim(variant, M, coeffs, header) for f in REF}
    script = []
    ops_between = ops_between or {}
    for i, x in enumerate(chunks):
        for op in ops_between.get(i, []):
            script.append(op)
            for o in objs.values():
                if op[0] == "reset":
                    o.reset()
                elif op[0] == "set_left_shift":
                    o.set_left_shift(op[1])
                elif op[0] == "set_coeffs":
                    o.set_coeffs(ARR[op[1]])
        ik = put(f"{name}__in{i}", P.as_kind(x, kin))
        outs = {f: objs[f].step(ARR[ik]) for f in objs}
        if variant != 0:
            assert same(outs["strict"], outs["fma"]), name
        if same(outs["strict"], outs["fma"]):
            k = put(f"{name}__out{i}", outs["strict"])
            script.append(["step", ik, {"strict": k, "fma": k}])
        else:
            ks = put(f"{name}__out{i}_strict", outs["strict"])
            kf = put(f"{name}__out{i}_fma", outs["fma"])
            script.append(["step", ik, {"strict": ks, "fma": kf}])
    CASES.append({"name": name, "op": "decim", "variant": variant, "M": M, "header": header,
                  "abs_mode": 1 if header == "fabs" else 0,
                  "coeffs": put(f"{name}__coeffs", coeffs), "script": script})


def gen_decim():
    h127 = hamming_sinc(127)
    h128 = np.concatenate([h127, [0.0]]).astype(np.float32)
    # headline shape (config 2), chained calls with history carry-over
    decim_case("decim_cf32_m4_h127", 0, 4, h127, [cf32(4096), cf32(1024), cf32(6144), cf32(128)])
    # the current header's 128-tap twin (trailing 0 tap), N % M == 0
    decim_case("decim_cf32_m4_h128_new", 0, 4, h128, [cf32(4096), cf32(2048)], header="new")
    # non-integer inputs, wide range -> saturation at +-32767 and float rounding
    decim_case("decim_cf32_m4_wide", 0, 4, h127, [cf32(8192, -60000, 60000, integer=False)])
    # quantiser edges: NaN/inf/out-of-int32 range -> INT_MIN -> 0; exact boundaries
    special = np.array([3e9, -3e9, -2147483648.0, 2147483520.0, np.nan, np.inf, -np.inf, 40000,
                        -40000, 32767.9, -32768.5, 1e-40, 32767.0, -32767.0, 32768.0, -32768.0],
                       np.float32)
    x = np.zeros(64, np.complex64)
    x.real[:16] = special
    x.imag[:16] = -special[::-1]
    decim_case("decim_cf32_m1_edge", 0, 1, np.array([1.0], np.float32), [x])
    decim_case("decim_cf32_m4_edge", 0, 4, np.array([1.0, 0.5, -0.25, 2.0], np.float32),
               [np.concatenate([x, cf32(192)])])
    # abs() binding: 127 taps of 0.9 (int binding: shift (INT_MIN)&31 = 0; fabs: 6)
    c09 = np.full(127, 0.9, np.float32)
    ones = np.full(1024, 100 + 0j, np.complex64)
    decim_case("decim_cf32_abs_int", 0, 4, c09, [ones, cf32(1024, -200, 200)])
    decim_case("decim_cf32_abs_fabs", 0, 4, c09, [ones, cf32(1024, -200, 200)], header="fabs")
    cbig = (hamming_sinc(64) * 37.0).astype(np.float32)   # sum|c| > 2 under both bindings
    decim_case("decim_cf32_bigc_int", 0, 4, cbig, [cf32(2048, -300, 300)])
    decim_case("decim_cf32_bigc_fabs", 0, 4, cbig, [cf32(2048, -300, 300)], header="fabs")
    # setLeftShiftBy2 and reset mid-stream
    decim_case("decim_cf32_leftshift", 0, 4, cbig, [cf32(1024, -300, 300)] * 1 + [cf32(1024, -300, 300),
               cf32(1024, -300, 300), cf32(1024, -300, 300)],
               ops_between={1: [["set_left_shift", 2]], 2: [["set_left_shift", -1]],
                            3: [["reset"], ["set_left_shift", 0]]})
    # other decimation ratios / tap counts
    decim_case("decim_cf32_m2_t31", 0, 2, hamming_sinc(31, 0.25), [cf32(2048), cf32(512)])
    decim_case("decim_cf32_m8_t63", 0, 8, hamming_sinc(63, 0.06), [cf32(4096), cf32(1024)])
    decim_case("decim_cf32_m3_t7", 0, 3, hamming_sinc(7, 0.15), [cf32(999), cf32(300)])
    decim_case("decim_cf32_m4_t1", 0, 4, np.array([0.75], np.float32), [cf32(400)])
    # fixed point, config-4 shape: ci16 x Q14 int32 coefficients
    cq = q14(h127)
    decim_case("decim_ci16_i32_m4_q14", 1, 4, cq, [ci(4096, -8192, 8191), ci(2048, -8192, 8191),
                                                   ci(1024, -8192, 8191)])
    decim_case("decim_ci16_i32_m4_sat", 1, 4, cq * 3, [ci(4096, -32768, 32767)])
    # wrapping int32 accumulation (huge coefficients)
    cw = RNG.integers(-2**30, 2**30, size=33).astype(np.int32)
    decim_case("decim_ci16_i32_m4_wrap", 1, 4, cw, [ci(1024, -32768, 32767)])
    # int16 coefficients: each product wraps to int16 (300*200 -> -5536)
    c16 = RNG.integers(-400, 400, size=32).astype(np.int16)
    decim_case("decim_ci16_i16_m4_wrap", 2, 4, c16, [ci(2048, -300, 300), ci(512, -32768, 32767)])
    decim_case("decim_ci32_i32_m4", 3, 4, cq, [ci(2048, -100000, 100000, np.int32),
                                               ci(1024, -2**31, 2**31 - 1, np.int32)])
    decim_case("decim_ci16_i32_m2_t31", 1, 2, q14(hamming_sinc(31, 0.25)), [ci(1024, -8192, 8191),
                                                                           ci(256, -8192, 8191)])
    decim_case("decim_ci16_i32_m8_t64", 1, 8, q14(hamming_sinc(64, 0.06)), [ci(2048, -8192, 8191)],
               header="new")


# ------------------------------------------------------------------ FilterFir
def fir_case(name, variant, coeffs, chunks, ops_between=None):
    kin, kout, kc = P.FIR_VARIANTS[variant]
    coeffs = P.coeff_array(coeffs, kc)
    objs = {f: REF[f].fir(variant, coeffs) for f in REF}
    script = []
    ops_between = ops_between or {}
    for i, x in enumerate(chunks):
        for op in ops_between.get(i, []):
            script.append(op)
            for o in objs.values():
                if op[0] == "reset":
                    o.reset()
                elif op[0] == "set_coeffs":
                    o.set_coeffs(ARR[op[1]])
        ik = put(f"{name}__in{i}", P.as_kind(x, kin))
        outs = {f: objs[f].step(ARR[ik]) for f in objs}
        if same(outs["strict"], outs["fma"]):
            k = put(f"{name}__out{i}", outs["strict"])
            script.append(["step", ik, {"strict": k, "fma": k}])
        else:
            ks = put(f"{name}__out{i}_strict", outs["strict"])
            kf = put(f"{name}__out{i}_fma", outs["fma"])
            script.append(["step", ik, {"strict": ks, "fma": kf}])
    CASES.append({"name": name, "op": "fir", "variant": variant, "abs_mode": 0,
                  "coeffs": put(f"{name}__coeffs", coeffs), "script": script})


def gen_fir():
    h31 = hamming_sinc(31, 0.2)
    # config 1: FilterFir<float, complex<float>, float, float>, 31 taps
    fir_case("fir_f32_t31", 1, h31, [RNG.integers(-2048, 2048, 4096).astype(np.float32),
                                     RNG.uniform(-40000, 40000, 2048).astype(np.float32)])
    fir_case("fir_cf32_t31", 0, h31, [cf32(4096), cf32(100), cf32(3000, -50000, 50000, False)])
    put("fir_cf32_reset__c2", (h31 * 3.0).astype(np.float32))
    fir_case("fir_cf32_reset", 0, h31, [cf32(512), cf32(512), cf32(512)],
             ops_between={1: [["reset"]], 2: [["set_coeffs", "fir_cf32_reset__c2"]]})
    fir_case("fir_ci16_i32_t31", 2, q14(h31), [ci(4096, -8192, 8191), ci(1024, -32768, 32767)])
    fir_case("fir_ci16_i32_t1", 2, np.array([16384], np.int32), [ci(300, -32768, 32767)])


# ------------------------------------------------------------------ upsampler
def up_case(name, variant, L, coeffs, calls):
    kin, kout, kc = P.UP_VARIANTS[variant]
    coeffs = P.coeff_array(coeffs, kc)
    objs = {f: REF[f].up(variant, L, coeffs) for f in REF}
    script = []
    for i, (x, flush, it) in enumerate(calls):
        if x is None:
            script.append(["reset"])
            for o in objs.values():
                o.reset()
            continue
        ik = put(f"{name}__in{i}", P.as_kind(x, kin))
        outs = {f: objs[f].step(ARR[ik], flush, it) for f in objs}
        assert same(outs["strict"], outs["fma"])
        k = put(f"{name}__out{i}", outs["strict"])
        script.append(["step_up", ik, bool(flush), bool(it), {"strict": k, "fma": k}])
    o = objs["strict"]
    CASES.append({"name": name, "op": "up", "variant": variant, "L": L,
                  "length": o.length, "imp_length": o.imp_length,
                  "coeffs": put(f"{name}__coeffs", coeffs), "script": script})


def gen_up():
    c32 = q14(hamming_sinc(32, 0.12) * 4)
    up_case("up_ci16_i32_l4", 0, 4, c32, [(ci(1024, -8192, 8191), False, False),
                                          (ci(512, -8192, 8191), False, False),
                                          (ci(256, -8192, 8191), True, False)])
    up_case("up_ci16_i32_l4_iter", 0, 4, c32 // 8, [(ci(512, -4000, 4000), False, True),
                                                   (ci(256, -4000, 4000), True, True)])
    up_case("up_ci16_i32_l4_sat", 0, 4, c32 * 4, [(ci(1024, -32768, 32767), False, False)])
    c16 = RNG.integers(-300, 300, size=24).astype(np.int16)
    up_case("up_ci16_i16_l4_wrap", 1, 4, c16, [(ci(512, -300, 300), False, False),
                                               (ci(256, -32768, 32767), True, False)])
    ct = np.concatenate([q14(hamming_sinc(13, 0.2)), np.zeros(3, np.int32)])  # 16 taps, 3 trailing 0
    up_case("up_i16_i32_l2_trail", 2, 2, ct,
            [(RNG.integers(-20000, 20000, 700).astype(np.int16), False, False),
             (None, False, False),
             (RNG.integers(-20000, 20000, 300).astype(np.int16), True, False)])
    up_case("up_ci16_i32_l3", 0, 3, q14(hamming_sinc(27, 0.15) * 3), [(ci(600, -8192, 8191), False, False),
                                                                      (ci(90, -8192, 8191), True, False)])
    up_case("up_ci16_i32_l8", 0, 8, q14(hamming_sinc(64, 0.06) * 8), [(ci(500, -8192, 8191), True, False)])


# ------------------------------------------------------------------ mixer
def mixer_case(name, N, script_in):
    objs = {f: REF[f].mixer(N) for f in REF}
    tab = objs["strict"].table()
    assert same(tab, objs["fma"].table())
    script = []
    for i, op in enumerate(script_in):
        if op[0] == "step":
            ik = put(f"{name}__in{i}", P.as_kind(op[1], "ci16"))
            outs = {f: objs[f].step(ARR[ik]) for f in objs}
            assert same(outs["strict"], outs["fma"])
            k = put(f"{name}__out{i}", outs["strict"])
            st = objs["strict"].state()
            script.append(["step", ik, {"strict": k, "fma": k}, list(st)])
        else:
            for o in objs.values():
                {"mixer_reset": o.reset, "mixer_set_frequency": o.set_frequency,
                 "mixer_adjust": o.adjust_frequency}[op[0]](op[1])
            st = objs["strict"].state()
            assert st == objs["fma"].state()
            script.append([op[0], float(op[1]), list(st)])
    CASES.append({"name": name, "op": "mixer", "N": N, "table": put(f"{name}__table", tab),
                  "script": script})


def gen_mixer():
    mixer_case("mixer_4096_f01", 4096, [["mixer_reset", 0.1], ["step", ci(4096, -8192, 8191)],
                                        ["step", ci(1000, -32768, 32767)], ["step", ci(3, -8192, 8191)]])
    mixer_case("mixer_4096_neg", 4096, [["mixer_reset", -0.3], ["step", ci(2048, -8192, 8191)],
                                        ["mixer_set_frequency", -1e-5], ["step", ci(512, -8192, 8191)],
                                        ["mixer_set_frequency", -1.0], ["step", ci(512, -8192, 8191)],
                                        ["mixer_set_frequency", 1.0], ["step", ci(512, -8192, 8191)]])
    mixer_case("mixer_4096_adjust", 4096, [["mixer_reset", 0.9], ["step", ci(777, -8192, 8191)],
                                           ["mixer_adjust", 0.25], ["step", ci(777, -8192, 8191)],
                                           ["mixer_adjust", -1.5], ["step", ci(777, -8192, 8191)],
                                           ["mixer_adjust", 0.3333], ["step", ci(777, -8192, 8191)]])
    mixer_case("mixer_1024_f037", 1024, [["mixer_reset", 0.37], ["step", ci(3000, -32768, 32767)]])
    mixer_case("mixer_256_fneg", 256, [["mixer_reset", -0.61], ["step", ci(1500, -8192, 8191)]])
    mixer_case("mixer_4096_nofreq", 4096, [["step", ci(64, -8192, 8191)]])  # ctor state: phi=freq=0


# ------------------------------------------------------------------ correlator
def corr_input(n, pattern, offsets, noise=125, amp_scale=2, S=1):
    x = RNG.integers(-noise, noise + 1, size=(n, 2)).astype(np.int32)
    for off in offsets:
        for m in range(len(pattern)):
            i = off + m * S
            if i < n:
                x[i] += pattern[m] * amp_scale
    return np.clip(x, -32768, 32767).astype(np.int16)


def corr_case(name, N, S, pattern, thr, calls):
    objs = {f: REF[f].corr(N, S) for f in REF}
    for o in objs.values():
        o.set_pattern(pattern, thr)
    script = []
    for i, x in enumerate(calls):
        if x is None:
            script.append(["reset"])
            for o in objs.values():
                o.reset()
            continue
        ik = put(f"{name}__in{i}", P.as_kind(x, "ci16"))
        res = {f: objs[f].step(ARR[ik]) for f in objs}
        assert res["strict"] == res["fma"]
        found, idx = res["strict"]
        bits = objs["strict"].bit_samples()
        st = objs["strict"].status()
        assert same(bits, objs["fma"].bit_samples()) and st == objs["fma"].status()
        bk = put(f"{name}__bits{i}", bits)
        script.append(["corr_step", ik, bool(found), int(idx) if found else -1, bk, st])
    CASES.append({"name": name, "op": "corr", "N": N, "S": S, "threshold": thr,
                  "pattern": put(f"{name}__pattern", pattern), "script": script})


def gen_corr():
    p32 = qpsk_pattern(32, 500, seed=1)
    # N=32, S=4: pattern at stride 4 embedded, detection, then keep stepping
    x = corr_input(6000, p32, [3000], S=4)
    corr_case("corr_32x4_detect", 32, 4, p32, 0.8, [x[:2000], x[2000:], corr_input(3000, p32, [1000], S=4)])
    p1k = qpsk_pattern(1024, 500, seed=2)
    x = corr_input(65536, p1k, [49152])
    corr_case("corr_1024x1_detect", 1024, 1, p1k, 0.8, [x[:20000], x[20000:], x[:4096]])
    corr_case("corr_1024x1_noise", 1024, 1, p1k, 0.8, [corr_input(8192, p1k, []), corr_input(4096, p1k, [])])
    p16 = qpsk_pattern(16, 2000, seed=3)
    # detection whose peak straddles the call boundary, and reset
    x = corr_input(4000, p16, [1000, 2600], noise=60, amp_scale=4)
    corr_case("corr_16x1_boundary", 16, 1, p16, 0.8,
              [x[:1016], x[1016:1017], x[1017:2000], None, x[2000:]])
    p64 = qpsk_pattern(64, 700, seed=4)
    corr_case("corr_64x2", 64, 2, p64, 0.8, [corr_input(5000, p64, [700, 4000], S=2)])
    # energy wrap (full-scale input) and an all-zero pattern (coeffScaling INT_MIN)
    big = RNG.integers(-32768, 32768, size=(3000, 2)).astype(np.int16)
    corr_case("corr_16x1_fullscale", 16, 1, p16, 0.8, [big])
    corr_case("corr_16x1_zero_pattern", 16, 1, np.zeros((16, 2), np.int32), 0.8, [big[:500]])
    p128 = qpsk_pattern(128, 1000, seed=5)
    corr_case("corr_128x1_two", 128, 1, p128, 0.8,
              [corr_input(9000, p128, [1000, 5000]), corr_input(2000, p128, [])])


def main():
    gen_decim()
    gen_fir()
    gen_up()
    gen_mixer()
    gen_corr()
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **ARR)
    meta = {"generator": "tests/golden/gen_golden.py",
            "reference": "dogjin/SrcDsp headers compiled by oracle/refbuild (g++ -O2 strict, -O2 -mfma)",
            "abs_binding": "::abs(int) (canonical include order), except cases with header 'fabs'",
            "cases": CASES}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(meta, f, indent=1)
    total = sum(a.nbytes for a in ARR.values())
    print(f"{len(CASES)} cases, {len(ARR)} arrays, {total/1e6:.2f} MB raw, "
          f"{os.path.getsize(os.path.join(HERE, 'golden.npz'))/1e6:.2f} MB on disk")


if __name__ == "__main__":
    main()
