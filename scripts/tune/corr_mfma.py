#!/usr/bin/env python3
"""Config 5's correlator on the integer matrix cores (tuning probe, VERDICT r5
item 3; the kernel is scripts/tune/corr_mfma.hip and never ships).

1. Builds the config-5 buffer exactly as bench.py's corr workload (2^26
   complex<int16_t>, noise +-125 and the +-1000 pattern copy at 3/4) and the
   B tables of the limb formulation (corr_mfma.hip's header).
2. Runs the probe with every sample's (corr, energy) registers stored and
   compares ALL of them with the oracle (orc_corr_registers: the reference's
   corrValue[0] / energyValue[0] of correlators.h:244-250 for every sample,
   in parallel windows primed with their 1024-sample history), bit for bit.
3. Times the probe (stores suppressed) and the product's corr_scan_s1 on the
   same box with HIP events, and reports both per scanned sample against
   their peaks: the I8 MFMA rate (32x32x32 i8: 32 cycles per SIMD = 1024 MACs
   per clock per SIMD, 2.52e15 MAC/s at 2.4 GHz) and the v_dot2 rate the
   product is graded on (39.3e12 lane-ops/s).

--emulate N: no GPU; replays the kernel's lane fragments and table addresses
in numpy for the first N outputs (N a multiple of 1024) and checks them
against the oracle (validates the host tables and index algebra)."""
import argparse
import concurrent.futures as cf
import ctypes as C
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle  # noqa: E402
from srcdsp_amd.design import qpsk_pattern  # noqa: E402

NP = 1024
CHUNKS = 66
BENT, BSTRIDE = 1096, 2192  # corr_mfma.hip's B copy geometry (checked against the library at run time)
COPY_OFF = (0, 2360, 4728, 7096)  # copy sigma's base in a kind: {0, 56, 120, 184} mod 256 (bank-conflict free)
BKIND = COPY_OFF[3] + BSTRIDE
I8_PEAK = 1024 * 1024 * 2.4e9    # MACs/s: 1024 SIMDs x 1024 i8 MACs per clock (32x32x32 in 32 cycles)
DOT2_PEAK = 39.32e12             # v_dot2 lane-ops/s (bench.py VALU_PEAK_TOPS)


def config5_buffer(L):
    """bench.py CorrWorkload's buffer (same RNG calls)."""
    p = qpsk_pattern(1024, 500, seed=2)
    rng = np.random.default_rng(0)
    x = rng.integers(-125, 126, size=(L, 2)).astype(np.int32)
    off = (3 * L) // 4
    x[off:off + 1024] += 2 * p
    return p, np.clip(x, -32768, 32767).astype(np.int16)


def limbs(v):
    """v (int64 array) = 256 vh + vl, vl in [-128, 127]."""
    vl = ((v + 128) & 255) - 128
    vh = (v - vl) >> 8
    if vh.min() < -128 or vh.max() > 127:
        raise ValueError("coefficient outside the 2-limb range (|v| >= 32640)")
    return vl.astype(np.int8), vh.astype(np.int8)


def factor(p):
    """(scale, q) with p = scale * q and every q component in [-128, 127] (the
    gcd of the nonzero components), or None: config 5's +-500 QPSK pattern is
    500 * (+-1)."""
    a = np.abs(p.astype(np.int64)).reshape(-1)
    a = a[a > 0]
    g = int(np.gcd.reduce(a)) if len(a) else 1
    q = p.astype(np.int64) // g
    if q.min() < -128 or q.max() > 127:
        return None
    return g, q


def btables(p, pl=2):
    """The kernel's LDS B image, per kind 4 copies shifted by sigma; copy sigma
    entry e holds the coefficient pair of tap k = e - sigma - 32 (zero outside
    [0, 1023]); pair = (comp 0, comp 1) = re output: (c.re, -c.im) = (p.re,
    p.im); im output: (c.im, c.re) = (-p.im, p.re), with c = conj(p)
    (correlators.h:173-176).  pl = 2: kinds re lo, re hi, im lo, im hi of p;
    pl = 1: kinds re, im of q = p / scale (factor()).  Returns (image, bias,
    scale)."""
    scale = 1
    if pl == 1:
        scale, p = factor(p)
    p = p.astype(np.int64)
    pairs = {"re": np.stack([p[:, 0], p[:, 1]], 1), "im": np.stack([-p[:, 1], p[:, 0]], 1)}
    kinds = [("re", 0), ("re", 1), ("im", 0), ("im", 1)] if pl == 2 else [("re", None), ("im", None)]
    img = np.zeros(len(kinds) * BKIND, np.uint8)
    bias = {}
    for ki, (out, limb) in enumerate(kinds):
        if limb is None:
            v = pairs[out].astype(np.int8).view(np.uint8)
        else:
            lo, hi = limbs(pairs[out])
            v = (lo if limb == 0 else hi).view(np.uint8)  # (1024, 2)
        bias[out] = int((128 * pairs[out].sum()) % (1 << 32))
        for sig in range(4):
            base = ki * BKIND + COPY_OFF[sig]
            e = np.arange(BENT)
            k = e - sig - 32
            ok = (k >= 0) & (k < NP)
            a = np.zeros((BENT, 2), np.uint8)
            a[ok] = v[k[ok]]
            img[base:base + 2 * BENT] = a.reshape(-1)
    return img, bias, scale


def coeff_scaling(p):
    o = pyoracle.Oracle(0)
    c = o.corr(NP, 1)
    c.set_pattern(p)
    return c.status()["coeff_scaling"]


def oracle_registers(p, x, win=1 << 20, workers=16):
    n = len(x)
    corr = np.empty(n, np.uint32)
    en = np.empty(n, np.uint32)

    def job(s):
        o = pyoracle.Oracle(0)
        c = o.corr(NP, 1)
        c.set_pattern(p)
        if s:
            c.prime(x[max(0, s - NP - 2):s])
        a, b = c.registers(x[s:s + win])
        corr[s:s + len(a)] = a
        en[s:s + len(b)] = b

    with cf.ThreadPoolExecutor(max(1, min(workers, os.cpu_count() or 1))) as ex:
        list(ex.map(job, range(0, n, win)))
    return corr, en


def emulate(p, x, n_out, pl=2):
    """numpy replay of corr_mfma_i8<pl>'s fragments for outputs [0, n_out)."""
    img, bias, scale = btables(p, pl)
    cs = coeff_scaling(p)
    L = len(x)
    xs = np.zeros((n_out + NP, 2), np.int64)  # staged samples j = -1024 .. n_out - 1
    xs[NP:] = x[:n_out]
    xl = (xs & 255) - 128  # the low byte XOR 0x80, as a signed byte
    xh = (xs >> 8).astype(np.int64)
    assert np.array_equal(256 * xh + xl + 128, xs)
    kinds = img.view(np.int8).astype(np.int64)
    corr = np.empty(n_out, np.uint32)
    for iw in range(0, n_out, 1024):
        acc = {k: np.zeros((32, 32), np.int64) for k in ("s0r", "s1r", "s2r", "s0i", "s1i", "s2i")}
        for t in range(CHUNKS):
            A = {}
            for nm, plane in (("xl", xl), ("xh", xh)):
                a = np.zeros((32, 2, 16), np.int64)  # [row][h][byte]
                for h in range(2):
                    j = iw + 32 * np.arange(32)[:, None] + 16 * t + 8 * h + np.arange(8)[None, :]  # local (+1024)
                    a[:, h, :] = plane[j].reshape(32, 16)
                A[nm] = a
            B = {}
            names = ("rl", "rh", "il", "ih") if pl == 2 else ("rl", "il")
            for ki, nm in enumerate(names):
                b = np.zeros((32, 2, 16), np.int64)  # [col][h][byte]
                for col in range(32):
                    sig = (col + 1) & 3
                    for h in range(2):
                        addr = ki * BKIND + COPY_OFF[sig] + 2 * (8 * h - col + 31 + sig) + 32 * t
                        assert addr % 8 == 0
                        b[col, h] = kinds[addr:addr + 16]
                B[nm] = b

            def mm(a, b):
                return np.einsum("rhj,chj->rc", a, b)
            acc["s0r"] += mm(A["xl"], B["rl"]); acc["s0i"] += mm(A["xl"], B["il"])
            acc["s1r"] += mm(A["xh"], B["rl"]); acc["s1i"] += mm(A["xh"], B["il"])
            if pl == 2:
                acc["s1r"] += mm(A["xl"], B["rh"]); acc["s1i"] += mm(A["xl"], B["ih"])
                acc["s2r"] += mm(A["xh"], B["rh"]); acc["s2i"] += mm(A["xh"], B["ih"])
        m32 = (1 << 32) - 1
        cr = (scale * (acc["s0r"] + (acc["s1r"] << 8) + (acc["s2r"] << 16) + bias["re"])) & m32
        ci = (scale * (acc["s0i"] + (acc["s1i"] << 8) + (acc["s2i"] << 16) + bias["im"])) & m32
        tr = (cr.astype(np.uint32).view(np.int32).astype(np.int64) >> cs) >> 2
        ti = (ci.astype(np.uint32).view(np.int32).astype(np.int64) >> cs) >> 2
        c = (tr * tr + ti * ti) & m32
        corr[iw:iw + 1024] = c.reshape(-1).astype(np.uint32)  # row-major = i_w + 32 row + col
    return corr


def run_gpu(args, p, x):
    import torch
    lib = C.CDLL(os.path.join(HERE, args.lib))
    geo = (C.c_int * 8)()
    lib.tune_corr_mfma_geometry(geo)
    assert (geo[1], geo[2], geo[3], geo[4]) == (CHUNKS, BENT, BSTRIDE, BKIND), list(geo)
    lib.tune_corr_mfma.argtypes = [C.c_void_p, C.c_long, C.c_void_p, C.c_int, C.c_uint32, C.c_uint32, C.c_void_p,
                                   C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint32, C.c_void_p]
    cs = coeff_scaling(p)
    n = len(x)
    dx = torch.from_numpy(x).cuda()
    dc = torch.zeros(n, dtype=torch.int32, device="cuda")
    de = torch.zeros(n, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    variants = [int(v) for v in args.pattern_limbs.split(",")]
    if factor(p) is None:
        variants = [v for v in variants if v == 2]

    def timeit(fn, reps):
        for _ in range(args.warmup):
            fn()
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
        for a, b in ev:
            a.record(st)
            fn()
            b.record(st)
        torch.cuda.synchronize()
        return [a.elapsed_time(b) for a, b in ev]

    out = {"samples": n, "coeff_scaling": cs, "lib": args.lib, "tile": geo[0], "lds_2limb": geo[7]}
    want = None
    for pl in variants:
        if args.cold:
            break
        img, bias, scale = btables(p, pl)
        db = torch.from_numpy(img).cuda()

        def launch(store_all, grid=args.grid):
            rc = lib.tune_corr_mfma(C.c_void_p(dx.data_ptr()), n, C.c_void_p(db.data_ptr()), cs, bias["re"],
                                    bias["im"], C.c_void_p(dc.data_ptr()), C.c_void_p(de.data_ptr()), grid, store_all,
                                    pl, scale, C.c_void_p(st.cuda_stream))
            assert rc == 0, rc

        if args.only_probe:  # counter passes: the probe's launches alone
            for _ in range(args.reps):
                launch(0)
            torch.cuda.synchronize()
            continue
        v = {"pattern_limbs": pl, "scale": scale, "bias": bias}
        dc.zero_()
        de.zero_()
        launch(1)
        torch.cuda.synchronize()
        got_c = dc.cpu().numpy().view(np.uint32)
        got_e = de.cpu().numpy().view(np.uint32)
        if not args.no_check:
            t0 = time.time()
            if want is None:
                want = oracle_registers(p, x)
            v["oracle_s"] = round(time.time() - t0, 1)
            bc = np.nonzero(got_c != want[0])[0]
            be = np.nonzero(got_e != want[1])[0]
            v["corr_mismatches"] = int(len(bc))
            v["energy_mismatches"] = int(len(be))
            v["first_bad"] = [int(bc[0]) if len(bc) else None, int(be[0]) if len(be) else None]
            print(json.dumps({"check": v}), flush=True)
        ms = timeit(lambda: launch(0), args.reps)
        ms_store = timeit(lambda: launch(1), args.reps)
        t = float(np.mean(ms)) * 1e-3
        macs = (16896.0 if pl == 2 else 8448.0) * n  # 66 chunks x 8 (4) MFMAs x 32768 MACs per 1024 outputs
        v.update({"ms": round(float(np.mean(ms)), 4), "ms_min": round(float(np.min(ms)), 4),
                  "ms_with_stores": round(float(np.mean(ms_store)), 4), "gsamples_per_s": round(n / t / 1e9, 2),
                  "i8_macs_per_s": macs / t, "i8_peak_frac": round(macs / t / I8_PEAK, 4),
                  "useful_frac_of_macs": round(16384 / 16896, 4),
                  "bound_gsamples_per_s": round(I8_PEAK / (macs / n) / 1e9, 1)})
        out[f"probe_{pl}limb"] = v
    if args.only_probe:
        return
    if args.cold:
        # the driver's protocol: an idle pause, 5 untimed + 20 timed launches
        # (per-launch HIP events), probe (each variant) and product interleaved
        import srcdsp_amd as S
        g = S.FixedPatternCorrelator(NP, 1)
        g.setPattern(p)

        def prod_step():
            g.reset()
            g.step(dx)
        fns = {"product": prod_step}
        for pl in variants:
            img, bias, scale = btables(p, pl)
            dbv = torch.from_numpy(img).cuda()
            fns[f"probe_{pl}limb"] = (lambda dbv=dbv, bias=bias, scale=scale, pl=pl: lib.tune_corr_mfma(
                C.c_void_p(dx.data_ptr()), n, C.c_void_p(dbv.data_ptr()), cs, bias["re"], bias["im"],
                C.c_void_p(dc.data_ptr()), C.c_void_p(de.data_ptr()), args.grid, 0, pl, scale,
                C.c_void_p(st.cuda_stream)))
        cold = {}
        for rnd in range(3):
            for nm, fn in fns.items():
                torch.cuda.synchronize()
                time.sleep(args.idle)
                for _ in range(5):
                    fn()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
                for a, b in ev:
                    a.record(st)
                    fn()
                    b.record(st)
                torch.cuda.synchronize()
                cold.setdefault(nm, []).append(round(float(np.mean([a.elapsed_time(b) for a, b in ev])), 4))
        out["driver_protocol_ms"] = cold
        print(json.dumps(out), flush=True)
        return
    # the product on the same box: corr_scan_s1 through the Python mirror (stops at the detection)
    import srcdsp_amd as S
    g = S.FixedPatternCorrelator(NP, 1)
    g.setPattern(p)
    res = {}

    def prod():
        g.reset()
        res["r"] = g.step(dx)
    pms = timeit(prod, args.reps)
    found, idx = res["r"]
    scanned = idx + 2 if found else n
    tp = float(np.mean(pms)) * 1e-3
    out["product"] = {"ms": round(float(np.mean(pms)), 4), "detection": [bool(found), int(idx)],
                      "scanned_samples": int(scanned), "gsamples_per_s": round(scanned / tp / 1e9, 2),
                      "dot2_peak_frac": round(2048.0 * scanned / tp / DOT2_PEAK, 4)}
    for pl in variants:
        v = out[f"probe_{pl}limb"]
        v["speedup_per_sample_vs_product"] = round(v["gsamples_per_s"] / out["product"]["gsamples_per_s"], 2)
    out["bounds_gsamples_per_s"] = {"i8_mfma_2limb": round(I8_PEAK / 16896 / 1e9, 1),
                                    "i8_mfma_1limb": round(I8_PEAK / 8448 / 1e9, 1),
                                    "v_dot2": round(DOT2_PEAK / 2048 / 1e9, 1)}
    print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=1 << 26)
    ap.add_argument("--emulate", type=int, default=0)
    ap.add_argument("--grid", type=int, default=0, help="0: 256 x workgroups per CU")
    ap.add_argument("--lib", default="libcorrmfma.so", help="probe library (tuning builds of corr_mfma.hip)")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--no-check", action="store_true")
    ap.add_argument("--only-probe", action="store_true", help="launch the probe --reps times, nothing else")
    ap.add_argument("--cold", action="store_true",
                    help="the driver's protocol (after --idle s: 5 untimed + 20 timed launches), probe and product")
    ap.add_argument("--idle", type=float, default=8.0)
    ap.add_argument("--pattern-limbs", default="2,1",
                    help="variants: 2 (any pattern), 1 (pattern = gcd x int8, when it factors)")
    args = ap.parse_args()
    p, x = config5_buffer(args.samples)
    if args.emulate:
        n = args.emulate
        want, _ = oracle_registers(p, x[:n])
        nbad = 0
        for pl in (2, 1):
            got = emulate(p, x, n, pl)
            bad = np.nonzero(got != want)[0]
            nbad += len(bad)
            print(f"emulate ({pl}-limb pattern): {n} outputs, {len(bad)} differ from the oracle"
                  + (f" (first {bad[0]})" if len(bad) else ""))
        sys.exit(1 if nbad else 0)
    run_gpu(args, p, x)


if __name__ == "__main__":
    main()
