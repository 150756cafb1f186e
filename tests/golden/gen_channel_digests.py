#!/usr/bin/env python3
"""Digests of the decimated synthetic channels (SURVEY §8e:
1/2/4/8 GPUs must give outputs bit-identical to one GPU).

For every channel ch = 0..63 of bench.py's synthetic workload (splitmix64
complex<float> samples, seed 0x5EED, channel ch), the 127-tap
Hamming-sinc FilterDnsamplingFir<cf32,cf32,cf32,float,4> over the whole
channel from a fresh object (dnsampling_filters.h:84-172), one step():
sha256 of the output bytes (2^26 complex<float> at 2^28 samples), for both
float contracts (fma: the sequential fmaf chain = the reference built -mfma;
strict: mul then add = the reference's -O2 x86-64 build).  Sizes: 2^28
(configs[1]/[2]) and 2^20 (the CPU rehearsal of bench.py's N > 1 path).

The outputs come from the oracle's C restatement (oracle/liboracle.so) in
parallel windows (tests/fullsize.py, each window started 128 samples early
with an empty history: the single call's outputs).  Where the reference
build is present (oracle/_ref, this container), channels 0 and 63 at both
sizes are recomputed through the REAL reference templates (the same windows)
and must give the same digests.  bench.py checks its ranks' outputs against
this table after the timed region.

Run: python tests/golden/gen_channel_digests.py   (~10 min on 8 cores)"""
import hashlib
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import fullsize as F  # noqa: E402
import pyoracle  # noqa: E402
from srcdsp_amd.design import hamming_sinc  # noqa: E402

SEED = 0x5EED
CHANNELS = 64
SIZES = (1 << 20, 1 << 28)
OUT = os.path.join(HERE, "channel_digests.json")


def digest(make, x, out):
    F.decim_all(make, x, 4, 128, out)
    return hashlib.sha256(out.tobytes()).hexdigest()


def main():
    c = hamming_sinc(127)
    ora = {"strict": pyoracle.Oracle(0), "fma": pyoracle.Oracle(1)}
    ref = {fl: pyoracle.Reference(fl) for fl in ("strict", "fma") if pyoracle.reference_available(fl)}
    table = {"workload": "decim_cf32_m4_t127", "seed": SEED, "taps": "srcdsp_amd.design.hamming_sinc(127)",
             "generator": "splitmix64 cf32 in [-2048, 2047] (oracle gen_cf32 = srcdsp fill_synthetic)",
             "hash": "sha256 of the complex<float> output bytes of one fresh step() over the whole channel",
             "source": "oracle/liboracle.so (C restatement); channels 0 and 63 re-derived from the reference "
                       "build" + (" (present)" if ref else " (absent when generated)"),
             "digests": {fp: {str(n): {} for n in SIZES} for fp in ora}}
    ref_checked = []
    for n in SIZES:
        out = np.empty(n // 4, np.complex64)
        for ch in range(CHANNELS):
            t0 = time.time()
            x = ora["fma"].gen_cf32(SEED, ch, 0, n)
            for fp, o in ora.items():
                table["digests"][fp][str(n)][str(ch)] = digest(lambda: o.decim(0, 4, c), x, out)
                if fp in ref and ch in (0, CHANNELS - 1):
                    h = digest(lambda: ref[fp].decim(0, 4, c), x, out)
                    assert h == table["digests"][fp][str(n)][str(ch)], (fp, n, ch)
                    ref_checked.append(f"{fp}/{n}/{ch}")
            del x
            print(f"n={n} ch={ch} {time.time() - t0:.1f}s", flush=True)
    table["reference_checked"] = ref_checked
    with open(OUT, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print("wrote", OUT)


if __name__ == "__main__":
    main()
