"""Kernel time of the complex<int16_t> x int16-tap decimator across tap counts
and decimation factors, alone and with the mixer fused ahead of it (config
4's chain): the M = 4 tap counts compiled into decim_dot2_ci16
(63/64/127/128/255/256; the mixer at 127/128) next to any other count and
M = 2 / 8 / 16, which take decim_dot2_ci16<0, ...> with the tap count at run
time.

  python scripts/ci16_envelope.py [N ...]      (CI16_M="2 4 8 16": the decimation factors, default 4)

SRCDSP_HIP_LIB selects another build of the library (same-box A/B).  2^26
device-resident samples per shape, 20 warm-up launches, then the median of 50
timed launches.  One line per shape and chain: ms, Gsamples/s and the v_dot2
rate (N/M dot2 lane-ops per input sample at decimation M for the filter, +2
for the mixer) against the 39.3 T/s VALU peak."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import srcdsp_amd as S  # noqa: E402
from srcdsp_amd.design import hamming_sinc, q14  # noqa: E402

COMPILED = {"decim": (63, 64, 127, 128, 255, 256), "mixdecim": (127, 128)}
TAPS = (31, 63, 65, 100, 127, 129, 200, 255, 300, 511, 1024)
PEAK = 39.32


def main():
    taps = [int(a) for a in sys.argv[1:]] or list(TAPS)
    L = 1 << 26
    x = torch.empty((L, 2), dtype=torch.int16, device="cuda")
    S.fill_synthetic(x, "ci16", seed=0x5EED, channel=0, lo=-8192, hi=8191)
    lib = os.environ.get("SRCDSP_HIP_LIB", "tree")
    for M in [int(m) for m in os.environ.get("CI16_M", "4").split()]:
        envelope(M, taps, x, lib)


def envelope(M, taps, x, lib):
    L = x.shape[0] - x.shape[0] % M
    xm = x[:L]
    y = torch.empty((L // M, 2), dtype=torch.int16, device="cuda")
    for N in taps:
        cq = q14(hamming_sinc(N)) if N > 1 else np.array([16384], np.int32)
        for chain in ("decim", "mixdecim"):
            d = S.FilterDnsamplingFir(cq, M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
            if chain == "mixdecim":
                m = S.Mixer(4096)
                m.reset(0.1)
                op = S.MixerDecimatorChain(m, d)
            else:
                op = d
            for _ in range(20):
                op.step(xm, y)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
            for a, b in ev:
                a.record()
                op.step(xm, y)
                b.record()
            torch.cuda.synchronize()
            ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
            dps = N / M + (2 if chain == "mixdecim" else 0)
            kind = "compiled" if M == 4 and N in COMPILED[chain] else "runtime "
            print(f"{chain:8s} M={M:2d} N={N:4d} {kind}: {ms:.4f} ms {L / ms / 1e6:8.1f} Gsamp/s "
                  f"{dps * L / (ms * 1e-3) / 1e12 / PEAK * 100:5.1f} % dot2 peak  [{os.path.basename(lib)}]",
                  flush=True)


if __name__ == "__main__":
    main()
