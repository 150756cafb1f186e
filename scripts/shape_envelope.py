"""Kernel time of the complex<float> decimator across tap counts: the shapes
compiled into the headline kernel next to arbitrary tap counts, which take the
same kernel with the tap count at run time (decim_stream_cf32<0, ...>).

  python scripts/shape_envelope.py [M ...]

2^26 device-resident samples per shape, 20 warm-up launches, then the median
of 50 timed launches.  One line per shape: ms, Gsamples/s, GB/s (8 B in per
sample + 8 B out per output) and TMAC/s (complex MACs = N per output)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import srcdsp_amd as S  # noqa: E402
from srcdsp_amd.design import hamming_sinc  # noqa: E402

COMPILED = {4: (63, 64, 127, 128), 8: (127, 128, 255, 256), 16: (127, 128, 255, 256),
            2: (63, 64, 127, 128), 3: (63, 64, 127, 128), 1: (63, 64), 6: (), 12: ()}
SHAPES = {4: (31, 63, 95, 100, 126, 127, 129, 200, 255, 300, 511, 1024),
          1: (31, 62, 63, 100, 127, 129, 255, 300),
          2: (62, 63, 95, 127, 129, 200),
          3: (62, 63, 100, 127, 129),
          8: (126, 127, 129, 200, 255, 300),
          16: (126, 127, 129, 255, 300),
          6: (31, 63, 127, 255),
          12: (63, 127, 255)}


def main():
    Ms = [int(a) for a in sys.argv[1:]] or [4, 1, 2, 3, 8, 16]
    L = 1 << 26
    x = torch.empty(L, dtype=torch.complex64, device="cuda")
    S.fill_synthetic(x, "cf32", seed=0x5EED, channel=0)
    for M in Ms:
        for N in SHAPES[M]:
            c = hamming_sinc(N - (N % 2 == 0)) if N > 2 else np.ones(N, np.float32) / N
            if N > 2 and N % 2 == 0:
                c = np.concatenate([c, [0.0]]).astype(np.float32)
            f = S.FilterDnsamplingFir(c, M, fp="fma") if M > 1 else S.FilterFir(c, fp="fma")
            xm = x[: L - L % M]
            y = torch.empty(L // M, dtype=torch.complex64, device="cuda")
            for _ in range(20):
                f.step(xm, y)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
            for a, b in ev:
                a.record()
                f.step(xm, y)
                b.record()
            torch.cuda.synchronize()
            ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
            gbs = (8 * L + 8 * L // M) / (ms * 1e-3) / 1e9
            kind = "compiled" if N in COMPILED[M] else "runtime "
            print(f"M={M:2d} N={N:4d} {kind}: {ms:.4f} ms {L / ms / 1e6:8.1f} Gsamp/s {gbs:7.1f} GB/s "
                  f"{N * L / M / (ms * 1e-3) / 1e12:5.2f} TMAC/s", flush=True)


if __name__ == "__main__":
    main()
