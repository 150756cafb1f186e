"""Kernel time of the FixedPatternCorrelator step across (N, S): the fused
one-launch scan (S = 1, any N >= 48 or N % 16 = 0: config 5's shape among them),
the dot2 tiles for any other N and stride, and (past 8192 taps) the generic kernel.

  python scripts/corr_envelope.py [N:S ...]

SRCDSP_HIP_LIB selects another build of the library (same-box A/B).  2^24
noise samples (no detection: the whole buffer is scanned), reset + one step
per launch, 3 warm-up steps, median of 10.  One line per shape: ms,
Msamples/s and the v_dot2 rate (2 N dot2 lane-ops per sample) against the
39.3 T/s VALU peak."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import srcdsp_amd as S  # noqa: E402
from srcdsp_amd.design import qpsk_pattern  # noqa: E402

SHAPES = ((1024, 1), (1000, 1), (127, 1), (100, 1), (512, 2), (256, 4), (127, 2), (128, 8), (64, 16), (31, 3))
PEAK = 39.32


def main():
    shapes = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or list(SHAPES)
    L = 1 << 24
    x = torch.from_numpy(np.random.default_rng(0).integers(-125, 126, size=(L, 2)).astype(np.int16)).cuda()
    lib = os.environ.get("SRCDSP_HIP_LIB", "tree")
    for N, St in shapes:
        g = S.FixedPatternCorrelator(N, St)
        g.setPattern(qpsk_pattern(N, 500 if N <= 2048 else 200, seed=N))
        ms = []
        for k in range(13):
            g.reset()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            found, _ = g.step(x)
            b.record()
            torch.cuda.synchronize()
            if k >= 3:
                ms.append(a.elapsed_time(b))
        m = float(np.median(ms))
        print(f"N={N:5d} S={St:2d}: {m:8.3f} ms {L / m / 1e3:9.1f} Msamp/s "
              f"{2 * N * L / (m * 1e-3) / 1e12 / PEAK * 100:5.1f} % dot2 peak  found={found}  "
              f"[{os.path.basename(lib)}]", flush=True)


if __name__ == "__main__":
    main()
