"""Kernel time of the v_dot2 interpolator (complex<int16_t>, int16-range taps)
over phase lengths: 2^24 device-resident inputs, median of 50 launches.

  python scripts/up_envelope.py [L:ntaps ...]     (SRCDSP_HIP_LIB: another library build)"""
import os
import sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import srcdsp_amd as S
from srcdsp_amd.design import hamming_sinc, q14

n = 1 << 24
x = torch.empty((n, 2), dtype=torch.int16, device="cuda")
S.fill_synthetic(x, "ci16", seed=0x5EED, channel=0, lo=-8192, hi=8191)
SHAPES = ((4, 64), (4, 128), (4, 256), (2, 32), (2, 64), (2, 128), (8, 128), (8, 256), (8, 512), (8, 1000))
shapes = [tuple(int(v) for v in a.split(":")) for a in sys.argv[1:]] or SHAPES
for L, ntaps in shapes:
    f = S.FilterUpsamplingFir(q14(hamming_sinc(ntaps, 0.12) * L), L)
    y = torch.empty((L * n, 2), dtype=torch.int16, device="cuda")
    for _ in range(10):
        f.step(x, y)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
    for a, b in ev:
        a.record(); f.step(x, y); b.record()
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    dot2 = n * L * 2 * ((ntaps // L + 1) // 2)
    print(f"L={L} taps={ntaps:4d}: {ms:.4f} ms  {n / ms / 1e6:8.1f} Gsamp/s in  {dot2 / (ms * 1e-3) / 1e12:.1f} T dot2/s", flush=True)
