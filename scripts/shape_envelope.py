"""Kernel time of the cf32 decimator for shapes off the tiled path (other M,
other tap counts run decim_generic) next to the tiled headline shape.
Prints one line per shape; 2^26 device-resident samples, 50 timed launches."""
import sys, os
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import srcdsp_amd as S
from srcdsp_amd.design import hamming_sinc

L = 1 << 26
x = torch.empty(L, dtype=torch.complex64, device="cuda")
S.fill_synthetic(x, "cf32", seed=0x5EED, channel=0)
for M, N in ((4, 127), (4, 128), (4, 63), (4, 255), (2, 63), (2, 127), (8, 127), (8, 255), (3, 127), (16, 255), (1, 31), (1, 63), (1, 127), (1, 255)):
    f = S.FilterDnsamplingFir(hamming_sinc(N), M, fp="fma") if M > 1 else S.FilterFir(hamming_sinc(N), fp="fma")
    xm = x[: L - L % M]  # a whole number of outputs (M = 3)
    y = torch.empty(L // M, dtype=torch.complex64, device="cuda")
    for _ in range(10):
        f.step(xm, y)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
    for a, b in ev:
        a.record(); f.step(xm, y); b.record()
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    gbs = (8 * L + 8 * L // M) / (ms * 1e-3) / 1e9
    print(f"M={M} N={N:4d}: {ms:.3f} ms  {L / ms / 1e6:8.1f} Gsamp/s  {gbs:7.1f} GB/s  {N * L / M / (ms * 1e-3) / 1e12:.1f} TMAC/s", flush=True)

# complex<int16_t> with Q14 int32 taps (config 4's decimator type)
from srcdsp_amd.design import q14
xi = torch.empty((L, 2), dtype=torch.int16, device="cuda")
S.fill_synthetic(xi, "ci16", seed=0x5EED, channel=0, lo=-8192, hi=8191)
for M, N in ((4, 127), (4, 63), (4, 255), (2, 63), (8, 255)):
    f = S.FilterDnsamplingFir(q14(hamming_sinc(N)), M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    y = torch.empty((L // M, 2), dtype=torch.int16, device="cuda")
    for _ in range(10):
        f.step(xi, y)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(50)]
    for a, b in ev:
        a.record(); f.step(xi, y); b.record()
    torch.cuda.synchronize()
    ms = float(np.median([a.elapsed_time(b) for a, b in ev]))
    print(f"ci16 M={M} N={N:4d}: {ms:.3f} ms  {L / ms / 1e6:8.1f} Gsamp/s  {N * L / M / (ms * 1e-3) / 1e12:.1f} TMAC/s", flush=True)
