"""Time FilterFir<cf32,cf32,cf32,float> at a given tap count on 2^26 device-resident
samples (100 warm-up steps, mean of 200 timed with HIP events on the launch stream).
Library from SRCDSP_HIP_LIB (A/B runs).  Usage: python scripts/fir_cf32_time.py [ntaps]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

import srcdsp_amd as S

nt = int(sys.argv[1]) if len(sys.argv) > 1 else 31
n = 1 << 26
c = (np.hanning(nt + 2)[1:-1] / nt).astype(np.float32)
g = S.FilterFir(c, "complex<float>", "complex<float>", "complex<float>", "float")
x = torch.randint(-30000, 30000, (n, 2), dtype=torch.int32, device="cuda").to(torch.float32)
x = torch.view_as_complex(x).contiguous()
y = torch.empty(n, dtype=torch.complex64, device="cuda")
st = torch.cuda.current_stream()
for _ in range(100):
    g.step(x, y)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(200)]
for a, b in ev:
    a.record(st)
    g.step(x, y)
    b.record(st)
torch.cuda.synchronize()
ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
print(f"cf32 FIR {nt} taps, 2^26: {ms:.4f} ms  {16 * n / ms / 1e6:.1f} GB/s")
