#!/usr/bin/env python3
"""Launch one tune_decim variant N times back to back (for rocprofv3 PMC passes;
tuning only).  usage: launch_variant.py VARIANT GRID [N]"""
import ctypes as C
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", ".."))
import srcdsp_amd as S  # noqa: E402
from srcdsp_amd.design import hamming_sinc  # noqa: E402

lib = C.CDLL(os.path.join(HERE, "libtune.so"))
lib.tune_decim.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p,
                           C.c_void_p, C.c_void_p]
var, grid = int(sys.argv[1]), int(sys.argv[2])
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
L = 1 << 28
x = torch.empty(L, dtype=torch.complex64, device="cuda")
S.fill_synthetic(x, "cf32")
y = torch.empty(L // 4, dtype=torch.complex64, device="cuda")
h0 = torch.zeros(126, dtype=torch.complex64, device="cuda")
h1 = torch.zeros(126, dtype=torch.complex64, device="cuda")
cdev = torch.from_numpy(hamming_sinc(127)).cuda()
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
for _ in range(n):
    rc = lib.tune_decim(var, grid, C.c_void_p(cdev.data_ptr()), C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()),
                        L, C.c_void_p(h0.data_ptr()), C.c_void_p(h1.data_ptr()), st)
    assert rc == 0, rc
torch.cuda.synchronize()
print("launched", var, grid, n)
