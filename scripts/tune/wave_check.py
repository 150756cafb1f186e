#!/usr/bin/env python3
"""Bit-exact check of tuning decimator variants against the product headline
(FilterDnsamplingFir.step), on the full 2^28 workload and on ragged sizes
(tuning only).  usage: wave_check.py VARIANT [VARIANT ...]"""
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


def main():
    st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
    c = hamming_sinc(127)
    cdev = torch.from_numpy(c).cuda()
    ok = True
    for L in (1 << 28, (1 << 20) + 4 * 777, 4096, 1024 + 4, 4 * 300000 + 8):
        x = torch.empty(L, dtype=torch.complex64, device="cuda")
        S.fill_synthetic(x, "cf32")
        ref = torch.empty(L // 4, dtype=torch.complex64, device="cuda")
        S.FilterDnsamplingFir(c, 4).step(x, ref)
        h0 = torch.zeros(126, dtype=torch.complex64, device="cuda")
        for v in map(int, sys.argv[1:]):
            y = torch.full((L // 4,), float("nan"), dtype=torch.complex64, device="cuda")
            h1 = torch.zeros(126, dtype=torch.complex64, device="cuda")
            for grid in (1024, 512, 7):
                y.fill_(float("nan"))
                rc = lib.tune_decim(v, grid, C.c_void_p(cdev.data_ptr()), C.c_void_p(x.data_ptr()),
                                    C.c_void_p(y.data_ptr()), L, C.c_void_p(h0.data_ptr()), C.c_void_p(h1.data_ptr()), st)
                if rc == -2:  # the variant does not take this shape (whole ring chunks only)
                    print(f"L={L} variant {v}: shape not supported, skipped", flush=True)
                    break
                assert rc == 0, rc
                torch.cuda.synchronize()
                same = torch.equal(torch.view_as_real(y).view(torch.int32), torch.view_as_real(ref).view(torch.int32))
                hist_ok = torch.equal(h1, x[-126:]) if L >= 126 else True
                print(f"L={L} variant {v} grid {grid}: {'bit-exact' if same else 'MISMATCH'}"
                      f"{'' if hist_ok else ' HISTORY MISMATCH'}", flush=True)
                ok &= same and hist_ok
    print("ALL OK" if ok else "FAILED", flush=True)
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
