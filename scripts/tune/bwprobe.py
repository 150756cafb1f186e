#!/usr/bin/env python3
"""HBM streaming probes (scripts/tune/bwprobe.hip; not part of the product):
GB/s of read:write mixes, load/store policies and work distributions over a
2 GiB input, min over interleaved rounds."""
import ctypes as C
import os

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "libbwprobe.so"))
lib.bw_probe.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_void_p, C.c_long, C.c_void_p]

CASES = {0: ("copy 1:1", 1), 12: ("copy 1:1 nt-store", 1), 1: ("4:1 gs U1", 4), 2: ("4:1 gs U2", 4),
         11: ("4:1 gs U4", 4), 3: ("4:1 gs U2 nt-store", 4), 4: ("4:1 gs U2 nt-load", 4),
         5: ("4:1 gs U2 nt-both", 4), 6: ("4:1 contig U1", 4), 7: ("4:1 contig U2", 4),
         8: ("4:1 contig U2 nt-store", 4), 9: ("read-only U2", 0), 10: ("read-only U2 nt", 0),
         20: ("write-only fill", -1)}


def main():
    n16 = 1 << 27  # 2 GiB of input granules
    x = torch.ones(n16 * 4, dtype=torch.float32, device="cuda")
    y = torch.empty(n16 * 4, dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream()
    sp = C.c_void_p(st.cuda_stream)
    res = {}
    grids = (1024, 2048, 4096, 8192)
    if os.environ.get("BW_AUX"):
        CASES.clear()
        for la in (0, 2):
            for k, sa in enumerate((0, 1, 2, 3, 16, 17, 18, 19)):
                CASES[100 + 10 * (la // 2) + k] = (f"4:1 contig ld aux {la} st aux {sa}", 4)
        for k, la in enumerate((1, 3, 16, 17, 18, 19)):
            CASES[120 + k] = (f"4:1 contig ld aux {la} st aux 2", 4)
        grids = (1024, 2048)
    if os.environ.get("BW_EXPAND"):
        CASES.clear()
        CASES.update({30: ("1:2 expand", -2), 31: ("1:2 expand nt-both", -2), 32: ("1:2 expand nt-store", -2),
                      0: ("copy 1:1", 1), 20: ("write-only fill", -1), 10: ("read-only U2 nt", 0)})
        grids = (1024, 2048, 4096, 8192)
    if os.environ.get("BW_BURST"):
        CASES.clear()
        CASES.update({13: ("4:1 contig U2 nt-both", 4), 5: ("4:1 gs U2 nt-both", 4),
                      40: ("4:1 burst K1 nt-both", 4), 41: ("4:1 burst K2 nt-both", 4),
                      42: ("4:1 burst K4 nt-both", 4), 43: ("4:1 burst K8 nt-both", 4),
                      44: ("4:1 burst K4 nt-load", 4), 10: ("read-only U2 nt", 0), 20: ("write-only fill", -1)})
        grids = (512, 1024, 2048, 4096)
    off_g = int(os.environ.get("BW_OUT_OFFSET", "0"))  # output base offset in 16-B granules
    if off_g:
        y = torch.empty(n16 * 4 + off_g * 4, dtype=torch.float32, device="cuda")[off_g * 4:]
        print(f"output base offset: {off_g * 16} B (address {y.data_ptr():#x}, input {x.data_ptr():#x})")
    for rnd in range(4):
        for cid in CASES:
            for g in grids:
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(4)]
                for a, b in ev:
                    a.record(st)
                    rc = lib.bw_probe(cid, g, C.c_void_p(x.data_ptr()), C.c_void_p(y.data_ptr()), n16, sp)
                    b.record(st)
                    assert rc == 0, rc
                torch.cuda.synchronize()
                t = min(a.elapsed_time(b) for a, b in ev[1:])
                res.setdefault((cid, g), []).append(t)
    for cid, (name, ratio) in CASES.items():
        if ratio > 0:
            byt = n16 * 16 + n16 // ratio * 16
        elif ratio == 0:
            byt = n16 * 16
        elif ratio == -2:  # 1:2 expansion: n16/2 granules read, n16 written
            byt = n16 // 2 * 16 + n16 * 16
        else:
            byt = n16 // 4 * 16
        row = []
        for g in grids:
            t = min(res[(cid, g)])
            row.append(f"{g:5d}: {byt / (t * 1e-3) / 1e9:7.1f}")
        print(f"{name:24s} GB/s  " + "  ".join(row), flush=True)


if __name__ == "__main__":
    main()
