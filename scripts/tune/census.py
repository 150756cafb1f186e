#!/usr/bin/env python3
"""Workgroup placement census (tuning only): 1024 workgroups of 512 lanes with
75 KB of LDS each (the headline's residency, 2 per CU) record HW_ID and
XCC_ID.  Prints, per (XCC, SE, SH, CU), the TG_ID slots the workgroups got,
and whether the two co-resident workgroups of a CU differ in TG_ID parity
(the stagger experiment of decim_stream_x keys on it)."""
import collections
import ctypes as C
import json
import os

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "libtune.so"))
lib.tune_census.argtypes = [C.c_int, C.c_void_p, C.c_void_p]
B = 1024
out = torch.zeros(2 * B, dtype=torch.int32, device="cuda")
lib.tune_census(B, C.c_void_p(out.data_ptr()), C.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
v = out.view(-1, 2).cpu().numpy().astype("uint32")
cus = collections.defaultdict(list)
for b, (hw, xcc) in enumerate(v):
    key = (int(xcc) & 0xF, (int(hw) >> 13) & 0x7, (int(hw) >> 12) & 1, (int(hw) >> 8) & 0xF)
    cus[key].append((b, (int(hw) >> 16) & 0xF))
tg = collections.Counter(t for l in cus.values() for _, t in l)
first = {k: sorted(l)[:2] for k, l in cus.items()}
mixed = sum(1 for l in first.values() if len(l) == 2 and (l[0][1] & 1) != (l[1][1] & 1))
print(json.dumps({"workgroups": B, "cus_seen": len(cus), "tg_id_histogram": dict(sorted(tg.items())),
                  "first_two_per_cu_differ_in_tg_parity": mixed,
                  "example": {str(k): l[:6] for k, l in list(cus.items())[:6]}}))
