#!/usr/bin/env python3
"""Layout and numerics of v_mfma_f32_4x4x1_16b_f32 (tuning only): which lane
holds which A/B/D element, and whether K steps equal a sequential fmaf chain
bit for bit (host chain through libm fmaf)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "libtune.so"))
libm = C.CDLL("libm.so.6")
libm.fmaf.restype = C.c_float
libm.fmaf.argtypes = [C.c_float, C.c_float, C.c_float]


def run(a, b):
    K = a.shape[0]
    da, db = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    d = torch.zeros(256, dtype=torch.float32, device="cuda")
    lib.tune_mfma4x4_probe(C.c_void_p(da.data_ptr()), C.c_void_p(db.data_ptr()), C.c_void_p(d.data_ptr()), K,
                           C.c_void_p(torch.cuda.current_stream().cuda_stream))
    torch.cuda.synchronize()
    return d.cpu().numpy().reshape(64, 4)


def main():
    # one step, distinct powers: A[l] = l + 1, B[l] = 1000 (l + 1)
    a = (np.arange(64, dtype=np.float32) + 1)[None, :]
    b = (1000 * (np.arange(64, dtype=np.float32) + 1))[None, :]
    d = run(a, b)
    ok = True
    for l in range(64):
        for r in range(4):
            blk, col = l // 4, l % 4
            want = a[0, 4 * blk + r] * b[0, 4 * blk + col]
            if d[l, r] != want:
                ok = False
    print("layout A[lane=4*blk+row] B[lane=4*blk+col] D[lane=4*blk+col][reg=row]:", "MATCH" if ok else "NO MATCH")
    if not ok:
        print("D (lane, reg) / 1000:")
        for l in range(16):
            print(l, d[l] / 1000)
    # numerics: K random steps vs the sequential fmaf chain per (blk, row, col)
    rng = np.random.default_rng(1)
    K = 300
    a = (rng.standard_normal((K, 64)) * np.exp2(rng.integers(-20, 20, (K, 64)))).astype(np.float32)
    b = (rng.standard_normal((K, 64)) * np.exp2(rng.integers(-20, 20, (K, 64)))).astype(np.float32)
    a[rng.random((K, 64)) < 0.1] = 0.0
    d = run(a, b)
    bad = 0
    for l in range(64):
        for r in range(4):
            blk, col = l // 4, l % 4
            y = C.c_float(0.0)
            for k in range(K):
                y = C.c_float(libm.fmaf(float(a[k, 4 * blk + r]), float(b[k, 4 * blk + col]), y.value))
            if np.float32(y.value).view(np.uint32) != d[l, r].view(np.uint32):
                bad += 1
    print(f"K={K} random steps vs host fmaf chain: {256 - bad}/256 bit-exact")


if __name__ == "__main__":
    main()
