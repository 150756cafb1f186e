#!/usr/bin/env python3
"""Lane map and accumulator numerics of the gfx950 i8 MFMAs (tuning only).

A kernel that builds its own A and B fragments needs only this: lane l holds
16 int8 of A's row (l mod R) and 16 int8 of B's column (l mod R), R = 32 or
16, for the k slice of lane group l // R, with the SAME k order in A and B.
Then D[row][col] = sum over groups g and bytes j of
A_frag[row + R g][j] * B_frag[col + R g][j], whatever the hardware's k order
is.  The check builds random fragments, predicts D that way (int64, then
mod 2^32), and reads D from the CDNA C/D map (32x32: col = l & 31,
row = (i & 3) + 8 (i >> 2) + 4 (l >> 5); 16x16: col = l & 15,
row = 4 (l >> 4) + i).  Then the accumulator's overflow: C near 2^31 plus
positive products, repeated, must wrap modulo 2^32 (the reference's
complex<int32_t> sum wraps) and not saturate."""
import ctypes as C
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
lib = C.CDLL(os.path.join(HERE, "libmfmai8.so"))


def run(shape, fa, fb, c, reps=1):
    regs = 16 if shape == 32 else 4
    da = torch.from_numpy(np.ascontiguousarray(fa)).cuda()
    db = torch.from_numpy(np.ascontiguousarray(fb)).cuda()
    dc = torch.from_numpy(np.ascontiguousarray(c.astype(np.int32))).cuda()
    dd = torch.zeros((64, regs), dtype=torch.int32, device="cuda")
    rc = lib.tune_i8_mfma_raw(shape, C.c_void_p(da.data_ptr()), C.c_void_p(db.data_ptr()), C.c_void_p(dc.data_ptr()),
                              C.c_void_p(dd.data_ptr()), reps, C.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0, rc
    torch.cuda.synchronize()
    return dd.cpu().numpy()


def dmap(shape):
    """(lane, reg) -> (row, col) of the C/D operand."""
    R = shape
    regs = 16 if shape == 32 else 4
    m = np.zeros((64, regs, 2), np.int64)
    for l in range(64):
        for i in range(regs):
            if shape == 32:
                m[l, i] = ((i & 3) + 8 * (i >> 2) + 4 * (l >> 5), l & 31)
            else:
                m[l, i] = (4 * (l >> 4) + i, l & 15)
    return m


def predict(shape, fa, fb, c_full, reps):
    R = shape
    G = 64 // R
    D = c_full.astype(np.int64).copy()
    for row in range(R):
        for col in range(R):
            s = 0
            for g in range(G):
                s += int(np.dot(fa[row + R * g].astype(np.int64), fb[col + R * g].astype(np.int64)))
            D[row, col] += reps * s
    return ((D + (1 << 31)) % (1 << 32) - (1 << 31)).astype(np.int64)


def check(shape, rng, big=False):
    R = shape
    regs = 16 if shape == 32 else 4
    m = dmap(shape)
    fa = rng.integers(-128, 128, (64, 16)).astype(np.int8)
    fb = rng.integers(-128, 128, (64, 16)).astype(np.int8)
    reps = 1
    c_full = rng.integers(-1000, 1000, (R, R)).astype(np.int64)
    if big:  # every product positive and large, C just below 2^31: several steps cross it
        fa[:] = 127
        fb[:] = 127
        c_full[:] = (1 << 31) - 1000
        reps = 40  # 40 x K x 16129 (K = 32 or 64) >= 2.1e7 per element: crosses 2^31 from below
    c = np.zeros((64, regs), np.int64)
    for l in range(64):
        for i in range(regs):
            c[l, i] = c_full[m[l, i, 0], m[l, i, 1]]
    d = run(shape, fa, fb, c.astype(np.int32), reps)
    want = predict(shape, fa, fb, c_full, reps)
    got = np.zeros((R, R), np.int64)
    for l in range(64):
        for i in range(regs):
            got[m[l, i, 0], m[l, i, 1]] = d[l, i]
    bad = int((got != want).sum())
    sat = int((got == (1 << 31) - 1).sum())
    return bad, sat


def main():
    rng = np.random.default_rng(7)
    ok = True
    for shape in (32, 16):
        for trial in range(3):
            bad, _ = check(shape, rng)
            print(f"i8 {shape}x{shape}: random fragments trial {trial}: {bad} of {shape * shape} elements differ "
                  f"from the lane-group prediction")
            ok &= bad == 0
        bad, sat = check(shape, rng, big=True)
        print(f"i8 {shape}x{shape}: C = 2^31 - 1000 plus 40 x K x 127^2: {bad} differ from the mod-2^32 wrap, "
              f"{sat} saturated at INT32_MAX")
        ok &= bad == 0
    print("RESULT", "PASS" if ok else "FAIL")
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
