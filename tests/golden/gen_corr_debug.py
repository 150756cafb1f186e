#!/usr/bin/env python3
"""Golden debug files of the reference correlator built with CREATE_DEBUG_FILES
(correlators.h:29,107-111,128-132,253-257).

Compiles tests/cpp/corr_debug_main.cpp against the UNMODIFIED reference headers
where they lie (-I /root/reference, linked with its dsp_complex.cpp, in a
temporary directory: nothing of the reference is copied), runs it on three
inputs and stores, per case, the input file, the step log and the three files
the reference wrote (debug_corr_energy.dat, debug_corr_values.dat,
debug_corr_threshold.dat) as byte arrays in tests/golden/corr_debug.npz.
tests/test_dropin_cpp.py builds the same program against the drop-in on the
GPU box and requires identical bytes.  Run in the build container:
    python tests/golden/gen_corr_debug.py
"""
from __future__ import annotations

import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("REF_DIR", "/root/reference")
SRC = os.path.join(ROOT, "tests", "cpp", "corr_debug_main.cpp")
FILES = ("debug_corr_energy.dat", "debug_corr_values.dat", "debug_corr_threshold.dat")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def in_bin(chunk: int, pattern: np.ndarray, x: np.ndarray) -> bytes:
    return (struct.pack("<i", chunk) + np.ascontiguousarray(pattern, np.int32).tobytes()
            + np.ascontiguousarray(x, np.int16).tobytes())


def cases():
    from srcdsp_amd.design import qpsk_pattern
    import corr_ties as T
    rng = np.random.default_rng(77)
    out = []
    for N, S, n, chunk, amp in ((32, 4, 12000, 2500, 2), (1024, 1, 9000, 3000, 2)):
        p = qpsk_pattern(N, 500, seed=N + S)
        x = rng.integers(-125, 126, size=(n, 2)).astype(np.int32)
        for off in (n // 4, (2 * n) // 3):
            for m in range(N):
                if off + m * S < n:
                    x[off + m * S] += amp * p[m]
        out.append({"key": f"n{N}_s{S}", "N": N, "S": S, "chunk": chunk, "pattern": p,
                    "x": np.clip(x, -32768, 32767).astype(np.int16)})
    man, arr = T.load()
    case = [c for c in man["cases"] if c["key"] == "n16_s1"][0]
    out.append({"key": "ties_n16_s1", "N": 16, "S": 1, "chunk": 700, "pattern": T.pattern(case),
                "x": arr["n16_s1_x"]})
    return out


def main():
    arrays, meta = {}, []
    with tempfile.TemporaryDirectory() as d:
        for c in cases():
            exe = os.path.join(d, f"ref_{c['key']}")
            subprocess.run(["g++", "-std=gnu++11", "-O2", "-DCREATE_DEBUG_FILES", f"-DCORR_N={c['N']}",
                            f"-DCORR_S={c['S']}", "-I", REF, SRC, os.path.join(REF, "dsp_complex.cpp"), "-o", exe],
                           check=True)
            run = os.path.join(d, c["key"])
            os.makedirs(run)
            blob = in_bin(c["chunk"], c["pattern"], c["x"])
            with open(os.path.join(run, "in.bin"), "wb") as f:
                f.write(blob)
            subprocess.run([exe, "in.bin", "steps.txt"], cwd=run, check=True)
            arrays[c["key"] + "_in"] = np.frombuffer(blob, np.uint8)
            for name in ("steps.txt",) + FILES:
                with open(os.path.join(run, name), "rb") as f:
                    arrays[c["key"] + "_" + name] = np.frombuffer(f.read(), np.uint8)
            lines = open(os.path.join(run, "steps.txt")).read().split("\n")
            det = sum(1 for l in lines if l and l.split()[2] == "1")
            n_lines = arrays[c["key"] + "_" + FILES[0]].tobytes().count(b"\n")
            meta.append({"key": c["key"], "N": c["N"], "S": c["S"], "chunk": c["chunk"], "samples": len(c["x"]),
                         "detections": det, "debug_lines": n_lines})
            print(meta[-1])
    np.savez_compressed(os.path.join(HERE, "corr_debug.npz"), **arrays)
    with open(os.path.join(HERE, "corr_debug.json"), "w") as f:
        json.dump({"generator": "tests/golden/gen_corr_debug.py",
                   "source": "reference correlators.h built with -DCREATE_DEBUG_FILES (g++ -O2)",
                   "files": list(FILES), "cases": meta}, f, indent=1)


if __name__ == "__main__":
    main()
