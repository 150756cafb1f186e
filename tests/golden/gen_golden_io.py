#!/usr/bin/env python3
"""Golden fixtures for the two §8f "next" items, from the REAL reference
(oracle/_ref/strict/libref_io.so, built by ``make -C oracle``):

* buffers.h FifoWithTimeTrack -- scripted write/read/count/reset/
  getAbsoluteTime sequences, including the scenario of the reference's own
  buffers_test.cpp (T = double, N = 15; that file does not compile as shipped:
  it binds a uint32_t to read()'s uint64_t& -- the sequence is replayed here);
* dsptl_files.h saveBinarySamples / readBinarySamples -- the bytes the
  reference writes, and what its reader returns (sample count, which includes
  the spurious trailing sample its `while(is)` loop appends).

Run in the build container: ``python tests/golden/gen_golden_io.py``.
Writes tests/golden/io_golden.npz and tests/golden/io_manifest.json.
Script ops (replayed by tests/test_io_golden.py and the GPU tests):
  ["write", key, seconds, frac]            -> nothing
  ["read", n, start, err, start_after, key|None]
  ["count", value]
  ["reset"]
  ["abs", time_point, frac, seconds, frac_seconds]
"""
from __future__ import annotations

import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as P  # noqa: E402

ARR: dict[str, np.ndarray] = {}
CASES: list[dict] = []
RIO = P.ReferenceIO("strict")


def put(name, a):
    assert name not in ARR, name
    ARR[name] = np.ascontiguousarray(a)
    return name


class Rec:
    def __init__(self, name, kind, fs):
        self.name, self.kind, self.fs = name, kind, fs
        self.f = RIO.fifo(kind, fs)
        self.ops = []
        self.k = 0

    def key(self, tag):
        self.k += 1
        return f"{self.name}/{self.k:04d}_{tag}"

    def write(self, x, sec=0, frac=0.0):
        self.f.write(x, sec, frac)
        self.ops.append(["write", put(self.key("w"), x), int(sec), float(frac)])

    def read(self, n, start):
        err, st, out = self.f.read(n, start)
        self.ops.append(["read", int(n), int(start), int(err), int(st), None if err else put(self.key("r"), out)])

    def count(self):
        self.ops.append(["count", self.f.count()])

    def reset(self):
        self.f.reset()
        self.ops.append(["reset"])

    def abs(self, tp, frac=0.0):
        s, fs = self.f.absolute_time(tp, frac)
        self.ops.append(["abs", int(tp), float(frac), int(s), float(fs)])

    def done(self):
        dt, N = self.f.dtype, self.f.N
        CASES.append({"name": self.name, "kind": self.kind, "N": N, "elem": dt.str if dt.shape == () else "ci16",
                      "fs": self.fs, "ops": self.ops})


def buffers_test_scenario():
    r = Rec("fifo_buffers_test", 0, 0.0)  # FifoWithTimeTrack<double, 15> fifo; (fs defaults to 0)
    value = 0.0

    def block(n):
        nonlocal value
        v = np.arange(value + 1, value + n + 1, dtype=np.float64)
        value += n
        return v

    for _ in range(23):
        r.write(block(14))
    r.count()
    for n in (10, 5, 7):
        r.write(block(n))
        r.count()
    r.reset()
    r.count()
    value = 0.0
    r.write(block(7))
    r.read(3, 4)
    r.write(block(10))
    r.read(15, 3)
    r.write(block(4))
    r.read(4, 6)
    r.count()
    r.done()


def random_scenario(name, kind, fs, nops, seed, max_write):
    rng = np.random.default_rng(seed)
    r = Rec(name, kind, fs)
    N = r.f.N
    t_end = 0
    sec = 1000
    for i in range(nops):
        op = rng.choice(["write", "write", "read", "read", "count", "abs", "reset"], p=[.3, .1, .25, .15, .08, .1, .02])
        if op == "write":
            n = int(rng.integers(1, max_write + 1))
            x = rng.integers(-32768, 32767, size=(n, 2)).astype(np.int16)
            frac = float(rng.integers(0, 1 << 20)) / (1 << 20)
            r.write(x, sec, frac)
            sec += int(rng.integers(0, 3))
            t_end += n
        elif op == "read":
            n = int(rng.integers(1, N + 1))
            lo = max(0, t_end - N - 20)
            start = int(rng.integers(lo, t_end + 5))
            r.read(n, start)
        elif op == "count":
            r.count()
        elif op == "abs":
            tp = int(rng.integers(max(0, t_end - 3 * N), t_end + 3 * N))
            r.abs(tp, float(rng.integers(0, 8)) / 8)
        else:
            r.reset()
            t_end = 0
    r.count()
    r.done()


def iq_cases():
    rng = np.random.default_rng(7)
    out = []
    with tempfile.TemporaryDirectory() as d:
        for name, x in (("iq_ci16", rng.integers(-32768, 32767, size=(1000, 2)).astype(np.int16)),
                        ("iq_cf32", rng.standard_normal((777, 2)).astype(np.float32)),
                        ("iq_ci16_empty", np.zeros((0, 2), np.int16))):
            path = os.path.join(d, name + ".bin")
            RIO.iq_save(path, x)
            with open(path, "rb") as fh:
                raw = np.frombuffer(fh.read(), np.uint8)
            got, n = RIO.iq_read(path, x.dtype, cap=len(x) + 4)
            assert np.array_equal(got[:len(x)], x)
            out.append({"name": name, "samples": put(name + "/samples", x), "file": put(name + "/file", raw),
                        "ref_read_count": int(n)})
    return out


def main():
    buffers_test_scenario()
    random_scenario("fifo_ci16_n64", 1, 1.0e6, 400, 11, 63)
    random_scenario("fifo_ci16_n1000", 2, 30.72e6, 90, 12, 999)
    random_scenario("fifo_ci16_n64_fs3", 1, 3.0, 200, 13, 40)
    iq = iq_cases()
    np.savez_compressed(os.path.join(HERE, "io_golden.npz"), **ARR)
    with open(os.path.join(HERE, "io_manifest.json"), "w") as fh:
        json.dump({"fifo": CASES, "iq": iq}, fh, indent=0)
    print(f"{len(CASES)} fifo scripts ({sum(len(c['ops']) for c in CASES)} ops), {len(iq)} iq cases, "
          f"{os.path.getsize(os.path.join(HERE, 'io_golden.npz'))} bytes")


if __name__ == "__main__":
    main()
