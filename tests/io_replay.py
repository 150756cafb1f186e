"""Replays the FifoWithTimeTrack golden scripts (tests/golden/io_manifest.json,
generated from the real reference by tests/golden/gen_golden_io.py) on any
FIFO implementation exposing write/read/count/reset/absolute_time."""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load():
    with open(os.path.join(GOLDEN, "io_manifest.json")) as f:
        man = json.load(f)
    arr = np.load(os.path.join(GOLDEN, "io_golden.npz"))
    return man, arr


def elem_dtype(case) -> np.dtype:
    return np.dtype(("<i2", 2)) if case["elem"] == "ci16" else np.dtype(case["elem"])


def replay_fifo(fifo, case, arr, read=None):
    """fifo: object with write(x, sec, frac), count(), reset(),
    absolute_time(tp, frac) -> (sec, frac) and read(n, start) -> (err, start, data)
    (or pass `read` to override).  Asserts every op against the golden."""
    read = read or fifo.read
    for i, op in enumerate(case["ops"]):
        kind = op[0]
        where = f"{case['name']} op {i} {op[:3]}"
        if kind == "write":
            fifo.write(np.ascontiguousarray(arr[op[1]]), op[2], op[3])
        elif kind == "read":
            _, n, start, err, start_after, key = op
            e, st, data = read(n, start)
            assert (int(e), int(st)) == (err, start_after), where
            if not err:
                got = np.ascontiguousarray(data).view(np.uint8)
                assert np.array_equal(got.reshape(-1), np.ascontiguousarray(arr[key]).view(np.uint8).reshape(-1)), where
        elif kind == "count":
            assert fifo.count() == op[1], where
        elif kind == "reset":
            fifo.reset()
        elif kind == "abs":
            s, fs = fifo.absolute_time(op[1], op[2])
            assert s == op[3] and fs == op[4], (where, (s, fs), op[3:])
        else:
            raise AssertionError(f"unknown op {kind}")
