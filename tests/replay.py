"""Replay the golden scripts (tests/golden/manifest.json) against a backend.

A backend provides factories with the reference's operator surface:
  decim(case) -> .step(x) .reset() .set_left_shift(v) .set_coeffs(c)
  fir(case)   -> .step(x) .reset() .set_coeffs(c)
  up(case)    -> .step(x, flush, iterator) .reset()
  mixer(case) -> .table() .step(x) .reset(f) .set_frequency(f) .adjust_frequency(f) .state()
  corr(case)  -> .set_pattern(p, thr) .step(x) -> (found, idx) .bit_samples() .status() .reset()
and an ``fp`` attribute ("strict" or "fma") selecting which reference output a
float case is compared with.  Comparison is bit-exact (bytes) everywhere.
"""
from __future__ import annotations

import json
import os

import numpy as np

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


class Golden:
    def __init__(self):
        with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
            self.meta = json.load(f)
        self.arr = dict(np.load(os.path.join(GOLDEN_DIR, "golden.npz"), allow_pickle=False))
        self.cases = {c["name"]: c for c in self.meta["cases"]}

    def __getitem__(self, k):
        return self.arr[k]

    def names(self, op=None):
        return [c["name"] for c in self.meta["cases"] if op is None or c["op"] == op]


_G = None


def load_golden() -> Golden:
    global _G
    if _G is None:
        _G = Golden()
    return _G


def bytes_equal(a, b) -> bool:
    a, b = np.ascontiguousarray(a), np.ascontiguousarray(b)
    return a.shape == b.shape and np.array_equal(a.view(np.uint8), b.view(np.uint8))


def _diff(name, step, got, exp):
    g, e = np.asarray(got), np.asarray(exp)
    if g.shape != e.shape:
        return f"{name} step {step}: shape {g.shape} != {e.shape}"
    bad = np.nonzero(np.ascontiguousarray(g).view(np.uint8) != np.ascontiguousarray(e).view(np.uint8))[0]
    return f"{name} step {step}: {len(bad)} differing bytes, first at byte {bad[0] if len(bad) else -1}"


def replay(case: dict, G: Golden, backend) -> list[str]:
    """Replay one case; return a list of failure strings (empty = pass)."""
    fails: list[str] = []
    op = case["op"]
    name = case["name"]
    fp = backend.fp
    if op == "decim":
        obj = backend.decim(case)
    elif op == "fir":
        obj = backend.fir(case)
    elif op == "up":
        obj = backend.up(case)
    elif op == "mixer":
        obj = backend.mixer(case)
        if not bytes_equal(obj.table(), G[case["table"]]):
            fails.append(f"{name}: LO table differs")
    elif op == "corr":
        obj = backend.corr(case)
        obj.set_pattern(G[case["pattern"]], case["threshold"])
    else:
        raise ValueError(op)
    for i, s in enumerate(case["script"]):
        kind = s[0]
        if kind == "reset":
            obj.reset()
        elif kind == "set_left_shift":
            obj.set_left_shift(s[1])
        elif kind == "set_coeffs":
            obj.set_coeffs(G[s[1]])
        elif kind in ("mixer_reset", "mixer_set_frequency", "mixer_adjust"):
            {"mixer_reset": obj.reset, "mixer_set_frequency": obj.set_frequency,
             "mixer_adjust": obj.adjust_frequency}[kind](np.float32(s[1]))
            if list(obj.state())[:2] != s[2][:2]:
                fails.append(f"{name} op {i}: mixer state {obj.state()} != {s[2]}")
        elif kind == "step":
            y = obj.step(G[s[1]])
            exp = G[s[2][fp]]
            if not bytes_equal(y, exp):
                fails.append(_diff(name, i, y, exp))
            if op == "mixer" and list(obj.state())[:2] != s[3][:2]:
                fails.append(f"{name} op {i}: mixer state {obj.state()} != {s[3]}")
        elif kind == "step_up":
            y = obj.step(G[s[1]], s[2], s[3])
            exp = G[s[4][fp]]
            if not bytes_equal(y, exp):
                fails.append(_diff(name, i, y, exp))
        elif kind == "corr_step":
            found, idx = obj.step(G[s[1]])
            if found != s[2] or (found and idx != s[3]):
                fails.append(f"{name} op {i}: ({found},{idx}) != ({s[2]},{s[3]})")
            if not bytes_equal(obj.bit_samples(), G[s[4]]):
                fails.append(f"{name} op {i}: bitSamples differ")
            st = obj.status()
            for k in ("energy", "corr", "coeffs_energy", "coeff_scaling"):
                if st[k] != s[5][k]:
                    fails.append(f"{name} op {i}: status {k} {st[k]} != {s[5][k]}")
        else:
            raise ValueError(kind)
    return fails


class OracleBackend:
    """The C restatement (oracle/liboracle.so) as a replay backend."""

    def __init__(self, fp: str):
        import pyoracle
        self.fp = fp
        self.o = pyoracle.Oracle(fp_mode=0 if fp == "strict" else 1)
        self.G = load_golden()

    def decim(self, c):
        return self.o.decim(c["variant"], c["M"], self.G[c["coeffs"]], abs_mode=c["abs_mode"])

    def fir(self, c):
        return self.o.fir(c["variant"], self.G[c["coeffs"]], abs_mode=c["abs_mode"])

    def up(self, c):
        return self.o.up(c["variant"], c["L"], self.G[c["coeffs"]])

    def mixer(self, c):
        return self.o.mixer(c["N"])

    def corr(self, c):
        return self.o.corr(c["N"], c["S"])
