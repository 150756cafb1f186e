"""Host stand-in for the srcdsp_amd operators bench.py's decim workload uses
(test infrastructure only).

bench.main(argv, S=<this module>, dev=bench.HostDevice()) then runs the whole
N > 1 path of the driver's command on CPU ranks over gloo -- warm-up, timed
steps, max over ranks, the parity digests, configs[2]'s share, the gather to
rank 0 and the JSON line -- with the oracle's decimator behind the
FilterDnsamplingFir / fill_synthetic / decim_step_batched calls, so a Python
error anywhere on that path fails `pytest -m "not gpu"` instead of a GPU
lease.  Its times are host times of the oracle, never measurements.

STUB_CORRUPT_CHANNEL=<id> flips one input sample of that channel id, so the
parity check must report exactly one mismatching channel."""
import os

import numpy as np

import pyoracle

_O = pyoracle.Oracle(1)  # the FMA contract: bench.py's default --fp fma


def lib():
    return None


def fill_synthetic(t, kind, seed, channel, lo=None, hi=None):
    assert kind == "cf32" and t.dtype.is_complex and t.device.type == "cpu"
    x = _O.gen_cf32(seed, channel, 0, t.numel())
    if os.environ.get("STUB_CORRUPT_CHANNEL") == str(channel):
        x[len(x) // 2] += 1.0
    t.numpy()[:] = x


class FilterDnsamplingFir:
    def __init__(self, coeffs, M=4, fp="fma"):
        assert fp == "fma" and M == 4
        self.c = np.asarray(coeffs, np.float32)
        self.M = M
        self.reset()

    def reset(self):
        self._f = _O.decim(0, self.M, self.c)

    def step(self, x, y=None):
        r = self._f.step(x.numpy())
        if y is None:
            import torch
            return torch.from_numpy(r)
        y.numpy()[:] = r
        return y


def decim_step_batched(filters, x, y):
    for k, f in enumerate(filters):
        f.step(x[k], y[k])
    return y
