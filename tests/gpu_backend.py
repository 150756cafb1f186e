"""Replay backend running the golden scripts through srcdsp_amd (the HIP path).

``device=True`` feeds torch tensors resident on cuda:0 (srcdsp_*_step, the
async device entry points); ``device=False`` feeds numpy arrays
(srcdsp_*_step_host, pinned staging).  Results come back as numpy for the
byte comparison in replay.py.
"""
from __future__ import annotations

import numpy as np

import srcdsp_amd as S
from replay import load_golden

_DECIM_T = {0: ("complex<float>", "complex<float>", "complex<float>", "float"),
            1: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t"),
            2: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int16_t"),
            3: ("complex<int32_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")}
_FIR_T = {0: ("complex<float>", "complex<float>", "complex<float>", "float"),
          1: ("float", "complex<float>", "float", "float"),
          2: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")}
_UP_T = {0: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t"),
         1: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int16_t"),
         2: ("int16_t", "int16_t", "int32_t", "int32_t")}


def to_dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).to("cuda:0")


def to_host(t):
    return t.cpu().numpy()


class _Wrap:
    """Adapts an operator so step() takes/returns numpy, optionally via the device."""

    def __init__(self, op, device):
        self.op, self.device = op, device

    def __getattr__(self, k):
        return getattr(self.op, k)

    def step(self, x, *args):
        if self.device:
            r = self.op.step(to_dev(x), None, *args) if args else self.op.step(to_dev(x))
            if isinstance(r, tuple):
                return r
            return to_host(r)
        return self.op.step(x, None, *args) if args else self.op.step(x)


class _UpWrap(_Wrap):
    def step(self, x, flush=False, iterator=False):
        if self.device:
            return to_host(self.op.step(to_dev(x), None, flush, iterator))
        return self.op.step(x, None, flush, iterator)


class _CorrWrap(_Wrap):
    def step(self, x):
        return self.op.step(to_dev(x) if self.device else x)


class GpuBackend:
    def __init__(self, fp: str, device: bool = True):
        self.fp, self.device = fp, device
        self.G = load_golden()

    def decim(self, c):
        t = _DECIM_T[c["variant"]]
        op = S.FilterDnsamplingFir(self.G[c["coeffs"]], c["M"], *t,
                                   abs_binding="fabs" if c["abs_mode"] else "int", fp=self.fp)
        return _Wrap(op, self.device)

    def fir(self, c):
        op = S.FilterFir(self.G[c["coeffs"]], *_FIR_T[c["variant"]],
                         abs_binding="fabs" if c["abs_mode"] else "int", fp=self.fp)
        return _Wrap(op, self.device)

    def up(self, c):
        return _UpWrap(S.FilterUpsamplingFir(self.G[c["coeffs"]], c["L"], *_UP_T[c["variant"]]), self.device)

    def mixer(self, c):
        return _Wrap(S.Mixer(c["N"]), self.device)

    def corr(self, c):
        return _CorrWrap(S.FixedPatternCorrelator(c["N"], c["S"]), self.device)
