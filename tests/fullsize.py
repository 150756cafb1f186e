"""Whole-output oracle runs at the BASELINE sizes, in parallel windows.

The oracle (test infrastructure) is scalar C; the full-size GPU tests compare
EVERY output with it by splitting the stream into independent windows that
run on a thread pool (ctypes releases the GIL during the C call):

* decimator: window [s0, s1) of outputs starts its input `lead` samples early
  (lead >= N - 1, a multiple of M) with an empty history, so its outputs from
  s0 on equal the single-call outputs (dnsampling_filters.h:140-167 reads at
  most N - 1 samples back);
* correlator: window [s, e) of samples is primed with the corr_halo() = N*S+2
  samples before it (history and the three registers), then stepped; the
  first window that detects holds the single call's first detection
  (correlators.h:291 stops there).

Worker count: the GPU box's share of host cores (16, the pool's limit for one
GPU), or fewer where the machine has fewer."""
from __future__ import annotations

import concurrent.futures as cf
import os

import numpy as np

WORKERS = max(1, min(16, os.cpu_count() or 1))


def decim_all(make, x: np.ndarray, M: int, lead: int, out: np.ndarray, win_out: int = 1 << 20) -> np.ndarray:
    """Fill out[:] with the decimator's outputs over all of x (fresh state).
    make() returns a fresh oracle decimator."""
    n_out = len(x) // M
    assert len(out) == n_out and lead % M == 0

    def job(s0):
        s1 = min(n_out, s0 + win_out)
        lo = max(0, M * s0 - lead)
        r = make().step(x[lo:M * s1])
        out[s0:s1] = r[(M * s0 - lo) // M:]

    with cf.ThreadPoolExecutor(WORKERS) as ex:
        list(ex.map(job, range(0, n_out, win_out)))
    return out


def up_all(make, x: np.ndarray, L: int, lead: int, out: np.ndarray, win_in: int = 1 << 18) -> np.ndarray:
    """Fill out[:] with the interpolator's L * len(x) outputs (fresh state):
    window [j0, j1) of inputs starts `lead` inputs early (lead >= the ring's
    taps / L inputs, upsampling_filters.h:166-184) and keeps outputs from
    L * j0 on."""
    n = len(x)
    assert len(out) == L * n

    def job(j0):
        j1 = min(n, j0 + win_in)
        lo = max(0, j0 - lead)
        r = make().step(x[lo:j1])
        out[L * j0:L * j1] = r[L * (j0 - lo):]

    with cf.ThreadPoolExecutor(WORKERS) as ex:
        list(ex.map(job, range(0, n, win_in)))
    return out


def first_bad(got: np.ndarray, want: np.ndarray):
    """Index of the first differing output (byte compare), or None."""
    g = np.ascontiguousarray(got).view(np.uint8).reshape(len(got), -1)
    w = np.ascontiguousarray(want).view(np.uint8).reshape(len(want), -1)
    assert g.shape == w.shape
    step = 1 << 22
    for s in range(0, len(g), step):
        ne = np.nonzero((g[s:s + step] != w[s:s + step]).any(axis=1))[0]
        if len(ne):
            return s + int(ne[0])
    return None


def corr_first(make, x: np.ndarray, N: int, S: int, win: int = 1 << 20):
    """The single call's first detection over all of x, from windows primed
    with their halos.  Returns (found, corrIndex, bitSamples, status) with
    corrIndex global, or (False, -1, None, None)."""
    n = len(x)
    halo = N * S + 2
    starts = list(range(0, n, win))

    def job(s):
        c = make()
        if s:
            c.prime(x[max(0, s - halo):s])
        found, idx = c.step(x[s:s + win])
        return (True, s + idx, c.bit_samples(), c.status()) if found else None

    with cf.ThreadPoolExecutor(WORKERS) as ex:
        futs = [ex.submit(job, s) for s in starts]
        for i, f in enumerate(futs):
            r = f.result()
            if r is not None:
                for g in futs[i + 1:]:
                    g.cancel()
                return r
    return False, -1, None, None
