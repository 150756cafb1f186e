"""Host-side mirror of SrcDsp's hot-path operator classes over libsrcdsp_hip.so.

Each class keeps the reference's name, constructor arguments, template
parameters (as constructor arguments) and ``step()`` contract; the compute runs
in the HIP kernels behind the C ABI (include/srcdsp_hip.h).  Buffers may be

* numpy arrays (host) -- staged through pinned memory, synchronous, like the
  reference's std::vector calls;
* torch tensors on the GPU -- device-resident, asynchronous on torch's current
  stream (the benchmark path).

Sample layouts match std::complex<T> in memory: complex<float> -> complex64[n]
(or float32[n,2]); complex<int16_t> -> int16[n,2]; complex<int32_t> -> int32[n,2];
float -> float32[n]; int16_t -> int16[n].

Like the reference, ``step(in, out)`` requires ``out`` pre-sized; ``step(in)``
allocates and returns it.  Size violations the reference asserts on raise
``SrcdspError`` (code SRCDSP_ERR_SIZE).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _capi as A

_ALIASES = {
    "cf32": "cf32", "complex<float>": "cf32", "std::complex<float>": "cf32",
    "ci16": "ci16", "complex<int16_t>": "ci16", "std::complex<int16_t>": "ci16", "complex<short>": "ci16",
    "ci32": "ci32", "complex<int32_t>": "ci32", "std::complex<int32_t>": "ci32", "complex<int>": "ci32",
    "f32": "f32", "float": "f32",
    "i16": "i16", "int16_t": "i16", "short": "i16",
    "i32": "i32", "int32_t": "i32", "int": "i32",
}
_NP = {"cf32": np.complex64, "ci16": np.int16, "ci32": np.int32, "f32": np.float32, "i16": np.int16,
       "i32": np.int32}
_BYTES = {"cf32": 8, "ci16": 4, "ci32": 8, "f32": 4, "i16": 2, "i32": 4}


def _kind(t: str) -> str:
    try:
        return _ALIASES[t.replace(" ", "")]
    except KeyError:
        raise TypeError(f"unknown sample/coefficient type {t!r}") from None


def _is_device(x) -> bool:
    return hasattr(x, "data_ptr") and getattr(x, "is_cuda", False)


def _nsamples(x, kind: str) -> int:
    if _is_device(x):
        nb = x.numel() * x.element_size()
    else:
        nb = np.asarray(x).nbytes
    return nb // _BYTES[kind]


def _host(x, kind: str) -> np.ndarray:
    a = np.ascontiguousarray(x)
    if kind in ("ci16", "ci32"):
        a = np.ascontiguousarray(a, _NP[kind]).reshape(-1, 2)
    elif kind == "cf32" and a.dtype != np.complex64:
        a = np.ascontiguousarray(a, np.float32).reshape(-1, 2).view(np.complex64).reshape(-1)
    else:
        a = np.ascontiguousarray(a, _NP[kind])
    return a


def _alloc_like(x, kind: str, n: int):
    if _is_device(x):
        import torch
        dt = {"cf32": torch.complex64, "ci16": torch.int16, "ci32": torch.int32, "f32": torch.float32,
              "i16": torch.int16, "i32": torch.int32}[kind]
        shape = (n, 2) if kind in ("ci16", "ci32") else (n,)
        return torch.empty(shape, dtype=dt, device=x.device)
    if kind in ("ci16", "ci32"):
        return np.zeros((n, 2), _NP[kind])
    return np.zeros(n, _NP[kind])


def _ptr(x) -> C.c_void_p:
    if _is_device(x):
        if not x.is_contiguous():
            raise ValueError("device buffers must be contiguous")
        return C.c_void_p(x.data_ptr())
    return C.c_void_p(x.ctypes.data)


def _stream(x):
    import torch
    return C.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)


def _coeffs(c, kind: str) -> np.ndarray:
    return np.ascontiguousarray(c, _NP[kind])


class _Handle:
    _destroy = ""
    _clone = ""  # the C ABI's copy of the object with its state (the reference classes are value types)

    def __copy__(self):
        """A copy as the reference's implicit copy constructor makes it: the
        configuration AND the current streaming state (history, phase,
        registers), so the copy continues the stream like the original."""
        if not self._clone:
            raise TypeError(f"{type(self).__name__} is not copyable")
        c = object.__new__(type(self))
        c.__dict__.update(self.__dict__)
        c._h = C.c_void_p()
        A.call(self._clone, self._h, C.byref(c._h))
        return c

    def __deepcopy__(self, memo):
        return self.__copy__()

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                getattr(A.lib(), self._destroy)(h)
            except Exception:
                pass
            self._h = C.c_void_p()


# ===================================================================== decimator
_DECIM_VARIANTS = {("cf32", "cf32", "cf32", "f32"): 0, ("ci16", "ci16", "ci32", "i32"): 1,
                   ("ci16", "ci16", "ci32", "i16"): 2, ("ci32", "ci16", "ci32", "i32"): 3}


class FilterDnsamplingFir(_Handle):
    """dsptl::FilterDnsamplingFir<InType, OutType, InternalType, CoefType, M>
    (dnsampling_filters.h:49-172).  ``abs_binding`` selects how coeffScaling
    sums |c| for float taps ('int' = canonical ::abs(int), 'fabs'); ``fp`` the
    float contract ('fma' = sequential FMA chain, 'strict' = mul then add)."""

    _destroy = "srcdsp_decim_destroy"
    _clone = "srcdsp_decim_clone"

    def __init__(self, coeffs, M: int = 4, InType="complex<float>", OutType="complex<float>",
                 InternalType="complex<float>", CoefType="float", abs_binding: str = "int", fp: str = "fma"):
        key = tuple(_kind(t) for t in (InType, OutType, InternalType, CoefType))
        if key not in _DECIM_VARIANTS:
            raise TypeError(f"FilterDnsamplingFir<{InType},{OutType},{InternalType},{CoefType}> "
                            "is not an instantiation the reference compiles (SURVEY §8c)")
        self.variant = _DECIM_VARIANTS[key]
        self.kin, self.kout, _, self.kc = key
        self.M = int(M)
        self.flags = (A.FLAG_ABS_FABS if abs_binding == "fabs" else 0) | (A.FLAG_FP_STRICT if fp == "strict" else 0)
        c = _coeffs(coeffs, self.kc)
        self._h = C.c_void_p()
        A.call("srcdsp_decim_create", C.byref(self._h), self.variant, self.M, c.ctypes.data, len(c), self.flags)
        self.ntaps = len(c)

    def setCoeffs(self, coeffs, require_multiple: bool = True):
        """dsptl_dnsampling_filters.h:114-134 (asserts N % M == 0)."""
        c = _coeffs(coeffs, self.kc)
        A.call("srcdsp_decim_set_coeffs", self._h, c.ctypes.data, len(c), int(require_multiple))
        self.ntaps = len(c)

    set_coeffs = setCoeffs

    def setLeftShiftBy2(self, left_shift: int):
        A.call("srcdsp_decim_set_left_shift", self._h, int(left_shift))

    set_left_shift = setLeftShiftBy2

    def reset(self):
        A.call("srcdsp_decim_reset", self._h)

    def state(self):
        cs, ls = C.c_uint(), C.c_int()
        hist = np.zeros(max(self.ntaps - 1, 0) * _BYTES[self.kin], np.uint8)
        A.call("srcdsp_decim_get_state", self._h, C.byref(cs), C.byref(ls),
               hist.ctypes.data if hist.size else None)
        return {"coeff_scaling": cs.value, "left_shift": ls.value, "history": hist}

    def step(self, inp, out=None):
        n_in = _nsamples(inp, self.kin)
        if out is None:
            out = _alloc_like(inp, self.kout, n_in // self.M)
        n_out = _nsamples(out, self.kout)
        if _is_device(inp):
            A.call("srcdsp_decim_step", self._h, _ptr(inp), n_in, _ptr(out), n_out, _stream(inp))
        else:
            x = _host(inp, self.kin)
            A.call("srcdsp_decim_step_host", self._h, _ptr(x), n_in, _ptr(out), n_out)
        return out


def decim_step_batched(filters, inp, out):
    """Step C same-configuration decimators over a [C, L] device batch in one
    launch (grid.y = channel)."""
    hs = (C.c_void_p * len(filters))(*[f._h.value for f in filters])
    f0 = filters[0]
    ch = len(filters)
    n_in = _nsamples(inp, f0.kin) // ch
    n_out = _nsamples(out, f0.kout) // ch
    if n_out * f0.M != n_in:
        raise ValueError("batched decimator: output length * M must equal input length")
    A.call("srcdsp_decim_step_batched", hs, ch, _ptr(inp), n_in, _ptr(out), n_out, n_in, _stream(inp))
    return out


# ===================================================================== FilterFir
_FIR_VARIANTS = {("cf32", "cf32", "cf32", "f32"): 0, ("f32", "cf32", "f32", "f32"): 1,
                 ("ci16", "ci16", "ci32", "i32"): 2}


class FilterFir(_Handle):
    """::FilterFir<InType, OutType, InternalType, CoefType> (filters.h:42-169)."""

    _destroy = "srcdsp_fir_destroy"
    _clone = "srcdsp_fir_clone"

    def __init__(self, coeffs, InType="complex<float>", OutType="complex<float>", InternalType="complex<float>",
                 CoefType="float", abs_binding: str = "int", fp: str = "fma"):
        key = tuple(_kind(t) for t in (InType, OutType, InternalType, CoefType))
        if key not in _FIR_VARIANTS:
            raise TypeError(f"FilterFir<{InType},{OutType},{InternalType},{CoefType}> is not an instantiation "
                            "the reference compiles (filters.h:164 needs a complex output)")
        self.variant = _FIR_VARIANTS[key]
        self.kin, self.kout, _, self.kc = key
        flags = (A.FLAG_ABS_FABS if abs_binding == "fabs" else 0) | (A.FLAG_FP_STRICT if fp == "strict" else 0)
        c = _coeffs(coeffs, self.kc)
        self._h = C.c_void_p()
        A.call("srcdsp_fir_create", C.byref(self._h), self.variant, c.ctypes.data, len(c), flags)

    def setCoeffs(self, coeffs):
        c = _coeffs(coeffs, self.kc)
        A.call("srcdsp_fir_set_coeffs", self._h, c.ctypes.data, len(c))

    set_coeffs = setCoeffs

    def reset(self):
        A.call("srcdsp_fir_reset", self._h)

    def step(self, inp, out=None):
        n = _nsamples(inp, self.kin)
        if out is None:
            out = _alloc_like(inp, self.kout, n)
        n_out = _nsamples(out, self.kout)
        if _is_device(inp):
            A.call("srcdsp_fir_step", self._h, _ptr(inp), n, _ptr(out), n_out, _stream(inp))
        else:
            x = _host(inp, self.kin)
            A.call("srcdsp_fir_step_host", self._h, _ptr(x), n, _ptr(out), n_out)
        return out


# ============================================================ FilterUpsamplingFir
_UP_VARIANTS = {("ci16", "ci16", "ci32", "i32"): 0, ("ci16", "ci16", "ci32", "i16"): 1,
                ("i16", "i16", "i32", "i32"): 2}


class FilterUpsamplingFir(_Handle):
    """dsptl::FilterUpsamplingFir<InType, OutType, InternalType, CoefType, L>
    (upsampling_filters.h:36-326)."""

    _destroy = "srcdsp_up_destroy"
    _clone = "srcdsp_up_clone"

    def __init__(self, coeffs, L: int = 4, InType="complex<int16_t>", OutType="complex<int16_t>",
                 InternalType="complex<int32_t>", CoefType="int32_t"):
        key = tuple(_kind(t) for t in (InType, OutType, InternalType, CoefType))
        if key not in _UP_VARIANTS:
            raise TypeError(f"FilterUpsamplingFir<{InType},{OutType},{InternalType},{CoefType}> is not an "
                            "instantiation the reference compiles (dsp_complex.h:87 needs integer types)")
        self.variant = _UP_VARIANTS[key]
        self.kin, self.kout, _, self.kc = key
        self.L = int(L)
        c = _coeffs(coeffs, self.kc)
        self._h = C.c_void_p()
        A.call("srcdsp_up_create", C.byref(self._h), self.variant, self.L, c.ctypes.data, len(c))

    def setCoefficients(self, coeffs):
        c = _coeffs(coeffs, self.kc)
        A.call("srcdsp_up_set_coeffs", self._h, c.ctypes.data, len(c))

    def reset(self):
        A.call("srcdsp_up_reset", self._h)

    def _lengths(self):
        a, b, r = C.c_int(), C.c_int(), C.c_int()
        A.call("srcdsp_up_get_length", self._h, C.byref(a), C.byref(b), C.byref(r))
        return a.value, b.value, r.value

    def getLength(self):
        return self._lengths()[0]

    def getImpLength(self):
        return self._lengths()[1]

    def getUpsamplingRatio(self):
        return self._lengths()[2]

    length = property(getLength)

    def step(self, inp, out=None, flush: bool = False, iterator: bool = False):
        n = _nsamples(inp, self.kin)
        if out is None:
            extra = self.L * (self.getLength() // self.L) if flush else 0
            out = _alloc_like(inp, self.kout, n * self.L + extra)
        n_out = _nsamples(out, self.kout)
        if _is_device(inp):
            A.call("srcdsp_up_step", self._h, _ptr(inp), n, _ptr(out), n_out, int(flush), int(iterator),
                   _stream(inp))
        else:
            x = _host(inp, self.kin)
            A.call("srcdsp_up_step_host", self._h, _ptr(x), n, _ptr(out), n_out, int(flush), int(iterator))
        return out


# ========================================================================= Mixer
class Mixer(_Handle):
    """dsptl::Mixer<complex<int16_t>, complex<int16_t>, int16_t, N> (mixers.h:130-188)."""

    _destroy = "srcdsp_mixer_destroy"
    _clone = "srcdsp_mixer_clone"

    def __init__(self, N: int = 4096, InType="complex<int16_t>", OutType="complex<int16_t>", PhaseType="int16_t"):
        if (_kind(InType), _kind(OutType), _kind(PhaseType)) != ("ci16", "ci16", "i16"):
            raise TypeError("only Mixer<complex<int16_t>, complex<int16_t>, int16_t, N> is defined (mixers.h:120-131)")
        self.N = int(N)
        self._h = C.c_void_p()
        A.call("srcdsp_mixer_create", C.byref(self._h), self.N)

    def setFrequency(self, f):
        A.call("srcdsp_mixer_set_frequency", self._h, C.c_float(f))

    def reset(self, f=0.0):
        A.call("srcdsp_mixer_reset", self._h, C.c_float(f))

    def adjustFrequency(self, f=0.0):
        A.call("srcdsp_mixer_adjust_frequency", self._h, C.c_float(f))

    set_frequency, adjust_frequency = setFrequency, adjustFrequency

    def setPhase(self, phi: int):
        """Not a reference method: set the phase accumulator, e.g.
        to phaseAt(k) for a buffer segment starting at sample k."""
        A.call("srcdsp_mixer_set_phase", self._h, int(phi))

    def phaseAt(self, k: int) -> int:
        """Closed form of mixers.h:177: the phase after k samples from now."""
        phi, freq = self.state()[:2]
        return (phi + (k % self.N) * freq) % self.N

    def state(self):
        p, fr, nom = C.c_int(), C.c_int(), C.c_float()
        A.call("srcdsp_mixer_get_state", self._h, C.byref(p), C.byref(fr), C.byref(nom))
        return p.value, fr.value, nom.value

    def table(self):
        t = np.zeros(self.N, np.int16)
        A.call("srcdsp_mixer_get_table", self._h, t.ctypes.data_as(A.I16P))
        return t

    def step(self, inp, out=None):
        n = _nsamples(inp, "ci16")
        if out is None:
            out = _alloc_like(inp, "ci16", n)
        if _is_device(inp):
            A.call("srcdsp_mixer_step", self._h, _ptr(inp), n, _ptr(out), _stream(inp))
        else:
            x = _host(inp, "ci16")
            A.call("srcdsp_mixer_step_host", self._h, _ptr(x), n, _ptr(out))
        return out


class MixerDecimatorChain:
    """mixer.step(in, tmp); decim.step(tmp, out) fused into one device pass
    (config 4).  Both operators' state advances exactly as the two calls."""

    def __init__(self, mixer: Mixer, decim: FilterDnsamplingFir):
        self.mixer, self.decim = mixer, decim

    def step(self, inp, out=None):
        n = _nsamples(inp, "ci16")
        if out is None:
            out = _alloc_like(inp, "ci16", n // self.decim.M)
        if not _is_device(inp):
            return self.decim.step(self.mixer.step(inp), out)
        A.call("srcdsp_mixdecim_step", self.mixer._h, self.decim._h, _ptr(inp), n, _ptr(out),
               _nsamples(out, "ci16"), _stream(inp))
        return out


# ======================================================== FixedPatternCorrelator
class FixedPatternCorrelator(_Handle):
    """dsptl::FixedPatternCorrelator<int16_t, int32_t, N, S> (correlators.h:54-316)."""

    _destroy = "srcdsp_corr_destroy"
    _clone = "srcdsp_corr_clone"

    def __init__(self, N: int = 32, S: int = 4, InType="int16_t", CompType="int32_t"):
        if (_kind(InType), _kind(CompType)) != ("i16", "i32"):
            raise TypeError("FixedPatternCorrelator is provided for <int16_t, int32_t, N, S>")
        self.N, self.S = int(N), int(S)
        self._h = C.c_void_p()
        A.call("srcdsp_corr_create", C.byref(self._h), self.N, self.S)

    def setPattern(self, pattern, thresholdCoeff: float = 0.8):
        p = np.ascontiguousarray(pattern, np.int32).reshape(-1, 2)
        if len(p) != self.N:
            raise ValueError(f"pattern must have N={self.N} complex<int32_t> entries")
        A.call("srcdsp_corr_set_pattern", self._h, p.ctypes.data_as(A.I32P), C.c_double(thresholdCoeff))

    set_pattern = setPattern

    def reset(self):
        A.call("srcdsp_corr_reset", self._h)

    def step(self, inp):
        """Returns (found, corrIndex); corrIndex is meaningful only if found."""
        n = _nsamples(inp, "ci16")
        found, idx = C.c_int(0), C.c_int(-1)
        if _is_device(inp):
            A.call("srcdsp_corr_step", self._h, _ptr(inp), n, C.byref(found), C.byref(idx), _stream(inp))
        else:
            x = _host(inp, "ci16")
            A.call("srcdsp_corr_step_host", self._h, _ptr(x), n, C.byref(found), C.byref(idx))
        return bool(found.value), idx.value

    def step_trace(self, inp):
        """step() as the reference's CREATE_DEBUG_FILES build runs it
        (correlators.h:253-257): (found, corrIndex, corr, energy), where corr[k]
        / energy[k] are corrValue[0] / energyValue[0] after each processed
        input sample (numpy uint32)."""
        n = _nsamples(inp, "ci16")
        found, idx, cnt = C.c_int(0), C.c_int(-1), C.c_size_t(0)
        corr, en = np.zeros(max(n, 1), np.uint32), np.zeros(max(n, 1), np.uint32)
        cp, ep = corr.ctypes.data_as(A.U32P), en.ctypes.data_as(A.U32P)
        if _is_device(inp):
            A.call("srcdsp_corr_step_trace", self._h, _ptr(inp), n, C.byref(found), C.byref(idx), cp, ep,
                   C.byref(cnt), _stream(inp))
        else:
            x = _host(inp, "ci16")
            A.call("srcdsp_corr_step_host_trace", self._h, _ptr(x), n, C.byref(found), C.byref(idx), cp, ep,
                   C.byref(cnt))
        k = cnt.value
        return bool(found.value), idx.value, corr[:k], en[:k]

    def prime(self, inp):
        """Not a reference method: leave the state step() would
        leave after streaming `inp` with no detection test -- seeds a time
        segment of a split buffer with its halo.  Device input only."""
        if not _is_device(inp):
            raise TypeError("prime() takes a device-resident buffer")
        A.call("srcdsp_corr_prime", self._h, _ptr(inp), _nsamples(inp, "ci16"), _stream(inp))

    def getRefBitSamples(self):
        b = np.zeros((self.N, 2), np.int16)
        A.call("srcdsp_corr_get_bit_samples", self._h, b.ctypes.data_as(A.I16P))
        return b

    bit_samples = getRefBitSamples

    def getStatus(self):
        e3, c3 = (C.c_uint32 * 3)(), (C.c_uint32 * 3)()
        ce, cs, tf = C.c_uint32(), C.c_int(), C.c_double()
        A.call("srcdsp_corr_get_status", self._h, e3, c3, C.byref(ce), C.byref(cs), C.byref(tf))
        return {"energy": list(e3), "corr": list(c3), "coeffs_energy": ce.value, "coeff_scaling": cs.value,
                "threshold_factor": tf.value}

    status = getStatus


def fill_synthetic(t, kind: str, seed: int = 0x5EED, channel: int = 0, offset: int = 0, lo: int = -2048,
                   hi: int = 2047):
    """Fill a device tensor with the counter-based synthetic samples."""
    k = {"cf32": 0, "ci16": 1}[kind]
    n = _nsamples(t, kind)
    A.call("srcdsp_fill_synthetic", _ptr(t), k, n, seed, channel, offset, lo, hi, _stream(t))
    return t


# ================================================================ FIFO (8f.3)
class FifoWithTimeTrack(_Handle):
    """dsptl::FifoWithTimeTrack<T, N> (buffers.h:58-459) with its N-element
    ring in HBM.  T is a numpy dtype (e.g. np.dtype(("<i2", 2)) for
    complex<int16_t>, np.float64, np.complex64).  write() takes host (numpy,
    staged through double-buffered pinned memory) or device (torch) input;
    read() returns (error, start, out) -- the reference's bool, its start
    after the call (raised to timeStart when it asked for older samples), and
    the values (device tensor when `out` is one, else numpy)."""

    _destroy = "srcdsp_fifo_destroy"

    def __init__(self, dtype, N: int, samplingFrequency: float = 0.0):
        self.dtype, self.N = np.dtype(dtype), int(N)
        self._h = C.c_void_p()
        A.call("srcdsp_fifo_create", C.byref(self._h), self.dtype.itemsize, self.N, float(samplingFrequency))

    def _count_elems(self, x) -> int:
        nb = x.numel() * x.element_size() if _is_device(x) else np.asarray(x).nbytes
        if nb % self.dtype.itemsize:
            raise ValueError("buffer is not a whole number of FIFO elements")
        return nb // self.dtype.itemsize

    def write(self, inp, seconds: int = 0, fracSeconds: float = 0.0):
        n = self._count_elems(inp)
        if _is_device(inp):
            A.call("srcdsp_fifo_write_device", self._h, _ptr(inp), n, int(seconds), float(fracSeconds), _stream(inp))
        else:
            x = np.ascontiguousarray(inp)  # raw element bytes (a subarray dtype would broadcast)
            A.call("srcdsp_fifo_write", self._h, C.c_void_p(x.ctypes.data), n, int(seconds), float(fracSeconds))

    def read(self, out, start: int):
        """out: an element count (host numpy result) or a buffer to fill."""
        if isinstance(out, (int, np.integer)):
            out = np.zeros(int(out), self.dtype)
        n = self._count_elems(out)
        st, err = C.c_uint64(int(start)), C.c_int(0)
        if _is_device(out):
            A.call("srcdsp_fifo_read", self._h, _ptr(out), n, C.byref(st), C.byref(err), _stream(out))
        else:
            A.call("srcdsp_fifo_read_host", self._h, C.c_void_p(out.ctypes.data), n, C.byref(st), C.byref(err))
        return bool(err.value), st.value, out

    def count(self) -> int:
        c = C.c_size_t()
        A.call("srcdsp_fifo_count", self._h, C.byref(c))
        return c.value

    def reset(self):
        A.call("srcdsp_fifo_reset", self._h)

    def state(self):
        """(writePtr, timeStart, timeEnd, rolloverFlag) -- what dumpInfo() prints."""
        wp, ts, te, ro = C.c_size_t(), C.c_uint64(), C.c_uint64(), C.c_int()
        A.call("srcdsp_fifo_get_state", self._h, C.byref(wp), C.byref(ts), C.byref(te), C.byref(ro))
        return wp.value, ts.value, te.value, bool(ro.value)

    def getAbsoluteTime(self, timePoint: int, fracTimePoint: float = 0.0):
        s, fs = C.c_uint(), C.c_double()
        A.call("srcdsp_fifo_get_absolute_time", self._h, int(timePoint), float(fracTimePoint), C.byref(s),
               C.byref(fs))
        return s.value, fs.value
