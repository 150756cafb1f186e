"""ctypes front-end to the oracle (test infrastructure only).

Two back-ends expose the same Python interface:

* ``Oracle(fp_mode)`` -- the plain-C restatement ``oracle/liboracle.so``;
* ``Reference(flavour)`` -- the real SrcDsp headers compiled from
  ``/root/reference`` into ``oracle/_ref/<flavour>/`` ("strict" = -O2,
  "fma" = -O2 -mfma).

Only tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline leg may
import this module.  The product path (``srcdsp_amd``) never does.

Sample layouts (identical to std::complex<T> in memory):
  cf32 -> numpy complex64 [n];  ci16 -> int16 [n, 2];  ci32 -> int32 [n, 2];
  f32 -> float32 [n];  i16 -> int16 [n].
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# (in, out, coef) per variant -- matches oracle/refbuild/ref_api.h
DECIM_VARIANTS = {0: ("cf32", "cf32", "f32"), 1: ("ci16", "ci16", "i32"),
                  2: ("ci16", "ci16", "i16"), 3: ("ci32", "ci16", "i32")}
FIR_VARIANTS = {0: ("cf32", "cf32", "f32"), 1: ("f32", "cf32", "f32"), 2: ("ci16", "ci16", "i32")}
UP_VARIANTS = {0: ("ci16", "ci16", "i32"), 1: ("ci16", "ci16", "i16"), 2: ("i16", "i16", "i32")}

_NP = {"f32": np.float32, "i16": np.int16, "i32": np.int32}


def empty(kind: str, n: int) -> np.ndarray:
    if kind == "cf32":
        return np.zeros(n, np.complex64)
    if kind == "ci16":
        return np.zeros((n, 2), np.int16)
    if kind == "ci32":
        return np.zeros((n, 2), np.int32)
    return np.zeros(n, _NP[kind])


def as_kind(a, kind: str) -> np.ndarray:
    if kind == "cf32":
        return np.ascontiguousarray(a, np.complex64)
    if kind == "ci16":
        return np.ascontiguousarray(a, np.int16).reshape(-1, 2)
    if kind == "ci32":
        return np.ascontiguousarray(a, np.int32).reshape(-1, 2)
    return np.ascontiguousarray(a, _NP[kind])


def coeff_array(c, kind: str) -> np.ndarray:
    return np.ascontiguousarray(c, _NP[kind])


def _ptr(a: np.ndarray):
    return C.c_void_p(a.ctypes.data)


def _sig(lib, name, res, *args):
    f = getattr(lib, name)
    f.restype = res
    f.argtypes = list(args)
    return f


VP, I, U, L, F, D = C.c_void_p, C.c_int, C.c_uint, C.c_long, C.c_float, C.c_double


class _Handle:
    def __init__(self, h, destroy):
        if not h:
            raise ValueError("oracle/reference rejected the configuration")
        self._h = h
        self._destroy = destroy

    def __del__(self):
        if getattr(self, "_h", None):
            self._destroy(self._h)
            self._h = None


# ----------------------------------------------------------------------------
# C restatement
# ----------------------------------------------------------------------------
class Oracle:
    """The plain-C restatement, fp_mode 0 = strict (mul then add), 1 = fma."""

    def __init__(self, fp_mode: int = 0, abs_mode: int = 0, path: str | None = None):
        self.lib = C.CDLL(path or os.path.join(HERE, "liboracle.so"))
        self.fp_mode, self.abs_mode = fp_mode, abs_mode
        lib = self.lib
        self.f = {
            "decim_create": _sig(lib, "orc_decim_create", VP, I, U, VP, I, I, I),
            "decim_step": _sig(lib, "orc_decim_step", None, VP, VP, L, VP),
            "decim_reset": _sig(lib, "orc_decim_reset", None, VP),
            "decim_ls": _sig(lib, "orc_decim_set_left_shift", None, VP, I),
            "decim_scaling": _sig(lib, "orc_decim_coeff_scaling", U, VP),
            "decim_set": _sig(lib, "orc_decim_set_coeffs", I, VP, VP, I, I),
            "fir_set": _sig(lib, "orc_fir_set_coeffs", I, VP, VP, I, I),
            "decim_destroy": _sig(lib, "orc_decim_destroy", None, VP),
            "fir_create": _sig(lib, "orc_fir_create", VP, I, VP, I, I, I),
            "fir_step": _sig(lib, "orc_fir_step", None, VP, VP, L, VP),
            "fir_reset": _sig(lib, "orc_fir_reset", None, VP),
            "fir_destroy": _sig(lib, "orc_fir_destroy", None, VP),
            "up_create": _sig(lib, "orc_up_create", VP, I, U, VP, I),
            "up_step": _sig(lib, "orc_up_step", None, VP, VP, L, VP, I, I),
            "up_reset": _sig(lib, "orc_up_reset", None, VP),
            "up_len": _sig(lib, "orc_up_get_length", I, VP),
            "up_destroy": _sig(lib, "orc_up_destroy", None, VP),
            "mix_create": _sig(lib, "orc_mixer_create", VP, U),
            "mix_table": _sig(lib, "orc_mixer_table", None, VP, VP),
            "mix_reset": _sig(lib, "orc_mixer_reset", None, VP, F),
            "mix_setf": _sig(lib, "orc_mixer_set_frequency", None, VP, F),
            "mix_adj": _sig(lib, "orc_mixer_adjust_frequency", None, VP, F),
            "mix_state": _sig(lib, "orc_mixer_state", None, VP, VP, VP, VP),
            "mix_step": _sig(lib, "orc_mixer_step", None, VP, VP, L, VP),
            "mix_destroy": _sig(lib, "orc_mixer_destroy", None, VP),
            "corr_create": _sig(lib, "orc_corr_create", VP, U, U),
            "corr_pattern": _sig(lib, "orc_corr_set_pattern", None, VP, VP, D),
            "corr_reset": _sig(lib, "orc_corr_reset", None, VP),
            "corr_step": _sig(lib, "orc_corr_step", I, VP, VP, L, VP),
            "corr_prime": _sig(lib, "orc_corr_prime", None, VP, VP, L),
            "corr_registers": _sig(lib, "orc_corr_registers", None, VP, VP, L, VP, VP),
            "corr_bits": _sig(lib, "orc_corr_bit_samples", None, VP, VP),
            "corr_status": _sig(lib, "orc_corr_status", None, VP, VP, VP, VP, VP, VP),
            "corr_destroy": _sig(lib, "orc_corr_destroy", None, VP),
            "gen_cf32": _sig(lib, "orc_gen_cf32", None, C.c_uint64, C.c_uint64, C.c_uint64, L, I, I, VP),
            "gen_ci16": _sig(lib, "orc_gen_ci16", None, C.c_uint64, C.c_uint64, C.c_uint64, L, I, I, VP),
            "fifo_create": _sig(lib, "orc_fifo_create", VP, C.c_size_t, C.c_size_t, D),
            "fifo_write": _sig(lib, "orc_fifo_write", I, VP, VP, C.c_size_t, U, D),
            "fifo_read": _sig(lib, "orc_fifo_read", I, VP, VP, C.c_size_t, VP),
            "fifo_count": _sig(lib, "orc_fifo_count", C.c_size_t, VP),
            "fifo_reset": _sig(lib, "orc_fifo_reset", None, VP),
            "fifo_abs": _sig(lib, "orc_fifo_absolute_time", None, VP, C.c_uint64, D, VP, VP),
            "fifo_destroy": _sig(lib, "orc_fifo_destroy", None, VP),
        }

    def fifo(self, dtype, N, sampling_frequency=0.0):
        """FifoWithTimeTrack<T, N> restated (buffers.h:58-459); dtype = numpy
        dtype of one element (e.g. complex<int16_t> -> ("<i2", 2) rows)."""
        return _Fifo(self, np.dtype(dtype), N, sampling_frequency)

    # factories --------------------------------------------------------------
    def decim(self, variant, M, coeffs, abs_mode=None):
        return _Decim(self, variant, M, coeffs, self.abs_mode if abs_mode is None else abs_mode)

    def fir(self, variant, coeffs, abs_mode=None):
        return _Fir(self, variant, coeffs, self.abs_mode if abs_mode is None else abs_mode)

    def up(self, variant, L_, coeffs):
        return _Up(self, variant, L_, coeffs)

    def mixer(self, N=4096):
        return _Mixer(self, N)

    def corr(self, N, S):
        return _Corr(self, N, S)

    def gen_cf32(self, seed, ch, off, n, lo=-2048, hi=2047):
        out = np.zeros(n, np.complex64)
        self.f["gen_cf32"](seed, ch, off, n, lo, hi, _ptr(out))
        return out

    def gen_ci16(self, seed, ch, off, n, lo=-8192, hi=8191):
        out = np.zeros((n, 2), np.int16)
        self.f["gen_ci16"](seed, ch, off, n, lo, hi, _ptr(out))
        return out


class _Decim(_Handle):
    def __init__(self, o, variant, M, coeffs, abs_mode):
        self.o, self.variant, self.M, self.abs_mode = o, variant, M, abs_mode
        self.kin, self.kout, self.kc = DECIM_VARIANTS[variant]
        c = coeff_array(coeffs, self.kc)
        super().__init__(o.f["decim_create"](variant, M, _ptr(c), len(c), abs_mode, o.fp_mode),
                         o.f["decim_destroy"])

    def step(self, x):
        x = as_kind(x, self.kin)
        y = empty(self.kout, len(x) // self.M)
        self.o.f["decim_step"](self._h, _ptr(x), len(x), _ptr(y))
        return y

    def reset(self):
        self.o.f["decim_reset"](self._h)

    def set_left_shift(self, ls):
        self.o.f["decim_ls"](self._h, ls)

    def set_coeffs(self, coeffs):
        c = coeff_array(coeffs, self.kc)
        self.o.f["decim_set"](self._h, _ptr(c), len(c), self.abs_mode)

    @property
    def coeff_scaling(self):
        return self.o.f["decim_scaling"](self._h)


class _Fir(_Handle):
    def __init__(self, o, variant, coeffs, abs_mode):
        self.o, self.abs_mode = o, abs_mode
        self.kin, self.kout, self.kc = FIR_VARIANTS[variant]
        c = coeff_array(coeffs, self.kc)
        super().__init__(o.f["fir_create"](variant, _ptr(c), len(c), abs_mode, o.fp_mode), o.f["fir_destroy"])

    def step(self, x):
        x = as_kind(x, self.kin)
        y = empty(self.kout, len(x))
        self.o.f["fir_step"](self._h, _ptr(x), len(x), _ptr(y))
        return y

    def reset(self):
        self.o.f["fir_reset"](self._h)

    def set_coeffs(self, coeffs):
        c = coeff_array(coeffs, self.kc)
        self.o.f["fir_set"](self._h, _ptr(c), len(c), self.abs_mode)


class _Up(_Handle):
    def __init__(self, o, variant, L_, coeffs):
        self.o, self.L = o, L_
        self.kin, self.kout, self.kc = UP_VARIANTS[variant]
        c = coeff_array(coeffs, self.kc)
        super().__init__(o.f["up_create"](variant, L_, _ptr(c), len(c)), o.f["up_destroy"])

    @property
    def length(self):
        return self.o.f["up_len"](self._h)

    def step(self, x, flush=False, iterator=False):
        x = as_kind(x, self.kin)
        n_out = len(x) * self.L + (self.L * (self.length // self.L) if flush else 0)
        y = empty(self.kout, n_out)
        self.o.f["up_step"](self._h, _ptr(x), len(x), _ptr(y), int(flush), int(iterator))
        return y

    def reset(self):
        self.o.f["up_reset"](self._h)


class _Mixer(_Handle):
    def __init__(self, o, N):
        self.o, self.N = o, N
        super().__init__(o.f["mix_create"](N), o.f["mix_destroy"])

    def table(self):
        t = np.zeros(self.N, np.int16)
        self.o.f["mix_table"](self._h, _ptr(t))
        return t

    def reset(self, f=0.0):
        self.o.f["mix_reset"](self._h, f)

    def set_frequency(self, f):
        self.o.f["mix_setf"](self._h, f)

    def adjust_frequency(self, f):
        self.o.f["mix_adj"](self._h, f)

    def state(self):
        p, fr, nom = C.c_int(), C.c_int(), C.c_float()
        self.o.f["mix_state"](self._h, C.byref(p), C.byref(fr), C.byref(nom))
        return p.value, fr.value, nom.value

    def step(self, x):
        x = as_kind(x, "ci16")
        y = empty("ci16", len(x))
        self.o.f["mix_step"](self._h, _ptr(x), len(x), _ptr(y))
        return y


class _Corr(_Handle):
    def __init__(self, o, N, S):
        self.o, self.N, self.S = o, N, S
        super().__init__(o.f["corr_create"](N, S), o.f["corr_destroy"])

    def set_pattern(self, pattern, threshold_coeff=0.8):
        p = np.ascontiguousarray(pattern, np.int32).reshape(-1, 2)
        assert len(p) == self.N
        self.o.f["corr_pattern"](self._h, _ptr(p), threshold_coeff)

    def reset(self):
        self.o.f["corr_reset"](self._h)

    def step(self, x):
        x = as_kind(x, "ci16")
        idx = C.c_int(-12345)
        found = self.o.f["corr_step"](self._h, _ptr(x), len(x), C.byref(idx))
        return bool(found), idx.value

    def prime(self, x):
        """State after streaming x with no detection (not a reference call)."""
        x = as_kind(x, "ci16")
        self.o.f["corr_prime"](self._h, _ptr(x), len(x))

    def registers(self, x):
        """Stream x with no detection (not a reference call) and return every
        sample's (corrValue[0], energyValue[0]) as uint32 arrays
        (correlators.h:244-250)."""
        x = as_kind(x, "ci16")
        c = np.zeros(len(x), np.uint32)
        e = np.zeros(len(x), np.uint32)
        self.o.f["corr_registers"](self._h, _ptr(x), len(x), _ptr(c), _ptr(e))
        return c, e

    def bit_samples(self):
        b = np.zeros((self.N, 2), np.int16)
        self.o.f["corr_bits"](self._h, _ptr(b))
        return b

    def status(self):
        e3 = np.zeros(3, np.uint32)
        c3 = np.zeros(3, np.uint32)
        ce, cs, tf = C.c_uint32(), C.c_int(), C.c_double()
        self.o.f["corr_status"](self._h, _ptr(e3), _ptr(c3), C.byref(ce), C.byref(cs), C.byref(tf))
        return {"energy": e3.tolist(), "corr": c3.tolist(), "coeffs_energy": ce.value,
                "coeff_scaling": cs.value, "threshold_factor": tf.value}


class _Fifo(_Handle):
    """Common Python face of the FIFO restatement and the reference build."""

    def __init__(self, o, dtype, N, fs):
        self.o, self.dtype, self.N = o, dtype, N
        super().__init__(o.f["fifo_create"](dtype.itemsize, N, fs), o.f["fifo_destroy"])

    def write(self, x, seconds=0, frac_seconds=0.0):
        x = np.ascontiguousarray(x)  # raw element bytes (a subarray dtype would broadcast)
        assert x.nbytes % self.dtype.itemsize == 0
        return self.o.f["fifo_write"](self._h, _ptr(x), x.nbytes // self.dtype.itemsize, seconds, frac_seconds)

    def read(self, n, start):
        """-> (error flag as the reference's bool, start after the call, data)"""
        out = np.zeros(n, self.dtype)
        st = C.c_uint64(start)
        err = self.o.f["fifo_read"](self._h, _ptr(out), n, C.byref(st))
        return err, st.value, out

    def count(self):
        return int(self.o.f["fifo_count"](self._h))

    def reset(self):
        self.o.f["fifo_reset"](self._h)

    def absolute_time(self, time_point, frac=0.0):
        sec, fs = C.c_uint(), C.c_double()
        self.o.f["fifo_abs"](self._h, time_point, frac, C.byref(sec), C.byref(fs))
        return sec.value, fs.value


# ----------------------------------------------------------------------------
# real reference (oracle/_ref)
# ----------------------------------------------------------------------------
def reference_available(flavour: str = "strict") -> bool:
    d = os.path.join(HERE, "_ref", flavour)
    return all(os.path.exists(os.path.join(d, f)) for f in
               ("libref_decim_old.so", "libref_decim_new.so", "libref_decim_fabs.so", "libref_ops.so"))


class Reference:
    """The real SrcDsp templates, compiled by oracle/refbuild (flavour strict|fma)."""

    def __init__(self, flavour: str = "strict"):
        d = os.path.join(HERE, "_ref", flavour)
        self.flavour = flavour
        self.old = C.CDLL(os.path.join(d, "libref_decim_old.so"))
        self.new = C.CDLL(os.path.join(d, "libref_decim_new.so"))
        self.fabs = C.CDLL(os.path.join(d, "libref_decim_fabs.so"))
        self.ops = C.CDLL(os.path.join(d, "libref_ops.so"))
        f = {}
        for pre, lib in (("ref_decim", self.old), ("ref_decim2", self.new)):
            f[pre + "_create"] = _sig(lib, pre + "_create", VP, I, U, VP, I)
            f[pre + "_step"] = _sig(lib, pre + "_step", None, VP, VP, L, VP)
            f[pre + "_reset"] = _sig(lib, pre + "_reset", None, VP)
            f[pre + "_ls"] = _sig(lib, pre + "_set_left_shift", None, VP, I)
            f[pre + "_destroy"] = _sig(lib, pre + "_destroy", None, VP)
        f["ref_decim2_set_coeffs"] = _sig(self.new, "ref_decim2_set_coeffs", None, VP, VP, I)
        f["ref_decim_fabs_create"] = _sig(self.fabs, "ref_decim_fabs_create", VP, I, U, VP, I)
        f["ref_decim_fabs_step"] = _sig(self.fabs, "ref_decim_fabs_step", None, VP, VP, L, VP)
        f["ref_decim_fabs_destroy"] = _sig(self.fabs, "ref_decim_fabs_destroy", None, VP)
        o = self.ops
        f.update({
            "fir_create": _sig(o, "ref_fir_create", VP, I, VP, I),
            "fir_set": _sig(o, "ref_fir_set_coeffs", None, VP, VP, I),
            "fir_reset": _sig(o, "ref_fir_reset", None, VP),
            "fir_step": _sig(o, "ref_fir_step", None, VP, VP, L, VP),
            "fir_destroy": _sig(o, "ref_fir_destroy", None, VP),
            "up_create": _sig(o, "ref_up_create", VP, I, U, VP, I),
            "up_reset": _sig(o, "ref_up_reset", None, VP),
            "up_len": _sig(o, "ref_up_get_length", I, VP),
            "up_implen": _sig(o, "ref_up_get_imp_length", I, VP),
            "up_step": _sig(o, "ref_up_step", None, VP, VP, L, VP, I),
            "up_step_iter": _sig(o, "ref_up_step_iter", None, VP, VP, L, VP, I),
            "up_destroy": _sig(o, "ref_up_destroy", None, VP),
            "mix_create": _sig(o, "ref_mixer_create", VP, U),
            "mix_reset": _sig(o, "ref_mixer_reset", None, VP, F),
            "mix_setf": _sig(o, "ref_mixer_set_frequency", None, VP, F),
            "mix_adj": _sig(o, "ref_mixer_adjust_frequency", None, VP, F),
            "mix_step": _sig(o, "ref_mixer_step", None, VP, VP, L, VP),
            "mix_state": _sig(o, "ref_mixer_state", None, VP, VP, VP, VP),
            "mix_table": _sig(o, "ref_mixer_table", None, VP, VP),
            "mix_destroy": _sig(o, "ref_mixer_destroy", None, VP),
            "corr_create": _sig(o, "ref_corr_create", VP, U, U),
            "corr_pattern": _sig(o, "ref_corr_set_pattern", None, VP, VP, D),
            "corr_reset": _sig(o, "ref_corr_reset", None, VP),
            "corr_step": _sig(o, "ref_corr_step", I, VP, VP, L, VP),
            "corr_bits": _sig(o, "ref_corr_bit_samples", None, VP, VP),
            "corr_status": _sig(o, "ref_corr_status", None, VP, VP, VP, VP, VP, VP),
            "corr_destroy": _sig(o, "ref_corr_destroy", None, VP),
        })
        self.f = f

    def decim(self, variant, M, coeffs, header="old"):
        return _RefDecim(self, variant, M, coeffs, header)

    def fir(self, variant, coeffs):
        return _RefFir(self, variant, coeffs)

    def up(self, variant, L_, coeffs):
        return _RefUp(self, variant, L_, coeffs)

    def mixer(self, N=4096):
        return _RefMixer(self, N)

    def corr(self, N, S):
        return _RefCorr(self, N, S)


class _RefDecim(_Handle):
    def __init__(self, r, variant, M, coeffs, header):
        self.r, self.M = r, M
        self.kin, self.kout, self.kc = DECIM_VARIANTS[variant]
        self.pre = {"old": "ref_decim", "new": "ref_decim2", "fabs": "ref_decim_fabs"}[header]
        c = coeff_array(coeffs, self.kc)
        super().__init__(r.f[self.pre + "_create"](variant, M, _ptr(c), len(c)), r.f[self.pre + "_destroy"])

    def step(self, x):
        x = as_kind(x, self.kin)
        y = empty(self.kout, len(x) // self.M)
        self.r.f[self.pre + "_step"](self._h, _ptr(x), len(x), _ptr(y))
        return y

    def reset(self):
        self.r.f[self.pre + "_reset"](self._h)

    def set_left_shift(self, ls):
        self.r.f[self.pre + "_ls"](self._h, ls)

    def set_coeffs(self, coeffs):
        assert self.pre == "ref_decim2"
        c = coeff_array(coeffs, self.kc)
        self.r.f["ref_decim2_set_coeffs"](self._h, _ptr(c), len(c))


class _RefFir(_Handle):
    def __init__(self, r, variant, coeffs):
        self.r = r
        self.kin, self.kout, self.kc = FIR_VARIANTS[variant]
        c = coeff_array(coeffs, self.kc)
        super().__init__(r.f["fir_create"](variant, _ptr(c), len(c)), r.f["fir_destroy"])

    def step(self, x):
        x = as_kind(x, self.kin)
        y = empty(self.kout, len(x))
        self.r.f["fir_step"](self._h, _ptr(x), len(x), _ptr(y))
        return y

    def reset(self):
        self.r.f["fir_reset"](self._h)

    def set_coeffs(self, coeffs):
        c = coeff_array(coeffs, self.kc)
        self.r.f["fir_set"](self._h, _ptr(c), len(c))


class _RefUp(_Handle):
    def __init__(self, r, variant, L_, coeffs):
        self.r, self.L = r, L_
        self.kin, self.kout, self.kc = UP_VARIANTS[variant]
        c = coeff_array(coeffs, self.kc)
        super().__init__(r.f["up_create"](variant, L_, _ptr(c), len(c)), r.f["up_destroy"])

    @property
    def length(self):
        return self.r.f["up_len"](self._h)

    @property
    def imp_length(self):
        return self.r.f["up_implen"](self._h)

    def step(self, x, flush=False, iterator=False):
        x = as_kind(x, self.kin)
        n_out = len(x) * self.L + (self.L * (self.length // self.L) if flush else 0)
        y = empty(self.kout, n_out)
        fn = self.r.f["up_step_iter" if iterator else "up_step"]
        fn(self._h, _ptr(x), len(x), _ptr(y), int(flush))
        return y

    def reset(self):
        self.r.f["up_reset"](self._h)


class _RefMixer(_Mixer):
    def __init__(self, r, N):
        self.o, self.N = r, N
        _Handle.__init__(self, r.f["mix_create"](N), r.f["mix_destroy"])


class _RefCorr(_Corr):
    def __init__(self, r, N, S):
        self.o, self.N, self.S = r, N, S
        h = r.f["corr_create"](N, S)
        _Handle.__init__(self, h, r.f["corr_destroy"])


# ------------------------------------------------ reference buffers.h / files
class ReferenceIO:
    """buffers.h FifoWithTimeTrack and dsptl_files.h binary I/Q functions of
    the reference build (oracle/_ref/<flavour>/libref_io.so)."""
    KINDS = {("<f8", 15): 0, ("<i2", 64): 1, ("<i2", 1000): 2}

    def __init__(self, flavour: str = "strict"):
        lib = C.CDLL(os.path.join(HERE, "_ref", flavour, "libref_io.so"))
        self.f = {
            "create": _sig(lib, "ref_fifo_create", VP, I, D),
            "write": _sig(lib, "ref_fifo_write", None, VP, VP, L, U, D),
            "read": _sig(lib, "ref_fifo_read", I, VP, VP, L, VP),
            "count": _sig(lib, "ref_fifo_count", C.c_ulong, VP),
            "reset": _sig(lib, "ref_fifo_reset", None, VP),
            "abs": _sig(lib, "ref_fifo_abs_time", None, VP, C.c_uint64, D, VP, VP),
            "destroy": _sig(lib, "ref_fifo_destroy", None, VP),
            "iq_save": _sig(lib, "ref_iq_save", None, C.c_char_p, I, VP, L),
            "iq_read": _sig(lib, "ref_iq_read", L, C.c_char_p, I, VP, L),
        }

    def fifo(self, kind: int, fs: float = 0.0):
        """kind 0: <double, 15>, 1: <complex<int16_t>, 64>, 2: <complex<int16_t>, 1000>"""
        return _RefFifo(self, kind, fs)

    def iq_save(self, path: str, x: np.ndarray):
        x = np.ascontiguousarray(x)
        t = 0 if x.dtype == np.int16 else 1
        self.f["iq_save"](path.encode(), t, _ptr(x), x.shape[0])

    def iq_read(self, path: str, component_dtype, cap: int = 1 << 22):
        t = 0 if np.dtype(component_dtype) == np.int16 else 1
        out = np.zeros((cap, 2), component_dtype)
        n = self.f["iq_read"](path.encode(), t, _ptr(out), cap)
        return out[:min(n, cap)], n


class _RefFifo:
    def __init__(self, r, kind, fs):
        self.r, self.kind = r, kind
        self.dtype, self.N = ((np.dtype("<f8"), 15), (np.dtype(("<i2", 2)), 64), (np.dtype(("<i2", 2)), 1000))[kind]
        self._h = r.f["create"](kind, fs)

    def __del__(self):
        if getattr(self, "_h", None):
            self.r.f["destroy"](self._h)
            self._h = None

    def write(self, x, seconds=0, frac_seconds=0.0):
        x = np.ascontiguousarray(x)  # raw element bytes (a subarray dtype would broadcast)
        n = x.nbytes // self.dtype.itemsize
        assert n * self.dtype.itemsize == x.nbytes and n < self.N, "the reference asserts inSize < N"
        self.r.f["write"](self._h, _ptr(x), n, seconds, frac_seconds)
        return 0

    def read(self, n, start):
        assert n > 0, "the reference asserts out.size() != 0"
        out = np.zeros(n, self.dtype)
        st = C.c_uint64(start)
        err = self.r.f["read"](self._h, _ptr(out), n, C.byref(st))
        return err, st.value, out

    def count(self):
        return int(self.r.f["count"](self._h))

    def reset(self):
        self.r.f["reset"](self._h)

    def absolute_time(self, time_point, frac=0.0):
        sec, fs = C.c_uint(), C.c_double()
        self.r.f["abs"](self._h, time_point, frac, C.byref(sec), C.byref(fs))
        return sec.value, fs.value
