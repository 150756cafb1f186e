"""ctypes binding of libsrcdsp_hip.so (the C ABI declared in include/srcdsp_hip.h).

The library is the ONLY compute path of this package: if it is missing or
fails to load, importing the operators raises -- there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import os
import re

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
LIB_PATH = os.environ.get("SRCDSP_HIP_LIB", os.path.join(PKG, "lib", "libsrcdsp_hip.so"))
HEADER = os.path.join(ROOT, "include", "srcdsp_hip.h")

VP, I, U, SZ, F, D = C.c_void_p, C.c_int, C.c_uint, C.c_size_t, C.c_float, C.c_double
U64, I32P, U32P, I16P = C.c_uint64, C.POINTER(C.c_int32), C.POINTER(C.c_uint32), C.POINTER(C.c_int16)
IP, UP, FP, DP = C.POINTER(C.c_int), C.POINTER(C.c_uint), C.POINTER(C.c_float), C.POINTER(C.c_double)
HP = C.POINTER(C.c_void_p)

OK, ERR_ARG, ERR_UNSUPPORTED, ERR_SIZE, ERR_HIP, ERR_NOMEM = 0, -1, -2, -3, -4, -5
FLAG_ABS_FABS, FLAG_FP_STRICT = 1, 2

# name -> (restype, argtypes)
SIGNATURES = {
    "srcdsp_decim_create": (I, [HP, I, U, VP, I, U]),
    "srcdsp_decim_destroy": (I, [VP]),
    "srcdsp_decim_clone": (I, [VP, HP]),
    "srcdsp_decim_set_coeffs": (I, [VP, VP, I, I]),
    "srcdsp_decim_set_left_shift": (I, [VP, I]),
    "srcdsp_decim_reset": (I, [VP]),
    "srcdsp_decim_step": (I, [VP, VP, SZ, VP, SZ, VP]),
    "srcdsp_decim_step_host": (I, [VP, VP, SZ, VP, SZ]),
    "srcdsp_decim_step_batched": (I, [HP, I, VP, SZ, VP, SZ, SZ, VP]),
    "srcdsp_decim_get_state": (I, [VP, UP, IP, VP]),
    "srcdsp_fir_create": (I, [HP, I, VP, I, U]),
    "srcdsp_fir_destroy": (I, [VP]),
    "srcdsp_fir_clone": (I, [VP, HP]),
    "srcdsp_fir_set_coeffs": (I, [VP, VP, I]),
    "srcdsp_fir_reset": (I, [VP]),
    "srcdsp_fir_step": (I, [VP, VP, SZ, VP, SZ, VP]),
    "srcdsp_fir_step_host": (I, [VP, VP, SZ, VP, SZ]),
    "srcdsp_up_create": (I, [HP, I, U, VP, I]),
    "srcdsp_up_destroy": (I, [VP]),
    "srcdsp_up_clone": (I, [VP, HP]),
    "srcdsp_up_set_coeffs": (I, [VP, VP, I]),
    "srcdsp_up_reset": (I, [VP]),
    "srcdsp_up_get_length": (I, [VP, IP, IP, IP]),
    "srcdsp_up_step": (I, [VP, VP, SZ, VP, SZ, I, I, VP]),
    "srcdsp_up_step_host": (I, [VP, VP, SZ, VP, SZ, I, I]),
    "srcdsp_mixer_create": (I, [HP, U]),
    "srcdsp_mixer_destroy": (I, [VP]),
    "srcdsp_mixer_clone": (I, [VP, HP]),
    "srcdsp_mixer_set_frequency": (I, [VP, F]),
    "srcdsp_mixer_reset": (I, [VP, F]),
    "srcdsp_mixer_adjust_frequency": (I, [VP, F]),
    "srcdsp_mixer_get_state": (I, [VP, IP, IP, FP]),
    "srcdsp_mixer_set_phase": (I, [VP, I]),
    "srcdsp_mixer_get_table": (I, [VP, I16P]),
    "srcdsp_mixer_step": (I, [VP, VP, SZ, VP, VP]),
    "srcdsp_mixer_step_host": (I, [VP, VP, SZ, VP]),
    "srcdsp_mixdecim_step": (I, [VP, VP, VP, SZ, VP, SZ, VP]),
    "srcdsp_corr_create": (I, [HP, U, U]),
    "srcdsp_corr_destroy": (I, [VP]),
    "srcdsp_corr_clone": (I, [VP, HP]),
    "srcdsp_corr_set_pattern": (I, [VP, I32P, D]),
    "srcdsp_corr_reset": (I, [VP]),
    "srcdsp_corr_step": (I, [VP, VP, SZ, IP, IP, VP]),
    "srcdsp_corr_prime": (I, [VP, VP, SZ, VP]),
    "srcdsp_corr_step_host": (I, [VP, VP, SZ, IP, IP]),
    "srcdsp_corr_step_trace": (I, [VP, VP, SZ, IP, IP, U32P, U32P, C.POINTER(C.c_size_t), VP]),
    "srcdsp_corr_step_host_trace": (I, [VP, VP, SZ, IP, IP, U32P, U32P, C.POINTER(C.c_size_t)]),
    "srcdsp_corr_get_bit_samples": (I, [VP, I16P]),
    "srcdsp_corr_get_status": (I, [VP, U32P, U32P, U32P, IP, DP]),
    "srcdsp_fifo_create": (I, [HP, SZ, SZ, D]),
    "srcdsp_fifo_destroy": (I, [VP]),
    "srcdsp_fifo_write": (I, [VP, VP, SZ, U, D]),
    "srcdsp_fifo_write_device": (I, [VP, VP, SZ, U, D, VP]),
    "srcdsp_fifo_read": (I, [VP, VP, SZ, C.POINTER(C.c_uint64), IP, VP]),
    "srcdsp_fifo_read_host": (I, [VP, VP, SZ, C.POINTER(C.c_uint64), IP]),
    "srcdsp_fifo_count": (I, [VP, C.POINTER(C.c_size_t)]),
    "srcdsp_fifo_reset": (I, [VP]),
    "srcdsp_fifo_get_state": (I, [VP, C.POINTER(C.c_size_t), C.POINTER(C.c_uint64), C.POINTER(C.c_uint64), IP]),
    "srcdsp_fifo_get_absolute_time": (I, [VP, U64, D, UP, DP]),
    "srcdsp_iq_save": (I, [C.c_char_p, VP, SZ, SZ, I, VP]),
    "srcdsp_iq_save_host": (I, [C.c_char_p, VP, SZ, SZ, I]),
    "srcdsp_iq_count": (I, [C.c_char_p, SZ, C.POINTER(C.c_size_t)]),
    "srcdsp_iq_load": (I, [C.c_char_p, SZ, VP, SZ, C.POINTER(C.c_size_t), VP]),
    "srcdsp_iq_load_host": (I, [C.c_char_p, SZ, VP, SZ, C.POINTER(C.c_size_t)]),
    "srcdsp_comm_create": (I, [HP, I, IP]),
    "srcdsp_comm_destroy": (I, [VP]),
    "srcdsp_comm_info": (I, [VP, IP, IP]),
    "srcdsp_comm_stream": (I, [VP, I, HP]),
    "srcdsp_comm_synchronize": (I, [VP]),
    "srcdsp_comm_wait_stream": (I, [VP, I, VP]),
    "srcdsp_comm_signal_stream": (I, [VP, I, VP]),
    "srcdsp_decim_sharded_create": (I, [HP, VP, I, I, U, VP, I, U]),
    "srcdsp_decim_sharded_destroy": (I, [VP]),
    "srcdsp_decim_sharded_partition": (I, [VP, I, IP, IP]),
    "srcdsp_decim_sharded_channel": (I, [VP, I, HP]),
    "srcdsp_decim_sharded_step": (I, [VP, HP, SZ, HP, SZ, SZ]),
    "srcdsp_decim_sharded_reset": (I, [VP]),
    "srcdsp_decim_sharded_step_host": (I, [VP, HP, HP, SZ]),
    "srcdsp_decim_sharded_gather": (I, [VP, HP, SZ, SZ, VP, I]),
    "srcdsp_last_error": (C.c_char_p, []),
    "srcdsp_version": (C.c_char_p, []),
    "srcdsp_build_flags": (C.c_int, [C.POINTER(C.c_uint)]),
    "srcdsp_fill_synthetic": (I, [VP, I, SZ, U64, U64, U64, I, I, VP]),
}


def header_symbols(path: str = HEADER) -> list[str]:
    """Every function the public header declares (SRCDSP_API ... name( )."""
    with open(path) as f:
        text = f.read()
    return re.findall(r"SRCDSP_API\s+[\w\s\*]+?\b(srcdsp_\w+)\s*\(", text)


class SrcdspError(RuntimeError):
    def __init__(self, fn: str, code: int, msg: str):
        super().__init__(f"{fn} failed ({code}): {msg}")
        self.code = code


_LIB = None


def lib() -> C.CDLL:
    """Load libsrcdsp_hip.so once.  torch (if installed) is imported first so the
    library binds to the same HIP runtime instance torch uses."""
    global _LIB
    if _LIB is not None:
        return _LIB
    try:
        import torch  # noqa: F401  (shares libamdhip64.so.7 with torch)
    except ImportError:
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"libsrcdsp_hip.so not built at {LIB_PATH}: run `python -m srcdsp_amd.build` "
                          "(hipcc, gfx950). There is no CPU fallback.")
    lib_ = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib_, name)
        fn.restype = res
        fn.argtypes = args
    _LIB = lib_
    return lib_


def call(name: str, *args) -> int:
    rc = getattr(lib(), name)(*args)
    if rc != OK:
        raise SrcdspError(name, rc, lib().srcdsp_last_error().decode(errors="replace"))
    return rc
