"""CPU-side checks of the C-ABI boundary: the library loads without a GPU and
exports every entry point include/srcdsp_hip.h declares; the ctypes signature
table matches the header; no compute call is made here."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def capi():
    from srcdsp_amd import _capi
    if not os.path.exists(_capi.LIB_PATH):
        from srcdsp_amd.build import build
        build()
    return _capi


def test_library_exports_every_header_symbol(capi):
    lib = capi.lib()
    declared = capi.header_symbols()
    assert len(declared) >= 40
    missing = [s for s in declared if not hasattr(lib, s)]
    assert not missing, missing


def test_signature_table_matches_header(capi):
    assert set(capi.header_symbols()) == set(capi.SIGNATURES)


def test_header_is_plain_c(capi):
    """No C++ or framework types in the boundary (compiles as C99)."""
    import subprocess
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "t.c")
        with open(src, "w") as f:
            f.write('#include "srcdsp_hip.h"\nint main(void){return SRCDSP_OK;}\n')
        r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), src,
                            "-o", os.path.join(d, "t")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
    code = re.sub(r"/\*.*?\*/", "", open(capi.HEADER).read(), flags=re.S)
    assert not re.search(r"\b(torch|std::|hipStream_t|at::)", code)


def test_every_entry_point_cites_the_reference(capi):
    """Each operator block in the header names the reference file:line it replaces."""
    text = open(capi.HEADER).read()
    for f in ("dnsampling_filters.h", "filters.h", "upsampling_filters.h", "mixers.h", "correlators.h"):
        assert re.search(re.escape(f) + r":\d+", text), f


def test_version_and_error_strings(capi):
    lib = capi.lib()
    assert lib.srcdsp_version().decode().endswith("gfx950")
    assert isinstance(lib.srcdsp_last_error(), bytes)


def test_argument_errors_need_no_gpu(capi):
    """Argument validation happens before any HIP call."""
    import ctypes as C
    lib = capi.lib()
    h = C.c_void_p()
    assert lib.srcdsp_decim_create(C.byref(h), 9, 4, None, 0, 0) == capi.ERR_UNSUPPORTED
    assert lib.srcdsp_decim_create(None, 0, 4, None, 0, 0) == capi.ERR_ARG
    assert lib.srcdsp_decim_step(None, None, 0, None, 0, None) == capi.ERR_ARG
    assert lib.srcdsp_mixer_create(C.byref(h), 2) == capi.ERR_ARG
    assert lib.srcdsp_fill_synthetic(None, 0, 5, 0, 0, 0, 0, 1, None) == capi.ERR_ARG


def test_library_does_not_link_rccl(capi):
    """RCCL is dlopened by srcdsp_comm_create only (multi.hip), so single-GPU
    users neither link nor load it: no DT_NEEDED entry for librccl."""
    import subprocess
    out = subprocess.run(["readelf", "-d", capi.LIB_PATH], capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("readelf unavailable")
    needed = re.findall(r"\(NEEDED\)\s+Shared library: \[([^\]]+)\]", out.stdout)
    assert needed and not [n for n in needed if "rccl" in n], needed
