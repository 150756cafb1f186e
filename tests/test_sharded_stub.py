"""The C-ABI multi-device path (srcdsp_amd/csrc/multi.hip) at ndev > 1 on ONE
GPU (VERDICT r3 Next #2).

tests/cpp/sharded_main.cpp drives dsptl::ShardedDnsamplingFir over a
communicator whose ranks all name device 0.  Real RCCL refuses that, so the
child process loads tests/rccl_stub (a test-only librccl.so.1: grouped
Gather / Send / Recv as stream-ordered device copies) through LD_LIBRARY_PATH,
and links the test build of the library whose multi.hip honours
SRCDSP_COMM_SHARED_DEVICES=1 (tests/_build/shared_dev/libsrcdsp_hip.so: the
product objects with multi.hip compiled -DSRCDSP_TEST_SHARED_DEVICES; the
shipped library refuses a device listed twice whatever the environment says).
What runs is
the product's own multi-device code: the block partition, one host thread
per rank in step_host, one batched launch per rank on its comm stream, the
even-partition ncclGather, and for uneven or strided rows the root's
hipMemcpy2DAsync plus the ncclSend/ncclRecv loop and its destination offsets.
Every channel is compared bit-exactly with its own oracle decimator.

The stub is never part of the product: it is built here, into the test's
temporary directory."""
import os
import subprocess

import numpy as np
import pytest

from test_dropin_cpp import INC, ROOT, _read, _rec

pytestmark = pytest.mark.gpu
STUB = os.path.join(ROOT, "tests", "rccl_stub", "rccl_stub.cpp")
SHARED_DEV_DIR = os.path.join(ROOT, "tests", "_build", "shared_dev")
HIPFLAGS = ["-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include"]


@pytest.fixture(scope="module")
def built(tmp_path_factory):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    d = tmp_path_factory.mktemp("stub")
    so = str(d / "librccl.so.1")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-shared", "-fPIC", *HIPFLAGS, STUB, "-o", so,
                        "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    exe = str(d / "sharded_main")
    assert os.path.exists(os.path.join(SHARED_DEV_DIR, "libsrcdsp_hip.so")), \
        "tests/_build/shared_dev not built: run python -c 'import __graft_entry__ as g; g.build()'"
    r = subprocess.run(["g++", "-std=c++14", "-O2", *HIPFLAGS, "-I", INC,
                        os.path.join(ROOT, "tests", "cpp", "sharded_main.cpp"), "-o", exe, "-L", SHARED_DEV_DIR,
                        "-lsrcdsp_hip", "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{SHARED_DEV_DIR}",
                        "-Wl,-rpath,/opt/rocm/lib"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return str(d), exe


def _run(built, tmp_path, ndev, C, root, n=40000, shared=True):
    import pyoracle
    from srcdsp_amd.design import hamming_sinc
    d, exe = built
    O = pyoracle.Oracle(1)
    c = hamming_sinc(127)
    xs = [O.gen_cf32(11, ch, 0, n) for ch in range(C)]
    fin = tmp_path / "in.bin"
    with open(fin, "wb") as f:
        _rec(f, 1, c)
        _rec(f, 2, np.array([C], np.int32))
        for ch in range(C):
            _rec(f, 10 + ch, xs[ch])
    env = dict(os.environ, LD_LIBRARY_PATH=d + ":" + os.environ.get("LD_LIBRARY_PATH", ""),
               SHARDED_ROOT=str(root), RCCL_STUB_LOG="1")
    if shared:
        env["SRCDSP_COMM_SHARED_DEVICES"] = "1"
    r = subprocess.run([exe, str(fin), str(tmp_path / "out.bin"), *["0"] * ndev], capture_output=True, text=True,
                       timeout=120, env=env)
    return r, xs, c, O


@pytest.mark.parametrize("ndev,C,root", [(2, 5, 0), (2, 5, 1), (3, 5, 2), (3, 7, 1), (8, 5, 6), (8, 16, 3),
                                         (8, 19, 0)],
                         ids=lambda v: str(v))
def test_sharded_decim_ndev_on_one_gpu(built, tmp_path, ndev, C, root):
    """ndev ranks on device 0: uneven shares (5 over 2/3, 7 over 3, 19 over 8),
    ranks with no channel (5 over 8, root 6 among them), an even partition
    (16 over 8: the ncclGather branch), a non-zero root, strided output rows,
    and the operator outliving its communicator."""
    r, xs, c, O = _run(built, tmp_path, ndev, C, root)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "rccl_stub:" in r.stderr, "the stub communicator did not carry the gather"
    got = _read(tmp_path / "out.bin")
    n = len(xs[0])
    half = (n // 2) & ~3
    alls = []
    for ch in range(C):
        dch = O.decim(0, 4, c)
        exp = np.concatenate([dch.step(xs[ch][:half]), dch.step(xs[ch][half:])])
        assert got[100 + ch] == exp.tobytes(), ch
        alls.append(O.decim(0, 4, c).step(xs[ch]))
    want = np.concatenate(alls).tobytes()
    assert got[200] == want
    assert got[201] == want  # strided rows: root's hipMemcpy2DAsync + per-row ncclSend/ncclRecv
    assert got[202] == want  # operator outliving its communicator
    assert got[203] == want  # caller streams ordered by waitFor / signal, no synchronize()
    q, rem = divmod(C, ndev)
    transfers = [l for l in r.stderr.splitlines() if l.startswith("rccl_stub:")]
    # three contiguous gathers (records 200, 202 and 203) and one strided (201)
    if rem == 0:
        # ncclGather for every contiguous gather (each rank incl. the root) and,
        # for the strided one, one Send/Recv per non-root row
        assert len(transfers) == 3 * ndev + (C - q)
    else:
        nonroot_ranks = sum(1 for k in range(ndev) if k != root and q + (k < rem) > 0)
        nonroot_rows = C - (q + (root < rem))
        assert len(transfers) == 3 * nonroot_ranks + nonroot_rows


def test_shared_devices_refused_by_the_product(S, monkeypatch):
    """The shipped library refuses a device listed twice before any
    communicator is made (as real RCCL would), even with the test build's
    opt-in variable set: the knob exists only in tests/_build/shared_dev."""
    import ctypes as C
    monkeypatch.setenv("SRCDSP_COMM_SHARED_DEVICES", "1")
    lib = S.lib()
    h = C.c_void_p()
    devs = (C.c_int * 2)(0, 0)
    rc = lib.srcdsp_comm_create(C.byref(h), 2, devs)
    assert rc != 0 and not h.value
    lib.srcdsp_last_error.restype = C.c_char_p
    assert b"listed twice" in lib.srcdsp_last_error()
