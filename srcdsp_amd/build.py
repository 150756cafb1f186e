"""Build libsrcdsp_hip.so in-tree (hipcc, gfx950).

``python -m srcdsp_amd.build`` compiles every ``csrc/*.hip`` to an object in
``build/`` (in parallel) and links ``srcdsp_amd/lib/libsrcdsp_hip.so``.  The
shared object is git-ignored but travels to the GPU box with the snapshot.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
OBJ = os.path.join(ROOT, "build", "srcdsp_hip")
LIB_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(LIB_DIR, "libsrcdsp_hip.so")
ARCH = os.environ.get("SRCDSP_OFFLOAD_ARCH", "gfx950")
ROCM_LIB = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "lib")

CXXFLAGS = [
    f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-fvisibility=hidden",
    # taps are accumulated exactly as written: explicit __builtin_fmaf where the
    # FMA contract is wanted, separately rounded mul/add otherwise
    "-ffp-contract=off",
    "-Wall", "-Wno-unused-function",
]


def _hipcc() -> str:
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libsrcdsp_hip.so)")


def _headers() -> list[str]:
    return glob.glob(os.path.join(CSRC, "*.h")) + [os.path.join(ROOT, "include", "srcdsp_hip.h")]


# the translation unit that holds each bench workload's dominant kernel
WORKLOAD_TU = {"decim": "decim.hip", "mixdecim": "decim.hip", "ci16decim": "decim.hip", "fir": "decim.hip",
               "up": "upsamp.hip", "corr": "corr.hip", "fifo": "fifo.hip", "iq": "fifo.hip"}


def _tu_files(tu: str) -> list[str]:
    """`tu` and every local header it reaches through #include "..." (csrc/, include/)."""
    seen, todo = [], [os.path.join(CSRC, tu)]
    while todo:
        f = todo.pop()
        if f in seen or not os.path.exists(f):
            continue
        seen.append(f)
        with open(f) as fh:
            for line in fh:
                line = line.strip()
                if line.startswith("#include \""):
                    name = line.split('"')[1]
                    for d in (os.path.dirname(f), CSRC, os.path.join(ROOT, "include")):
                        if os.path.exists(os.path.join(d, name)):
                            todo.append(os.path.normpath(os.path.join(d, name)))
                            break
    return seen


def source_digest(workload: str | None = None) -> str:
    """sha256 (16 hex) over kernel sources: stamps measured evidence
    (profiles/pmc_traffic.json) with the code it was measured on, so a later
    change shows it as stale.  With a bench workload: only the translation
    unit of its kernel and the headers that unit includes; without one: every
    csrc/*.hip, csrc/*.h and the C ABI header."""
    import hashlib
    h = hashlib.sha256()
    if workload is not None:
        files = sorted(_tu_files(WORKLOAD_TU[workload]))
    else:
        files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + _headers())
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def _stale(target: str, deps: list[str]) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, jobs: int = 8, defines: tuple[str, ...] = (), lib: str | None = None) -> str:
    """Compile and link the library.  `defines`/`lib`: a tuning build (e.g.
    ("SRCDSP_TUNING", "SRCDSP_PHASE_CLOCK") into scripts/tune/ab/...), with its
    own object directory; the product build takes neither."""
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")))
    obj_dir = OBJ if not defines else OBJ + "_" + "_".join(d.lower() for d in defines)
    LIB = lib or globals()["LIB"]
    os.makedirs(obj_dir, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    hipcc = _hipcc()
    hdrs = _headers()

    def compile_one(src: str) -> str:
        obj = os.path.join(obj_dir, os.path.basename(src) + ".o")
        if _stale(obj, [src] + hdrs):
            cmd = [hipcc, *CXXFLAGS, *[f"-D{d}" for d in defines], "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), file=sys.stderr)
            r = subprocess.run(cmd, capture_output=True, text=True)
            if r.returncode != 0:
                raise RuntimeError(f"hipcc failed on {src}:\n{r.stderr[-6000:]}")
        return obj

    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        objs = list(ex.map(compile_one, srcs))
    if _stale(LIB, objs):
        # no -lrccl: multi.hip dlopens librccl at the first srcdsp_comm_create, so
        # single-GPU users of the library neither link nor load RCCL
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", LIB, *objs, "-ldl",
               f"-Wl,-rpath,{ROCM_LIB}"]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr[-6000:]}")
    return LIB


TEST_BUILD = os.path.join(ROOT, "tests", "_build")
CORR_HIT_PROBE = os.path.join(TEST_BUILD, "libcorr_hit_probe.so")
# Test-only variants of the library: the product's objects with ONE translation
# unit recompiled under a test define.  Never loaded by the package.
#   corr_exact: the correlator's detection test always on the correctly rounded
#     square roots (corr_hit.h), so the suite can require identical detections
#     with and without the fast sign test;
#   shared_dev: multi.hip honouring SRCDSP_COMM_SHARED_DEVICES=1, so the
#     multi-device C ABI can be rehearsed at ndev > 1 on one GPU through the
#     test-only communicator library (tests/rccl_stub); named libsrcdsp_hip.so in
#     its own directory so the C++ test program links it as -lsrcdsp_hip.
TEST_VARIANTS = {
    "corr_exact": ("corr.hip", "SRCDSP_CORR_ALWAYS_EXACT", os.path.join(TEST_BUILD, "libsrcdsp_hip_corr_exact.so")),
    "shared_dev": ("multi.hip", "SRCDSP_TEST_SHARED_DEVICES", os.path.join(TEST_BUILD, "shared_dev", "libsrcdsp_hip.so")),
}
CORR_EXACT_LIB = TEST_VARIANTS["corr_exact"][2]
SHARED_DEV_LIB = TEST_VARIANTS["shared_dev"][2]


def build_test_probes(verbose: bool = False) -> list[str]:
    """Test-only artefacts (tests/_build/, git-ignored, travel to the GPU box
    like the library): the corr_hit probe kernel and the TEST_VARIANTS builds."""
    build(verbose=verbose)
    os.makedirs(TEST_BUILD, exist_ok=True)
    hipcc = _hipcc()
    hdrs = _headers()

    def run(cmd):
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"hipcc failed:\n{r.stderr[-6000:]}")

    probe_src = os.path.join(ROOT, "tests", "hip", "corr_hit_probe.hip")
    if _stale(CORR_HIT_PROBE, [probe_src] + hdrs):
        run([hipcc, *CXXFLAGS, "-shared", probe_src, "-o", CORR_HIT_PROBE])
    out = [CORR_HIT_PROBE]
    for name, (tu, define, lib) in TEST_VARIANTS.items():
        obj_dir = OBJ + "_test_" + name
        os.makedirs(obj_dir, exist_ok=True)
        os.makedirs(os.path.dirname(lib), exist_ok=True)
        src = os.path.join(CSRC, tu)
        obj = os.path.join(obj_dir, tu + ".o")
        if _stale(obj, [src] + hdrs):
            run([hipcc, *CXXFLAGS, f"-D{define}", "-c", src, "-o", obj])
        objs = [obj if os.path.basename(s) == tu else os.path.join(OBJ, os.path.basename(s) + ".o")
                for s in sorted(glob.glob(os.path.join(CSRC, "*.hip")))]
        if _stale(lib, objs):
            run([hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", lib, *objs, "-ldl",
                 f"-Wl,-rpath,{ROCM_LIB}"])
        out.append(lib)
    return out


if __name__ == "__main__":
    # python -m srcdsp_amd.build [NAME DEFINE...]: with arguments, a tuning
    # build scripts/tune/ab/libsrcdsp_hip_NAME.so compiled with -DDEFINE...
    if len(sys.argv) > 2:
        print(build(verbose=True, defines=tuple(sys.argv[2:]),
                    lib=os.path.join(ROOT, "scripts", "tune", "ab", f"libsrcdsp_hip_{sys.argv[1]}.so")))
    else:
        print(build(verbose=True))
