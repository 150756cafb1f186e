"""Child process of tests/test_gpu_corr_hit.py: runs the
always-exact correlator build (tests/_build/libsrcdsp_hip_corr_exact.so,
corr.hip with -DSRCDSP_CORR_ALWAYS_EXACT) with NO product library in the
process, so every C-ABI call and kernel launch is that build's own.

  python tests/corr_exact_child.py EXACT_SO OUT.json

OUT.json: whether the product library got mapped (it must not), the build
flags a kernel of the loaded library reports, the tie-point streams' mismatch
lists (tests/golden/corr_ties.*) and the band sweep's mismatch lists against
the oracle (test_gpu_corr_hit.sweep_case / sweep_vs_oracle)."""
import ctypes as C
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, HERE, os.path.join(ROOT, "oracle")):
    sys.path.insert(0, p)


def main():
    exact, out = sys.argv[1], sys.argv[2]
    os.environ["SRCDSP_HIP_LIB"] = exact  # should anything ask srcdsp_amd for "the library"
    import torch  # noqa: F401  (the HIP runtime instance the library binds to)
    lib = C.CDLL(exact, mode=C.RTLD_LOCAL)
    import corr_ties as T
    import pyoracle
    import test_gpu_corr_hit as G
    G._bind(lib)
    f = C.c_uint(99)
    assert lib.srcdsp_build_flags(C.byref(f)) == 0
    res = {"build_flags": int(f.value), "ties": {}, "sweep": {}}
    man, arr = T.load()
    for case in man["cases"]:
        res["ties"][case["key"]] = T.replay(case, arr, G.CapiCorr(lib, case["N"], case["S"]))
    for N, S_ in G.SWEEP:
        p, x = G.sweep_case(N, S_)
        res["sweep"][f"{N}_{S_}"] = G.sweep_vs_oracle(G.CapiCorr(lib, N, S_), pyoracle.Oracle(1).corr(N, S_), p, x)
    product = os.path.join(ROOT, "srcdsp_amd", "lib", "libsrcdsp_hip.so")
    with open("/proc/self/maps") as m:
        res["product_mapped"] = product in m.read()
    with open(out, "w") as fh:
        json.dump(res, fh)


if __name__ == "__main__":
    main()
