"""The correlator's detection test at its tie points (correlators.h:262-268).

The GPU kernels decide `sqrt(c) > sqrt(e) * 2.7 && sqrt(e) > 300` by the sign
of c - 7.29 e and take correctly rounded square roots only inside a 1e-9
relative band (srcdsp_amd/csrc/corr_hit.h).  Random noise never reaches that
band, so it is forced here three ways:

1. crafted registers through the test-only probe kernel
   (tests/hip/corr_hit_probe.hip -> tests/_build/libcorr_hit_probe.so): every
   exact tie c = 729 k, e = 100 k in the uint32 range, ties +-1 on c and on e,
   e = 90000 / 90001, c / e = 7.29 (1 +- 2e-9), the uint32 maxima and the
   peak conditions, each against the host's IEEE double evaluation;
2. the tie-point streams generated from the reference build
   (tests/golden/corr_ties.*), replayed through the C ABI on corr_scan_s1
   (S = 1) and corr_eval(_dot2) + corr_detect (S > 1);
3. a library built with the band widened to infinity (corr.hip with
   -DSRCDSP_CORR_ALWAYS_EXACT -> tests/_build/libsrcdsp_hip_corr_exact.so)
   must give the product's detections on the fixtures and a fuzz sweep.
"""
import ctypes as C
import os

import numpy as np
import pytest

import corr_ties as T

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "tests", "_build")
PROBE = os.path.join(BUILD, "libcorr_hit_probe.so")
EXACT = os.path.join(BUILD, "libsrcdsp_hip_corr_exact.so")
MAN, ARR = T.load()
U32MAX = (1 << 32) - 1


def _need(path):
    # built by __graft_entry__.build() (srcdsp_amd.build.build_test_probes); a
    # missing artefact is a failure, not a skip
    assert os.path.exists(path), f"{path} not built: run python -c 'import __graft_entry__ as g; g.build()'"
    return path


@pytest.fixture(scope="module")
def probe(S):
    lib = C.CDLL(_need(PROBE), mode=C.RTLD_LOCAL)
    for name in ("corr_hit_probe", "crsqrt_probe"):
        getattr(lib, name).restype = C.c_int
        getattr(lib, name).argtypes = [C.c_void_p, C.c_long, C.c_void_p, C.c_void_p]
    return lib


def host_hit(q: np.ndarray) -> np.ndarray:
    """The reference's expression in IEEE double (numpy's sqrt is correctly
    rounded, its multiply is one rounded product, as on the reference's x86-64)."""
    c2, c1, c0, e1 = (q[:, i].astype(np.float64) for i in range(4))
    sc, se = np.sqrt(c1), np.sqrt(e1)
    return (q[:, 1] > q[:, 0]) & (q[:, 1] > q[:, 2]) & (sc > se * 2.7) & (se > 300)


def crafted_cases() -> np.ndarray:
    rng = np.random.default_rng(29)
    rows = []

    def add(c1, e1, c2=None, c0=None):
        c1 = np.asarray(c1, np.int64)
        e1 = np.broadcast_to(np.asarray(e1, np.int64), c1.shape)
        c2 = np.zeros_like(c1) if c2 is None else np.broadcast_to(np.asarray(c2, np.int64), c1.shape)
        c0 = np.zeros_like(c1) if c0 is None else np.broadcast_to(np.asarray(c0, np.int64), c1.shape)
        ok = (c1 >= 0) & (c1 <= U32MAX) & (e1 >= 0) & (e1 <= U32MAX)
        rows.append(np.stack([c2[ok], c1[ok], c0[ok], e1[ok]], 1))

    k = np.arange(900, U32MAX // 729 + 1, dtype=np.int64)  # every tie c = 729 k, e = 100 k, e >= 90000
    for dc, de in ((0, 0), (1, 0), (-1, 0), (0, 1), (0, -1), (1, 1), (-1, -1)):
        add(729 * k + dc, 100 * k + de)
    sq = np.arange(300, 2428, dtype=np.int64)  # perfect-square ties c = (27 s)^2, e = (10 s)^2 and neighbours
    for dc in (-1, 0, 1):
        for de in (-1, 0, 1):
            add((27 * sq) ** 2 + dc, (10 * sq) ** 2 + de)
    cs = np.arange(0, 1 << 22, 997, dtype=np.int64)  # the energy floor: sqrt(e) > 300 <=> e >= 90001
    for e in (89999, 90000, 90001, 90002):
        add(cs, e)
        add(np.array([656100, 656101, 656108, 656109, 656110, U32MAX]), e)
    e = rng.integers(90001, U32MAX // 7, size=1 << 18, dtype=np.int64)  # c / e = 7.29 (1 +- 2e-9), +- a few
    for rel in (-2e-9, -1e-9, -5e-10, 0.0, 5e-10, 1e-9, 2e-9):
        base = np.floor(7.29 * e * (1 + rel)).astype(np.int64)
        for d in (-1, 0, 1):
            add(base + d, e)
    top = np.arange(0, 64, dtype=np.int64)  # the uint32 maxima
    add(U32MAX - top, U32MAX)
    add(U32MAX - top, U32MAX - top)
    add(U32MAX - top, int(U32MAX / 7.29) + top - 32)
    add(np.full(64, U32MAX), (U32MAX * 100) // 729 + top - 32)
    add(np.full(3, U32MAX), [0, 90000, 90001])
    c1 = rng.integers(1, U32MAX, size=1 << 16, dtype=np.int64)  # the peak conditions
    ee = (c1 * 100) // 729
    add(c1, ee, c2=c1)
    add(c1, ee, c0=c1)
    add(c1, ee, c2=c1 - 1, c0=c1 - 1)
    add(c1, ee, c2=c1 + 1)
    add(c1, ee, c0=np.minimum(c1 + 1, U32MAX))
    r = rng.integers(0, 1 << 32, size=(1 << 20, 4), dtype=np.int64)  # random registers
    rows.append(r)
    return np.ascontiguousarray(np.concatenate(rows).astype(np.uint32))


def test_corr_hit_crafted_registers_vs_host_double(probe):
    """Fast test (as shipped) and always-exact test against the host's double
    evaluation on ~48 M crafted register sets; ~19 M of them are peaks inside
    the band (the exact branch), with both verdicts."""
    import torch
    q = crafted_cases()
    n = len(q)
    dq = torch.from_numpy(q.view(np.int32)).cuda()
    out = torch.empty(2 * n, dtype=torch.uint8, device="cuda")
    assert probe.corr_hit_probe(C.c_void_p(dq.data_ptr()), n, C.c_void_p(out.data_ptr()),
                                C.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    got = out.cpu().numpy().reshape(n, 2).astype(bool)
    want = host_hit(q)
    bad = np.nonzero(got[:, 0] != want)[0]
    assert len(bad) == 0, f"fast test: {len(bad)} mismatches, first {q[bad[:5]].tolist()}"
    bad = np.nonzero(got[:, 1] != want)[0]
    assert len(bad) == 0, f"exact test: {len(bad)} mismatches, first {q[bad[:5]].tolist()}"
    c1, e1 = q[:, 1].astype(np.float64), q[:, 3].astype(np.float64)
    peak = (q[:, 1] > q[:, 0]) & (q[:, 1] > q[:, 2]) & (q[:, 3] > 90000)
    in_band = peak & (np.abs(c1 - 7.29 * e1) <= 1e-9 * c1)
    assert in_band.sum() > 100000 and want[in_band].any() and (~want[in_band]).any()


def test_crsqrt_u32_correctly_rounded(probe):
    """crsqrt_u32 (the band's square root) equals the host's correctly rounded
    sqrt bit for bit: all n < 2^20, k^2 + (-2..2) for every k < 2^16, the top
    of the range and 4 M random values."""
    import torch
    rng = np.random.default_rng(31)
    ks = np.arange(1, 1 << 16, dtype=np.int64)
    v = np.concatenate([np.arange(1 << 20, dtype=np.int64), *[ks * ks + d for d in (-2, -1, 0, 1, 2)],
                        U32MAX - np.arange(1 << 16, dtype=np.int64),
                        rng.integers(0, 1 << 32, size=1 << 22, dtype=np.int64)])
    v = v[(v >= 0) & (v <= U32MAX)].astype(np.uint32)
    dv = torch.from_numpy(v.view(np.int32)).cuda()
    out = torch.empty(len(v), dtype=torch.float64, device="cuda")
    assert probe.crsqrt_probe(C.c_void_p(dv.data_ptr()), len(v), C.c_void_p(out.data_ptr()),
                              C.c_void_p(torch.cuda.current_stream().cuda_stream)) == 0
    got = out.cpu().numpy()
    want = np.sqrt(v.astype(np.float64))
    bad = np.nonzero(got.view(np.uint64) != want.view(np.uint64))[0]
    assert len(bad) == 0, f"{len(bad)} mismatches, first n = {v[bad[:5]].tolist()}"


# ------------------------------------------------ the C ABI on the tie streams
class CapiCorr:
    """The oracle's correlator face over any build of the library's C ABI
    (device-resident input on the current stream, or host-staged)."""

    def __init__(self, lib, N, S, host=False):
        self.lib, self.N, self.host = lib, N, host
        self.h = C.c_void_p()
        assert lib.srcdsp_corr_create(C.byref(self.h), N, S) == 0

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.srcdsp_corr_destroy(self.h)

    def set_pattern(self, p, th=0.8):
        p = np.ascontiguousarray(p, np.int32)
        assert self.lib.srcdsp_corr_set_pattern(self.h, p.ctypes.data_as(C.POINTER(C.c_int32)), C.c_double(th)) == 0

    def step(self, x):
        import torch
        x = np.ascontiguousarray(x, np.int16)
        found, idx = C.c_int(0), C.c_int(-1)
        if self.host:
            rc = self.lib.srcdsp_corr_step_host(self.h, C.c_void_p(x.ctypes.data), len(x), C.byref(found),
                                                 C.byref(idx))
        else:
            d = torch.from_numpy(x).cuda()
            rc = self.lib.srcdsp_corr_step(self.h, C.c_void_p(d.data_ptr()), len(x), C.byref(found), C.byref(idx),
                                           C.c_void_p(torch.cuda.current_stream().cuda_stream))
        assert rc == 0
        return bool(found.value), idx.value

    def bit_samples(self):
        b = np.zeros((self.N, 2), np.int16)
        assert self.lib.srcdsp_corr_get_bit_samples(self.h, b.ctypes.data_as(C.POINTER(C.c_int16))) == 0
        return b

    def status(self):
        e3, c3 = (C.c_uint32 * 3)(), (C.c_uint32 * 3)()
        ce, cs, tf = C.c_uint32(), C.c_int(), C.c_double()
        assert self.lib.srcdsp_corr_get_status(self.h, e3, c3, C.byref(ce), C.byref(cs), C.byref(tf)) == 0
        return {"energy": list(e3), "corr": list(c3)}


def _bind(lib):
    from srcdsp_amd._capi import SIGNATURES
    for name, (res, args) in SIGNATURES.items():
        if name.startswith("srcdsp_corr_") or name == "srcdsp_build_flags":
            fn = getattr(lib, name)
            fn.restype, fn.argtypes = res, args
    return lib


# ------------------------------------- the always-exact build, in its own process
def sweep_case(N, S_):
    """The fuzz stream of the band sweep: QPSK pattern copies at three
    amplitudes in noise (detections inside and outside the 1e-9 band)."""
    from srcdsp_amd.design import qpsk_pattern
    p = qpsk_pattern(N, 500, seed=N + 7)
    rng = np.random.default_rng(N * 31 + S_)
    n = 1 << 16 if N >= 1000 else 1 << 17
    x = rng.integers(-125, 126, size=(n, 2)).astype(np.int32)
    for off in (n // 5, n // 2, (4 * n) // 5):
        amp = int(rng.integers(1, 4))
        for m in range(N):
            if off + m * S_ < n:
                x[off + m * S_] += amp * p[m]
    return p, np.clip(x, -32768, 32767).astype(np.int16)


def sweep_vs_oracle(obj, oracle, p, x) -> list[str]:
    """Step obj and the oracle through x, stepping on after every detection;
    detections, indices, bitSamples and registers must agree."""
    fails = []
    for o in (obj, oracle):
        o.set_pattern(p)
    pos, n = 0, len(x)
    while pos < n and not fails:
        xs = x[pos:pos + 17000]
        r, w = obj.step(xs), oracle.step(xs)
        if (r[0], r[0] and r[1]) != (w[0], w[0] and w[1]):
            fails.append(f"at {pos}: {r} vs oracle {w}")
        elif not np.array_equal(obj.bit_samples(), oracle.bit_samples()):
            fails.append(f"at {pos}: bitSamples")
        else:
            st, so = obj.status(), oracle.status()
            if st["energy"] != list(so["energy"]) or st["corr"] != list(so["corr"]):
                fails.append(f"at {pos}: registers {st} vs {so}")
        pos += (w[1] + 2) if w[0] else len(xs)
    return fails


SWEEP = [(1024, 1), (32, 4), (64, 2), (33, 1), (127, 2), (16, 16), (1000, 1), (48, 3), (256, 4), (17, 1), (129, 1)]


@pytest.fixture(scope="module")
def exact_results(S, tmp_path_factory):
    """the always-exact build runs in a CHILD process that loads
    only that library (tests/corr_exact_child.py), so its C-ABI calls and
    kernel launches cannot resolve to the product library this process holds
    (a kernel of each library reports its build switch: round 6 saw the
    RTLD_LOCAL copy launch the product's kernel in-process)."""
    import json
    import subprocess
    import sys
    out = str(tmp_path_factory.mktemp("exact") / "exact.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tests", "corr_exact_child.py"), _need(EXACT), out],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    return json.load(open(out))


def test_exact_build_runs_its_own_kernels(S, exact_results):
    """The child holds no product library and its kernel reports the
    always-exact switch; the product's kernel reports none."""
    assert exact_results["product_mapped"] is False
    assert exact_results["build_flags"] == 1  # SRCDSP_BUILD_CORR_ALWAYS_EXACT
    f = C.c_uint(99)
    assert S.lib().srcdsp_build_flags(C.byref(f)) == 0 and f.value == 0


@pytest.mark.parametrize("host", [False, True], ids=["device", "host"])
@pytest.mark.parametrize("case", MAN["cases"], ids=lambda c: c["key"])
def test_tie_streams_through_the_product(S, case, host):
    """The reference's outputs on the tie-point streams (detections at band
    peaks it accepts, none at those it rejects, bitSamples, registers at
    every step) from the product library: corr_scan_s1 at S = 1,
    corr_eval + corr_detect at (32, 4), corr_eval_dot2 + corr_detect at (64, 2)."""
    assert T.replay(case, ARR, CapiCorr(S.lib(), case["N"], case["S"], host=host)) == []


@pytest.mark.parametrize("case", MAN["cases"], ids=lambda c: c["key"])
def test_tie_streams_through_the_always_exact_build(exact_results, case):
    assert exact_results["ties"][case["key"]] == []


@pytest.mark.parametrize("N,S_", SWEEP)
def test_band_sweep_product_and_always_exact_vs_oracle(S, O, exact_results, N, S_):
    """Threshold sweep: the build whose band is infinite (every peak decided
    by the correctly rounded square roots, in the child process) and the
    product each give the oracle's detections, indices, bitSamples and
    registers on the fuzz streams, stepping on after every detection; so the
    product's fast sign test equals the exact one there."""
    p, x = sweep_case(N, S_)
    assert sweep_vs_oracle(CapiCorr(S.lib(), N, S_), O["fma"].corr(N, S_), p, x) == []
    assert exact_results["sweep"][f"{N}_{S_}"] == []


def _oracle_trace(o, x):
    """Per-sample corrValue[0] / energyValue[0] of the reference semantics:
    the oracle stepped one sample at a time (a detection at a one-sample call
    reports corrIndex -1, and the caller resumes at the next sample, exactly
    the chunked protocol), so a detection's dropped history slot
    (correlators.h:291) is reproduced."""
    c, e = np.zeros(len(x), np.uint32), np.zeros(len(x), np.uint32)
    for k in range(len(x)):
        o.step(x[k:k + 1])
        st = o.status()
        c[k], e[k] = st["corr"][0], st["energy"][0]
    return c, e


@pytest.mark.parametrize("device", [True, False], ids=["device", "host"])
@pytest.mark.parametrize("which", ["n16_s1", "n32_s4", "n64_s2", "rand_1024_1", "rand_32_4"])
def test_step_trace_registers_vs_oracle(S, O, which, device):
    """srcdsp_corr_step(_host)_trace (the CREATE_DEBUG_FILES registers): every
    processed sample's corrValue[0] / energyValue[0] across chunked calls with
    detections, against the oracle stepped sample by sample; the detections
    equal step()'s."""
    import torch
    from srcdsp_amd.design import qpsk_pattern
    if which.startswith("rand"):
        _, N, S_ = which.split("_")
        N, S_ = int(N), int(S_)
        p = qpsk_pattern(N, 500, seed=3)
        rng = np.random.default_rng(N)
        x = rng.integers(-125, 126, size=(6000, 2)).astype(np.int32)
        for off in (1000, 4000):
            for m in range(N):
                if off + m * S_ < len(x):
                    x[off + m * S_] += 2 * p[m]
        x = np.clip(x, -32768, 32767).astype(np.int16)
    else:
        case = [c for c in MAN["cases"] if c["key"] == which][0]
        N, S_, p, x = case["N"], case["S"], T.pattern(case), ARR[which + "_x"]
    o = O["fma"].corr(N, S_)
    o.set_pattern(p)
    wc, we = _oracle_trace(o, x)
    g = S.FixedPatternCorrelator(N, S_)
    g.setPattern(p)
    gc, ge, pos, hits = [], [], 0, 0
    while pos < len(x):
        xs = x[pos:pos + 1700]
        found, idx, c, e = g.step_trace(torch.from_numpy(xs).cuda() if device else xs)
        assert len(c) == ((idx + 2) if found else len(xs))
        gc.append(c)
        ge.append(e)
        hits += found
        pos += (idx + 2) if found else len(xs)
    gc, ge = np.concatenate(gc), np.concatenate(ge)
    assert np.array_equal(gc, wc) and np.array_equal(ge, we)
    assert hits >= 1
