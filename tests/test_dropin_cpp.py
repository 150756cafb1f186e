"""The C++ drop-in headers (include/srcdsp/): reference-style code builds
against them unchanged and reproduces the reference's results.

CPU: every supported instantiation compiles; an instantiation the reference
cannot compile fails to compile here too.  GPU: tests/cpp/dropin_main.cpp runs
on the box and its outputs are compared bit-exactly with the oracle."""
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include", "srcdsp")
LIBDIR = os.path.join(ROOT, "srcdsp_amd", "lib")


def _compile(src_text, out, tmp, link=False):
    src = os.path.join(tmp, "t.cpp")
    with open(src, "w") as f:
        f.write(src_text)
    cmd = ["g++", "-std=c++14", "-Wall", "-I", INC, src, "-o", out]
    if link:
        cmd += ["-L", LIBDIR, "-lsrcdsp_hip", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib"]
    else:
        cmd = cmd[:-2] + ["-fsyntax-only"]
    return subprocess.run(cmd, capture_output=True, text=True)


def test_dropin_headers_compile_all_supported_instantiations(tmp_path):
    src = """
#include "dnsampling_filters.h"
#include "filters.h"
#include "upsampling_filters.h"
#include "mixers.h"
#include "correlators.h"
#include "buffers.h"
#include "dsptl_files.h"
using cf32 = std::complex<float>; using ci16 = std::complex<int16_t>; using ci32 = std::complex<int32_t>;
template class dsptl::FifoWithTimeTrack<ci16, 1 << 20>;
template class dsptl::FifoWithTimeTrack<double, 15>;
template void dsptl::saveBinarySamples<int16_t>(std::vector<ci16> &, std::ofstream &);
template void dsptl::readBinarySamples<float>(std::ifstream &, std::vector<cf32> &);
template size_t dsptl::readBinarySamples<int16_t>(const char *, dsptl::DeviceSpan<ci16>, void *);
template class dsptl::FilterDnsamplingFir<cf32, cf32, cf32, float, 4>;
template class dsptl::FilterDnsamplingFir<ci16, ci16, ci32, int32_t, 4>;
template class dsptl::FilterDnsamplingFir<ci16, ci16, ci32, int16_t, 2>;
template class dsptl::FilterDnsamplingFir<ci32, ci16, ci32, int32_t, 8>;
template class FilterFir<cf32, cf32, cf32, float>;
template class FilterFir<float, cf32, float, float>;
template class FilterFir<ci16, ci16, ci32, int32_t>;
template class dsptl::FilterUpsamplingFir<ci16, ci16, ci32, int32_t, 4>;
template class dsptl::FilterUpsamplingFir<ci16, ci16, ci32, int16_t, 4>;
template class dsptl::FilterUpsamplingFir<int16_t, int16_t, int32_t, int32_t, 2>;
template class dsptl::Mixer<ci16, ci16, int16_t, 4096>;
template class dsptl::FixedPatternCorrelator<int16_t, int32_t, 1024, 1>;
template class dsptl::FixedPatternCorrelator<int16_t, int32_t, 32, 4>;
int main() { return 0; }
"""
    r = _compile(src, str(tmp_path / "a.out"), str(tmp_path))
    assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("inst", [
    "dsptl::FilterDnsamplingFir<float, float, float, float, 4>",        # dsptl_dnsampling_filters.h:215
    "FilterFir<float, float, float, float>",                            # filters.h:164
    "dsptl::FilterUpsamplingFir<std::complex<float>, std::complex<float>, std::complex<float>, float, 4>",
])
def test_dropin_rejects_what_the_reference_cannot_compile(tmp_path, inst):
    src = ('#include "dnsampling_filters.h"\n#include "filters.h"\n#include "upsampling_filters.h"\n'
           f"template class {inst};\nint main(){{return 0;}}\n")
    r = _compile(src, str(tmp_path / "a.out"), str(tmp_path))
    assert r.returncode != 0


def _rec(f, tag, arr):
    b = np.ascontiguousarray(arr).tobytes()
    f.write(struct.pack("<iq", tag, len(b)))
    f.write(b)


def _read(path):
    out = {}
    with open(path, "rb") as f:
        while True:
            h = f.read(12)
            if len(h) < 12:
                return out
            tag, nb = struct.unpack("<iq", h)
            out[tag] = f.read(nb)


@pytest.mark.gpu
def test_dropin_program_matches_oracle(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pyoracle
    from srcdsp_amd.design import hamming_sinc, q14, qpsk_pattern
    exe = str(tmp_path / "dropin_main")
    r = subprocess.run(["g++", "-std=c++14", "-O2", "-I", INC, os.path.join(ROOT, "tests", "cpp", "dropin_main.cpp"),
                        "-o", exe, "-L", LIBDIR, "-lsrcdsp_hip", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    O = pyoracle.Oracle(1)
    c = hamming_sinc(127)
    cq = q14(c)
    x = O.gen_cf32(1, 0, 0, 40000)
    xi = O.gen_ci16(2, 0, 0, 20000, -8192, 8191)
    cf = hamming_sinc(31, 0.2)
    xf = np.random.default_rng(3).integers(-2048, 2048, 5000).astype(np.float32)
    cu = q14(hamming_sinc(32, 0.12) * 4)
    p = qpsk_pattern(32, 500, seed=1)
    xc = np.random.default_rng(4).integers(-125, 126, size=(6000, 2)).astype(np.int32)
    for m in range(32):
        xc[3000 + 4 * m] += 2 * p[m]
    xc = xc.astype(np.int16)
    fin = tmp_path / "in.bin"
    with open(fin, "wb") as f:
        for tag, a in ((1, c), (2, x), (3, xi), (4, cq), (5, cf), (6, xf), (7, cu), (8, p), (9, xc)):
            _rec(f, tag, a)
    r = subprocess.run([exe, str(fin), str(tmp_path / "out.bin")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = _read(tmp_path / "out.bin")

    d = O.decim(0, 4, c)
    h = (len(x) // 2) & ~3
    exp = np.concatenate([d.step(x[:h]), d.step(x[h:])])
    assert got[101] == exp.tobytes()
    assert got[102] == O.decim(1, 4, cq).step(xi).tobytes()
    mix = O.mixer(4096)
    mix.reset(0.1)
    mixed = mix.step(xi)
    assert got[103] == mixed.tobytes()
    assert got[104] == O.decim(1, 4, cq).step(mixed).tobytes()
    assert got[105] == O.fir(1, cf).step(xf).tobytes()
    u = O.up(0, 4, cu)
    exp_u = np.concatenate([u.step(xi[:1000]), u.step(xi[1000:1500], flush=True, iterator=True)])
    assert got[106] == exp_u.tobytes()
    corr = O.corr(32, 4)
    corr.set_pattern(p)
    found, idx = corr.step(xc)
    st = corr.status()
    res = np.frombuffer(got[107], np.int32)
    assert res[0] == int(found) and (not found or res[1] == idx)
    assert list(res[2:]) == [np.int32(np.uint32(st["corr"][0])), np.int32(np.uint32(st["energy"][0])),
                             st["coeff_scaling"]]
    assert got[108] == corr.bit_samples().tobytes()
    # FIFO: the reference's buffers_test.cpp scenario vs the golden recorded from the reference
    from io_replay import load
    man, arr = load()
    bt = next(c for c in man["fifo"] if c["name"] == "fifo_buffers_test")
    exp = []
    for op in bt["ops"]:
        if op[0] == "count":
            exp.append(float(op[1]))
        elif op[0] == "read":
            exp += [float(op[3]), float(op[4])] + list(arr[op[5]].astype(np.float64))
    assert np.array_equal(np.frombuffer(got[109], np.float64), np.array(exp))
    # I/Q: whole samples only, output replaced
    assert got[110] == xi.tobytes()
    # value semantics: copies continue from the original's state, bit-exact
    h = (len(x) // 2) & ~3
    d = O.decim(0, 4, c)
    d.step(x[:h])
    exp_b = d.step(x[h:])
    assert got[111] == exp_b.tobytes() and got[112] == exp_b.tobytes()
    exp_bank = d.step(x[:h])  # the state after both halves, stepped with the first half
    assert got[113] == exp_bank.tobytes() and got[123] == exp_bank.tobytes() and got[124] == exp_bank.tobytes()
    assert got[114] == exp_bank.tobytes()
    mix = O.mixer(4096)
    mix.reset(0.1)
    mix.step(xi[:1000])
    exp_m = mix.step(xi[1000:2000])
    assert got[115] == exp_m.tobytes() and got[116] == exp_m.tobytes()
    fo = O.fir(2, cq)
    fo.step(xi[:1000])
    exp_f = fo.step(xi[1000:2000])
    assert got[117] == exp_f.tobytes() and got[118] == exp_f.tobytes()
    uo = O.up(0, 4, cu)
    uo.step(xi[:1000])
    exp_u2 = uo.step(xi[1000:2000])
    assert got[119] == exp_u2.tobytes() and got[120] == exp_u2.tobytes()
    co = O.corr(32, 4)
    co.set_pattern(p)
    co.step(xc[:2000])
    f2, i2 = co.step(xc[2000:])
    r = np.frombuffer(got[121], np.int32)
    assert f2 and r[0] == 1 and r[2] == 1 and r[1] == i2 and r[3] == i2
    assert got[122] == co.bit_samples().tobytes()


def test_sharded_header_compiles(tmp_path):
    src = """
#include "sharded_filters.h"
using cf32 = std::complex<float>; using ci16 = std::complex<int16_t>; using ci32 = std::complex<int32_t>;
template class dsptl::ShardedDnsamplingFir<cf32, cf32, cf32, float, 4>;
template class dsptl::ShardedDnsamplingFir<ci16, ci16, ci32, int32_t, 4>;
int main() { return 0; }
"""
    r = _compile(src, str(tmp_path / "a.out"), str(tmp_path))
    assert r.returncode == 0, r.stderr


@pytest.mark.gpu
def test_sharded_program_matches_oracle(tmp_path):
    """tests/cpp/sharded_main.cpp: 5 complex<float> decim-4 channels through
    dsptl::ShardedDnsamplingFir on a 1-GPU communicator (ncclCommInitAll over
    device 0): host-vector step() in two chained calls, then reset(), device
    step() and the RCCL gather -- every channel bit-exact with its own oracle
    FilterDnsamplingFir (FMA flavour).  Unmeasured at more than one GPU."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import pyoracle
    from srcdsp_amd.design import hamming_sinc
    exe = str(tmp_path / "sharded_main")
    r = subprocess.run(["g++", "-std=c++14", "-O2", "-D__HIP_PLATFORM_AMD__", "-I", INC, "-I", "/opt/rocm/include",
                        os.path.join(ROOT, "tests", "cpp", "sharded_main.cpp"), "-o", exe, "-L", LIBDIR,
                        "-lsrcdsp_hip", "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{LIBDIR}",
                        "-Wl,-rpath,/opt/rocm/lib"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    O = pyoracle.Oracle(1)
    c = hamming_sinc(127)
    C, n = 5, 40000
    xs = [O.gen_cf32(7, ch, 0, n) for ch in range(C)]
    fin = tmp_path / "in.bin"
    with open(fin, "wb") as f:
        _rec(f, 1, c)
        _rec(f, 2, np.array([C], np.int32))
        for ch in range(C):
            _rec(f, 10 + ch, xs[ch])
    r = subprocess.run([exe, str(fin), str(tmp_path / "out.bin"), "0"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    got = _read(tmp_path / "out.bin")
    half = (n // 2) & ~3
    alls = []
    for ch in range(C):
        d = O.decim(0, 4, c)
        exp = np.concatenate([d.step(xs[ch][:half]), d.step(xs[ch][half:])])
        assert got[100 + ch] == exp.tobytes(), ch
        alls.append(O.decim(0, 4, c).step(xs[ch]))
    assert got[200] == np.concatenate(alls).tobytes()
    assert got[201] == got[200]  # strided rows through the Memcpy2D branch of the gather
    assert got[202] == got[200]  # operator outliving its GpuComm
    assert got[203] == got[200]  # caller streams ordered by waitFor / signal (real RCCL, one rank)


@pytest.mark.gpu
@pytest.mark.parametrize("ndebug", [False, True], ids=["assert", "NDEBUG"])
@pytest.mark.parametrize("device", [False, True], ids=["host", "device"])
def test_mixer_step_undersized_out_is_refused(tmp_path, ndebug, device):
    """Mixer::step with out shorter than in (mixers.h:172-175
    writes in.size() outputs regardless) asserts in a debug build and throws
    std::length_error under NDEBUG -- before anything is staged or launched,
    so nothing is written past out's end."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    src = r"""
#include <csignal>
#include <cstdio>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include "mixers.h"
using ci16 = std::complex<int16_t>;
// the assert's abort() ends the process with a plain exit status (9), not a
// SIGABRT death, so the GPU box sees an ordinary exit
extern "C" void on_abort(int) { _exit(9); }
int main() {
    std::signal(SIGABRT, on_abort);
    dsptl::Mixer<ci16, ci16, int16_t, 4096> m;
    m.reset(0.1f);
    std::vector<ci16> in(1000, ci16(100, -100)), out(999);
    try {
        if (DEVICE) {
            ci16 *din = nullptr, *dout = nullptr;
            if (hipMalloc(&din, 1000 * sizeof(ci16)) || hipMalloc(&dout, 999 * sizeof(ci16))) return 3;
            m.step(dsptl::DeviceSpan<const ci16>{din, 1000}, dsptl::DeviceSpan<ci16>{dout, 999});
        } else {
            m.step(in, out);
        }
    } catch (const std::length_error &e) {
        std::printf("length_error: %s\n", e.what());
        return 7;
    }
    std::printf("no error\n");
    return 0;
}
"""
    p = tmp_path / "t.cpp"
    p.write_text(src)
    exe = str(tmp_path / "t")
    cmd = ["g++", "-std=c++14", "-O1", "-D__HIP_PLATFORM_AMD__", f"-DDEVICE={int(device)}", "-I", INC,
           "-I", "/opt/rocm/include", str(p), "-o", exe, "-L", LIBDIR, "-lsrcdsp_hip", "-L/opt/rocm/lib",
           "-lamdhip64", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib"] + (["-DNDEBUG"] if ndebug else [])
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    if ndebug:
        assert r.returncode == 7 and "output buffer smaller" in r.stdout, (r.returncode, r.stdout, r.stderr)
    else:
        assert r.returncode == 9 and "output buffer smaller than the call writes" in r.stderr, (r.returncode, r.stderr)


@pytest.mark.gpu
@pytest.mark.parametrize("ndebug", [False, True], ids=["assert", "NDEBUG"])
@pytest.mark.parametrize("case", ["short_out", "ragged_in", "few_vectors"])
def test_sharded_step_bad_vectors_are_refused(tmp_path, ndebug, case):
    """ShardedDnsamplingFir::step(host vectors): the C ABI takes one length for
    every channel and no output sizes, so the wrapper checks every vector
    first -- an output of the wrong size, channels of different lengths, or
    fewer vectors than channels assert in a debug build and throw
    std::length_error under NDEBUG, before anything is copied or launched."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    src = r"""
#include <csignal>
#include <cstdio>
#include <unistd.h>
#include <hip/hip_runtime.h>
#include "sharded_filters.h"
using cf32 = std::complex<float>;
extern "C" void on_abort(int) { _exit(9); }
int main() {
    std::signal(SIGABRT, on_abort);
    dsptl::GpuComm comm(std::vector<int>{0});
    std::vector<float> taps(127, 0.01f);
    dsptl::ShardedDnsamplingFir<cf32, cf32, cf32, float, 4> f(comm, 3, taps);
    std::vector<std::vector<cf32>> in(3, std::vector<cf32>(4096)), out(3, std::vector<cf32>(1024));
    if (CASE == 0) out[2].resize(1023);
    if (CASE == 1) in[1].resize(4100);
    if (CASE == 2) { in.resize(2); out.resize(2); }
    try {
        f.step(in, out);
    } catch (const std::length_error &e) {
        std::printf("length_error: %s\n", e.what());
        return 7;
    }
    std::printf("no error\n");
    return 0;
}
"""
    p = tmp_path / "t.cpp"
    p.write_text(src)
    exe = str(tmp_path / "t")
    icase = ["short_out", "ragged_in", "few_vectors"].index(case)
    cmd = ["g++", "-std=c++14", "-O1", "-D__HIP_PLATFORM_AMD__", f"-DCASE={icase}", "-I", INC,
           "-I", "/opt/rocm/include", str(p), "-o", exe, "-L", LIBDIR, "-lsrcdsp_hip", "-L/opt/rocm/lib",
           "-lamdhip64", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib"] + (["-DNDEBUG"] if ndebug else [])
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    if ndebug:
        assert r.returncode == 7 and "ShardedDnsamplingFir::step" in r.stdout, (r.returncode, r.stdout, r.stderr)
    else:
        assert r.returncode == 9 and "buffer shapes do not match the call" in r.stderr, (r.returncode, r.stderr)


def _corr_debug_golden():
    import json
    g = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(g, "corr_debug.json")) as f:
        return json.load(f), np.load(os.path.join(g, "corr_debug.npz"))


def test_dropin_corr_debug_files_compile(tmp_path):
    """CREATE_DEBUG_FILES: tests/cpp/corr_debug_main.cpp compiles against the
    drop-in with the macro (the reference's move-only object included)."""
    for n, s_ in ((32, 4), (1024, 1)):
        r = subprocess.run(["g++", "-std=c++14", "-Wall", "-DCREATE_DEBUG_FILES", f"-DCORR_N={n}", f"-DCORR_S={s_}",
                            "-I", INC, "-I", "/opt/rocm/include", "-D__HIP_PLATFORM_AMD__", "-fsyntax-only",
                            os.path.join(ROOT, "tests", "cpp", "corr_debug_main.cpp")], capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
    # the move-only object under the macro: move construction AND move
    # assignment (the reference's implicit ones), copies rejected
    src = tmp_path / "corr_move.cpp"
    src.write_text('#include <cmath>\n#include <cassert>\n#include <complex>\n#include <cstdint>\n#include <vector>\n#include <array>\n#include "correlators.h"\n#include <utility>\n'
                   'int main() {\n  dsptl::FixedPatternCorrelator<int16_t, int32_t, 32, 4> a, b;\n'
                   '  dsptl::FixedPatternCorrelator<int16_t, int32_t, 32, 4> c(std::move(a));\n'
                   '  b = std::move(c);\n  return 0;\n}\n')
    cmd = ["g++", "-std=gnu++11", "-Wall", "-DCREATE_DEBUG_FILES", "-I", INC, "-I", "/opt/rocm/include",
           "-D__HIP_PLATFORM_AMD__", "-fsyntax-only", str(src)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    src.write_text(src.read_text().replace("b = std::move(c);", "b = c;"))
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode != 0 and "deleted" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("key", [c["key"] for c in _corr_debug_golden()[0]["cases"]])
def test_dropin_corr_debug_files_match_reference(tmp_path, key):
    """The reference built with CREATE_DEBUG_FILES writes sqrt(energy),
    sqrt(corr) and 2.5 sqrt(energy) for every processed sample
    (correlators.h:253-257).  The same program compiled against the drop-in
    with the macro (step() through srcdsp_corr_step_host_trace) writes the
    same three files byte for byte, and the same detections
    (tests/golden/corr_debug.*, made from the reference by gen_corr_debug.py)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    man, arr = _corr_debug_golden()
    case = [c for c in man["cases"] if c["key"] == key][0]
    exe = str(tmp_path / "corr_debug_main")
    r = subprocess.run(["g++", "-std=c++14", "-O2", "-DCREATE_DEBUG_FILES", f"-DCORR_N={case['N']}",
                        f"-DCORR_S={case['S']}", "-D__HIP_PLATFORM_AMD__", "-I", INC, "-I", "/opt/rocm/include",
                        os.path.join(ROOT, "tests", "cpp", "corr_debug_main.cpp"), "-o", exe, "-L", LIBDIR,
                        "-lsrcdsp_hip", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath,/opt/rocm/lib"],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    run = tmp_path / "run"
    run.mkdir()
    (run / "in.bin").write_bytes(arr[key + "_in"].tobytes())
    r = subprocess.run([exe, "in.bin", "steps.txt"], cwd=str(run), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert (run / "steps.txt").read_bytes() == arr[key + "_steps.txt"].tobytes()
    for name in man["files"]:
        got, want = (run / name).read_bytes(), arr[key + "_" + name].tobytes()
        assert got.count(b"\n") == case["debug_lines"] and got == want, name
