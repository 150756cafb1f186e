"""Seeded differential fuzzing of the HIP path against the C oracle (which
tests/test_oracle_golden.py pins to the reference): random operator shapes,
random chains of step() calls of ragged lengths (including 0 and 1), resets,
left shifts and coefficient changes, device-resident and host-staged calls
interleaved.  Every output byte must match.  Shapes are drawn to hit the tuned
kernels (63/64/127/128/255/256 taps at M = 1/2/3/4/8/16, M = 1, L = 2/4 with 16/32/64
taps per phase) as often as the generic ones."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

_DECIM_T = {0: ("complex<float>", "complex<float>", "complex<float>", "float"),
            1: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t"),
            2: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int16_t"),
            3: ("complex<int32_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")}
_FIR_T = {0: ("complex<float>", "complex<float>", "complex<float>", "float"),
          1: ("float", "complex<float>", "float", "float"),
          2: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")}
_UP_T = {0: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t"),
         1: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int16_t"),
         2: ("int16_t", "int16_t", "int32_t", "int32_t")}


@pytest.fixture(scope="module")
def O():
    import pyoracle
    return {"strict": pyoracle.Oracle(0), "fma": pyoracle.Oracle(1)}


def _dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


def _run(op, x, on_device):
    if on_device:
        return op.step(_dev(x)).cpu().numpy()
    return op.step(x)


def _taps(rng, variant, n):
    if variant == 0:
        return (rng.standard_normal(n) / max(2.0, n / 4)).astype(np.float32)
    if variant == 2:
        return rng.integers(-2000, 2000, n).astype(np.int16)
    kind = rng.integers(0, 3)  # int16 range (dot2), < 2^23 (mad24), wide
    lim = (32767, (1 << 23) - 1, 1 << 26)[kind]
    return rng.integers(-lim, lim + 1, n).astype(np.int32)


def _input(rng, O, variant, n):
    if variant == 0:
        x = O["fma"].gen_cf32(int(rng.integers(1 << 30)), 0, 0, n, -30000, 30000)
        if n and rng.random() < 0.2:  # a few large / special values
            k = rng.integers(0, n, 3)
            x[k] = np.array([3e9 + 1j, -np.inf + 0j, np.nan * 1j], np.complex64)[: len(k)]
        return x
    if variant == 3:
        return rng.integers(-(1 << 20), 1 << 20, size=(n, 2)).astype(np.int32)
    return O["fma"].gen_ci16(int(rng.integers(1 << 30)), 0, 0, n, -32768, 32767)


@pytest.mark.parametrize("seed", range(40))
def test_fuzz_decimator(S, O, seed):
    rng = np.random.default_rng(1000 + seed)
    variant = int(rng.integers(0, 4))
    M = int(rng.choice([1, 2, 3, 4, 4, 4, 5, 8, 16]))
    ntaps = int(rng.choice([1, 2, 7, 31, 63, 64, 127, 127, 128, 129, 200, 255, 256]))
    fp = str(rng.choice(["fma", "strict"]))
    c = _taps(rng, variant, ntaps)
    g = S.FilterDnsamplingFir(c, M, *_DECIM_T[variant], fp=fp)
    r = O[fp].decim(variant, M, c)
    for op in range(10):
        u = rng.random()
        if u < 0.08:
            g.reset()
            r.reset()
        elif u < 0.14:
            ls = int(rng.integers(0, 3))
            g.setLeftShiftBy2(ls)
            r.set_left_shift(ls)
        elif u < 0.2:
            c = _taps(rng, variant, int(rng.choice([ntaps, 1, 63, 64, 127, 128, 255])))
            g.setCoeffs(c, require_multiple=False)
            r.set_coeffs(c)
        n = M * int(rng.choice([0, 1, 3, 17, 1024, 4099, 20000, int(rng.integers(0, 30000))]))
        x = _input(rng, O, variant, n)
        got, exp = _run(g, x, bool(rng.integers(0, 2))), r.step(x)
        assert got.tobytes() == exp.tobytes(), (seed, op, variant, M, ntaps, fp, n)


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_fir(S, O, seed):
    rng = np.random.default_rng(2000 + seed)
    variant = int(rng.integers(0, 3))
    ntaps = int(rng.choice([1, 3, 31, 31, 100, 128, 129, 500, 1100]))
    fp = str(rng.choice(["fma", "strict"]))
    tv = {0: 0, 1: 0, 2: 1}[variant]
    c = _taps(rng, tv, ntaps).astype(np.float32 if variant < 2 else np.int32)
    g = S.FilterFir(c, *_FIR_T[variant], fp=fp)
    r = O[fp].fir(variant, c)
    for op in range(8):
        if rng.random() < 0.1:
            g.reset()
            r.reset()
        n = int(rng.choice([0, 1, 5, 2048, 2049, 9000, int(rng.integers(0, 20000))]))
        if variant == 1:
            x = O["fma"].gen_cf32(int(rng.integers(1 << 30)), 0, 0, n, -30000, 30000).real.astype(np.float32)
        else:
            x = _input(rng, O, 0 if variant == 0 else 1, n)
        got, exp = _run(g, x, bool(rng.integers(0, 2))), r.step(x)
        assert got.tobytes() == exp.tobytes(), (seed, op, variant, ntaps, fp, n)


@pytest.mark.parametrize("seed", range(16))
def test_fuzz_upsampler(S, O, seed):
    rng = np.random.default_rng(3000 + seed)
    variant = int(rng.integers(0, 3))
    L = int(rng.choice([1, 2, 3, 4, 4, 8]))
    H = int(rng.choice([1, 2, 5, 16, 32, 33, 64, 70]))
    lim = {0: int(rng.choice([32767, 1 << 22, 1 << 26])), 1: 32767, 2: 30000}[variant]
    c = rng.integers(-lim, lim + 1, L * H)
    g = S.FilterUpsamplingFir(c, L, *_UP_T[variant])
    r = O["fma"].up(variant, L, c)
    for op in range(8):
        if rng.random() < 0.1:
            g.reset()
            r.reset()
        n = int(rng.choice([0, 1, 7, 2048, 2049, int(rng.integers(0, 9000))]))
        x = O["fma"].gen_ci16(int(rng.integers(1 << 30)), 0, 0, n, -32768, 32767)
        if variant == 2:
            x = np.ascontiguousarray(x[:, 0])
        flush, it = bool(rng.random() < 0.2), bool(rng.random() < 0.3)
        if bool(rng.integers(0, 2)):
            got = g.step(_dev(x), None, flush, it).cpu().numpy()
        else:
            got = g.step(x, None, flush, it)
        exp = r.step(x, flush, it)
        assert got.tobytes() == exp.tobytes(), (seed, op, variant, L, H, n, flush, it)


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_mixer_and_chain(S, O, seed):
    rng = np.random.default_rng(4000 + seed)
    N = int(rng.choice([16, 1000, 4096, 4096]))
    f = float(rng.uniform(-1, 1))
    m, om = S.Mixer(N), O["fma"].mixer(N)
    m.reset(f)
    om.reset(f)
    fused = bool(rng.integers(0, 2))
    if fused:
        from srcdsp_amd.design import hamming_sinc, q14
        # M = 4 x 127/128 is the fused kernel; the others run as the two calls
        Md = int(rng.choice([4, 4, 4, 2, 8]))
        cq = q14(hamming_sinc(int(rng.choice([127, 128, 63])), 0.12))
        d = S.FilterDnsamplingFir(cq, Md, *_DECIM_T[1])
        chain = S.MixerDecimatorChain(m, d)
        od = O["fma"].decim(1, Md, cq)
    for op in range(8):
        u = rng.random()
        if u < 0.15:
            a = float(rng.uniform(-0.5, 0.5))
            m.adjustFrequency(a)
            om.adjust_frequency(a)
        elif u < 0.25:
            f = float(rng.uniform(-1, 1))
            m.setFrequency(f)
            om.set_frequency(f)
        n = 8 * int(rng.choice([0, 1, 7, 1000, 4097, int(rng.integers(0, 20000))]))
        x = O["fma"].gen_ci16(int(rng.integers(1 << 30)), 0, 0, n, -32768, 32767)
        if fused:
            got = chain.step(_dev(x)).cpu().numpy()
            exp = od.step(om.step(x))
        else:
            got = _run(m, x, bool(rng.integers(0, 2)))
            exp = om.step(x)
        assert got.tobytes() == exp.tobytes(), (seed, op, N, fused, n)
        assert m.state()[:2] == om.state()[:2]


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_correlator(S, O, seed):
    from srcdsp_amd.design import qpsk_pattern
    rng = np.random.default_rng(5000 + seed)
    N, Sx = [(32, 1), (32, 4), (64, 2), (1024, 1), (48, 1), (16, 3)][seed % 6]
    p = qpsk_pattern(N, int(rng.choice([200, 500])), seed=seed)
    g, r = S.FixedPatternCorrelator(N, Sx), O["fma"].corr(N, Sx)
    g.setPattern(p)
    r.set_pattern(p)
    for op in range(6):
        if rng.random() < 0.1:
            g.reset()
            r.reset()
        n = int(rng.choice([0, 1, 5, 5000, 30000, int(rng.integers(0, 40000))]))
        x = rng.integers(-125, 126, size=(n, 2))
        for _ in range(int(rng.integers(0, 3))):  # embedded copies of the pattern (strided by S)
            if n > N * Sx + 10:
                at = int(rng.integers(0, n - N * Sx))
                x[at:at + N * Sx:Sx] += 2 * p
        x = np.clip(x, -32768, 32767).astype(np.int16)
        got = g.step(_dev(x)) if bool(rng.integers(0, 2)) else g.step(x)
        exp = r.step(x)
        assert got[0] == exp[0] and (not exp[0] or got[1] == exp[1]), (seed, op, N, Sx, n, got, exp)
        if exp[0]:
            assert np.array_equal(g.getRefBitSamples(), r.bit_samples())
        st = r.status()
        gs = g.getStatus()
        assert list(gs["corr"]) == st["corr"] and list(gs["energy"]) == st["energy"], (seed, op)


# --- the run-time-shape kernels of round 3, drawn over their whole ranges ---
# (decim_stream_cf32 / decim_dot2_ci16 at any N <= 1024 and M in {1, 2, 3, 4,
# 6, 8, 12, 16}; up_tile_dot2 at L = 2..8 and any taps per phase;
# corr_eval_dot2 at any N >= 48 and stride S; the fused chain at any N)

def _any_taps(rng):
    return int(rng.choice([int(rng.integers(2, 48)), int(rng.integers(48, 400)), int(rng.integers(400, 1025)),
                           int(rng.integers(1025, 1300))]))


@pytest.mark.parametrize("seed", range(24))
def test_fuzz_decimator_any_shape(S, O, seed):
    rng = np.random.default_rng(6000 + seed)
    variant = int(rng.choice([0, 0, 1, 1, 2]))
    M = int(rng.choice([1, 2, 3, 4, 6, 8, 12, 16]))
    ntaps = _any_taps(rng)
    fp = str(rng.choice(["fma", "strict"]))
    c = _taps(rng, variant, ntaps)
    if variant == 1 and rng.random() < 0.6:  # int16-range taps in an int32 filter: the dot2 kernel
        c = rng.integers(-32768, 32768, ntaps).astype(np.int32)
    g = S.FilterDnsamplingFir(c, M, *_DECIM_T[variant], fp=fp)
    r = O[fp].decim(variant, M, c)
    for op in range(6):
        if rng.random() < 0.1:
            g.reset()
            r.reset()
        n = M * int(rng.choice([0, 1, 5, 2047, 8193, int(rng.integers(0, 24000))]))
        x = _input(rng, O, variant, n)
        got, exp = _run(g, x, bool(rng.integers(0, 2))), r.step(x)
        assert got.tobytes() == exp.tobytes(), (seed, op, variant, M, ntaps, fp, n)


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_upsampler_any_shape(S, O, seed):
    rng = np.random.default_rng(7000 + seed)
    L = int(rng.integers(2, 9))
    H = int(rng.choice([int(rng.integers(1, 20)), int(rng.integers(20, 140))]))
    c = rng.integers(-32767, 32768, L * H)
    g = S.FilterUpsamplingFir(c, L, *_UP_T[0])
    r = O["fma"].up(0, L, c)
    for op in range(6):
        if rng.random() < 0.1:
            g.reset()
            r.reset()
        n = int(rng.choice([0, 1, 7, 2048, 4099, int(rng.integers(0, 12000))]))
        x = O["fma"].gen_ci16(int(rng.integers(1 << 30)), 0, 0, n, -32768, 32767)
        flush, it = bool(rng.random() < 0.2), bool(rng.random() < 0.3)
        if bool(rng.integers(0, 2)):
            got = g.step(_dev(x), None, flush, it).cpu().numpy()
        else:
            got = g.step(x, None, flush, it)
        exp = r.step(x, flush, it)
        assert got.tobytes() == exp.tobytes(), (seed, op, L, H, n, flush, it)


@pytest.mark.parametrize("seed", range(12))
def test_fuzz_correlator_any_shape(S, O, seed):
    from srcdsp_amd.design import qpsk_pattern
    rng = np.random.default_rng(8000 + seed)
    N, Sx = int(rng.integers(48, 330)), int(rng.integers(1, 6))
    p = qpsk_pattern(N, int(rng.choice([200, 500])), seed=seed)
    g, r = S.FixedPatternCorrelator(N, Sx), O["fma"].corr(N, Sx)
    g.setPattern(p)
    r.set_pattern(p)
    for op in range(5):
        if rng.random() < 0.1:
            g.reset()
            r.reset()
        n = int(rng.choice([0, 1, 5, 9000, int(rng.integers(0, 40000))]))
        x = rng.integers(-125, 126, size=(n, 2))
        for _ in range(int(rng.integers(0, 3))):
            if n > N * Sx + 10:
                at = int(rng.integers(0, n - N * Sx))
                x[at:at + N * Sx:Sx] += 2 * p
        x = np.clip(x, -32768, 32767).astype(np.int16)
        got = g.step(_dev(x)) if bool(rng.integers(0, 2)) else g.step(x)
        exp = r.step(x)
        assert got[0] == exp[0] and (not exp[0] or got[1] == exp[1]), (seed, op, N, Sx, n, got, exp)
        if exp[0]:
            assert np.array_equal(g.getRefBitSamples(), r.bit_samples())
        st, gs = r.status(), g.getStatus()
        assert list(gs["corr"]) == st["corr"] and list(gs["energy"]) == st["energy"], (seed, op, N, Sx)


@pytest.mark.parametrize("seed", range(10))
def test_fuzz_chain_any_shape(S, O, seed):
    rng = np.random.default_rng(9000 + seed)
    N = int(rng.choice([16, 1000, 4096]))
    f = float(rng.uniform(-1, 1))
    m, om = S.Mixer(N), O["fma"].mixer(N)
    m.reset(f)
    om.reset(f)
    Md = int(rng.choice([1, 2, 4, 8, 16]))
    nt = int(rng.integers(2, 1025))
    c = rng.integers(-32768, 32768, nt).astype(np.int32)
    d = S.FilterDnsamplingFir(c, Md, *_DECIM_T[1])
    chain = S.MixerDecimatorChain(m, d)
    od = O["fma"].decim(1, Md, c)
    for op in range(6):
        if rng.random() < 0.15:
            a = float(rng.uniform(-0.5, 0.5))
            m.adjustFrequency(a)
            om.adjust_frequency(a)
        n = 16 * int(rng.choice([0, 1, 7, 1000, int(rng.integers(0, 12000))]))
        x = O["fma"].gen_ci16(int(rng.integers(1 << 30)), 0, 0, n, -32768, 32767)
        got = chain.step(_dev(x)).cpu().numpy()
        exp = od.step(om.step(x))
        assert got.tobytes() == exp.tobytes(), (seed, op, N, Md, nt, n)
        assert m.state()[:2] == om.state()[:2]
