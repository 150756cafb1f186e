"""Parity of the HIP path (through the C ABI) with the reference.

* every golden script (reference outputs, tests/golden) replayed on the GPU,
  device-resident and host-staged, in both float contracts -- bit-exact;
* larger seeded cases against the C oracle (pinned to the reference by
  test_oracle_golden.py) -- bit-exact;
* the headline size (2^28 samples) through size-independent checks.
"""
import numpy as np
import pytest

from replay import OracleBackend, load_golden, replay

pytestmark = pytest.mark.gpu
G = load_golden()


@pytest.fixture(scope="module")
def S():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import srcdsp_amd
    srcdsp_amd.lib()
    return srcdsp_amd


@pytest.fixture(scope="module")
def O():
    import pyoracle
    return {"strict": pyoracle.Oracle(0), "fma": pyoracle.Oracle(1)}


def dev(x):
    import torch
    return torch.from_numpy(np.ascontiguousarray(x)).cuda()


# ------------------------------------------------------------------ goldens
@pytest.mark.parametrize("device", [True, False], ids=["device", "host"])
@pytest.mark.parametrize("fp", ["fma", "strict"])
@pytest.mark.parametrize("name", G.names())
def test_golden_replay_on_gpu(S, name, fp, device):
    from gpu_backend import GpuBackend
    fails = replay(G.cases[name], G, GpuBackend(fp, device))
    assert not fails, "\n".join(fails)


# ------------------------------------------------------- decimator, larger
def _chunks(total, sizes):
    out, i, k = [], 0, 0
    while i < total:
        n = min(sizes[k % len(sizes)], total - i)
        out.append((i, n))
        i += n
        k += 1
    return out


@pytest.mark.parametrize("fp", ["fma", "strict"])
@pytest.mark.parametrize("M,ntaps", [(4, 63), (4, 64), (4, 127), (4, 128), (4, 255), (4, 256),
                                     (8, 127), (8, 128), (8, 255), (8, 256), (2, 63), (2, 64), (2, 127), (2, 128),
                                     (1, 63), (1, 64), (1, 127), (1, 128), (3, 63), (3, 64), (3, 127), (3, 128),
                                     (16, 127), (16, 128), (16, 255), (16, 256)])
def test_decim_cf32_tile_kernel_vs_oracle(S, O, fp, M, ntaps):
    """The headline kernel at every (M, tap count) it is compiled for: many
    tiles, tail tiles, history carried over uneven calls (incl. calls shorter
    than a tile)."""
    from srcdsp_amd.design import hamming_sinc
    c = hamming_sinc(ntaps - (ntaps % 2 == 0))
    if ntaps % 2 == 0:  # an even count: a trailing zero tap, as the 128-tap form of the 127-tap filter
        c = np.concatenate([c, [0.0]]).astype(np.float32)
    x = O[fp].gen_cf32(0x5EED, 3, 0, 1 << 20, -32768, 32767)
    x = x + np.float32(0.37)  # non-integer inputs exercise rounding
    ref = O[fp].decim(0, M, c)
    g = S.FilterDnsamplingFir(c, M, fp=fp)
    for off, n in _chunks(len(x), [400000, 8, 2048 * M + M, 131072, 128, 300004]):
        n -= n % M
        if n == 0:
            continue
        xs = x[off:off + n]
        y = g.step(dev(xs)).cpu().numpy()
        assert np.array_equal(y.view(np.uint32), ref.step(xs).view(np.uint32)), (off, n)


@pytest.mark.parametrize("fp", ["fma", "strict"])
@pytest.mark.parametrize("M,ntaps", [(2, 1), (2, 16), (2, 17), (2, 63), (2, 128), (4, 2), (4, 15), (4, 48),
                                     (4, 63), (4, 255), (4, 1024), (8, 8), (8, 49), (8, 255), (8, 1000),
                                     (3, 1), (3, 13), (3, 95), (5, 21), (5, 100), (6, 11), (6, 72), (16, 17),
                                     (16, 256)])
def test_decim_cf32_any_taps_tile_vs_oracle(S, O, fp, M, ntaps):
    """decim_tile_cf32 (M in 2/4/8, runtime tap count <= 1024): tail tiles,
    calls shorter than the filter, chained uneven calls, both float contracts."""
    rng = np.random.default_rng(M * 10000 + ntaps)
    c = (rng.standard_normal(ntaps) / max(2, ntaps) ** 0.5).astype(np.float32)
    x = O[fp].gen_cf32(33 + ntaps, M, 0, 200000)
    g = S.FilterDnsamplingFir(c, M, fp=fp)
    r = O[fp].decim(0, M, c)
    for off, n in _chunks(len(x), [65536, M, 8 * M, 70000, 4 * M * 1000 + 8]):
        n -= n % M
        xs = x[off:off + n]
        assert np.array_equal(g.step(dev(xs)).cpu().numpy(), r.step(xs)), (off, n)


RT_SHAPES = [(4, n) for n in (1, 2, 5, 31, 95, 100, 129, 200, 300, 511, 700, 1024)] + \
    [(1, n) for n in (1, 31, 100, 300, 1024)] + [(2, n) for n in (3, 95, 200, 513)] + \
    [(3, n) for n in (4, 50, 301)] + [(8, n) for n in (7, 129, 1000)] + [(16, n) for n in (9, 200, 1023)] + \
    [(6, n) for n in (1, 13, 127, 600)] + [(12, n) for n in (5, 127, 1024)]


@pytest.mark.parametrize("fp", ["fma", "strict"])
@pytest.mark.parametrize("M,ntaps", RT_SHAPES)
def test_decim_cf32_runtime_taps_vs_oracle(S, O, fp, M, ntaps):
    """The headline kernel with the tap count at run time (any N <= 1024 at
    M in 1/2/3/4/6/8/12/16, decim_stream_cf32<0, ...>): full chunks, the guarded
    last chunk, taps past N never applied (inf / NaN samples in the stream and
    the history would turn a 0 * x into NaN), tail tiles and chained uneven
    calls, both float contracts."""
    rng = np.random.default_rng(M * 7919 + ntaps)
    c = (rng.standard_normal(ntaps) / max(2, ntaps) ** 0.5).astype(np.float32)
    x = O[fp].gen_cf32(91 + ntaps, M, 0, 300000, -32768, 32767) + np.float32(0.37)
    # a few special values, so a tap past N multiplied by one would show
    for i, v in ((5000, np.inf), (77777, -np.inf), (150001, np.nan), (299990, np.inf)):
        x[i] = np.complex64(complex(v, 1.0))
    g = S.FilterDnsamplingFir(c, M, fp=fp) if M > 1 else S.FilterFir(c, "complex<float>", "complex<float>",
                                                                      "complex<float>", "float", fp=fp)
    r = O[fp].decim(0, M, c) if M > 1 else O[fp].fir(0, c)
    for off, n in _chunks(len(x), [65536, M, 8 * M, 70001 * M, 4 * M * 1000 + 8, 3]):
        n -= n % M
        if n == 0:
            continue
        xs = x[off:off + n]
        y = g.step(dev(xs)).cpu().numpy()
        assert np.array_equal(y.view(np.uint32), r.step(xs).view(np.uint32)), (off, n)


@pytest.mark.parametrize("kind", ["i16", "i24", "i32", "t16"])
@pytest.mark.parametrize("M,ntaps", [(2, 1), (2, 33), (2, 127), (4, 17), (4, 63), (4, 200), (8, 16), (8, 255),
                                     (8, 1024), (3, 40), (5, 61), (6, 13), (16, 100)])
def test_decim_ci16_any_taps_tile_vs_oracle(S, O, kind, M, ntaps):
    """decim_tile for complex<int16_t> (M in 2/4/8, runtime tap count <= 1024):
    int32 taps in int16 / i24 / wider range (v_mad_i32_i24 or full 32-bit
    products) and int16 taps (products wrapped to int16, "t16"); full-scale
    inputs so the accumulators wrap and the outputs saturate."""
    rng = np.random.default_rng(M * 100 + ntaps + len(kind))
    lim = {"i16": 32767, "i24": (1 << 23) - 1, "i32": 1 << 24, "t16": 32767}[kind]
    c = rng.integers(-lim, lim + 1, size=ntaps).astype(np.int32)
    c[0] = lim
    x = O["strict"].gen_ci16(7 + ntaps, M, 0, 150000, -32768, 32767)
    if kind == "t16":
        c = c.astype(np.int16)
        g = S.FilterDnsamplingFir(c, M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int16_t")
        r = O["strict"].decim(2, M, c)
    else:
        g = S.FilterDnsamplingFir(c, M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
        r = O["strict"].decim(1, M, c)
    for off, n in _chunks(len(x), [65536, M, 8 * M, 60000, 2 * M * 1000 + 4]):
        n -= n % M
        xs = x[off:off + n]
        assert np.array_equal(g.step(dev(xs)).cpu().numpy(), r.step(xs)), (off, n)


@pytest.mark.parametrize("kind,M,ntaps", [("cf32", 2, 63), ("cf32", 4, 63), ("cf32", 3, 95), ("cf32", 8, 1000),
                                          ("cf32", 4, 600), ("i24", 4, 63), ("t16", 2, 127), ("i16", 5, 61),
                                          ("i32", 16, 300)])
def test_decim_tile_large_calls_vs_oracle(S, O, kind, M, ntaps):
    """decim_tile on calls of 2^23-2^24 samples (thousands of tiles, more
    workgroups than the chip holds at once), long halos (600 and 1000 taps),
    a ragged last tile and a call shorter than the filter; chained calls carry
    the history.  Bit-exact against the oracle on every output."""
    rng = np.random.default_rng(M * 7 + ntaps)
    total = (1 << 24) + 3 * M * 1000 + 5 * M
    if kind == "cf32":
        c = (rng.standard_normal(ntaps) / max(2, ntaps) ** 0.5).astype(np.float32)
        x = O["fma"].gen_cf32(99 + ntaps, M, 0, total)
        g = S.FilterDnsamplingFir(c, M, fp="fma")
        r = O["fma"].decim(0, M, c)
    else:
        lim = {"i16": 32767, "i24": (1 << 23) - 1, "i32": 1 << 24, "t16": 32767}[kind]
        c = rng.integers(-lim, lim + 1, size=ntaps).astype(np.int32)
        x = O["strict"].gen_ci16(5 + ntaps, M, 0, total, -32768, 32767)
        if kind == "t16":
            c = c.astype(np.int16)
            g = S.FilterDnsamplingFir(c, M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int16_t")
            r = O["strict"].decim(2, M, c)
        else:
            g = S.FilterDnsamplingFir(c, M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
            r = O["strict"].decim(1, M, c)
    for off, n in _chunks(len(x), [1 << 23, (1 << 23) + 3 * M * 1000, 5 * M]):
        n -= n % M
        xs = x[off:off + n]
        assert np.array_equal(g.step(dev(xs)).cpu().numpy(), r.step(xs)), (off, n)


@pytest.mark.parametrize("ntaps", [63, 64, 127, 128, 255, 256])
def test_decim_ci16_dot2_tap_counts_vs_oracle(S, O, ntaps):
    """The v_dot2 decimator (int16-range taps, M = 4) at every tap count it is
    compiled for: full-scale inputs (accumulator wrap, output saturation), many
    tiles, a tail tile, history carried over uneven calls."""
    rng = np.random.default_rng(1000 + ntaps)
    c = rng.integers(-32768, 32768, size=ntaps).astype(np.int32)
    c[0], c[-1] = 32767, -32768
    x = O["strict"].gen_ci16(77 + ntaps, 4, 0, 1 << 20, -32768, 32767)
    g = S.FilterDnsamplingFir(c, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    r = O["strict"].decim(1, 4, c)
    for off, n in _chunks(len(x), [400000, 8, 2048 * 4 + 4, 131072, 128, 300004]):
        n -= n % 4
        xs = x[off:off + n]
        assert np.array_equal(g.step(dev(xs)).cpu().numpy(), r.step(xs)), (off, n)


DOT2_RT_TAPS = [1, 2, 3, 5, 17, 31, 62, 65, 100, 126, 129, 200, 257, 300, 511, 600, 1000, 1023, 1024]


DOT2_RT_SHAPES = ([(4, n) for n in DOT2_RT_TAPS] +
                  [(2, n) for n in (1, 2, 7, 31, 63, 64, 65, 127, 200, 1024)] +
                  [(8, n) for n in (1, 9, 63, 127, 128, 255, 300, 1024)] +
                  [(16, n) for n in (1, 17, 127, 255, 256, 511, 1024)] +
                  [(1, n) for n in (1, 2, 3, 16, 17, 31, 64, 127, 300, 1024)])


@pytest.mark.parametrize("M,ntaps", DOT2_RT_SHAPES)
def test_decim_ci16_dot2_runtime_taps_vs_oracle(S, O, M, ntaps):
    """The v_dot2 decimator with the tap count at run time (int16-range taps,
    any N <= 1024 at M = 1 (even / odd output passes), 2, 8, 16, and at M = 4 off the compiled
    63/64/127/128/255/256): the pairs padded with zero pairs to whole 4-pair
    steps, chunk tails, the longest halos; full-scale inputs (accumulator
    wrap, saturation), a call shorter than the filter, history carried over
    uneven calls."""
    rng = np.random.default_rng(2000 + 7 * M + ntaps)
    c = rng.integers(-32768, 32768, size=ntaps).astype(np.int32)
    c[0], c[-1] = 32767, -32768 if ntaps > 1 else 32767
    x = O["strict"].gen_ci16(31 + ntaps + M, 4, 0, 600000, -32768, 32767)
    g = S.FilterDnsamplingFir(c, M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    r = O["strict"].decim(1, M, c)
    for off, n in _chunks(len(x), [200000, 8 * M, 2048 * M + 4 * M, M * ((ntaps + 3) // 4) + M, 131072, 128]):
        n -= n % M
        xs = x[off:off + n]
        assert np.array_equal(g.step(dev(xs)).cpu().numpy(), r.step(xs)), (off, n)


@pytest.mark.parametrize("M,ntaps,N,f", [(4, 1, 4096, 0.1), (4, 31, 4096, 0.1), (4, 63, 1000, -0.37),
                                         (4, 64, 4096, 0.5), (4, 129, 4096, 0.1), (4, 200, 3000, 0.3),
                                         (4, 255, 4093, 0.1), (4, 1024, 4096, 0.73), (2, 63, 4096, 0.1),
                                         (2, 127, 4093, -0.2), (8, 127, 4096, 0.1), (8, 255, 1000, 0.37),
                                         (16, 255, 4096, 0.1), (16, 1024, 4093, 0.3), (1, 31, 4096, 0.1),
                                         (1, 128, 4093, -0.45)])
def test_mixdecim_chain_runtime_taps(S, O, M, ntaps, N, f):
    """Config 4's fused mixer -> decimator off the compiled M = 4 x 127/128:
    the run-time-tap dot2 kernel with the mixer in its staging pass at
    M = 1, 2, 4, 8, 16, both mixer table forms (N = 4093 at f = 0.1 / -0.2 /
    0.3: the doubled phase table), Q14 taps of the design filter and
    full-scale inputs; the same outputs and mixer state as the two
    reference calls."""
    from srcdsp_amd.design import hamming_sinc, q14
    cq = q14(hamming_sinc(ntaps)) if ntaps > 1 else np.array([16384], np.int32)
    x = O["strict"].gen_ci16(0xF00 + ntaps, 3, 0, 400000, -32768, 32767)
    m = S.Mixer(N)
    m.reset(f)
    d = S.FilterDnsamplingFir(cq, M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    chain = S.MixerDecimatorChain(m, d)
    om, od = O["strict"].mixer(N), O["strict"].decim(1, M, cq)
    om.reset(f)
    for off, n in _chunks(len(x), [131072, 8 * M, 4100, 200000]):
        n -= n % M
        xs = x[off:off + n]
        assert np.array_equal(chain.step(dev(xs)).cpu().numpy(), od.step(om.step(xs))), (off, n)
        assert m.state()[:2] == om.state()[:2]


@pytest.mark.parametrize("kind", ["i16", "i24", "i32"])
@pytest.mark.parametrize("ntaps", [1, 16, 17, 31, 100, 1024])
def test_fir_ci16_tile_vs_oracle(S, O, kind, ntaps):
    """FilterFir<ci16,ci16,ci32,int32_t> (filters.h:131-169) on decim_tile with
    M = 1: int32 taps in the three product ranges, full-scale inputs, chained
    uneven calls."""
    rng = np.random.default_rng(ntaps * 3 + len(kind))
    lim = {"i16": 32767, "i24": (1 << 23) - 1, "i32": 1 << 24}[kind]
    c = rng.integers(-lim, lim + 1, size=ntaps).astype(np.int32)
    c[0] = lim
    x = O["strict"].gen_ci16(5 + ntaps, 3, 0, 90000, -32768, 32767)
    g = S.FilterFir(c, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    r = O["strict"].fir(2, c)
    for off, n in _chunks(len(x), [40000, 1, 7, 4096 + 3, 30000]):
        xs = x[off:off + n]
        assert np.array_equal(g.step(dev(xs)).cpu().numpy(), r.step(xs)), (off, n)


def test_decim_fma_vs_strict_tolerance(S, O):
    """Stated float tolerance: the FMA contract differs from the
    -O2 x86-64 reference by at most 1 output LSB on at most 1e-4 of outputs."""
    from srcdsp_amd.design import hamming_sinc
    c = hamming_sinc(127)
    x = O["strict"].gen_cf32(0x5EED, 0, 0, 1 << 22)
    y = S.FilterDnsamplingFir(c, 4, fp="fma").step(dev(x)).cpu().numpy()
    r = O["strict"].decim(0, 4, c).step(x)
    d = np.abs(y.view(np.float32) - r.view(np.float32))
    assert d.max() <= 1.0
    assert np.count_nonzero(d) <= 1e-4 * d.size


def test_decim_ci16_tile_and_mixer_chain_vs_oracle(S, O):
    from srcdsp_amd.design import hamming_sinc, q14
    cq = q14(hamming_sinc(127))
    x = O["strict"].gen_ci16(0x5EED, 1, 0, 1 << 20, -8192, 8191)
    # plain fixed-point decimator (tile kernel, v_mad_i32_i24)
    g = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    r = O["strict"].decim(1, 4, cq)
    for off, n in _chunks(len(x), [262144, 4, 1024, 500000]):
        n -= n % 4
        xs = x[off:off + n]
        assert np.array_equal(g.step(dev(xs)).cpu().numpy(), r.step(xs)), (off, n)
    # config 4: mixer -> decimator fused, against the two reference calls
    m = S.Mixer(4096)
    m.reset(0.1)
    d = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    chain = S.MixerDecimatorChain(m, d)
    om, od = O["strict"].mixer(4096), O["strict"].decim(1, 4, cq)
    om.reset(0.1)
    for off, n in _chunks(len(x), [300000, 12, 65536, 700000]):
        n -= n % 4
        xs = x[off:off + n]
        y = chain.step(dev(xs)).cpu().numpy()
        assert np.array_equal(y, od.step(om.step(xs))), (off, n)
        assert m.state()[:2] == om.state()[:2]


@pytest.mark.parametrize("ntaps", [127, 128])
@pytest.mark.parametrize("kind", ["i16", "i24", "i32"])
def test_decim_ci16_tap_ranges_vs_oracle(S, O, ntaps, kind):
    """int16-range taps run the v_dot2 kernel, |c| < 2^23 the v_mad_i32_i24
    kernel, anything wider the generic one; all bit-exact, including int32
    accumulator wrap-around and saturation on full-scale inputs."""
    rng = np.random.default_rng(ntaps + len(kind))
    lim = {"i16": 32767, "i24": (1 << 23) - 1, "i32": (1 << 24)}[kind]
    c = rng.integers(-lim, lim + 1, size=ntaps).astype(np.int32)
    c[0], c[-1], c[ntaps // 2] = lim, -lim - 1 if kind == "i16" else -lim, 1
    x = O["strict"].gen_ci16(99, 2, 0, (1 << 18) + 4096, -32768, 32767)
    g = S.FilterDnsamplingFir(c, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    r = O["strict"].decim(1, 4, c)
    for off, n in _chunks(len(x), [65536, 4, 8196, 100000]):
        n -= n % 4
        xs = x[off:off + n]
        assert np.array_equal(g.step(dev(xs)).cpu().numpy(), r.step(xs)), (off, n)


@pytest.mark.parametrize("N,f", [(1000, -0.37), (4096, 0.73), (2048, 0.0), (4096, 0.1), (4096, 0.5),
                                 (3000, 0.3), (1022, 0.9), (4093, 0.1), (4096, -1.0 / 1024)])
def test_mixdecim_chain_table_sizes(S, O, N, f):
    """Fused mixer (LDS (cos, sin) table, dot2 complex multiply) at
    non-power-of-two and power-of-two table sizes, several chained calls.
    The sequence table's period Pe = lcm(N / gcd(freq, N), 4) spans 4 (f = 0,
    0.5), 20, 200, 2044 (lane offsets wrap), 4096, and 16372 for N = 4093
    (over the LDS budget: the doubled phase table instead)."""
    from srcdsp_amd.design import hamming_sinc, q14
    cq = q14(hamming_sinc(127))
    x = O["strict"].gen_ci16(0xBEE, 3, 0, 400000, -32768, 32767)
    m = S.Mixer(N)
    m.reset(f)
    d = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    chain = S.MixerDecimatorChain(m, d)
    om, od = O["strict"].mixer(N), O["strict"].decim(1, 4, cq)
    om.reset(f)
    for off, n in _chunks(len(x), [131072, 8, 4100, 200000]):
        n -= n % 4
        xs = x[off:off + n]
        assert np.array_equal(chain.step(dev(xs)).cpu().numpy(), od.step(om.step(xs))), (off, n)
        assert m.state()[:2] == om.state()[:2]


@pytest.mark.parametrize("case", ["m3", "t63_i24", "t16taps", "wide_taps", "n8192", "out_offset", "in_offset"])
def test_mixdecim_chain_unfused_configs(S, O, case):
    """Chain configurations the fused kernels do not cover run as the two
    reference calls (mixer launch into a stream-ordered scratch buffer, then the
    decimator): M = 3, 63 taps beyond the int16 range (the fused v_mad_i32_i24
    kernel is compiled for 127/128 only), int16 taps (variant 2), taps beyond
    2^23, a table of 8192 entries, 4-B-offset output / input views.  Same
    outputs and the same mixer and decimator state as the two oracle calls."""
    import torch
    from srcdsp_amd.design import hamming_sinc, q14
    M, ntaps, N, variant = 4, 127, 4096, 1
    if case == "m3":
        M = 3
    elif case == "t63_i24":
        ntaps = 63
    elif case == "t16taps":
        variant = 2
    elif case == "n8192":
        N = 8192
    cq = q14(hamming_sinc(ntaps))
    if case == "t63_i24":
        cq = cq.astype(np.int32) * 64  # |c| < 2^23, beyond int16
    if case == "wide_taps":
        cq = cq.astype(np.int64) * 1024
        cq[0] = 1 << 24
        cq = cq.astype(np.int32)
    ctype = "int16_t" if variant == 2 else "int32_t"
    if variant == 2:
        cq = cq.astype(np.int16)
    x = O["strict"].gen_ci16(0xC0DE, 5, 0, 300001, -32768, 32767)
    m = S.Mixer(N)
    m.reset(0.13)
    d = S.FilterDnsamplingFir(cq, M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", ctype)
    chain = S.MixerDecimatorChain(m, d)
    om, od = O["strict"].mixer(N), O["strict"].decim(variant, M, cq)
    om.reset(0.13)
    xd = dev(x)
    for off, n in _chunks(300000, [131072, 8, 4100, 200000]):
        n -= n % M
        if n == 0:
            continue
        ioff = 1 if case == "in_offset" else 0
        xs = x[off + ioff:off + ioff + n]
        if case == "out_offset":
            obuf = torch.zeros((n // M + 1, 2), dtype=torch.int16, device="cuda")
            y = chain.step(xd[off:off + n], obuf[1:])
            assert not obuf[0].any()
        else:
            y = chain.step(xd[off + ioff:off + ioff + n])
        assert np.array_equal(y.cpu().numpy(), od.step(om.step(xs))), (case, off, n)
        assert m.state()[:2] == om.state()[:2]


@pytest.mark.parametrize("M,ntaps", [(4, 127), (2, 127), (3, 127)])
def test_mixdecim_chain_alternating_streams(S, O, M, ntaps):
    """Chain steps issued on two streams in turn with no host synchronisation
    between them: the handles' stream ordering (and, for the unfused M = 3
    chain, the stream-ordered scratch buffer) keep every step in call order.
    Bit-exact against the two oracle calls."""
    import torch
    from srcdsp_amd.design import hamming_sinc, q14
    cq = q14(hamming_sinc(ntaps))
    x = O["strict"].gen_ci16(0xA5, 2, 0, 1 << 20, -32768, 32767)
    m = S.Mixer(4096)
    m.reset(-0.3)
    d = S.FilterDnsamplingFir(cq, M, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    chain = S.MixerDecimatorChain(m, d)
    om, od = O["strict"].mixer(4096), O["strict"].decim(1, M, cq)
    om.reset(-0.3)
    xd = dev(x)
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    outs, exps = [], []
    for k, (off, n) in enumerate(_chunks(len(x), [262144, 4096, 131072, 8, 300000])):
        n -= n % M
        s = streams[k % 2]
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            outs.append(chain.step(xd[off:off + n]))
        exps.append(od.step(om.step(x[off:off + n])))
    torch.cuda.synchronize()
    for k, (y, e) in enumerate(zip(outs, exps)):
        assert np.array_equal(y.cpu().numpy(), e), k
    assert m.state()[:2] == om.state()[:2]


@pytest.mark.parametrize("fp", ["fma", "strict"])
@pytest.mark.parametrize("ntaps", [1, 2, 3, 5, 12, 13, 31, 127, 1000, 1030])
def test_fir_float_tile_kernel_vs_oracle(S, O, fp, ntaps):
    """FilterFir<cf32,cf32,cf32,float> and <float,cf32,float,float>: the
    single-rate tile kernel (runtime tap count <= 1024; 1030 takes the generic
    kernel), chained calls of uneven length, bit-exact per float contract."""
    rng = np.random.default_rng(ntaps)
    c = (rng.standard_normal(ntaps) / max(4, ntaps)).astype(np.float32)
    xc = O[fp].gen_cf32(21, 0, 0, 70001)
    xr = np.ascontiguousarray(xc.view(np.float32)[:, 0]) if xc.ndim == 2 else xc.real.astype(np.float32)
    for kind in ("cf32", "f32"):
        if kind == "cf32":
            g = S.FilterFir(c, fp=fp)
            r = O[fp].fir(0, c)
            x = xc
        else:
            g = S.FilterFir(c, "float", "complex<float>", "float", "float", fp=fp)
            r = O[fp].fir(1, c)
            x = xr
        for off, n in _chunks(len(x), [16384, 3, 4096 + 8, 40000, 1]):
            xs = x[off:off + n]
            assert np.array_equal(g.step(dev(xs)).cpu().numpy(), r.step(xs)), (kind, off, n)


@pytest.mark.parametrize("M,ntaps,L", [(4, 127, 98304), (2, 63, 98304), (8, 200, 98304), (3, 50, 98304),
                                       (1, 127, 98304), (3, 128, 98304), (8, 255, 98304), (16, 255, 98304),
                                       (4, 255, 98304), (4, 127, 4 * 24575), (2, 64, 2 * 24575)])
def test_decim_batched_equals_single(S, O, M, ntaps, L):
    """The batched step (configs[2]'s layout: one launch per channel on the
    headline kernel, grid.y = channel elsewhere) at each compiled (M, taps)
    and on the any-tap tile kernel: per-channel
    history across steps.  An odd output row count makes the output row stride
    8-B aligned only: those launches must leave the 16-B-store kernels."""
    import torch
    from srcdsp_amd.design import hamming_sinc
    c = hamming_sinc(ntaps)
    C = 8
    L -= L % M
    x = np.stack([O["fma"].gen_cf32(0x5EED, ch, 0, L) for ch in range(C)])
    fs = [S.FilterDnsamplingFir(c, M) for _ in range(C)]
    xd = dev(x)
    for rep in range(2):  # two steps: history per channel
        out = torch.empty((C, L // M), dtype=torch.complex64, device="cuda")
        S.decim_step_batched(fs, xd, out)
        if rep == 0:
            refs = [O["fma"].decim(0, M, c) for _ in range(C)]
        for ch in range(C):
            assert np.array_equal(out[ch].cpu().numpy(), refs[ch].step(x[ch])), (rep, ch)


def test_decim_generic_paths_vs_oracle(S, O):
    """Unaligned device input and shapes without a tile kernel use the
    generic kernel; results are still bit-exact."""
    import torch
    from srcdsp_amd.design import hamming_sinc
    x = O["fma"].gen_cf32(7, 0, 0, 40001)
    c = hamming_sinc(63, 0.06)
    g = S.FilterDnsamplingFir(c, 8)
    r = O["fma"].decim(0, 8, c)
    assert np.array_equal(g.step(dev(x[:40000])).cpu().numpy(), r.step(x[:40000]))
    # misaligned (8-byte offset) input through the M=4 path
    c127 = hamming_sinc(127)
    g4, r4 = S.FilterDnsamplingFir(c127, 4), O["fma"].decim(0, 4, c127)
    buf = dev(x)  # 40001 samples; view starting at sample 1 is 8-B aligned only
    view = buf[1:40001]
    assert np.array_equal(g4.step(view).cpu().numpy(), r4.step(x[1:40001]))
    del torch


@pytest.mark.parametrize("M,ntaps", [(4, 127), (4, 255), (2, 63), (3, 128), (8, 255), (16, 127), (1, 127), (1, 300)])
def test_decim_cf32_misaligned_views_vs_oracle(S, O, M, ntaps):
    """Caller-supplied input / output views that are 8-B but not 16-B aligned
    at every tuned complex<float> shape: the 16-B-store kernels must not take
    them (they fall back to the generic path), results stay bit-exact."""
    import torch
    from srcdsp_amd.design import hamming_sinc
    c = hamming_sinc(ntaps, 0.4 / M)
    n = 6000 * M
    x = O["fma"].gen_cf32(11 + M, 0, 0, n + 1)
    for in_off, out_off in [(0, 1), (1, 0), (1, 1)]:
        g, r = S.FilterDnsamplingFir(c, M), O["fma"].decim(0, M, c)
        xin = dev(x)[in_off:in_off + n]
        obuf = torch.zeros(n // M + 1, dtype=torch.complex64, device="cuda")
        for rep in range(2):  # history carried across the fallback
            y = obuf[out_off:out_off + n // M]
            g.step(xin, y)
            exp = r.step(x[in_off:in_off + n])
            assert np.array_equal(y.cpu().numpy().view(np.uint32), exp.view(np.uint32)), (in_off, out_off, rep)
        if out_off:
            assert obuf[0].item() == 0  # nothing written before the view


@pytest.mark.parametrize("ntaps", [127, 255])
def test_decim_ci16_misaligned_output_vs_oracle(S, O, ntaps):
    """complex<int16_t> outputs into a 4-B-offset view: the dot2 / mad24
    kernels' 16-B stores are not taken; bit-exact through the fallback."""
    import torch
    rng = np.random.default_rng(ntaps)
    c = rng.integers(-3000, 3000, ntaps).astype(np.int32)
    n = 4 * 5000
    x = O["fma"].gen_ci16(99, 0, 0, n, -32768, 32767)
    g, r = S.FilterDnsamplingFir(c, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t"), O["fma"].decim(1, 4, c)
    obuf = torch.zeros((n // 4 + 1, 2), dtype=torch.int16, device="cuda")
    for rep in range(2):
        y = obuf[1:1 + n // 4]
        g.step(dev(x), y)
        assert np.array_equal(y.cpu().numpy(), r.step(x)), rep


def test_decim_errors_and_empty(S):
    import torch
    from srcdsp_amd._capi import ERR_SIZE, SrcdspError
    g = S.FilterDnsamplingFir(np.ones(5, np.float32), 4)
    with pytest.raises(SrcdspError) as e:
        g.step(torch.zeros(10, dtype=torch.complex64, device="cuda"), torch.zeros(2, dtype=torch.complex64,
                                                                                 device="cuda"))
    assert e.value.code == ERR_SIZE
    out = g.step(torch.zeros(0, dtype=torch.complex64, device="cuda"))
    assert out.numel() == 0
    with pytest.raises(TypeError):
        S.FilterDnsamplingFir(np.ones(5, np.float32), 4, "float", "float", "float", "float")
    d2 = S.FilterDnsamplingFir(np.ones(8, np.float32), 4)
    with pytest.raises(SrcdspError):
        d2.setCoeffs(np.ones(7, np.float32))  # dsptl_dnsampling_filters.h:122 assert


def test_headline_whole_output(S, O):
    """Config 2 at full size (2^28 complex<float> samples, device-resident, one
    step()), both float contracts: EVERY one of the 2^26 outputs
    of the FMA contract against the FMA oracle, and of the strict contract
    (SRCDSP_FLAG_FP_STRICT: a rounded multiply then a rounded add per tap, the
    reference's own makefile build has no FMA, makefile:17;
    dnsampling_filters.h:150-167) against the strict oracle, byte for byte;
    then the stated tolerance over all 2^26 outputs: the FMA contract differs
    from the strict reference by at most 1 output LSB (|delta| <= 1.0 on a
    component) on at most 1e-4 of the outputs.  The oracle runs in parallel
    windows on the host (tests/fullsize.py); the device generator equals the
    host one on the first, a seam and the last window."""
    import torch
    import fullsize as F
    from srcdsp_amd.design import hamming_sinc
    c = hamming_sinc(127)
    L = 1 << 28
    x = torch.empty(L, dtype=torch.complex64, device="cuda")
    S.fill_synthetic(x, "cf32", seed=0x5EED, channel=0)
    y = {fp: S.FilterDnsamplingFir(c, 4, fp=fp).step(x).cpu().numpy() for fp in ("fma", "strict")}
    xh = x.cpu().numpy()
    del x
    torch.cuda.empty_cache()
    for lo in (0, (1 << 27) - 5000, L - 8192):
        assert np.array_equal(xh[lo:lo + 8192], O["fma"].gen_cf32(0x5EED, 0, lo, 8192)), lo
    want = {}
    for fp in ("fma", "strict"):
        want[fp] = F.decim_all(lambda: O[fp].decim(0, 4, c), xh, 4, 128, np.empty(L // 4, np.complex64))
        bad = F.first_bad(y[fp], want[fp])
        assert bad is None, f"fp={fp}: first differing output {bad}"
    del xh
    d = np.abs(y["fma"].view(np.float32) - want["strict"].view(np.float32)).reshape(-1, 2)
    assert d.max() <= 1.0, f"max |fma - strict reference| = {d.max()}"
    n_diff = int(np.count_nonzero(d.max(axis=1)))
    assert n_diff <= 1e-4 * len(d), f"{n_diff} of {len(d)} outputs differ from the strict reference"


def test_config3_per_gpu_share_whole_channels(S, O):
    """Config 3's per-GPU share at full size: 8 channels x 2^28 complex<float>
    samples (channels 8..15 of the 64, i.e. rank 1 of 8), one batched step as
    bench.py --gpus N runs it.  EVERY output of all 8 channels (8 x 2^26)
    against the oracle, channel by channel, so a grid.y / channel-stride
    mapping error on any channel fails; each channel's input equals the host
    generator on a first, an interior and a last window; each channel's
    history is its own tail."""
    import torch
    import fullsize as F
    from srcdsp_amd.design import hamming_sinc
    c = hamming_sinc(127)
    C, L = 8, 1 << 28
    ch0 = 8
    x = torch.empty((C, L), dtype=torch.complex64, device="cuda")
    for k in range(C):
        S.fill_synthetic(x[k], "cf32", seed=0x5EED, channel=ch0 + k)
    y = torch.empty((C, L // 4), dtype=torch.complex64, device="cuda")
    fs = [S.FilterDnsamplingFir(c, 4, fp="fma") for _ in range(C)]
    S.decim_step_batched(fs, x, y)
    torch.cuda.synchronize()
    want = np.empty(L // 4, np.complex64)
    for k in range(C):
        xh = x[k].cpu().numpy()
        for lo in (0, (1 << 27) + 12345, L - 8192):
            assert np.array_equal(xh[lo:lo + 8192], O["fma"].gen_cf32(0x5EED, ch0 + k, lo, 8192)), (k, lo)
        F.decim_all(lambda: O["fma"].decim(0, 4, c), xh, 4, 128, want)
        bad = F.first_bad(y[k].cpu().numpy(), want)
        assert bad is None, f"channel {ch0 + k}: first differing output {bad}"
        assert fs[k].state()["history"].tobytes() == xh[L - 126:].tobytes(), k
        del xh
    del x, y
    torch.cuda.empty_cache()


def test_config4_whole_output(S, O):
    """Config 4 at full size (2^28 complex<int16_t>, device-resident, one fused
    mixer -> decimator step): EVERY output against the reference pair -- the
    oracle mixer over the whole call (so the NCO phase is checked across all
    2^28 samples), then the oracle decimator over the mixed stream in parallel
    windows started 128 samples early with an empty history."""
    import torch
    import fullsize as F
    from srcdsp_amd.design import hamming_sinc, q14
    cq = q14(hamming_sinc(127))
    L = 1 << 28
    x = torch.empty((L, 2), dtype=torch.int16, device="cuda")
    S.fill_synthetic(x, "ci16", seed=0x5EED, channel=0, lo=-8192, hi=8191)
    m = S.Mixer(4096)
    m.reset(0.1)
    d = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    y = S.MixerDecimatorChain(m, d).step(x)
    torch.cuda.synchronize()
    xh = x.cpu().numpy()
    for lo in (0, L - 8192):
        assert np.array_equal(xh[lo:lo + 8192], O["strict"].gen_ci16(0x5EED, 0, lo, 8192, -8192, 8191)), lo
    om = O["strict"].mixer(4096)
    om.reset(0.1)
    mixed = om.step(xh)
    assert m.state()[:2] == om.state()[:2]  # the phase after the call
    del xh
    want = F.decim_all(lambda: O["strict"].decim(1, 4, cq), mixed, 4, 128, np.empty((L // 4, 2), np.int16))
    bad = F.first_bad(y.cpu().numpy(), want)
    assert bad is None, f"first differing output {bad}"
    del x, y
    torch.cuda.empty_cache()


def test_ci16decim_bench_whole_output(S, O):
    """Row a2 as the ci16decim bench workload runs it: FilterDnsamplingFir<ci16,
    ci16,ci32,int32_t,4>, 127 Q14 taps, 2^28 complex<int16_t> samples of the
    synthetic generator, one step(): EVERY one of the 2^26 outputs against the
    oracle (dnsampling_filters.h:150-167 with dsp_complex.cpp:23-29 products)."""
    import torch
    import fullsize as F
    from srcdsp_amd.design import hamming_sinc, q14
    cq = q14(hamming_sinc(127))
    L = 1 << 28
    x = torch.empty((L, 2), dtype=torch.int16, device="cuda")
    S.fill_synthetic(x, "ci16", seed=0x5EED, channel=0, lo=-8192, hi=8191)
    d = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    y = d.step(x).cpu().numpy()
    xh = x.cpu().numpy()
    want = F.decim_all(lambda: O["strict"].decim(1, 4, cq), xh, 4, 128, np.empty((L // 4, 2), np.int16))
    bad = F.first_bad(y, want)
    assert bad is None, f"first differing output {bad}"
    assert d.state()["history"].tobytes() == xh[L - 126:].tobytes()
    del x
    torch.cuda.empty_cache()


def test_decim_cf32_beyond_4gib_one_channel(S, O):
    """One channel past 4 GiB: 2^30 + a ragged tail of complex<float> samples
    (8 GiB in, one step()), so byte offsets pass 2^32 and sample indices 2^29:
    spot windows around the 4 GiB boundary, random interior, the ragged last
    tile, and the history left for the next call, against the oracle on the
    same input windows."""
    import torch
    from srcdsp_amd.design import hamming_sinc
    c = hamming_sinc(127)
    L = (1 << 30) + 4 * 1237
    x = torch.empty(L, dtype=torch.complex64, device="cuda")
    S.fill_synthetic(x, "cf32", seed=0x5EED, channel=5)
    f = S.FilterDnsamplingFir(c, 4, fp="fma")
    y = torch.empty(L // 4, dtype=torch.complex64, device="cuda")
    f.step(x, y)
    torch.cuda.synchronize()
    n_out = L // 4
    b4 = (1 << 29) // 4  # the output whose inputs straddle byte offset 2^32
    rng = np.random.default_rng(6)
    for s0 in [0, b4 - 40, b4 - 1, b4 + 7, n_out - 64, *map(int, rng.integers(40, n_out - 64, 4))]:
        lo = max(0, 4 * s0 - 128)
        xin = x[lo:4 * (s0 + 64)].cpu().numpy()
        assert np.array_equal(xin, O["fma"].gen_cf32(0x5EED, 5, lo, len(xin))), s0
        r = O["fma"].decim(0, 4, c).step(xin)[(4 * s0 - lo) // 4:]
        got = y[s0:s0 + 64].cpu().numpy()
        assert np.array_equal(got, r[:len(got)]), s0
    assert f.state()["history"].tobytes() == x[L - 126:].cpu().numpy().tobytes()
    del x, y
    torch.cuda.empty_cache()


def test_mixdecim_beyond_2p31_samples(S, O):
    """Config 4's fused chain on one call of 2^31 + a ragged tail of
    complex<int16_t> samples (8 GiB in): sample indices pass 2^31, so the
    NCO phase (phi0 + k*freq) mod N and every tile offset must be 64-bit.
    Output windows before and after sample 2^31 and at the end against the
    reference mixer -> decimator pair on the same input windows (the oracle
    mixer advanced by stepping zeros: the phase does not depend on the data)."""
    import torch
    from srcdsp_amd.design import hamming_sinc, q14
    cq = q14(hamming_sinc(127))
    L = (1 << 31) + 4 * 2048 * 3 + 4 * 77
    x = torch.empty((L, 2), dtype=torch.int16, device="cuda")
    S.fill_synthetic(x, "ci16", seed=0x5EED, channel=3, lo=-8192, hi=8191)
    m = S.Mixer(4096)
    m.reset(0.1)
    d = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")
    y = S.MixerDecimatorChain(m, d).step(x)
    torch.cuda.synchronize()
    om = O["strict"].mixer(4096)
    om.reset(0.1)
    n_out = L // 4
    b31 = (1 << 31) // 4
    starts = [0, 2048 - 3, b31 - 100, b31 + 5, n_out - 64]
    zeros = np.zeros((1 << 24, 2), np.int16)
    pos = 0
    for s0 in starts:
        lo = max(0, 4 * s0 - 128)
        hi = 4 * (s0 + 64)
        while pos < lo:
            k = min(lo - pos, len(zeros))
            om.step(zeros[:k])
            pos += k
        xin = x[lo:hi].cpu().numpy()
        assert np.array_equal(xin, O["strict"].gen_ci16(0x5EED, 3, lo, hi - lo, -8192, 8191)), s0
        mixed = om.step(xin)
        pos = hi
        r = O["strict"].decim(1, 4, cq).step(mixed)[(4 * s0 - lo) // 4:]
        got = y[s0:s0 + 64].cpu().numpy()
        assert np.array_equal(got, r[:len(got)]), s0
    del x, y
    torch.cuda.empty_cache()


def test_fir_and_up_bench_whole_output(S, O):
    """The fir and up bench workloads at their full sizes: EVERY output of the
    31-tap FilterFir<float,cf32,float,float> over 2^28 float samples, and of
    the 128-tap x4 interpolator over 2^26 complex<int16_t> inputs (2^28
    outputs), against the oracle in parallel windows started early enough to
    fill the history (tests/fullsize.py)."""
    import torch
    import fullsize as F
    from srcdsp_amd.design import hamming_sinc, q14
    L = 1 << 28
    x = torch.randint(-2048, 2048, (L,), device="cuda").float()
    c = hamming_sinc(31, 0.2)
    xh = x.cpu().numpy()
    for fp in ("fma", "strict"):  # both float contracts (filters.h:153-164 in ascending k)
        y = S.FilterFir(c, "float", "complex<float>", "float", "float", fp=fp).step(x).cpu().numpy()
        want = F.decim_all(lambda: O[fp].fir(1, c), xh, 1, 32, np.empty(L, np.complex64))
        bad = F.first_bad(y, want)
        assert bad is None, f"fir ({fp}): first differing output {bad}"
    del x, y, xh, want
    n = 1 << 26
    xu = torch.empty((n, 2), dtype=torch.int16, device="cuda")
    S.fill_synthetic(xu, "ci16", seed=0x5EED, channel=0, lo=-8192, hi=8191)
    cu = q14(hamming_sinc(128, 0.12) * 4)
    yu = S.FilterUpsamplingFir(cu, 4).step(xu)
    torch.cuda.synchronize()
    want = F.up_all(lambda: O["fma"].up(0, 4, cu), xu.cpu().numpy(), 4, 40, np.empty((4 * n, 2), np.int16))
    bad = F.first_bad(yu.cpu().numpy(), want)
    assert bad is None, f"up: first differing output {bad}"
    del xu, yu
    torch.cuda.empty_cache()


# ----------------------------------------------------- other operators
def test_mixer_large_vs_oracle(S, O):
    x = O["fma"].gen_ci16(11, 0, 0, (1 << 20) + 3, -32768, 32767)
    for N, f in ((4096, 0.1), (1024, -0.37), (256, 0.999)):
        m, r = S.Mixer(N), O["fma"].mixer(N)
        m.reset(f)
        r.reset(f)
        for off, n in _chunks(len(x), [333333, 1, 65536, 400000]):
            xs = x[off:off + n]
            assert np.array_equal(m.step(dev(xs)).cpu().numpy(), r.step(xs)), (N, off)
            assert m.state()[:2] == r.state()[:2]


def test_upsampler_vs_oracle(S, O):
    from srcdsp_amd.design import hamming_sinc, q14
    c = q14(hamming_sinc(32, 0.12) * 4)
    x = O["fma"].gen_ci16(5, 0, 0, 1 << 16, -8192, 8191)
    for it in (False, True):
        g = S.FilterUpsamplingFir(c if not it else c // 8, 4)
        r = O["fma"].up(0, 4, c if not it else c // 8)
        for off, n in _chunks(len(x), [30000, 3, 20000]):
            xs = x[off:off + n]
            last = off + n >= len(x)
            assert np.array_equal(g.step(dev(xs), None, last, it).cpu().numpy(), r.step(xs, last, it)), (it, off)


_UP_TYPES = {0: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t"),
             1: ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int16_t"),
             2: ("int16_t", "int16_t", "int32_t", "int32_t")}


@pytest.mark.parametrize("variant", [0, 1, 2])
@pytest.mark.parametrize("L,H", [(2, 1), (2, 7), (4, 32), (4, 33), (8, 16), (3, 5), (4, 2000), (3, 6000), (16, 1100)])
def test_upsampler_tile_kernel_vs_oracle(S, O, variant, L, H):
    """Tiled interpolator (L in 2/4/8, <= 4096 taps) and the generic one (other
    L, int16 input, longer filters; past 16384 taps it reads them through the
    cache): flush and iterator overloads, wide taps
    (|c| >= 2^23 takes the exact 32-bit multiply), int16 product wrap."""
    rng = np.random.default_rng(L * 1000 + H + 7 * variant)
    n = L * H
    lim = {0: 1 << 24, 1: 32767, 2: 20000}[variant]
    c = rng.integers(-lim, lim + 1, size=n)
    c[-1] = 0  # trailing zero tap: length < ImpLength (upsampling_filters.h:121-123)
    c[0] = lim
    x = O["fma"].gen_ci16(L + H, variant, 0, 50000, -32768, 32767)
    if variant == 2:
        x = np.ascontiguousarray(x[:, 0]) if x.ndim == 2 else x
    g = S.FilterUpsamplingFir(c, L, *_UP_TYPES[variant])
    r = O["fma"].up(variant, L, c)
    for it in (False, True):
        for off, m in _chunks(len(x), [20000, 1, 4099, 30000]):
            xs = x[off:off + m]
            last = off + m >= len(x)
            assert np.array_equal(g.step(dev(xs), None, last, it).cpu().numpy(), r.step(xs, last, it)), (it, off)
        g.reset()
        r.reset()


@pytest.mark.parametrize("L,H", [(2, 1), (2, 2), (2, 7), (2, 16), (2, 24), (2, 31), (2, 64), (4, 1), (4, 15), (4, 16),
                                 (4, 24), (4, 32), (4, 33), (4, 63), (4, 64), (4, 300), (8, 1), (8, 2), (8, 7),
                                 (8, 15), (8, 16), (8, 17), (8, 32), (8, 33), (8, 100), (3, 1), (3, 16), (3, 33),
                                 (5, 7), (5, 40), (6, 16), (7, 9), (7, 64)])
def test_upsampler_dot2_kernel_vs_oracle(S, O, L, H):
    """<ci16,ci16,ci32,int32_t> with int16-range taps (incl. -32768, 32767) runs
    the v_dot2 interpolator (L = 2 .. 8); full-scale inputs so the int32
    accumulators wrap; flush and iterator overloads; uneven chained calls."""
    rng = np.random.default_rng(100 * L + H)
    c = rng.integers(-32768, 32768, size=L * H)
    c[0], c[-1] = -32768, 32767
    x = O["fma"].gen_ci16(7 * L + H, 0, 0, 40000, -32768, 32767)
    g = S.FilterUpsamplingFir(c, L, *_UP_TYPES[0])
    r = O["fma"].up(0, L, c)
    for it in (False, True):
        for off, m in _chunks(len(x), [9000, 1, 2049, 4097, 30000]):
            xs = x[off:off + m]
            last = off + m >= len(x)
            assert np.array_equal(g.step(dev(xs), None, last, it).cpu().numpy(), r.step(xs, last, it)), (it, off)
        g.reset()
        r.reset()


@pytest.mark.parametrize("in_off,out_off", [(1, 0), (0, 1), (1, 1), (2, 2)])
def test_offset_views_up_mixer_corr(S, O, in_off, out_off):
    """Upsampler (the dot2 shape L = 4 x 128 and the wide-tap tile kernel),
    mixer and correlator on device views 4-B (one complex<int16_t>) off
    16-B alignment: the vector kernels are not taken for them, results stay
    bit-exact and the state carries over to aligned calls."""
    import torch
    from srcdsp_amd.design import qpsk_pattern
    rng = np.random.default_rng(in_off * 10 + out_off)
    n = 20001
    x = O["fma"].gen_ci16(3 + in_off, 0, 0, n + 4, -32768, 32767)
    xd = dev(x)
    for c in (rng.integers(-32768, 32768, 128), rng.integers(-(1 << 24), 1 << 24, 128)):
        g, r = S.FilterUpsamplingFir(c, 4, *_UP_TYPES[0]), O["fma"].up(0, 4, c)
        for k, (a, b) in enumerate([(0, 7000), (7000, n)]):
            xs = xd[a + in_off:b + in_off] if k == 0 else xd[a:b]  # offset view, then aligned
            obuf = torch.zeros((4 * (b - a) + out_off, 2), dtype=torch.int16, device="cuda")
            y = obuf[out_off:] if k == 0 else obuf[:4 * (b - a)]
            g.step(xs, y)
            exp = r.step(x[a + in_off:b + in_off] if k == 0 else x[a:b])
            assert np.array_equal(y.cpu().numpy(), exp), (k, c[0])
    m, om = S.Mixer(4096), O["fma"].mixer(4096)
    m.reset(0.21)
    om.reset(0.21)
    for k, (a, b) in enumerate([(0, 10000), (10000, n)]):
        xs = xd[a + in_off:b + in_off] if k == 0 else xd[a:b]
        obuf = torch.zeros((b - a + out_off, 2), dtype=torch.int16, device="cuda")
        y = obuf[out_off:] if k == 0 else obuf[:b - a]
        m.step(xs, y)
        exp = om.step(x[a + in_off:b + in_off] if k == 0 else x[a:b])
        assert np.array_equal(y.cpu().numpy(), exp), k
        assert m.state()[:2] == om.state()[:2]
    p = qpsk_pattern(64, 500, seed=3)
    xc = rng.integers(-125, 126, size=(n + 4, 2))
    xc[12000:12000 + 64] += 2 * p
    xc = np.clip(xc, -32768, 32767).astype(np.int16)
    g, r = S.FixedPatternCorrelator(64, 1), O["fma"].corr(64, 1)
    g.setPattern(p)
    r.set_pattern(p)
    xcd = dev(xc)
    for k, (a, b) in enumerate([(0, 5000), (5000, n)]):
        xs = xcd[a + in_off:b + in_off] if k == 0 else xcd[a:b]
        fg, ig = g.step(xs)
        fr, ir = r.step(xc[a + in_off:b + in_off] if k == 0 else xc[a:b])
        assert (fg, fg and ig) == (fr, fr and ir), (k, fg, ig, fr, ir)
        assert np.array_equal(g.getRefBitSamples(), r.bit_samples())


@pytest.mark.parametrize("N,S_", [(1024, 1), (32, 4), (64, 2), (1, 1), (7, 5), (33, 1), (100, 1), (127, 2),
                                  (31, 3), (16, 16), (1000, 1), (8200, 1), (48, 3), (50, 7), (256, 4),
                                  (17, 1), (47, 1), (129, 1), (8185, 1)])
def test_correlator_vs_oracle(S, O, N, S_):
    """FixedPatternCorrelator at (N, S): the fused one-launch scan (S = 1, any
    N <= 8192, the pattern front-padded with zero taps to a multiple of 16), the
    dot2 tiles at any N >= 48 and stride S > 1 (one phase of the stride per
    grid row), and the generic kernel below 48 taps at S > 1 and past 8192 taps; stepping on after
    every detection, bitSamples and registers compared at each."""
    from srcdsp_amd.design import qpsk_pattern
    p = qpsk_pattern(N, 500 if N <= 2048 else 200, seed=N)
    rng = np.random.default_rng(N)
    n = 1 << 16 if N == 1024 else 1 << 17
    x = rng.integers(-125, 126, size=(n, 2)).astype(np.int32)
    for off in (n // 3, (3 * n) // 4):
        for m in range(N):
            if off + m * S_ < n:
                x[off + m * S_] += 2 * p[m]
    x = np.clip(x, -32768, 32767).astype(np.int16)
    g, r = S.FixedPatternCorrelator(N, S_), O["fma"].corr(N, S_)
    g.setPattern(p)
    r.set_pattern(p)
    pos, events = 0, 0
    while pos < n:  # keep stepping after detections, like a receiver would
        xs = x[pos:pos + 20000]
        fg, ig = g.step(dev(xs))
        fr, ir = r.step(xs)
        assert (fg, fg and ig) == (fr, fr and ir)
        assert np.array_equal(g.getRefBitSamples(), r.bit_samples())
        st, sr = g.getStatus(), r.status()
        assert all(st[k] == sr[k] for k in ("energy", "corr", "coeffs_energy", "coeff_scaling"))
        events += fr
        pos += (ir + 2) if fr else len(xs)
    # these shapes' scaled statistics stay under the threshold for this
    # signal (in the reference too): they check the registers at every step
    assert events >= 1 or (N, S_) in {(1, 1), (7, 5), (16, 16), (48, 3), (50, 7), (17, 1), (47, 1)}


@pytest.mark.parametrize("N,S_,n,chunk", [(32, 2100, 1 << 18, 50000), (64, 70000, 5_500_000, 1_000_000),
                                           (64, 600, 1 << 18, 70000)])
def test_correlator_long_window_vs_oracle(S, O, N, S_, n, chunk):
    """Windows N*S too long to stage in LDS (corr_eval_g: one output per lane
    through the cache) and strides past one grid row per phase (S > 65535 leaves
    the dot2 tiles); (64, 600) is the dot2 tile kernel at a long stride.  Bytes,
    detections, bitSamples and registers against the oracle at every step."""
    from srcdsp_amd.design import qpsk_pattern
    p = qpsk_pattern(N, 500, seed=N)
    rng = np.random.default_rng(N + S_)
    x = rng.integers(-125, 126, size=(n, 2)).astype(np.int32)
    off = n - N * S_ - 1000
    for m in range(N):
        x[off + m * S_] += 2 * p[m]
    x = np.clip(x, -32768, 32767).astype(np.int16)
    g, r = S.FixedPatternCorrelator(N, S_), O["fma"].corr(N, S_)
    g.setPattern(p)
    r.set_pattern(p)
    pos, events = 0, 0
    while pos < n:
        xs = x[pos:pos + chunk]
        fg, ig = g.step(dev(xs))
        fr, ir = r.step(xs)
        assert (fg, fg and ig) == (fr, fr and ir)
        assert np.array_equal(g.getRefBitSamples(), r.bit_samples())
        st, sr = g.getStatus(), r.status()
        assert all(st[k] == sr[k] for k in ("energy", "corr", "coeffs_energy", "coeff_scaling"))
        events += fr
        pos += (ir + 2) if fr else len(xs)
    assert events >= 1


def test_config5_whole_buffer(S, O):
    """Config 5 at full size (2^26 samples, device-resident, one step): the
    bench's buffer (noise +-125, the 1024-sample QPSK pattern x2 at 3/4).  The
    oracle scans the WHOLE buffer (parallel windows, each primed with its
    N*S+2-sample halo: tests/fullsize.py): no detection before the GPU's, the
    same index, and equal bitSamples and registers there."""
    import fullsize as F
    from srcdsp_amd.design import qpsk_pattern
    L = 1 << 26
    p = qpsk_pattern(1024, 500, seed=2)
    rng = np.random.default_rng(0)
    x = rng.integers(-125, 126, size=(L, 2)).astype(np.int32)
    off = (3 * L) // 4
    x[off:off + 1024] += 2 * p
    x = np.clip(x, -32768, 32767).astype(np.int16)
    g = S.FixedPatternCorrelator(1024, 1)
    g.setPattern(p)
    fg, ig = g.step(dev(x))

    def make():
        r = O["fma"].corr(1024, 1)
        r.set_pattern(p)
        return r

    fr, ir, bits, st_r = F.corr_first(make, x, 1024, 1, win=1 << 19)
    assert fg and fr and ig == ir, (fg, ig, fr, ir)
    assert np.array_equal(g.getRefBitSamples(), bits)
    st = g.getStatus()
    assert all(st[k] == st_r[k] for k in ("energy", "corr", "coeffs_energy", "coeff_scaling"))


def test_time_split_segments_equal_single_call(S, O):
    """SURVEY 8e, one long buffer split in time (W = 3 segments run one after
    another here, as 3 ranks would): decimator seeded by stepping its halo,
    mixer by setPhase(phaseAt(start)), correlator by prime(); outputs and the
    first detection are bit-identical to the unsplit call."""
    import torch
    from srcdsp_amd import dist as D
    from srcdsp_amd.design import hamming_sinc, q14, qpsk_pattern
    W = 3
    # decimator (cf32)
    c = hamming_sinc(127)
    x = dev(O["fma"].gen_cf32(0x5EED, 0, 0, 3 * 65536 + 12))
    ref = S.FilterDnsamplingFir(c, 4).step(x).cpu().numpy()
    parts = []
    for r in range(W):
        s0, s1 = D.time_segment(x.shape[0], W, r, align=4)
        h = min(s0, D.decim_halo(127, 4))
        parts.append(S.FilterDnsamplingFir(c, 4).step(x[s0 - h:s1].contiguous())[h // 4:].cpu().numpy())
    assert np.array_equal(np.concatenate(parts), ref)
    # mixer -> decimator chain (ci16): mixer phase in closed form at the halo start
    cq = q14(hamming_sinc(127))
    xi = dev(O["fma"].gen_ci16(0x5EED, 1, 0, 3 * 65536 + 12, -32768, 32767))
    dtypes = ("complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t")

    def chain(f):
        m = S.Mixer(4096)
        m.reset(f)
        return m, S.MixerDecimatorChain(m, S.FilterDnsamplingFir(cq, 4, *dtypes))

    m0, ch0 = chain(0.1)
    ref = ch0.step(xi).cpu().numpy()
    parts = []
    for r in range(W):
        s0, s1 = D.time_segment(xi.shape[0], W, r, align=4)
        h = min(s0, D.decim_halo(127, 4))
        m, ch = chain(0.1)
        m.setPhase(m.phaseAt(s0 - h))
        parts.append(ch.step(xi[s0 - h:s1].contiguous())[h // 4:].cpu().numpy())
    assert np.array_equal(np.concatenate(parts), ref)
    # correlator: pattern straddling a segment boundary, and inside segment 2
    p = qpsk_pattern(1024, 500, seed=2)
    rng = np.random.default_rng(3)
    for where in (None, 200000 - 500, 300000):
        xc = rng.integers(-125, 126, size=(400000, 2))
        if where is not None:
            xc[where:where + 1024] += 2 * p
        xd = dev(xc.astype(np.int16))
        g = S.FixedPatternCorrelator(1024, 1)
        g.setPattern(p)
        found, idx = g.step(xd)
        bits = g.getRefBitSamples()
        first, owner = D.NO_DETECTION, None
        for r in range(W):
            s0, s1 = D.time_segment(xd.shape[0], W, r)
            hc = min(s0, D.corr_halo(1024, 1))
            gr = S.FixedPatternCorrelator(1024, 1)
            gr.setPattern(p)
            loc = D.corr_segment_search(gr, xd[s0 - hc:s0].contiguous() if hc else None, xd[s0:s1].contiguous(), s0)
            if loc is not None and loc < first:
                first, owner = loc, gr
        assert (found, idx if found else D.NO_DETECTION) == (where is not None, first)
        if found:
            assert np.array_equal(owner.getRefBitSamples(), bits)
    del torch


def test_mixer_decimator_correlator_pipeline_device_resident(S, O):
    """the chained mixer -> decimator -> correlator pipeline with
    device-resident intermediates (the decimated stream never leaves HBM):
    same detection, index and bitSamples as the three oracle calls."""
    from srcdsp_amd.design import hamming_sinc, q14, qpsk_pattern
    rng = np.random.default_rng(8)
    p = qpsk_pattern(64, 300, seed=4)
    # a baseband stream whose decimated output carries the pattern
    n = 1 << 18
    x = rng.integers(-500, 500, size=(n, 2))
    at = 150000
    x[at:at + 4 * 64] += 40 * np.repeat(p, 4, axis=0)  # each symbol held for M = 4 inputs
    x = np.clip(x, -32768, 32767).astype(np.int16)
    cq = q14(hamming_sinc(127, 0.12))
    m = S.Mixer(4096)
    m.reset(0.0)
    chain = S.MixerDecimatorChain(m, S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>",
                                                           "complex<int32_t>", "int32_t"))
    g = S.FixedPatternCorrelator(64, 1)
    g.setPattern(p)
    om, od, oc = O["fma"].mixer(4096), O["fma"].decim(1, 4, cq), O["fma"].corr(64, 1)
    om.reset(0.0)
    oc.set_pattern(p)
    xd = dev(x)
    hits = []
    for off in range(0, n, 1 << 16):  # four blocks, state carried on the device
        y = chain.step(xd[off:off + (1 << 16)])
        assert y.is_cuda
        hits.append(g.step(y))
        exp = oc.step(od.step(om.step(x[off:off + (1 << 16)])))
        assert hits[-1][0] == exp[0] and (not exp[0] or hits[-1][1] == exp[1]), (off, hits[-1], exp)
        if exp[0]:
            assert np.array_equal(g.getRefBitSamples(), oc.bit_samples())
    assert sum(h[0] for h in hits) == 1  # the pattern is found once, in the third block


# ------------------------------------------------------------ value semantics
def test_copies_continue_the_stream(S, O):
    """The reference operators are value types (implicit copy constructors:
    dnsampling_filters.h:52, filters.h:49, upsampling_filters.h:42,
    correlators.h:85, mixers.h:134): a copy taken mid-stream (srcdsp_*_clone)
    continues from the original's history / phase / registers, bit-exact with
    the original and the oracle."""
    import copy
    from srcdsp_amd.design import hamming_sinc, q14, qpsk_pattern
    o = O["fma"]
    x = o.gen_cf32(5, 0, 0, 60000)
    xi = o.gen_ci16(6, 0, 0, 40000, -8192, 8191)
    c = hamming_sinc(127)

    def check(op, ref, a, b, **kw):
        y1 = op.step(dev(a), **kw)
        ref.step(a, **kw)
        cp = copy.copy(op)
        ya, yb, yr = op.step(dev(b), **kw).cpu().numpy(), cp.step(dev(b), **kw).cpu().numpy(), ref.step(b, **kw)
        assert np.array_equal(ya.view(np.uint32), yr.view(np.uint32))
        assert np.array_equal(yb.view(np.uint32), yr.view(np.uint32))
        return y1

    check(S.FilterDnsamplingFir(c, 4), o.decim(0, 4, c), x[:30000], x[30000:])
    check(S.FilterDnsamplingFir(q14(c), 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int32_t"),
          o.decim(1, 4, q14(c)), xi[:20000], xi[20000:])
    check(S.FilterFir(hamming_sinc(31, 0.2)), o.fir(0, hamming_sinc(31, 0.2)), x[:30001], x[30001:])
    cu = q14(hamming_sinc(32, 0.12) * 4)
    check(S.FilterUpsamplingFir(cu, 4), o.up(0, 4, cu), xi[:5000], xi[5000:9000])
    m = S.Mixer(4096)
    m.reset(0.1)
    mo = o.mixer(4096)
    mo.reset(0.1)
    check(m, mo, xi[:17], xi[17:30000])
    # correlator: registers and history carried into the copy (detection in the second part)
    p = qpsk_pattern(32, 500, seed=3)
    xc = np.random.default_rng(8).integers(-125, 126, size=(8000, 2)).astype(np.int32)
    for k in range(32):
        xc[5000 + 4 * k] += 2 * p[k]
    xc = xc.astype(np.int16)
    g = S.FixedPatternCorrelator(32, 4)
    g.setPattern(p)
    go = o.corr(32, 4)
    go.set_pattern(p)
    assert not g.step(dev(xc[:4000]))[0] and not go.step(xc[:4000])[0]
    g2 = copy.copy(g)
    r1, r2, rr = g.step(dev(xc[4000:])), g2.step(dev(xc[4000:])), go.step(xc[4000:])
    assert r1 == r2 == rr and rr[0]
