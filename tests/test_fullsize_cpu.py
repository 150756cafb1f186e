"""CPU: the parallel-window oracle runs behind the full-size GPU tests
(tests/fullsize.py) equal one single oracle call."""
import numpy as np
import pytest

import fullsize as F


@pytest.mark.parametrize("variant,kind", [(0, "cf32"), (1, "ci16")])
def test_decim_all_equals_single_call(O, variant, kind):
    from srcdsp_amd.design import hamming_sinc, q14
    c = hamming_sinc(127) if variant == 0 else q14(hamming_sinc(127))
    o = O["fma"]
    n = (1 << 18) + 4 * 37
    x = o.gen_cf32(7, 0, 0, n) if kind == "cf32" else o.gen_ci16(7, 0, 0, n)
    want = o.decim(variant, 4, c).step(x)
    got = F.decim_all(lambda: o.decim(variant, 4, c), x, 4, 128, np.empty_like(want), win_out=5000)
    assert F.first_bad(got, want) is None
    got[12345] += 1
    assert F.first_bad(got, want) == 12345


@pytest.mark.parametrize("where", [None, 40000, 65536 - 700, 65536 - 1023, 131072 + 3])
def test_corr_first_equals_single_call(O, where):
    """Pattern inside a window, straddling a window edge, ending right at one,
    and absent; index, bitSamples and registers as one call."""
    from srcdsp_amd.design import qpsk_pattern
    N = 256
    p = qpsk_pattern(N, 500, seed=5)
    rng = np.random.default_rng(11)
    x = rng.integers(-125, 126, size=(200000, 2)).astype(np.int32)
    if where is not None:
        x[where:where + N] += 2 * p
    x = np.clip(x, -32768, 32767).astype(np.int16)

    def make():
        r = O["fma"].corr(N, 1)
        r.set_pattern(p)
        return r

    one = make()
    f1, i1 = one.step(x)
    f2, i2, bits, st = F.corr_first(make, x, N, 1, win=65536)
    assert (f1, i1 if f1 else -1) == (f2, i2)
    if f1:
        assert i1 == where + N - 1
        assert np.array_equal(bits, one.bit_samples())
        s1 = one.status()
        assert all(s1[k] == st[k] for k in ("energy", "corr"))


def test_fir_and_up_windows_equal_single_call(O):
    """The window runs behind the fir / up whole-output GPU tests equal one call."""
    from srcdsp_amd.design import hamming_sinc, q14
    o = O["fma"]
    rng = np.random.default_rng(3)
    x = rng.integers(-2048, 2048, size=150000).astype(np.float32)
    c = hamming_sinc(31, 0.2)
    want = o.fir(1, c).step(x)
    got = F.decim_all(lambda: o.fir(1, c), x, 1, 32, np.empty_like(want), win_out=7000)
    assert F.first_bad(got, want) is None
    xu = o.gen_ci16(5, 0, 0, 70000)
    cu = q14(hamming_sinc(128, 0.12) * 4)
    want = o.up(0, 4, cu).step(xu)
    got = F.up_all(lambda: o.up(0, 4, cu), xu, 4, 40, np.empty_like(want), win_in=6000)
    assert F.first_bad(got, want) is None
