"""Stream behaviour of the operators' host-side entry points: reset() clears
the history on the handle's own stream and waits for that stream only, so it
does not stall behind unrelated work queued on other streams (a device-wide
synchronize would wait for it)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_reset_does_not_wait_for_other_streams(S):
    import torch
    from srcdsp_amd.design import hamming_sinc, qpsk_pattern
    ops = [S.FilterDnsamplingFir(hamming_sinc(127), 4), S.FilterFir(hamming_sinc(31)),
           S.FilterUpsamplingFir(np.arange(1, 129, dtype=np.int32), 4), S.FixedPatternCorrelator(64, 1)]
    ops[3].setPattern(qpsk_pattern(64, 500, seed=1))
    side = torch.cuda.Stream()
    torch.cuda.synchronize()
    with torch.cuda.stream(side):
        torch.cuda._sleep(int(2e9))  # ~1 s of busy cycles on a stream no operator uses
    for op in ops:
        op.reset()
    still_busy = not side.query()
    side.synchronize()
    assert still_busy, "reset() waited for another stream's work"


def test_one_mixer_feeding_two_decimators_on_two_streams(S, O):
    """one Mixer chained into two FilterDnsamplingFir objects whose
    steps run on two streams, through the unfused chain (int16 taps: the mixer
    writes its scratch buffer, the decimator reads it).  The second chain's
    mixer launch must wait for the FIRST chain's decimator (the scratch's
    reader), not only for the first mixer launch: both outputs equal the two
    reference call pairs, with the mixer's phase carried from one to the next."""
    import torch
    from srcdsp_amd.design import hamming_sinc, q14
    cq = q14(hamming_sinc(512, 0.1)).astype(np.int16)
    nA, nB = 1 << 22, 1 << 18
    x = O["strict"].gen_ci16(0xBEEF, 3, 0, nA + nB, -32768, 32767)
    m = S.Mixer(4096)
    m.reset(0.07)
    dA = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int16_t")
    dB = S.FilterDnsamplingFir(cq, 4, "complex<int16_t>", "complex<int16_t>", "complex<int32_t>", "int16_t")
    a, b = S.MixerDecimatorChain(m, dA), S.MixerDecimatorChain(m, dB)
    xa = torch.from_numpy(x[:nA]).cuda()
    xb = torch.from_numpy(x[nA:]).cuda()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    torch.cuda.synchronize()
    for _ in range(3):
        with torch.cuda.stream(s1):
            ya = a.step(xa)
        with torch.cuda.stream(s2):
            yb = b.step(xb)
    torch.cuda.synchronize()
    om = O["strict"].mixer(4096)
    om.reset(0.07)
    oa, ob = O["strict"].decim(2, 4, cq), O["strict"].decim(2, 4, cq)
    for _ in range(3):
        ra = oa.step(om.step(x[:nA]))
        rb = ob.step(om.step(x[nA:]))
    assert np.array_equal(ya.cpu().numpy(), ra)
    assert np.array_equal(yb.cpu().numpy(), rb)
    assert m.state()[:2] == om.state()[:2]
