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
