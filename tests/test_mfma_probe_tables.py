"""The integer matrix-core tuning probes' host side (scripts/tune/corr_mfma.py,
scripts/tune/mixdecim_mfma.py; never shipped): their
numpy replay of the kernels' lane fragments, limb planes and Toeplitz B tables
must reproduce the oracle bit for bit (config 5's correlator registers on a
buffer holding the pattern; config 4's mixer -> decimator outputs with the
zero history), so a GPU run of a probe checks the kernel, not its tables."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts", "tune"))


def test_corr_probe_tables_replay_the_oracle():
    import corr_mfma as M
    p, x = M.config5_buffer(8192)  # the pattern copy at 6144: detection-sized correlations
    got = M.emulate(p, x, 8192)
    want, _ = M.oracle_registers(p, x)
    assert np.array_equal(got, want)


def test_corr_probe_limb_split_range():
    import corr_mfma as M
    lo, hi = M.limbs(np.array([-32640, -1, 0, 127, 128, 32639]))
    assert np.array_equal(256 * hi.astype(np.int64) + lo, [-32640, -1, 0, 127, 128, 32639])
    try:
        M.limbs(np.array([32640]))
    except ValueError:
        pass
    else:
        raise AssertionError("32640 needs a third limb")


def test_mixdecim_probe_tables_replay_the_oracle():
    import mixdecim_mfma as M
    import pyoracle
    from srcdsp_amd.design import hamming_sinc, q14
    c = q14(hamming_sinc(127))
    x = pyoracle.Oracle(0).gen_ci16(M.SEED, 0, 0, 4096, -32768, 32767)  # full scale: the clamps engage
    assert np.array_equal(M.emulate(x, c, 4096), M.oracle_chain(x, c))
