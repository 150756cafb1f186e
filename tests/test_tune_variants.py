"""The tuning libraries of scripts/tune/variant_lib.py are patched copies of
the product sources: every patch site must still occur exactly once, and the
files a variant adds must exist, or the variant no longer builds (CPU only,
nothing is compiled)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "scripts", "tune"))

import variant_lib as V  # noqa: E402

CSRC = os.path.join(ROOT, "srcdsp_amd", "csrc")


@pytest.mark.parametrize("name", sorted(V.PATCHES))
def test_patch_sites_present_once(name):
    if name in V.STALE:
        pytest.skip(f"stale variant: {V.STALE[name]}")
    for fname, old, new in V.PATCHES[name]:
        text = open(os.path.join(CSRC, fname)).read()
        assert text.count(old) == 1, (name, fname, old[:80])
        assert old != new
    for fname in V.EXTRA.get(name, []):
        assert os.path.exists(os.path.join(V.HERE, fname)), fname


def test_corrmfma_never_in_the_product():
    """north_star: the product path uses no MFMA -- the matrix-core scan lives
    only in the tuning header, never in the product sources."""
    for f in os.listdir(CSRC):
        text = open(os.path.join(CSRC, f)).read()
        assert "corr_mfma_scan.h" not in text and "mfma_i32" not in text, f
