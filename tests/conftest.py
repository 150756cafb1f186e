import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box)")
    # the oracle is test infrastructure; build it on demand (gcc, seconds)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "liboracle.so"], check=True,
                       stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def golden():
    from replay import load_golden
    return load_golden()


@pytest.fixture(scope="session")
def S():
    """The product package with its HIP library loaded (GPU tests only)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import srcdsp_amd
    srcdsp_amd.lib()
    return srcdsp_amd


@pytest.fixture(scope="session")
def O():
    """The oracle (test infrastructure): strict and FMA float contracts."""
    import pyoracle
    return {"strict": pyoracle.Oracle(0), "fma": pyoracle.Oracle(1)}
