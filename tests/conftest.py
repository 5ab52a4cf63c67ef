import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "go-audio-resampler_amd")
for p in (ROOT, PKG, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "slow: full BASELINE-size GPU runs")


@pytest.fixture(scope="session")
def O():
    """The CPU oracle (test infrastructure only)."""
    from oracle import oracle as mod
    mod.build()
    return mod


@pytest.fixture(scope="session")
def gar():
    """The product package; builds libgar.so in-tree if it is missing (no fallback)."""
    lib = os.path.join(PKG, "libgar.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j", os.environ.get("MAX_JOBS", "8"), "-C", PKG], check=True)
    import gar as mod
    mod.lib()
    return mod


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch
