import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "lightfieldmicroscopy_pc-bzip2_amd")
for p in (REPO, PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

REFERENCE = "/root/reference"
GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu)")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def oracle():
    import lfm_oracle
    lfm_oracle.lib()
    return lfm_oracle


@pytest.fixture(scope="session")
def lfmlib():
    import lfm
    lfm.lib()
    return lfm


@pytest.fixture(scope="session")
def gpu(lfmlib):
    import torch
    if not torch.cuda.is_available() or lfmlib.device_count() <= 0:
        pytest.fail("GPU test requested but no HIP device is visible")
    torch.cuda.init()
    return torch
