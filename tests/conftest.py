"""Shared test setup.

Markers:
  gpu  -- needs a real MI355X (run with `-m gpu` on the GPU box); everything
          else runs on the CPU-only container (`-m "not gpu"`).
The CPU oracle (oracle/) is imported here strictly as the checker.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "cuda-dct-idct_amd")
for p in (ROOT, PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP kernels run)")
    config.addinivalue_line("markers", "slow: long CPU-side checks (opt-in with -m slow)")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O


@pytest.fixture(scope="session")
def hp():
    import hpdct
    hpdct.load_library()  # raises HpdctLibraryError if the build is missing
    return hpdct


@pytest.fixture(scope="session")
def dev():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("gpu test selected but no HIP device is visible")
    return torch.device("cuda:0")
