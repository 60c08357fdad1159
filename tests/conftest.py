"""Test configuration: `gpu` marker, repo on sys.path, native build on demand."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")
    # build the native runtime if it is missing (the driver calls build() first)
    lib = os.path.join(ROOT, "dmlc_core_amd", "lib", "libdmlc.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-C", ROOT, "-j", "8", "all"], check=True)


@pytest.fixture(scope="session")
def has_gpu():
    import torch
    return torch.cuda.is_available()


@pytest.fixture
def tmpdir_path(tmp_path):
    return str(tmp_path)
