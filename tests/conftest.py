import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 GPU (run with -m gpu)")


@pytest.fixture(scope="session")
def oracle():
    """CPU oracle (test infrastructure): oracle/_build/liboracle.so."""
    so = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(so) and os.path.exists("/usr/bin/gcc"):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    from tests import oracle_ctypes
    return oracle_ctypes.Oracle(so)


@pytest.fixture(scope="session")
def golden():
    import json
    d = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(d, "lz4_golden.json")) as f:
        lz4 = json.load(f)
    with open(os.path.join(d, "zstd_golden.json")) as f:
        zs = json.load(f)
    return {"lz4": lz4, "zstd": zs}


@pytest.fixture(scope="session")
def lib():
    from juicefs_amd import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test requested but torch.cuda.is_available() is False")
    from juicefs_amd import _lib
    lib = _lib.load()
    assert lib.jfs_device_count() >= 1, "libjfsgpu found no gfx950 device"
    return torch.device("cuda:0")
