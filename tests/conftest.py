"""Test configuration.

`-m "not gpu"`: oracle vs golden fixtures, host logic (loaders, BVH, sampler, decoders),
C-ABI exports, gloo multi-process sharding. `-m gpu`: parity of the HIP path with the oracle,
called through the C ABI on a real MI355X.
"""
import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
for p in (ROOT, ROOT / "yulio-raytracer_amd"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

SCENES = ROOT / "scenes"
GOLDEN = ROOT / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run on the GPU box via gpurun)")


@pytest.fixture(scope="session")
def host_device():
    import yrt
    d = yrt.Device(host=True)
    yield d
    d.close()


@pytest.fixture(scope="session")
def gpu_device():
    import yrt
    d = yrt.Device(0)
    yield d
    d.close()
