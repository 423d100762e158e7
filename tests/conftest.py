import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# Tests that hand device buffers to the library use PyTorch for allocation.  Load torch (and with
# it its HIP runtime) before libdkg_amd.so can pull in /opt/rocm's, whatever subset of the tests
# runs: with the other order torch sees no GPU in this process.  Device counting only, no HIP init.
try:
    import torch  # noqa: F401,E402
except Exception:  # pragma: no cover - torch is part of the image
    torch = None


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built HIP library")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def gpu_available():
    try:
        import torch  # noqa: F401  (device counting only; no HIP init here)
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def golden():
    import json

    cache = {}

    def load(name):
        if name not in cache:
            with open(os.path.join(ROOT, "tests", "golden", name)) as f:
                cache[name] = json.load(f)
        return cache[name]

    return load
