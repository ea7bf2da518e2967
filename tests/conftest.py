"""Test configuration.

Markers:
  gpu  -- needs an MI355X (runs on the GPU box: `pytest -m gpu`); calls the
          HIP engine through the C ABI (libmde_hip.so) and checks it against
          the oracle / golden fixtures.
Everything unmarked runs on the CPU (`pytest -m "not gpu"`).
"""

import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import pytest  # noqa: E402

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X GPU and the built libmde_hip.so")


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """Fail (not skip) a gpu-marked test when no GPU is present: on the GPU
    box a missing device or library must be loud."""
    import torch
    assert torch.cuda.is_available(), "gpu-marked test run without a visible GPU"
    from monocular_depth_estimation_trt_amd import _lib
    _lib.lib()  # raises if libmde_hip.so is missing
    return torch.device("cuda:0")
