import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "adlm-inherently-interpretable-segmentation_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built libprotoseg_hip.so")


@pytest.fixture(scope="session")
def device():
    import torch
    assert torch.cuda.is_available(), "gpu tests need a ROCm device (run with -m 'not gpu' on CPU)"
    return torch.device("cuda:0")


@pytest.fixture
def bwd_kernel():
    """set(name): the bf16x3 training backward's kernel for this test ("wave" / "fused"; the
    library's protoseg_set_backward_kernel), back to automatic afterwards."""
    from protoseg_amd import _lib

    def set_kernel(name):
        _lib.call("protoseg_set_backward_kernel", name.encode() if name else b"")

    yield set_kernel
    set_kernel("")
