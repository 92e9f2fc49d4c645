import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "clear-vae_amd"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (ROCm) device and libclearvae_hip.so")


def pytest_collection_modifyitems(config, items):
    try:
        import torch

        has_gpu = torch.cuda.is_available()
    except Exception:  # pragma: no cover
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this environment")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(autouse=True)
def _gemm_workspace(request):
    """GPU tests run with the library's GEMM workspace registered, as the engine runs (the in-launch
    split-K of long-K convolutions is then exercised by the kernel tests too)."""
    if "gpu" in request.keywords:
        import torch

        if torch.cuda.is_available():
            from cvhip import _lib

            _lib.ensure_gemm_workspace(torch.device("cuda", 0))
    yield
