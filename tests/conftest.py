import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# hipRTC code objects on disk (jit.cpp): one fresh directory per test session,
# set before libdfmi.so is loaded (nothing is written outside it)
if "DFMI_JIT_CACHE_DIR" not in os.environ:
    import tempfile
    os.environ["DFMI_JIT_CACHE_DIR"] = tempfile.mkdtemp(prefix="dfmi_jit_tests_")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


def pytest_collection_modifyitems(config, items):
    try:
        import torch
        has_gpu = torch.cuda.is_available()
    except Exception:
        has_gpu = False
    if has_gpu:
        return
    skip = pytest.mark.skip(reason="no GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
