import os
import shutil
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

REF_DIR = os.environ.get("APM_REF_DIR", "/root/reference")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running test")


def have_node_and_reference() -> bool:
    return shutil.which("node") is not None and os.path.exists(os.path.join(REF_DIR, "entries.js"))


requires_reference = pytest.mark.skipif(not have_node_and_reference(),
                                        reason="node or the reference sources are not available")


@pytest.fixture(scope="session")
def gpu_available():
    import torch
    return torch.cuda.is_available()
