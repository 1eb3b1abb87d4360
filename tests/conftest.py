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


@pytest.fixture(autouse=True)
def _gpu_heartbeat(request):
    """GPU tests on the box: a line every 30 s under gpurun_out/ while a test runs, so a long
    multi-process test (elastic degrade, supervisor restarts: minutes with pytest capturing its
    output) is not taken for a hung command; pytest's own per-test timeout still ends a real hang."""
    root = os.environ.get("GRAFT_REPO_ROOT")
    if root is None or request.node.get_closest_marker("gpu") is None:
        yield
        return
    import threading
    import time
    path = os.path.join(root, "gpurun_out", "pytest_progress.log")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    stop = threading.Event()
    t0 = time.time()

    def beat():
        while not stop.wait(30.0):
            with open(path, "a") as f:
                f.write(f"[heartbeat] {request.node.nodeid} {time.time() - t0:.0f}s\n")

    with open(path, "a") as f:
        f.write(f"[start] {request.node.nodeid}\n")
    th = threading.Thread(target=beat, daemon=True)
    th.start()
    try:
        yield
    finally:
        stop.set()
        th.join(5)
        with open(path, "a") as f:
            f.write(f"[end] {request.node.nodeid} {time.time() - t0:.0f}s\n")
