import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")


@pytest.fixture(scope="session")
def tree_pattern():
    return os.path.join(ROOT, "patterns", "rmat_log2_tree_pattern")


@pytest.fixture(scope="session")
def cycle_pattern():
    return os.path.join(ROOT, "patterns", "rmat_log2_cycle4_pattern")


@pytest.fixture(autouse=True)
def _heartbeat():
    """Prints a line every 60 s while a test runs (long GPU / oracle cases are
    otherwise silent for minutes and look hung to the GPU runner)."""
    import threading
    import time
    stop = threading.Event()

    def beat():
        t0 = time.time()
        while not stop.wait(60):
            print(f"[heartbeat {time.time() - t0:.0f}s]", file=sys.stderr, flush=True)

    th = threading.Thread(target=beat, daemon=True)
    th.start()
    yield
    stop.set()
