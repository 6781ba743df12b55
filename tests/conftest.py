import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


def pytest_sessionstart(session):
    """GPU runs: bring torch's HIP context up before any test opens engine handles.  Tests that generate data in HBM
    (test_full_size, test_node) initialise torch lazily; after several hundred native handles had been opened and
    closed in one process, that late initialisation once reported "No HIP GPUs are available" on the box (the same
    tests pass when they run first, as in the default file order)."""
    if (session.config.getoption("markexpr", "") or "").strip() != "gpu":
        return
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
            torch.zeros(1, device="cuda:0")
    except Exception:   # a box without a GPU fails the GPU tests themselves, with their own messages
        pass
