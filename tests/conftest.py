import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# GPU test files that run last: the full-size goldens (10^8-10^9-triple inputs) take the longest, so every smaller
# parity test (sharded, paged driver, ingest, ...) has run before them
_LAST = ("test_gpu_full.py",)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (runs through the HIP C ABI)")


def pytest_collection_modifyitems(session, config, items):
    items.sort(key=lambda it: os.path.basename(str(it.fspath)) in _LAST)  # stable: file order kept otherwise
