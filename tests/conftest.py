"""Test configuration: `gpu` marker, package path, shared golden helpers."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "afivo-streamer_amd"))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# pytest-xdist workers each load the OpenMP oracle: one thread per worker
# (N workers x all-core OpenMP teams spin against each other and run the
# suite tens of times slower)
if "PYTEST_XDIST_WORKER" in os.environ and "OMP_NUM_THREADS" not in os.environ:
    os.environ["OMP_NUM_THREADS"] = "1"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")
