import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")
if GOLDEN not in sys.path:
    sys.path.insert(0, GOLDEN)

# torch first: it ships its own HIP runtime, which cannot enumerate the GPU
# once libcapf_gpu.so's runtime has initialised it in the same process
import torch  # noqa: E402,F401

import capf_import  # noqa: E402,F401


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: larger parity sizes")


def bag(rows):
    """okapi-testing Bag (OT/Bag.scala:29-51): multiset equality of records."""
    def norm(v):
        if v is None:
            return ("0null", 0.0, "")
        if isinstance(v, bool):
            return ("bool", float(v), "")
        if isinstance(v, (int, float)):
            if isinstance(v, float) and v != v:
                return ("nan", 0.0, "")
            return ("num", float(v), "")
        return ("str", 0.0, str(v))
    return sorted(tuple(sorted((k, norm(v)) for k, v in r.items())) for r in rows)


@pytest.fixture(scope="session")
def gpu_session():
    from capf_amd.table import GpuSession
    s = GpuSession(0)
    yield s
