import os
import sys

import pytest

# hardware queues for the whole test process (HIP reads GPU_MAX_HW_QUEUES when it initialises, so
# before torch): the tests run up to 20 one-stream slots, and the library refuses a pipeline that
# does not fit the process's queues (ssb_hw_queue_budget; the GPU box exports HIP's default, 4)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "0") or 0) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"
import torch  # noqa: E402,F401  (before libssbls.so: one HIP runtime per process, see _lib.load)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP engine)")


@pytest.fixture(scope="session")
def engine():
    from safestakeoperator_amd.build import build
    build(verbose=False)
    from safestakeoperator_amd import Engine
    e = Engine(0)
    yield e
    e.close()
