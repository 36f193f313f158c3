import os
import sys

import pytest
import torch  # noqa: F401  (before libssbls.so: one HIP runtime per process, see _lib.load)

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
