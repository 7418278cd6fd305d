import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


def _gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


def pytest_collection_modifyitems(config, items):
    if _gpu_available():
        return
    skip = pytest.mark.skip(reason="no HIP device visible")
    for item in items:
        if "gpu" in item.keywords:
            item.add_marker(skip)


@pytest.fixture(scope="session")
def ctx():
    """One device context for the whole GPU session (tests reuse it)."""
    from vrpms_amd.build import build_library
    build_library()
    from vrpms_amd.core import Context
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(scope="session")
def coracle():
    from oracle import coracle as co
    co.build()
    return co
