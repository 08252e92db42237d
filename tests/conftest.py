import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def blob():
    with open(os.path.join(GOLDEN, "blob.bin"), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def ctx():
    """One liblsmck context for the whole GPU session (one process, one GPU)."""
    from lsm_storage_engine_amd.device import Context
    c = Context(0)
    yield c
    c.close()
