import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "data"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running")


DATA = os.path.join(ROOT, "data")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def data(name: str) -> str:
    return os.path.join(DATA, name)


@pytest.fixture(scope="session")
def sponza_path():
    import gen_standin_sponza
    return gen_standin_sponza.ensure()


@pytest.fixture(scope="session")
def gpu():
    import toymeshpathtracer_amd as tm
    n = tm.device_count()
    if n < 1:
        raise RuntimeError("GPU test on a machine with no visible GPU")
    return 0
