import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def pkg():
    from mi355x_pkg import load_package
    return load_package()


@pytest.fixture(scope="session")
def backend(pkg):
    be = pkg.Backend(0)
    yield be
    be.free()


@pytest.fixture(scope="session")
def orc():
    import oracle_lib
    return oracle_lib.load()
