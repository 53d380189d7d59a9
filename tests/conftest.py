import importlib
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


@pytest.fixture(scope="session")
def pkg():
    return importlib.import_module("aa-admm_amd")


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    return pyoracle


@pytest.fixture(scope="session")
def ctx(pkg):
    c = pkg.capi.Context(0)
    yield c
    c.close()
