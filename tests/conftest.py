import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "3d-dycoreplanet_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs under -m gpu")


def _ensure_built():
    if not os.path.exists(os.path.join(PKG, "libdcp.so")):
        subprocess.check_call(["make", "-j8", "-C", PKG])
    if not os.path.exists(os.path.join(ORACLE, "build", "liboracle.so")):
        subprocess.check_call(["make", "-C", ORACLE])


_ensure_built()


@pytest.fixture(scope="session")
def classic():
    import dcp
    return dcp.classic_physics()
