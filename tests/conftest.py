import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "jepsen-etcd-demo_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


def gpu_available() -> bool:
    try:
        from lincheck import _native as N
        return N.lib().lc_device_count() > 0
    except Exception:
        return False


@pytest.fixture(scope="session")
def device():
    if not gpu_available():
        pytest.fail("no GPU visible: -m gpu tests need an MI355X")
    from lincheck.checker import Device
    return Device(0)
