import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "jepsen-etcd-demo_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT, os.path.dirname(os.path.abspath(__file__))):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    # Build what the tests load if a checkout has not been built yet
    # (the GPU box receives the prebuilt files; nothing is compiled there).
    if not os.path.exists(os.path.join(ORACLE, "_build", "liboracle.so")):
        subprocess.run(["make", "-C", ORACLE], check=True, capture_output=True)
    if not os.path.exists(os.path.join(PKG, "lincheck", "liblincheck.so")):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)


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
    return Device(0, count_probes=True)
