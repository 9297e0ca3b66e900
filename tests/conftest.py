import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and libgossip_hip.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    pyoracle.build()
    return pyoracle


def pytest_sessionfinish(session, exitstatus):
    """Hand the library's cached device blocks back before the process exits:
    the next process on the GPU (the driver's smoke and bench) waits while the
    driver clears the memory a previous process left, and
    a trim now lets that clearing start while this process winds down.  No-op
    where the library was never loaded (the CPU suite)."""
    mod = sys.modules.get("gossip_simulator_amd._lib")
    if mod is None or getattr(mod, "_lib", None) is None:
        return
    try:
        from gossip_simulator_amd import engine
        engine.trim()
    except Exception:  # a failed trim must not fail the session
        pass
