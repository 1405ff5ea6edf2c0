import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(Path(__file__).resolve().parent))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libmhmkc.so on the GPU)")
    config.addinivalue_line("markers", "slow: larger inputs (still minutes at most)")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """Native libraries are built in-tree (the GPU box receives the prebuilt .so files)."""
    from mhm2_proxy_amd import build

    if not build.SYNTH.exists() or not build.ORACLE.exists():
        build.build_synth()
        build.build_oracle()
    yield


@pytest.fixture(autouse=True)
def _debug_knobs_reset():
    """Every test starts and ends with the library's test-only switches at their defaults."""
    from mhm2_proxy_amd import _native as N

    N.debug_reset()
    yield
    N.debug_reset()


@pytest.fixture
def knob():
    """knob(name, value): set a test-only switch of libmhmkc (include/mhmkc_debug.h) for this test."""
    from mhm2_proxy_amd import _native as N

    return N.debug_set


def apply_env(d: dict) -> None:
    """Worker processes: "knob:<name>" entries set a test-only switch, the others an environment variable."""
    from mhm2_proxy_amd import _native as N

    for key, val in d.items():
        if key.startswith("knob:"):
            N.debug_set(key[5:], int(val))
        else:
            os.environ[key] = val
