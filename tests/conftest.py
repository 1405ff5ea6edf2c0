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
