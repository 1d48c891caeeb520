"""Test configuration: `gpu` marker, import paths and shared fixtures.

CPU suite:  python -m pytest tests -m "not gpu"   (oracle, host builder, loaders, ABI)
GPU suite:  python -m pytest tests -m gpu         (HIP kernels vs the oracle, via the C ABI)
"""
import os
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
for p in (REPO, REPO / "mass-raytrace_amd", REPO / "tools"):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))

GOLDEN = REPO / "tests" / "golden"


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: builds the 1M-triangle scenes")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def assets_dir():
    from gen_assets import ensure_assets
    return ensure_assets(REPO / "assets", mesh=True, textures=True, environment=True)


@pytest.fixture(scope="session")
def ctx():
    import massrt
    c = massrt.Context(0)  # raises loudly without a GPU: there is no fallback
    yield c
    c.close()
