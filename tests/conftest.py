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


@pytest.fixture(scope="session", autouse=True)
def _torch_hip_first(request):
    """In one process torch must initialise HIP before libmassrt does: torch
    ships its own HIP runtime, and once libmassrt's (/opt/rocm) has opened the
    device torch's init reports "No HIP GPUs are available" (measured on the
    MI355X box with this round's and round 2's library alike,
    tools/diag/torch_after_raw.py). bench.py and the multi-rank tests set the
    torch device first; the GPU test session does it here."""
    if any(item.get_closest_marker("gpu") for item in request.session.items):
        import torch

        if torch.cuda.is_available():
            torch.cuda.init()
    yield


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def assets_dir():
    from gen_assets import ensure_assets
    return ensure_assets(REPO / "assets", mesh=True, textures=True, environment=True)


@pytest.fixture(scope="session", params=["reference", "near_first"])
def ctx(request):
    """A context per walk (option traversal): every test that takes `ctx`
    runs on the reference's left-first walk and on the near-first walk."""
    import massrt
    walk = massrt.TRAVERSAL_REFERENCE if request.param == "reference" else massrt.TRAVERSAL_NEAR_FIRST
    c = massrt.Context(0, options={"traversal": walk})  # raises loudly without a GPU: there is no fallback
    yield c
    c.close()


# counters of the walk itself: the near-first walk does other work for the
# same hits (tests/test_gpu_nearfirst.py); the rest must match either way
WALK_COUNTERS = {"node_visits", "sphere_tests", "triangle_tests", "instance_entries", "model_entries", "box_exact",
                 "wave_slots", "lane_steps", "vnf_fallbacks", "alpha_taps",
                 "texel_taps"}  # texel taps: alpha tests during the walk sample textures too


def walk_keys(c, keys):
    """`keys` to compare with the oracle's counters for context c's current
    scene: all of them on the reference's walk, the walk-independent ones on
    the near-first walk."""
    import massrt
    if c.tuning()["traversal"] == massrt.TRAVERSAL_REFERENCE:
        return list(keys)
    return [k for k in keys if k not in WALK_COUNTERS]
