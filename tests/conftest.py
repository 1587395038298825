"""Shared test setup.

Markers: `gpu` tests need a HIP device (run on the MI355X box with -m gpu);
everything else runs on CPU.  Only tests/ (and smoke()/bench.py's
cpu_baseline) may use the oracle under oracle/ — as the checker.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ray-tracer-challenge-rs_amd")
ORACLE = os.path.join(ROOT, "oracle")
GOLDEN = os.path.join(ROOT, "tests", "golden")
REFERENCE = "/root/reference"
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long CPU test")


def _built():
    lib = os.path.join(PKG, "rtc_amd", "_lib", "librtc.so")
    olib = os.path.join(ORACLE, "_build", "liboracle.so")
    if not (os.path.exists(lib) and os.path.exists(olib)):
        import subprocess
        subprocess.run([sys.executable, "-c", "import __graft_entry__ as g; g.build()"], cwd=ROOT, check=True)


_built()


@pytest.fixture(scope="session")
def rtc():
    import rtc_amd
    return rtc_amd


@pytest.fixture(scope="session")
def oracle():
    import pyoracle
    return pyoracle


def scene_fixture(name):
    from rtc_amd import scene_io
    return scene_io.load(os.path.join(GOLDEN, "scenes", f"{name}.json"))


@pytest.fixture(scope="session")
def gpu_ctx():
    """One context for the whole GPU session (tests upload their own worlds)."""
    import rtc_amd
    if rtc_amd.device_count() < 1:
        pytest.fail("gpu test selected but no HIP device is visible — the render path has no CPU fallback")
    ctx = rtc_amd.Context(0)
    yield ctx
    ctx.close()
