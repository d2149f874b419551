"""Shared test setup.

Markers:
  gpu — needs an MI355X (run on the GPU box: `pytest tests -m gpu`).
Everything unmarked runs on CPU (`pytest tests -m "not gpu"`).
"""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.join(REPO, "tests")
PKG = os.path.join(REPO, "raytracer-challenge-rs_amd")
for p in (REPO, PKG, TESTS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct MI355X (gfx950) GPU")


def _ensure_built():
    lib = os.path.join(PKG, "lib", "librtamd.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", PKG], check=True)
    orc = os.path.join(REPO, "oracle", "_build", "liboracle.so")
    if not os.path.exists(orc):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)


_ensure_built()


@pytest.fixture(scope="session")
def rt():
    import rtamd
    return rtamd


@pytest.fixture(scope="session")
def oracle():
    from oracle import pyoracle
    return pyoracle
