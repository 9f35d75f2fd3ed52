"""Shared pytest setup.

* registers the ``gpu`` marker (tests that need an MI355X);
* puts the repo root (for ``oracle``) and ``gol-distributed-final_amd/`` (for
  the ``golhip`` package) on sys.path.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(ROOT, "gol-distributed-final_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (ROOT, PKG_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
