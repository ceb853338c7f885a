"""Shared test setup.

* ``gpu`` marker: tests that need a real MI355X (run on the GPU box with
  ``pytest -m gpu``); everything else must pass on a CPU-only container.
* Puts the product package directory (``llama3.np_amd/``, imported the way
  the reference is: ``import llama3``, ``from config import ModelArgs``) and
  the oracle on ``sys.path``.
"""

import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "llama3.np_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
REFERENCE = "/root/reference"

for p in (PKG, os.path.join(REPO, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden
