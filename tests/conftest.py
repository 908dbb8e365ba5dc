"""Shared pytest setup: the ``gpu`` marker, import paths and golden-fixture loaders."""
import glob
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "i-admm-lstm_amd")
for _p in (REPO, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


def golden_files():
    return sorted(glob.glob(os.path.join(GOLDEN, "*.npz")))


def load_golden(path):
    f = np.load(path)  # allow_pickle=False (default): data only
    return {k: f[k] for k in f.files}


@pytest.fixture(params=[os.path.basename(p)[:-4] for p in golden_files()])
def golden(request):
    return request.param, load_golden(os.path.join(GOLDEN, request.param + ".npz"))
