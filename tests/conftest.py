import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP kernels)")


@pytest.fixture(scope="session")
def golden():
    g = np.load(os.path.join(GOLDEN, "augment_output_linear.npz"))
    img = np.load(os.path.join(GOLDEN, "img_2112_70_bgr.npz"))["bgr"]
    return {"train": g["train"], "eval": g["eval"], "img": img}


@pytest.fixture(scope="session")
def oracle():
    import oracle as O
    O.lib()
    return O
