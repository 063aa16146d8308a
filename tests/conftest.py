import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
HERE = os.path.dirname(os.path.abspath(__file__))
if HERE not in sys.path:
    sys.path.insert(0, HERE)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    g = os.path.join(HERE, "golden")
    with open(os.path.join(g, "golden.json")) as f:
        meta = json.load(f)
    lo = np.load(os.path.join(g, "lengths_offsets.npz"))
    cfg = np.load(os.path.join(g, "configs.npz"))
    return {"meta": meta, "lo": lo, "cfg": cfg}
