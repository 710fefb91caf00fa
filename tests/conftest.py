import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


def golden(name):
    path = os.path.join(GOLDEN, name)
    return dict(np.load(path, allow_pickle=False))


def rel_l2(a, b):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.fixture(scope="session")
def states():
    import torch
    from audiolcm_amd import recipe
    torch.set_num_threads(max(1, min(8, len(os.sched_getaffinity(0)))))
    return dict(dit=recipe.dit_state(0), vae=recipe.vae_state(0), bigvgan=recipe.bigvgan_state(0))
