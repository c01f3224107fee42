import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG_DIR = os.path.join(REPO, "configurable-hierarchical-allreduce-algorithms_amd")
for p in (REPO, PKG_DIR, os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu on the GPU box)")
    config.addinivalue_line("markers", "slow: larger CPU cases")


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays


@pytest.fixture(scope="session")
def golden_mpich():
    """Golden vectors of the MPICH baselines testing/main.cpp drives (gen_golden.py mpich)."""
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "mpich_manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "mpich_outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays


@pytest.fixture(scope="session")
def golden_types():
    """Golden vectors of the integer types beyond int32 and the logical/bitwise ops, from the
    reference compiled here against MPICH (gen_golden.py types)."""
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "types_manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "types_outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays


@pytest.fixture(scope="session")
def golden_rsmpich():
    """Golden vectors of the MPICH baseline reduce-scatters that
    testing/mpich_implementations/reduce_scatter/main.cpp drives (gen_golden.py rsmpich)."""
    import json

    import numpy as np

    here = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(here, "rsmpich_manifest.json")) as f:
        manifest = json.load(f)
    arrays = np.load(os.path.join(here, "rsmpich_outputs.npz"), allow_pickle=False)
    return manifest["cases"], arrays
