import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

import __graft_entry__ as entry  # noqa: E402

# The build-kernel variant ids libgdp.so holds (gdp_build_variants; tests/test_abi.py checks the
# library against this list).  Round 5 kept the ids an autotune picked in round 4 plus v11.
BUILD_VARIANTS = (0, 8, 11, 15, 16, 17, 18, 20, 23, 27)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; run with -m gpu")


@pytest.fixture(scope="session", autouse=True)
def _built():
    """A fresh checkout has no built libraries (git-ignored): build them once (hipcc
    cross-compiles without a GPU)."""
    entry.ensure_built()


@pytest.fixture(scope="session")
def oracle():
    """The CPU checker (oracle/) — test infrastructure only."""
    mod = entry.load_oracle()
    mod.lib()  # builds liboracle.so on first use if needed
    return mod


@pytest.fixture(scope="session")
def pkg():
    """The product package; on a GPU box the HIP library MUST load (no fallback)."""
    return entry.load_package()


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np

    gdir = os.path.join(REPO, "tests", "golden")
    with open(os.path.join(gdir, "hashes.json")) as f:
        hashes = json.load(f)
    dumps = dict(np.load(os.path.join(gdir, "dumps.npz"), allow_pickle=False))
    taps = dict(np.load(os.path.join(gdir, "taps.npz"), allow_pickle=False))
    with open(os.path.join(gdir, "checksums.json")) as f:
        checksums = json.load(f)
    return {"hashes": hashes, "dumps": dumps, "taps": taps, "checksums": checksums}
