import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")

# MIOpen's first use of each convolution shape runs an exhaustive kernel search (~1-2 min per new
# fwd+bwd shape on a fresh box, profiles/r01_network.txt); the learner tests only need correct
# convolutions, so the suite asks for the fast search (set before torch initialises MIOpen).
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libffmp on cuda:0)")


# Tests whose GPU work runs in child processes, or that need most of the HBM free, go first: this
# process parks the pieces of every frame ring it creates for reuse and never unmaps them
# (DESIGN §4), so late in the session a child (or a placement retry) would find less free HBM than
# bench.py does on a fresh box.
EARLY_MODULES = ("test_gpu_timed_path", "test_gpu_distributed", "test_gpu_rank_shard")
EARLY_TESTS = ("test_partner_relocation_keeps_a_consistent_env",)


def pytest_collection_modifyitems(config, items):
    def rank(it):
        if it.module.__name__.rsplit(".", 1)[-1] in EARLY_MODULES:
            return 0
        return 1 if it.name in EARLY_TESTS else 2
    items.sort(key=rank)


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "ref_pinned.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_maps():
    with np.load(os.path.join(GOLDEN, "ref_maps.npz")) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def lib():
    """The built libffmp (host entry points work without a GPU)."""
    import __graft_entry__
    __graft_entry__.build()
    from flow_field_based_motion_planner_amd import _abi
    return _abi.load()
