import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and libfleetplace.so")


@pytest.fixture(scope="session")
def kats():
    with open(os.path.join(GOLDEN, "reference_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "synthetic_small.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def O():
    """C oracle (test infrastructure)."""
    from oracle import oracle
    oracle.lib()
    return oracle


@pytest.fixture(scope="session")
def P():
    """Pure-Python oracle twin (test infrastructure)."""
    from oracle import pyoracle
    return pyoracle


@pytest.fixture(scope="session")
def planner():
    """The product: one fp_ctx on cuda:0.  Fails loudly without the HIP library."""
    from fleetflow_amd import Planner
    p = Planner(0)
    yield p
    p.close()


@pytest.fixture
def opts(planner):
    """Set context options for one test (fp_ctx_set_option, fleetplace.h enum fp_option):
    ``opts(pipe_w=4, pipe_seg=4)``.  Every option goes back to FP_OPT_AUTO afterwards."""
    def set_(**kw):
        for k, v in kw.items():
            planner.set_option(k, v)
    yield set_
    planner.reset_options()
