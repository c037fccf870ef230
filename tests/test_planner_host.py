"""Host-side argument checks of the Python mirror (no GPU): every host-pointer call reads its arrays
for the lengths its sizes imply, so a short array is refused with ValueError before the library is
called -- the Rust binding's FP_EINVAL checks (integration/fleetflow-placement/src/lib.rs plan_stage,
place, place_batch).  ADVICE r05: Planner.plan_stage took V from has_deps and memcpy'd (V + 1) words
of row_ptr and V of each container field without checking."""
import numpy as np
import pytest

from fleetflow_amd.planner import Planner


class _NoLib:
    def __getattr__(self, name):  # any library call would be a failed check
        raise AssertionError(f"library called: {name}")


@pytest.fixture
def p():
    q = object.__new__(Planner)  # no context, no device: the checks come first
    q._L = _NoLib()
    return q


def _u(*xs):
    return tuple(np.array(x, np.uint32) for x in xs)


def test_plan_stage_row_ptr_length(p):
    with pytest.raises(ValueError, match="row_ptr"):
        p.plan_stage([0, 0], [], [0, 0])
    with pytest.raises(ValueError, match="row_ptr"):
        p.levelize([0, 0, 0, 0], [], [0, 0])


def test_plan_stage_container_and_node_lengths(p):
    rp, col, hd = [0, 0, 0], [], [0, 0]
    nodes = _u([9], [9], [0], [0]) + (np.ones(1, np.uint8),)
    with pytest.raises(ValueError, match="container"):
        p.plan_stage(rp, col, hd, _u([1], [1], [0], [0]), nodes)
    with pytest.raises(ValueError, match="node"):
        p.plan_stage(rp, col, hd, _u([1, 1], [1, 1], [0, 0], [0, 0]), _u([9], [9], [0, 0], [0]) + (np.ones(1, np.uint8),))


def test_place_and_batch_lengths(p):
    nodes = _u([9], [9], [0], [0]) + (np.ones(1, np.uint8),)
    with pytest.raises(ValueError, match="container"):
        p.place(_u([1, 1], [1], [0, 0], [0, 0]), nodes)
    with pytest.raises(ValueError, match="level"):
        p.place(_u([1], [1], [0], [0]), nodes, level=[0, 0])
    with pytest.raises(ValueError, match="node"):
        p.place(_u([1], [1], [0], [0]), _u([9], [9], [0], [0]) + (np.ones(2, np.uint8),))
    with pytest.raises(ValueError, match="container"):
        p.place_batch(2, 1, 1, _u([1], [1], [0], [0]), _u([9, 9], [9, 9], [0, 0], [0, 0]) + (np.ones(2, np.uint8),))
    with pytest.raises(ValueError, match="node"):
        p.place_batch(1, 1, 2, _u([1], [1], [0], [0]), nodes)
