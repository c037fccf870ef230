"""The benchmark's host DAG generator (fleetflow_amd/synth.py, SPEC.md 3.3) against the C
oracle's (oracle/fp_oracle.c fpo_gen_dag): same reversed CSR and has_deps on the same seed."""
import numpy as np
import pytest

from fleetflow_amd import synth


@pytest.mark.parametrize("params", [(0x5EED0005, 3, 4, 2, 5, 1), (7, 10, 20, 5, 30, 4), (9, 0, 0, 3, 10, 2),
                                    (11, 5, 1, 1, 2, 3), (0x5EED0005, 50, 100, 10, 400, 33)])
def test_gen_dag_matches_oracle(params, O):
    rp, col, hd = synth.gen_dag(*params)
    erp, ecol, ehd = O.gen_dag(*params)
    assert np.array_equal(rp, erp) and np.array_equal(col, ecol) and np.array_equal(hd, ehd)


def test_draw_matches_oracle(O, P):
    s = O.scenario_seed(0x5EED0004, 3)
    assert [int(x) for x in synth.draw(s, np.arange(5))] == [P.draw(s, k) for k in range(5)]
