"""CPU tests of the host-side front end (names -> ids -> reversed CSR)."""
import numpy as np

from fleetflow_amd.flow import Flow, LabelDict, Service, has_deps_vector, stage_graph


def test_has_deps_predicate_matches_engine_rs():
    # engine.rs:71-80: known && !depends_on.is_empty(); unknown names -> first bucket (0)
    flow = Flow(services={"api": Service(depends_on=["db"]), "db": Service()})
    assert list(has_deps_vector(["api", "db", "ghost"], flow)) == [1, 0, 0]


def test_stage_graph_reversed_csr_and_duplicates():
    flow = Flow(services={"app": Service(depends_on=["db", "cache", "db", "external"]),
                          "db": Service(), "cache": Service(depends_on=["db"])})
    names, pos2v, rp, col, hd = stage_graph(["db", "app", "cache", "db"], flow)
    assert names == ["db", "app", "cache"]
    assert list(pos2v) == [0, 1, 2, 0]           # duplicate -> first occurrence's vertex
    assert list(hd) == [0, 1, 1]
    # edges dep->dependent: db->app (x2), cache->app, db->cache; "external" is outside the set
    rows = {d: sorted(col[rp[d]:rp[d + 1]].tolist()) for d in range(3)}
    assert rows == {0: [1, 1, 2], 1: [], 2: [1]}
    assert rp[-1] == col.size == 4


def test_label_dictionary_is_sorted_and_dense():
    ld = LabelDict(["tier=web", "arch=arm64", "tier=web", "region=tk"])
    assert ld.bits == {"arch=arm64": 0, "region=tk": 1, "tier=web": 2}
    assert ld.mask(["tier=web", "arch=arm64"]) == 0b101


def test_empty_stage_graph():
    names, pos2v, rp, col, hd = stage_graph([], Flow())
    assert names == [] and rp.tolist() == [0] and col.size == 0 and np.asarray(hd).size == 0
