"""Two contexts planning at once on one device.

The control plane runs one deploy task per QUIC channel
(crates/fleetflow-controlplane/src/handlers/deploy.rs:13-20), so two host threads, each with its own
fp_ctx, can plan on the same GPU at the same time.  Bounded-link launches (FP_GEOM_BOUNDED) need
their segments co-resident; the library serialises them per device (fp_pipe.hip BoundedGate).
Each thread's plans must be bit-exact against the oracle, with no FP_EDEVICE.
"""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED = 0x5EED0C00


def _plan_loop(case, reps, out, barrier):
    from fleetflow_amd import Planner
    try:
        with Planner(0) as p:
            for k, v in case.get("opts", {}).items():
                p.set_option(k, v)
            cont, nodes = case["cont"], case["nodes"]
            out["geometry"] = p.geometry(1, cont[0].size, nodes[0].size)
            barrier.wait(timeout=60)
            out["plans"] = [p.place(cont, nodes) for _ in range(reps)]
    except Exception as e:  # reported by the main thread
        out["error"] = repr(e)


def test_two_contexts_bounded_at_once(O):
    cases = {
        "config2": O.gen_scenario(SEED + 2, 0, 10_000, 1_000, 1),
        "nodes100k": O.gen_scenario(SEED + 3, 0, 120_000, 100_000, 7),
    }
    reps = {"config2": 12, "nodes100k": 3}
    # config 2's 159-slot links already hold every container: 16-slot rings make it bounded too
    opts = {"config2": {"link_slots": 16}, "nodes100k": {}}
    outs = {k: {} for k in cases}
    barrier = threading.Barrier(len(cases))
    threads = [threading.Thread(target=_plan_loop, args=({"cont": c, "nodes": n, "opts": opts[k]}, reps[k], outs[k],
                                                              barrier))
               for k, (c, n) in cases.items()]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=280)
        assert not t.is_alive(), "a planning thread did not finish"
    for k, (cont, nodes) in cases.items():
        o = outs[k]
        assert "error" not in o, (k, o.get("error"))
        # both launches run bounded links: the case the per-device serialisation is for
        assert o["geometry"]["bounded"] == 1, (k, o["geometry"])
        ea, er, eafter, _ = O.place(cont, nodes)
        assert len(o["plans"]) == reps[k]
        for assign, reason, after in o["plans"]:
            assert np.array_equal(assign, ea), k
            assert np.array_equal(reason, er), k
            for i in (0, 1, 3):
                assert np.array_equal(after[i], eafter[i]), k
