"""Regenerate tests/golden/synthetic_small.json from the pure-Python oracle twin.

    python tests/golden/make_golden.py

The vectors are small SPEC.md section-3 instances (seeded SplitMix64) with the
expected planner outputs computed by oracle/pyoracle.py.  They pin the C oracle
and the HIP path to the same numbers; they are NOT reference-pinned (the
reference has no levels/FFD: see DESIGN.md "Oracle").
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import pyoracle as P  # noqa: E402

SEED = 0x5EED0000


def ffd_case(name, seed, scenario, C, N, flags, level=None):
    s = P.scenario_seed(seed, scenario)
    cpu, mem, req, conf = P.gen_containers(s, C, flags)
    cf, mf, lab, cu, sched = P.gen_nodes(s, N)
    assign, reason = P.place(cpu, mem, req, conf, cf, mf, lab, cu, sched, level)
    return {"name": name, "seed": seed, "scenario": scenario, "C": C, "N": N, "flags": flags,
            "cont": [cpu, mem, req, conf], "level": level,
            "assign": assign, "reason": reason, "cost": P.cost(assign, scenario),
            "nodes_after": [cf, mf, cu]}


def main():
    out = {"_about": __doc__.strip().splitlines()[0], "generator": {}, "ffd": [], "levelize": [],
           "feasibility": []}
    # generator spot values
    s = P.scenario_seed(SEED, 3)
    out["generator"] = {"seed": SEED, "scenario": 3, "draw_0_1_2": [P.draw(SEED, k) for k in range(3)],
                        "containers": [list(x) for x in P.gen_containers(s, 16, 7)],
                        "nodes": [list(x) for x in P.gen_nodes(s, 16)]}
    out["ffd"].append(ffd_case("c2-like", SEED + 2, 0, 300, 30, 1))
    out["ffd"].append(ffd_case("c3-like", SEED + 3, 0, 400, 40, 7))
    out["ffd"].append(ffd_case("c4-scen17", SEED + 4, 17, 250, 70, 7))
    out["ffd"].append(ffd_case("tiny-2x1", SEED + 9, 0, 2, 1, 7))
    # levelize on a small config-5-shaped DAG, then FFD with its levels
    V, row_ptr, col, has_deps = P.gen_dag(SEED + 5, 6, 7, 4, 9, 2)
    level, order = P.levelize(V, row_ptr, col, has_deps)
    out["levelize"].append({"name": "dag-6x7+4x9-2cyc", "seed": SEED + 5, "params": [6, 7, 4, 9, 2],
                            "row_ptr": row_ptr, "col": col, "has_deps": has_deps,
                            "level": level, "order": order})
    out["ffd"].append(ffd_case("dag-placed", SEED + 5, 0, V, 20, 7, level=level))
    # feasibility on initial node state
    s = P.scenario_seed(SEED + 6, 0)
    cpu, mem, req, conf = P.gen_containers(s, 130, 7)
    cf, mf, lab, cu, sched = P.gen_nodes(s, 70)
    first, count, bitmap = P.feasibility(cpu, mem, req, conf, cf, mf, lab, cu, sched)
    out["feasibility"].append({"name": "130x70", "seed": SEED + 6, "C": 130, "N": 70, "flags": 7,
                               "first": first, "count": count, "bitmap_hex": [f"{w:016x}" for w in bitmap]})
    with open(os.path.join(HERE, "synthetic_small.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", os.path.join(HERE, "synthetic_small.json"))


if __name__ == "__main__":
    main()
