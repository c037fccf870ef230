"""Generate tests/golden/ffd_big_digest.json: oracle FFD plans too large to recompute inside
a GPU test (the C oracle needs ~3 min for 2M containers x 200k nodes), stored as SHA-256
digests of the oracle's outputs plus a few sampled entries.

Inputs are the oracle's own seeded generator (oracle/fp_oracle.c fpo_gen_*), so the test
regenerates them bit-identically; the expected outputs are oracle/fp_oracle.c fpo_place
(the A6 restatement).  Test infrastructure only.

Usage: python tests/golden/make_big_digest.py   (from the repo root; minutes)
"""
import hashlib
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
from oracle import oracle as O  # noqa: E402

CASES = [
    # (name, seed, scenario, C, N, flags): the bounded-link workspace case
    ("c2m_n200k", 0x5EED0B16, 0, 2_000_000, 200_000, 7),
]


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def plan_record(assign, reason, after, N, scenario):
    idx = np.linspace(0, len(assign) - 1, 17).astype(np.int64)
    return {
        "assign_sha256": digest(assign.astype(np.uint32)),
        "reason_sha256": digest(reason.astype(np.uint8)),
        "cpu_free_sha256": digest(after[0].astype(np.uint32)),
        "mem_free_sha256": digest(after[1].astype(np.uint32)),
        "conflict_used_sha256": digest(after[3].astype(np.uint32)),
        "n_rejected": int((reason != 0).sum()),
        "cost": int(O.cost(assign, N, scenario)),
        "sample_index": idx.tolist(),
        "sample_assign": assign[idx].astype(np.int64).tolist(),
    }


def main():
    out = {"generator": "tests/golden/make_big_digest.py", "oracle": "oracle/fp_oracle.c fpo_place", "cases": []}
    for name, seed, scen, C, N, flags in CASES:
        cont, nodes = O.gen_scenario(seed, scen, C, N, flags)
        assign, reason, after, _ = O.place(cont, nodes)
        rec = {"name": name, "seed": seed, "scenario": scen, "C": C, "N": N, "flags": flags}
        rec.update(plan_record(assign, reason, after, N, scen))
        out["cases"].append(rec)
        print(name, rec["n_rejected"], flush=True)
    path = os.path.join(os.path.dirname(__file__), "ffd_big_digest.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
