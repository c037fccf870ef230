"""Debug: many-scenario dev_place_batch vs the oracle on a few scenarios.

    python tools/debug_batch.py S C N [S C N ...]     (env FLEETPLACE_* apply)
Prints per checked scenario: GPU vs oracle cost fields and the first FFD-order
container whose assignment differs."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import _opts  # noqa: E402  (tools/_opts.py)
from fleetflow_amd import DevBatch, Planner  # noqa: E402
from oracle import oracle as O  # noqa: E402

SEED = 0x5EED0004


def run(p, S, C, N, base=1024):
    db = DevBatch.allocate(S, C, N, "cuda:0", scen_base=base)
    p.dev_gen_batch(SEED, db, 7)
    p.dev_place_batch(db)
    p.sync()
    costs = db.cost.cpu().numpy().view(np.uint64)
    bad = 0
    for s in sorted({0, 1, S // 2, S - 1}):
        cont, nodes = O.gen_scenario(SEED, base + s, C, N, 7)
        ea, er, _, _ = O.place(cont, nodes)
        ga = db.assign[s * C:(s + 1) * C].cpu().numpy().view(np.uint32)
        gr = db.reason[s * C:(s + 1) * C].cpu().numpy()
        ec = O.cost(ea, N, base + s)
        gc = int(costs[s])
        line = f"S={S} C={C} N={N} s={s}: gpu rej/used {gc >> 40}/{(gc >> 16) & 0xFFFFFF} oracle {ec >> 40}/{(ec >> 16) & 0xFFFFFF}"
        if np.array_equal(ga, ea) and np.array_equal(gr, er):
            print(line, "plan OK", flush=True)
            continue
        bad += 1
        order = O.ffd_order(cont[0], cont[1])
        diff = np.nonzero(ga[order] != ea[order])[0]
        k = int(diff[0])
        j = int(order[k])
        print(line, f"plan DIFF: {diff.size} containers differ; first at FFD pos {k} (idx {j}) "
              f"cpu={cont[0][j]} mem={cont[1][j]} req={cont[2][j]:#x} conf={cont[3][j]:#x} "
              f"gpu={ga[j]:#x}/{gr[j]} oracle={ea[j]:#x}/{er[j]}; gpu NOFIT {int((gr == 1).sum())} "
              f"oracle NOFIT {int((er == 1).sum())}", flush=True)
        print("   next diffs (pos, gpu, oracle):", [(int(d), int(ga[order[d]]), int(ea[order[d]])) for d in diff[1:8]])
    del db
    torch.cuda.empty_cache()
    return bad


def main():
    a = [int(x) for x in sys.argv[1:]]
    p = Planner(0)
    _opts.apply_env(p)
    print("lib", os.environ.get("FLEETPLACE_LIB", "default"), "W", os.environ.get("FLEETPLACE_PIPE_W"),
          "SEG", os.environ.get("FLEETPLACE_PIPE_SEG"), flush=True)
    for i in range(0, len(a), 3):
        run(p, a[i], a[i + 1], a[i + 2])


if __name__ == "__main__":
    main()
