"""Quick config-3 timing under geometry env settings (tuning; the bench's config3 leg is the record).

    python tools/c3.py "name:ENV=V ENV2=V" ...      (empty env = defaults)
Each spec runs in a child process (the library reads its env at launch); prints FFD kernel ms and
the plan digest so geometries can be compared for identical output.
"""
import hashlib
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, hashlib
sys.path.insert(0, %r)
import torch
import _opts  # noqa: E402  (tools/_opts.py)
from fleetflow_amd import DevBatch, Planner
from fleetflow_amd._lib import FP_K_PLACE
C, N = int(%r), int(%r)
p = Planner(0)
_opts.apply_env(p)
db = DevBatch.allocate(1, C, N, "cuda:0")
p.dev_gen_batch(0x5EED0003, db, 7)
p.sync()
pristine = db.node_snapshot()
torch.cuda.synchronize()
for i in range(3):
    db.restore_nodes(pristine)
    torch.cuda.synchronize()
    if i == 1:
        p.profile(True)
    p.dev_place_batch(db)
    p.sync()
ms, n = p.kernel_stats(FP_K_PLACE)
h = hashlib.sha1(db.assign.cpu().numpy().tobytes()).hexdigest()[:12]
print(f"ffd_ms {ms / n:.2f} digest {h}")
"""


def main():
    C, N = os.environ.get("C", "1000000"), os.environ.get("N", "100000")
    for spec in sys.argv[1:] or [":"]:
        name, envs = spec.split(":", 1)
        env = dict(os.environ)
        for kv in envs.split():
            k, v = kv.split("=", 1)
            env[k] = v
        r = subprocess.run([sys.executable, "-c", CHILD % (ROOT, C, N)], env=env, capture_output=True, text=True,
                           timeout=240)
        out = (r.stdout.strip().splitlines() or ["(no output)"])[-1]
        print(f"{name:12s} {out}" + ("" if r.returncode == 0 else f"  rc={r.returncode} {r.stderr[-300:]}"), flush=True)


if __name__ == "__main__":
    main()
