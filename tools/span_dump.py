"""Per-stage spans of one config-3 launch (diagnostics build): for every global stage of
scenario 0, [0] start [1] first input [2] loop end (s_memrealtime, 100 MHz) [3] busy cycles
[4] batches [5] output-wait cycles [6] input-spin iterations [7] placements.
    python tools/span_dump.py out.json   (GPU box)"""
import ctypes as ct
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FLEETPLACE_LIB", os.path.join(ROOT, "fleetflow_amd", "libfleetplace_stats.so"))
import torch  # noqa: E402
import _opts  # noqa: E402  (tools/_opts.py)
from fleetflow_amd import DevBatch, Planner, _lib  # noqa: E402

p = Planner(0)
_opts.apply_env(p)
C, N = 1_000_000, 100_000
db = DevBatch.allocate(1, C, N, "cuda:0")
p.dev_gen_batch(0x5EED0003, db, 7)
p.sync()
pristine = db.node_snapshot()
L = _lib.load()
f = L.fp_debug_stage_span
f.argtypes = [ct.POINTER(ct.c_ulonglong)]
for _ in range(2):
    db.restore_nodes(pristine)
    torch.cuda.synchronize()
    p.dev_place_batch(db)
    p.sync()
buf = (ct.c_ulonglong * (4096 * 8))()
f(buf)
rows = [[buf[i * 8 + k] for k in range(8)] for i in range(1564)]
t0 = min(r[0] for r in rows if r[0])
out = [{"start_us": (r[0] - t0) / 100, "first_in_us": (r[1] - t0) / 100 if r[1] else None, "end_us": (r[2] - t0) / 100,
        "busy_Mcyc": r[3] / 1e6, "batches": r[4], "outwait_Mcyc": r[5] / 1e6, "in_spins": r[6], "placed": r[7]} for r in rows]
json.dump(out, open(sys.argv[1], "w"))
for i in list(range(0, 1564, 100)) + [1563]:
    print(i, {k: (round(v, 1) if isinstance(v, float) else v) for k, v in out[i].items()})
