"""Latency model of k_ffd_pipe from the diagnostics build (per-stage s_memtime
counters, libfleetplace_stats.so) for both bench legs; writes JSON that bench.py's
roofline reports as `latency_model`.

    FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_stats.so python tools/pipe_model.py out.json

Per leg: exact checks and placements per scenario, the candidate-loop cycles per
check, the prescan cycles, the stage lifetime and the pipeline overlap
(sum of the stages' busy cycles / one stage's lifetime).  The model:
  kernel_ms = ceil(S / resident) x (checks x cycles_per_check + prescan) / overlap / cycles_per_ms
i.e. the time of the sequential first-fit chain, not of any memory traffic."""
import ctypes as ct
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("FLEETPLACE_LIB", os.path.join(ROOT, "fleetflow_amd", "libfleetplace_stats.so"))

import torch  # noqa: E402

from fleetflow_amd import DevBatch, Planner, _lib  # noqa: E402

# (leg, scenarios in the diagnostics run, C, N, seed, scenarios resident at once on 256 CUs)
LEGS = [("config4", int(os.environ.get("S_DIAG", 768)), 50_000, 5_000, 0x5EED0004, 768),
        ("config3", 1, 1_000_000, 100_000, 0x5EED0003, 1)]


def measure(p, S, C, N, seed):
    db = DevBatch.allocate(S, C, N, "cuda:0")
    p.dev_gen_batch(seed, db, 7)
    p.sync()  # the generator runs on the planner stream; torch copies on its own
    pristine = db.node_snapshot()
    torch.cuda.synchronize()
    L = _lib.load()
    f = L.fp_debug_pipe_stats
    f.argtypes = [ct.POINTER(ct.c_ulonglong), ct.c_int]
    buf = (ct.c_ulonglong * 256)()
    p.profile(False)
    p.profile(True)
    for _ in range(2):
        db.restore_nodes(pristine)
        torch.cuda.synchronize()
        f(buf, 1)
        p.dev_place_batch(db)
        p.sync()
    ms, n = p.kernel_stats(_lib.FP_K_PLACE)
    print(f"  S={S} placed/scenario {int((db.reason == 0).sum().item()) / S:.0f}", flush=True)
    f(buf, 0)
    v = [[buf[w * 16 + i] for i in range(16)] for w in range(16)]
    v = [r for r in v if any(r)]
    del db, pristine
    torch.cuda.empty_cache()
    return ms / n, v  # last launch's counters (reset before it); time = mean of both


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pipe_model.json")
    p = Planner(0)
    res = {}
    for leg, S, C, N, seed, resident in LEGS:
        kms, v = measure(p, S, C, N, seed)
        checks = sum(r[1] for r in v) / S
        hits = sum(r[2] for r in v) / S
        cand = sum(r[10] for r in v) / S
        pre = sum(r[9] for r in v) / S
        # r[13] (whole loop) of stage slot w is summed over the scenario's segments
        life_sum = max(r[13] for r in v) / S
        stages = len(v)
        res[leg] = {"S_diag": S, "C": C, "N": N, "resident_scenarios": resident,
                    "stage_slots": stages, "kernel_ms_diag_build": kms,
                    "checks_per_scenario": checks, "placements_per_scenario": hits,
                    "cycles_per_check": cand / max(checks, 1), "cand_loop_cycles_per_scenario": cand,
                    "prescan_cycles_per_scenario": pre,
                    "stage_lifetime_cycles_summed_over_segments": life_sum,
                    "miss_reasons_per_scenario": {"cap_ok_label_or_conflict": sum(r[6] for r in v) / S,
                                                  "cap_label_ok_conflict": sum(r[7] for r in v) / S,
                                                  "cpu_ok_mem_fails": sum(r[14] for r in v) / S,
                                                  "mem_ok_cpu_fails": sum(r[15] for r in v) / S,
                                                  "note": "C++ loop diagnostics build only (FP_NO_ASM)"},
                    "per_stage": [{"visits": r[0] / S, "checks": r[1] / S, "hits": r[2] / S,
                                   "cand_Mcycles": r[10] / S / 1e6, "prescan_Mcycles": r[9] / S / 1e6,
                                   "input_Mcycles": r[8] / S / 1e6, "spin_in_per_batch": r[4] / max(r[3], 1),
                                   "fwd_Mcycles": r[11] / S / 1e6, "batches": r[3] / S,
                                   "life_Mcycles": r[13] / S / 1e6} for r in v]}
        print(leg, json.dumps(res[leg]), flush=True)
    with open(out_path, "w") as fo:
        json.dump(res, fo, indent=1)


if __name__ == "__main__":
    main()
