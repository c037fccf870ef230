"""bench.py --gpus N without an external launcher starts N rank processes itself
(RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, one rendezvous port, parent touches no GPU).
Checked on CPU through the --dry-launch hook, which makes each rank print its env."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_spawns_n_ranks():
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--dry-launch"],
                         env=env, capture_output=True, text=True, timeout=120, check=True).stdout
    recs = [json.loads(line) for line in out.splitlines() if line.startswith("{")]
    assert sorted(int(r["RANK"]) for r in recs) == [0, 1, 2]
    assert all(r["WORLD_SIZE"] == "3" and r["MASTER_ADDR"] == "127.0.0.1" for r in recs)
    assert len({r["MASTER_PORT"] for r in recs}) == 1
    assert all(r["LOCAL_RANK"] == r["RANK"] for r in recs)


def test_bench_under_external_launcher_does_not_respawn():
    env = dict(os.environ, WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_ADDR="127.0.0.1", MASTER_PORT="1")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-launch"],
                         env=env, capture_output=True, text=True, timeout=120, check=True).stdout
    recs = [json.loads(line) for line in out.splitlines() if line.startswith("{")]
    assert len(recs) == 1 and recs[0]["RANK"] == "1"
