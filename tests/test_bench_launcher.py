"""bench.py --gpus N without torchrun starts the N rank processes itself:
each child gets RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, the launcher waits for
all of them, and one failing rank fails the run (the others are stopped instead of waiting in a
collective).  CPU only: the children here are stand-in commands, the launcher never touches torch."""
import json
import os
import sys

import bench

CHILD = """
import json, os, sys
keys = ("RANK", "LOCAL_RANK", "WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "FFMP_BENCH_LAUNCHER")
out = sys.argv[1]
with open(os.path.join(out, "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys}, f)
"""


def test_launcher_sets_rank_environment(tmp_path):
    rc = bench.launch_ranks(3, [sys.executable, "-c", CHILD, str(tmp_path)])
    assert rc == 0
    got = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    assert [g["RANK"] for g in got] == ["0", "1", "2"] == [g["LOCAL_RANK"] for g in got]
    assert {g["WORLD_SIZE"] for g in got} == {"3"} and {g["MASTER_ADDR"] for g in got} == {"127.0.0.1"}
    assert len({g["MASTER_PORT"] for g in got}) == 1 and {g["FFMP_BENCH_LAUNCHER"] for g in got} == {"1"}


def test_launcher_fails_when_a_rank_fails(tmp_path):
    # rank 1 exits 3 at once; rank 0 would otherwise wait for a minute (a rank stuck in a collective)
    child = ("import os, sys, time\n"
             "if os.environ['RANK'] == '1': sys.exit(3)\n"
             "time.sleep(60)\n")
    import time
    t0 = time.time()
    rc = bench.launch_ranks(2, [sys.executable, "-c", child])
    assert rc == 3 and time.time() - t0 < 30


def test_world_size_mismatch_is_an_error(tmp_path):
    import subprocess
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, bench.__file__, "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus=2" in r.stderr
