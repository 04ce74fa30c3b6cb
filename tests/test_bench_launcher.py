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


def _rank_worker(rank, world, port, out_dir):
    """One stand-in rank: a fake FFMPVec whose launch choice and ring timing depend on the rank,
    gathered exactly as bench.run_leg does after its timed region."""
    import types
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    fused = rank % 2 == 1
    env = types.SimpleNamespace(
        fused=fused,
        placement={"shape_newest": {"cells_per_block": 4096 * (rank + 1), "flags": 37},
                   "fused": {"flags": 33 + rank}},
        ring_meta=({"pair_gbs_min": 6000.0 + rank,
                    "repair": [{"slot_ms": [2.3 + rank, 2.4 + rank], "slow": []}]} if rank != 2 else {}))
    rec = bench.rank_record(10.0 + rank, 1.5 * rank, 8192, 2.3 + 0.1 * rank, 0.9 - 0.01 * rank, env)
    table = bench.per_rank_table(bench._gather_floats(rec, world, None, "gloo"))
    if rank == 0:
        with open(os.path.join(out_dir, "per_rank.json"), "w") as f:
            json.dump(table, f)
    dist.barrier()
    dist.destroy_process_group()


def test_per_rank_records_gathered_in_rank_order(tmp_path):
    """one all_gather after the timed region brings every rank's kernel time,
    roofline fraction, launch choice and ring pairing to rank 0, in rank order (gloo, world 4)."""
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    mp.spawn(_rank_worker, args=(4, port, str(tmp_path)), nprocs=4, join=True)
    t = json.load(open(tmp_path / "per_rank.json"))
    assert set(t) == set(bench.RANK_FIELDS)
    assert t["elapsed_s"] == [10, 11, 12, 13] and t["n_envs"] == [8192] * 4
    assert t["construct_s"] == [0, 1.5, 3, 4.5]
    assert t["kernel_ms"] == [2.3, 2.4, 2.5, 2.6] and t["frac"] == [0.9, 0.89, 0.88, 0.87]
    assert t["fused"] == [0, 1, 0, 1]
    # two-launch ranks report their raster shape, one-launch ranks the fused kernel's flags
    assert t["shape_cells"] == [4096, None, 12288, None] and t["shape_flags"] == [37, 34, 37, 36]
    # rank 2 has no seamless ring: no slot times, no pairing
    assert t["slot_ms_min"] == [2.3, 3.3, None, 5.3] and t["slot_ms_max"] == [2.4, 3.4, None, 5.4]
    assert t["pair_gbs_min"] == [6000, 6001, None, 6003]
