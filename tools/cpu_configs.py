#!/usr/bin/env python3
"""CPU baseline per BASELINE config (BASELINE.md §3's CPU columns): the C restatement of the oracle
(oracle/ffmp_oracle.c, bit-identical to the NumPy oracle) stepping a bounded sample of each config's
workload on 1 thread and on every usable CPU (bench.py's host_cpus rule), ~SECONDS each, plus the
NumPy oracle on one env of C1 (the reference's CPU case).  Test infrastructure: the oracle is the
checker and the CPU baseline, never the product.  Prints one JSON line.
Usage: python tools/cpu_configs.py [SECONDS]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from bench import host_cpus  # noqa: E402
from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from oracle.ffmp_oracle import OracleVecEnv  # noqa: E402
from oracle.ffmp_oracle_c import COracleVecEnv  # noqa: E402


def rate(env, n, seconds, seed):
    rng = np.random.default_rng(seed)
    env.reset()
    env.step(rng.integers(0, 28, n))
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        env.step(rng.integers(0, 28, n))
        steps += 1
    return n * steps / (time.perf_counter() - t0), steps


def main():
    seconds = float(sys.argv[1]) if len(sys.argv) > 1 else 4.0
    cpus = host_cpus()
    threads = cpus["usable"]
    out = {"host_cpus": cpus, "seconds_per_leg": seconds, "configs": {}}
    for name in ("C1", "C2", "C3", "C5"):
        cfg = preset(name)
        r1, s1 = rate(COracleVecEnv(cfg, 2, threads=1), 2, seconds, 1)
        n = 4 * threads
        rn, sn = rate(COracleVecEnv(cfg, n, threads=threads), n, seconds, 2)
        out["configs"][name] = {"one_core": r1, "all_cores": rn, "cores": threads,
                                "sample": f"1 thread: 2 envs x {s1} steps; {threads} threads: {n} envs x {sn} steps"}
        print(name, round(r1), round(rn), file=sys.stderr, flush=True)
    r, s = rate(OracleVecEnv(preset("C1"), 1), 1, seconds, 3)
    out["c1_numpy_single_env"] = {"value": r, "steps": s}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
