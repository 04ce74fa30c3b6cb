"""One C3 FFMPVec in a fresh process under a placement policy variant; prints the tuned cycle
bandwidth, the chosen shapes / step mode and the per-slot raster ms (profiles/r01_ring.txt §7).
usage: python tools/ring_variants.py PAIR(0/1) XCD(0/1) REPAIR_ROUNDS"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from flow_field_based_motion_planner_amd.config import preset  # noqa: E402
from flow_field_based_motion_planner_amd.vec_env import FFMPVec  # noqa: E402

pair, xcd, rounds = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
FFMPVec.PAIR_SLOTS = bool(pair)
FFMPVec.XCD_SHAPES = bool(xcd)
FFMPVec.REPAIR_ROUNDS = rounds
env = FFMPVec(32768, preset("C3"), device="cuda:0")
pl = env.placement
rep = pl["ring"].get("repair", [])
ms = env._slot_ms()  # final per-slot ms (after any repair), current step mode
fu = pl.get("fused") or {}
print(f"pair={pair} xcd={xcd} rounds={rounds}: cycle {pl['gbs']} GB/s, newest {pl['shape_newest']}, fused {fu.get('chosen')} "
      f"flags {fu.get('flags')} | final slot ms {[round(v, 3) for _, v in sorted(ms.items())]} | mean {sum(ms.values()) / len(ms):.3f} "
      f"| rebuilds {pl['ring'].get('rebuilds')} probes {pl['ring'].get('pair_probes')}", flush=True)
