"""Diagnostic (not a test): run every GPU parity case and print mismatch details.
Usage on the GPU box:  python tests/parity_report.py"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


from tests.parity_util import exact_report, gpu_snapshot, oracle_snapshot  # noqa: E402
from tests.test_gpu_parity import CASES, _run  # noqa: E402

for name, (cfg, n, steps) in CASES.items():
    t = time.time()
    env, ref, problems, counts = _run(cfg, n, steps)
    rep = exact_report(gpu_snapshot(env), oracle_snapshot(ref))
    print(f"[{name}] {time.time() - t:.1f}s problems={len(problems)} counts={counts}")
    print("   non-bit-identical at end:", rep)
    for p in problems[:8]:
        print("   ", p)
    sys.stdout.flush()
