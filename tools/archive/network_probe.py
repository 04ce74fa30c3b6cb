#!/usr/bin/env python3
"""Time the reference Network (network.py) forward / forward+backward at batch B on cuda:0 under
MIOpen's default algorithm choice, exhaustive search (cudnn.benchmark), channels_last, bf16."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from flow_field_based_motion_planner_amd.network import Network  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
dev = torch.device("cuda:0")


def run(tag, bench=False, cl=False, bf16=False, reps=3):
    torch.backends.cudnn.benchmark = bench
    net = Network().to(dev)
    x = (torch.rand(B, 2, 100, 100, device=dev) > 0.9).float() * 255
    if cl:
        net = net.to(memory_format=torch.channels_last)
        x = x.to(memory_format=torch.channels_last)
    g = torch.rand(B, 2, device=dev)
    v = torch.rand(B, 2, device=dev)
    t = torch.rand(B, 1, device=dev)
    res = {}
    for mode in ("fwd", "fwd+bwd"):
        for r in range(reps + 1):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=bf16):
                if mode == "fwd":
                    with torch.no_grad():
                        q = net(x, g, v, t)
                else:
                    q = net(x, g, v, t)
                    q.float().sum().backward()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            if r == 0:
                first = dt
        res[mode] = (first, dt)
    print(f"{tag:28s} B={B}: fwd first {res['fwd'][0]*1e3:8.1f} ms, steady {res['fwd'][1]*1e3:8.1f} ms | "
          f"fwd+bwd first {res['fwd+bwd'][0]*1e3:8.1f} ms, steady {res['fwd+bwd'][1]*1e3:8.1f} ms", flush=True)


run("default")
run("benchmark", bench=True)
run("channels_last+benchmark", bench=True, cl=True)
run("bf16 autocast+benchmark", bench=True, bf16=True)
