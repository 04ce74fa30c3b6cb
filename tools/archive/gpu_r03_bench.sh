#!/bin/bash
# round 3: hbm-budget test, default bench (weak C3 + strong C4 legs), 2-rank gloo rehearsal of both legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_hbm_budget.py > gpurun_out/r03_budget.log 2>&1 || { tail -40 gpurun_out/r03_budget.log; exit 1; }
tail -3 gpurun_out/r03_budget.log
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03_bench_default.json 2> gpurun_out/r03_bench_default.err || { tail -30 gpurun_out/r03_bench_default.err; exit 1; }
timeout -k 10 500 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --cpu-seconds 0 > gpurun_out/r03_bench_2rank_gloo.json 2> gpurun_out/r03_bench_2rank_gloo.err || { tail -30 gpurun_out/r03_bench_2rank_gloo.err; exit 1; }
python - <<'PY'
import json
for f in ("gpurun_out/r03_bench_default.json", "gpurun_out/r03_bench_2rank_gloo.json"):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    s = d.get("strong") or {}
    print(f, round(d["value"] / 1e6, 3), "M", d["roofline"]["frac"], d.get("construct_s"), d.get("hbm_bytes"),
          "| strong", s.get("workload"), round(s.get("value", 0) / 1e6, 3), s.get("per_rank_ms_per_step"),
          s.get("construct_s"), "| cpu", (d.get("cpu_baseline") or {}).get("cores"), (d.get("cpu_baseline") or {}).get("host_cpus"))
PY
