#!/bin/bash
# HIP path vs the C oracle at whole-config batch sizes, then the default bench (C-oracle cpu_baseline)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_oracle_c.py tests/test_oracle_c.py -x -v --timeout 300 --timeout-method thread > gpurun_out/oraclec_pytest.log 2>&1 || { tail -40 gpurun_out/oraclec_pytest.log; exit 1; }
grep -E "PASS|FAIL|passed|failed" gpurun_out/oraclec_pytest.log | tail -14
timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || { tail -20 gpurun_out/bench_default.log; exit 1; }
python -c "
import json;d=json.loads([l for l in open('gpurun_out/bench_default.log') if l.startswith('{')][0])
print('value %.4g frac %.3f' % (d['value'], d['roofline']['frac'])); print(json.dumps(d['cpu_baseline']))"
