#!/bin/bash
# round 4: bench.py --gpus N starting its own ranks (no torchrun), rehearsed on the one GPU of the box with
# the gloo backend (RCCL refuses two ranks on one device): 2 and 4 ranks, 8,192 envs of C3 per rank; then
# the ring tests (a failed slot rebuild keeps the current ring)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04n
mkdir -p $O
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_ring.py -x -v --timeout 120 --timeout-method thread > $O/pytest_ring.log 2>&1 || { tail -30 $O/pytest_ring.log; exit 1; }
tail -3 $O/pytest_ring.log
for n in 2 4; do
  timeout -k 10 400 python $R/bench.py --gpus $n --dist-backend gloo --envs 8192 --steps 10 --warmup 3 > $O/bench_gpus$n.json 2> $O/bench_gpus$n.err || { grep -v '^\[rank[0-9]\]:   ' $O/bench_gpus$n.err | tail -20; exit 1; }
  python -c "
import json; d=json.loads(open('$O/bench_gpus$n.json').read().strip().splitlines()[-1]); c=d['config']; s=d['strong']
print('gpus', d['n_gpus'], c['launcher'], c['comm'], 'weak', round(d['value']/1e6,3), d['per_rank_ms_per_step'], 'strong', s['n_envs_total'], round(s['value']/1e6,3))"
done
