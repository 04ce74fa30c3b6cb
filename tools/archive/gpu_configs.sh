#!/bin/bash
# Evidence for the other BASELINE configs on the final code: C2, the C5 per-GPU share (f32),
# the whole C5 workload in the compact layout on one GPU, and a 2-rank gloo rehearsal.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/cfg
S="import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['config']['workload'], d['config']['obs_format'], d['config']['n_envs_per_gpu'], d['n_gpus'], round(d['value']/1e6,3), 'M', round(d['ms_per_step'],4), r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3))"
timeout -k 10 300 python3 $R/bench.py --config C2 --steps 200 --warmup 20 --cpu-seconds 0 --compact-steps 0 > $R/gpurun_out/cfg/c2.log 2>&1 || exit 1
grep '^{' $R/gpurun_out/cfg/c2.log | python3 -c "$S" || exit 1
timeout -k 10 400 python3 $R/bench.py --config C5 --steps 50 --warmup 10 --cpu-seconds 0 --compact-steps 0 > $R/gpurun_out/cfg/c5.log 2>&1 || exit 1
grep '^{' $R/gpurun_out/cfg/c5.log | python3 -c "$S" || exit 1
timeout -k 10 500 python3 $R/bench.py --config C5 --envs 131072 --obs-format u8f16 --steps 30 --warmup 5 --cpu-seconds 0 > $R/gpurun_out/cfg/c5c.log 2>&1 || exit 1
grep '^{' $R/gpurun_out/cfg/c5c.log | python3 -c "$S" || exit 1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 $R/bench.py --gpus 2 --envs 8192 --steps 30 --warmup 5 --dist-backend gloo --cpu-seconds 0 > $R/gpurun_out/cfg/dist2.log 2>&1 || { tail -20 $R/gpurun_out/cfg/dist2.log; exit 1; }
grep '^{' $R/gpurun_out/cfg/dist2.log | python3 -c "$S" || exit 1
