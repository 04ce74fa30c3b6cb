#!/bin/bash
# End-of-round evidence for every BASELINE config on the final code (one line per run):
# C2; C3 f32 / compact / with flow planes (f32 and compact); the C5 per-GPU share; C4 whole and
# the whole C5 workload (compact) on one GPU; a 2-rank gloo rehearsal of the multi-rank path.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/cfg
S="import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d['config']; print(c['workload'], c['obs_format'], 'flow' if c['flow'] else '-', c['n_envs_per_gpu'], 'x', d['n_gpus'], '%.3f M env-steps/s' % (d['value']/1e6), 'step %.4f ms' % d['ms_per_step'], r['kernel'], '%.4f ms' % r['kernel_ms'], '%.0f GB/s' % r['achieved'], 'frac %.3f' % r['frac'], 'fused' if c['fused'] else 'two-launch')"
run() {  # name, timeout, args...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t python3 $R/bench.py --cpu-seconds 0 --compact-steps 0 "$@" > $R/gpurun_out/cfg/$n.log 2>&1 || { tail -20 $R/gpurun_out/cfg/$n.log; exit 1; }
  grep '^{' $R/gpurun_out/cfg/$n.log | python3 -c "$S" || exit 1
}
run c2 300 --config C2 --steps 200 --warmup 20
run c3 300 --config C3 --steps 200 --warmup 20
run c3c 300 --config C3 --obs-format u8f16 --steps 200 --warmup 20
run c3f 300 --config C3 --flow --steps 100 --warmup 10
run c3fc 300 --config C3 --flow --obs-format u8f16 --steps 100 --warmup 10
run c5 400 --config C5 --steps 50 --warmup 10
run c4 400 --config C4 --envs 65536 --steps 50 --warmup 10
run c5c 500 --config C5 --envs 131072 --obs-format u8f16 --steps 30 --warmup 5
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 $R/bench.py --gpus 2 --envs 8192 --steps 30 --warmup 5 --dist-backend gloo --cpu-seconds 0 > $R/gpurun_out/cfg/dist2.log 2>&1 || { tail -20 $R/gpurun_out/cfg/dist2.log; exit 1; }
grep '^{' $R/gpurun_out/cfg/dist2.log | python3 -c "$S" || exit 1
