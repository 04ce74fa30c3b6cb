#!/bin/bash
# Full GPU evidence pass: build, GPU tests, multi-rank rehearsal, profiles, default bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
echo "== pytest gpu"; timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
echo "== 2-rank rehearsal (gloo, both ranks on cuda:0)"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --envs 8192 --dist-backend gloo > gpurun_out/rehearsal.log 2>&1 || { tail -20 gpurun_out/rehearsal.log; exit 1; }
grep '^{' gpurun_out/rehearsal.log | cut -c1-300
echo "== profile C3"; bash tools/gpu_profile.sh ${1:-r01} C3 > gpurun_out/profile.log 2>&1 || { tail -30 gpurun_out/profile.log; exit 1; }
tail -25 gpurun_out/profile.log
echo "== profile C3 compact"; bash tools/gpu_profile.sh ${1:-r01} C3 u8f16 > gpurun_out/profile_u8f16.log 2>&1 || { tail -30 gpurun_out/profile_u8f16.log; exit 1; }
tail -8 gpurun_out/profile_u8f16.log
echo "== bench default"; timeout -k 10 600 python bench.py > gpurun_out/bench_default.log 2>&1 || exit 1
grep '^{' gpurun_out/bench_default.log
echo "== bench C2 / C5-per-rank"
timeout -k 10 300 python bench.py --config C2 --cpu-seconds 10 > gpurun_out/bench_C2.log 2>&1 && grep '^{' gpurun_out/bench_C2.log | cut -c1-400
timeout -k 10 300 python bench.py --config C5 --steps 50 --cpu-seconds 10 > gpurun_out/bench_C5.log 2>&1 && grep '^{' gpurun_out/bench_C5.log | cut -c1-400
echo "== bench compact C3 / C5 whole"
timeout -k 10 300 python bench.py --config C3 --obs-format u8f16 --cpu-seconds 0 > gpurun_out/bench_C3_u8f16.log 2>&1 && grep '^{' gpurun_out/bench_C3_u8f16.log | cut -c1-400
timeout -k 10 300 python bench.py --config C5 --obs-format u8f16 --steps 50 --cpu-seconds 0 > gpurun_out/bench_C5_u8f16.log 2>&1 && grep '^{' gpurun_out/bench_C5_u8f16.log | cut -c1-400
exit $rc
