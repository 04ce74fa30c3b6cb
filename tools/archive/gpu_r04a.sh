# round 4, first GPU pass: the full GPU suite (new: timed path over every shape, RCCL world 1,
# C4 rank shards, pool trim, per-layer MFMA fallback), the driver's bench line, the env kernel split
set -o pipefail
mkdir -p gpurun_out/r04a
export FFMP_TIMED_PATH_OUT=gpurun_out/r04a
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread tests -m gpu > gpurun_out/r04a/pytest.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r04a/bench.json 2> gpurun_out/r04a/bench.err && \
timeout -k 10 300 python tools/env_kernel_breakdown.py --preset C3 --envs 32768 > gpurun_out/r04a/env_breakdown.txt 2>&1 && \
timeout -k 10 200 bash tools/gpu_env_pmc.sh > gpurun_out/r04a/env_pmc.txt 2>&1
