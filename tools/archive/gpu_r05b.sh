#!/bin/bash
# round 5: the data gradient with the batch as M (ffmp_conv2d_dgrad_bf16): float64 parity, then timing at B = 256 / 1024;
# the single-env surface (packed staging, cached footprint): golden tests + per-call latency; the env kernel's LDS fallback
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05b
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread $R/tests/test_gpu_conv_mfma.py -k "dgrad or autograd" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python $R/tools/conv_probe.py 256 1024 --mfma-only > $O/conv_probe.log 2>&1 || { tail -20 $O/conv_probe.log; exit 1; }
grep -v amdgpu.ids $O/conv_probe.log
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread $R/tests/test_gpu_legacy_api.py $R/tests/test_gpu_parity.py -k "legacy or footprint or rewarder or collision or goal or reward or gym or lds or lanes" > $O/pytest_legacy.log 2>&1 || { tail -40 $O/pytest_legacy.log; exit 1; }
tail -3 $O/pytest_legacy.log
timeout -k 10 300 python $R/tools/single_env_probe.py > $O/single_env.log 2>&1 || { tail -20 $O/single_env.log; exit 1; }
grep -v amdgpu.ids $O/single_env.log
