#!/bin/bash
# round 4: the 12-channel BEV option (ffmp_bev_image, FFMPVec.bev_maps, ReplayMemory(bev=True),
# Brain(input_channels=12), conv1 folded at 12 -> 16 channels) plus the suites it touches
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04o
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_bev_series.py $R/tests/test_gpu_conv_mfma.py $R/tests/test_gpu_replay.py \
  $R/tests/test_gpu_temporal_maps.py $R/tests/test_gpu_learner.py -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest.log | tail -60
exit $rc
