#!/bin/bash
# round 4: learner evidence with the shipped conv kernels: conv parity + learner tests, the conv2 kernels
# at B = 256, the train loop (examples/train_vec.py --amp) three times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04m
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_conv_mfma.py $R/tests/test_gpu_learner.py $R/tests/test_gpu_temporal_maps.py $R/tests/test_gpu_replay.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "learner parity: $(tail -1 $O/pytest.log)"
timeout -k 10 300 python $R/tools/conv_probe.py 256 --mfma-only 2>&1 | grep mfma || exit 1
for rep in 0 1 2; do
  timeout -k 10 300 python $R/examples/train_vec.py --amp --steps 100 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train_vec --amp', round(d['env_steps_per_s']), 'env-steps/s,', d['learner_updates'], 'updates')" || exit 1
done
