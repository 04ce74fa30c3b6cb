#!/bin/bash
# round 6 (e): the row-ring forward's tile picked by a grid-fill model (384-position tiles for conv2 at
# B = 256: 1,024 workgroups = 2 full rounds instead of 768 = 1.5): conv parity, A/B of the tile sizes,
# the train loop
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06e
mkdir -p $O
cd $R
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_mfma.py tests/test_gpu_learner.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head; ok $rc || exit 1
timeout -k 10 300 python -u tools/conv_ab.py 256 9 0:0:0:0:0:0:0:0:0 0:0:0:0:0:0:0:0:3 > $O/conv_ab.txt 2>&1 || { tail -20 $O/conv_ab.txt; exit 1; }
cat $O/conv_ab.txt
timeout -k 10 300 python -u tools/conv_ab.py 1024 5 0:0:0:0:0:0:0:0:0 0:0:0:0:0:0:0:0:3 > $O/conv_ab_1024.txt 2>&1 || { tail -20 $O/conv_ab_1024.txt; exit 1; }
cat $O/conv_ab_1024.txt
for rep in 0 1; do
  timeout -k 10 300 python examples/train_vec.py --amp --steps 100 > $O/train256_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/train256_$rep.json').read().splitlines()[-1]); print('B=256', round(d['env_steps_per_s']), 'env-steps/s', round(d['updates_per_s'],1), 'upd/s', round(d['conv_tflops_per_s'],1), 'conv TF/s')"
done
timeout -k 10 300 python examples/train_vec.py --amp --reference-hparams --steps 60 > $O/train1024.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('$O/train1024.json').read().splitlines()[-1]); print('B=1024 cap 20000', round(d['env_steps_per_s']), 'env-steps/s', round(d['updates_per_s'],1), 'upd/s', round(d['conv_tflops_per_s'],1), 'conv TF/s', d['learner_updates'])"
timeout -k 10 400 bash tools/gpu_conv_pmc.sh r06e_conv > $O/conv_pmc.txt 2>&1 || { tail -20 $O/conv_pmc.txt; exit 1; }
grep -v "^W20" $O/conv_pmc.txt | head -12
