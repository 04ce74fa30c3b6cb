#!/bin/bash
# round 6 (l): the train loop on the final conv defaults
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06l
mkdir -p $O
cd $R
for rep in 0 1; do
  timeout -k 10 300 python examples/train_vec.py --amp --steps 100 > $O/train256_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/train256_$rep.json').read().splitlines()[-1]); print('B=256', round(d['env_steps_per_s']), 'env-steps/s', round(d['updates_per_s'],1), 'upd/s', round(d['conv_tflops_per_s'],1), 'conv TF/s')"
done
timeout -k 10 300 python examples/train_vec.py --amp --reference-hparams --steps 60 > $O/train1024.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('$O/train1024.json').read().splitlines()[-1]); print('B=1024 cap 20000', round(d['env_steps_per_s']), 'env-steps/s', round(d['updates_per_s'],1), 'upd/s', round(d['conv_tflops_per_s'],1), 'conv TF/s', d['learner_updates'])"
