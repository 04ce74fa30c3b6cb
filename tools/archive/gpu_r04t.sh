#!/bin/bash
# round 4: conv2 forward tile quantization (FFMP_CONV_MBW) and three independent forwards on streams;
# Brain(overlap=True) — Q_main(s') and Q_target(s') on two side streams, a variant not kept: its
# parity test, then the train loop with and without it (profiles/r04t_conv_streams.txt)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04t
mkdir -p $O
for m in 4 2 1; do
  FFMP_CONV_MBW=$m timeout -k 10 120 python $R/tools/conv_tail_probe.py || exit 1
done
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_learner.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "learner tests: $(tail -1 $O/pytest.log)"
for rep in 0 1; do
  for flag in "" "--no-overlap"; do
    timeout -k 10 300 python $R/examples/train_vec.py --amp --steps 100 $flag 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train_vec --amp $flag', round(d['env_steps_per_s']), 'env-steps/s,', d['learner_updates'], 'updates')" || exit 1
  done
done
