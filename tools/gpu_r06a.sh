#!/bin/bash
# round 6 (a): closed-loop step graphs + policy kernel + fused-Adam pack fix; conv MFMA-shape A/B; C3/C2 with
# the closed-loop leg; the 8-GPU strong leg's per-rank shard (C4, 8,192 envs) on one GPU as rank 0 and rank 7.
# A failing test (rc 1) does not stop the run; a fault, abort or time limit does.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06a
mkdir -p $O
cd $R
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests/test_gpu_closed_loop.py tests/test_gpu_graph.py tests/test_gpu_conv_mfma.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -20; ok $rc || exit 1
timeout -k 10 300 python -u tools/conv_ab.py 256 7 > $O/conv_ab.txt 2>&1 || { tail -20 $O/conv_ab.txt; exit 1; }
cat $O/conv_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_learner.log 2>&1; rc=$?
tail -2 $O/pytest_learner.log; grep -E "^FAILED" $O/pytest_learner.log | head; ok $rc || exit 1
B="python $R/bench.py"
S="import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d.get('closed_loop') or {}; print(sys.argv[2], round(d['value']/1e6,3), round(d['ms_per_step'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), d['config']['graph'] and d['config']['graph']['skewed'], {k: (round(c[k]['value']/1e6,3), round(c[k]['hbm_roofline_pct_whole_step'],2)) for k in ('step_graph','step_plain','policy_graph') if k in c}, round(d['construct_s'],1))"
timeout -k 10 400 $B --steps 20 --warmup 5 --cpu-seconds 3 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "$S" $O/bench_default.json default
timeout -k 10 400 $B --steps 200 --warmup 20 --cpu-seconds 0 --compact-steps 0 --strong-config none > $O/bench_c3_200.json 2> $O/bench_c3_200.err || { tail -20 $O/bench_c3_200.err; exit 1; }
python -c "$S" $O/bench_c3_200.json C3_200
timeout -k 10 400 $B --config C2 --steps 200 --warmup 20 --cpu-seconds 0 --compact-steps 0 --strong-config none > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python -c "$S" $O/bench_c2.json C2
for off in 0 57344; do
  timeout -k 10 400 $B --config C4 --envs 8192 --env-offset $off --steps 20 --warmup 5 --cpu-seconds 0 --compact-steps 0 --strong-config none > $O/bench_c4_8192_$off.json 2> $O/bench_c4_8192_$off.err || { tail -20 $O/bench_c4_8192_$off.err; exit 1; }
  python -c "$S" $O/bench_c4_8192_$off.json C4s_off$off
  timeout -k 10 400 $B --config C4 --envs 8192 --env-offset $off --steps 200 --warmup 20 --cpu-seconds 0 --compact-steps 0 --strong-config none > $O/bench_c4_8192_${off}_200.json 2> $O/bench_c4_8192_${off}_200.err || { tail -20 $O/bench_c4_8192_${off}_200.err; exit 1; }
  python -c "$S" $O/bench_c4_8192_${off}_200.json C4s200_off$off
done
