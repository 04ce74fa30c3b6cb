#!/bin/bash
# round 6 (b): conv launch variants (MFMA shape, kernel rows per ring step, B through LDS): parity + A/B;
# legacy edges, closed loop, learner, HBM tests; re-warmed bench legs (C4 shard at the driver's 20 steps).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06b
mkdir -p $O
cd $R
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_mfma.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_conv.log 2>&1; rc=$?
tail -3 $O/pytest_conv.log; grep -E "^FAILED|Error" $O/pytest_conv.log | head -20; ok $rc || exit 1
timeout -k 10 300 python -u tools/conv_ab.py 256 7 0:0:0 32:1:0 32:1:1 32:2:0 32:4:0 16:4:0 > $O/conv_ab.txt 2>&1 || { tail -20 $O/conv_ab.txt; exit 1; }
cat $O/conv_ab.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_legacy_api.py tests/test_gpu_closed_loop.py tests/test_gpu_learner.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "^FAILED|Error" $O/pytest.log | head -20; ok $rc || exit 1
timeout -k 10 900 python -u -m pytest tests/test_gpu_hbm_budget.py -m gpu -v -s --timeout 600 --timeout-method thread > $O/pytest_hbm.log 2>&1; rc=$?
tail -15 $O/pytest_hbm.log; ok $rc || exit 1
B="python $R/bench.py"
S="import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d.get('closed_loop') or {}; print(sys.argv[2], round(d['value']/1e6,3), round(d['ms_per_step'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), d['config']['graph'] and d['config']['graph']['skewed'], {k: (round(c[k]['value']/1e6,3), round(c[k]['hbm_roofline_pct_whole_step'],2)) for k in ('step_graph','step_plain','policy_graph') if k in c}, round(d['construct_s'],1))"
for off in 0 57344; do
  timeout -k 10 400 $B --config C4 --envs 8192 --env-offset $off --steps 20 --warmup 5 --cpu-seconds 0 --compact-steps 0 --strong-config none > $O/bench_c4_8192_$off.json 2> $O/bench_c4_8192_$off.err || { tail -20 $O/bench_c4_8192_$off.err; exit 1; }
  python -c "$S" $O/bench_c4_8192_$off.json C4s_off$off
done
timeout -k 10 400 $B --steps 20 --warmup 5 --cpu-seconds 3 > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python -c "$S" $O/bench_default.json default
timeout -k 10 400 $B --config C2 --steps 200 --warmup 20 --cpu-seconds 0 --compact-steps 0 --strong-config none > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
python -c "$S" $O/bench_c2.json C2
