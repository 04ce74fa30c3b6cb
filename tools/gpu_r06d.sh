#!/bin/bash
# round 6 (d): the learner after the conv changes (A reads before MFMAs / next tap's during them, scalar wgrad offsets):
# conv A/B + parity, the train loop (B = 256 twice, reference hyper-parameters), its kernel split; the C5 share;
# the C-oracle CPU baseline per config on the box's host CPUs
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06d
mkdir -p $O
cd $R
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_conv_mfma.py tests/test_gpu_learner.py -m gpu -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log; grep -E "^FAILED" $O/pytest.log | head; ok $rc || exit 1
timeout -k 10 300 python -u tools/conv_ab.py 256 9 0:0:0:0:0 0:0:0:0:1 > $O/conv_ab.txt 2>&1 || { tail -20 $O/conv_ab.txt; exit 1; }
cat $O/conv_ab.txt
for rep in 0 1; do
  timeout -k 10 300 python examples/train_vec.py --amp --steps 100 > $O/train256_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/train256_$rep.json').read().splitlines()[-1]); print('B=256', round(d['env_steps_per_s']), 'env-steps/s', round(d['updates_per_s'],1), 'upd/s', round(d['conv_tflops_per_s'],1), 'conv TF/s')"
done
timeout -k 10 300 python examples/train_vec.py --amp --reference-hparams --steps 60 > $O/train1024.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('$O/train1024.json').read().splitlines()[-1]); print('B=1024 cap 20000', round(d['env_steps_per_s']), 'env-steps/s', round(d['updates_per_s'],1), 'upd/s', round(d['conv_tflops_per_s'],1), 'conv TF/s', d['learner_updates'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 $R/examples/train_vec.py --amp --steps 60 > $O/train_prof.log 2>&1 || { tail -20 $O/train_prof.log; exit 1; }
cd $R && python3 - > $O/kernel_split.txt <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/r06d/trace/**/run_kernel_stats.csv", recursive=True))[-1]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
U = 63
print(f"total kernel time {tot/1e6:.1f} ms, {tot/1e6/U:.2f} ms per loop step ({U} incl. warm-up)")
print(" share  ms/step  calls/step  mean_us  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    t = float(r["TotalDurationNs"])
    print(f"{100*t/tot:5.1f} {t/1e6/U:8.3f} {int(r['Calls'])/U:10.1f} {float(r['AverageNs'])/1e3:8.1f}  {r['Name'][:110]}")
PY
head -16 $O/kernel_split.txt
timeout -k 10 500 python bench.py --config C5 --steps 40 --warmup 10 --cpu-seconds 0 --compact-steps 0 --strong-config none --closed-loop 0 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_c5.json').read().strip().splitlines()[-1]); print('C5', round(d['value']/1e6,3), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), d['config']['n_envs_per_gpu'])"
timeout -k 10 200 python tools/cpu_configs.py 4 > $O/cpu_configs.json 2> $O/cpu_configs.err || { tail -5 $O/cpu_configs.err; exit 1; }
cat $O/cpu_configs.err
