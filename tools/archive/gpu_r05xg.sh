#!/bin/bash
# round 5 (late): the learner with the on-the-fly fold staged by dword-aligned 16-byte loads (+ fused Adam, fragment order): learner / replay / BEV parity, the train loop at
# B = 256 (twice) and at the reference's own hyper-parameters (B = 1024, capacity 20,000), and the loop's
# kernel split (rocprofv3 kernel trace + stats)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05xg
mkdir -p $O
timeout -k 10 600 python -u -m pytest $R/tests/test_gpu_conv_mfma.py $R/tests/test_gpu_learner.py $R/tests/test_gpu_replay.py $R/tests/test_gpu_bev_series.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "learner parity: $(tail -1 $O/pytest.log)"
for rep in 0 1; do
  timeout -k 10 300 python $R/examples/train_vec.py --amp --steps 100 > $O/train256_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('$O/train256_$rep.json').read().splitlines()[-1]); print('B=256', round(d['env_steps_per_s']), 'env-steps/s', round(d['updates_per_s'],1), 'upd/s', round(d['conv_tflops_per_s'],1), 'conv TF/s')"
done
timeout -k 10 300 python $R/examples/train_vec.py --amp --reference-hparams --steps 60 > $O/train1024.json 2>/dev/null || exit 1
python -c "import json; d=json.loads(open('$O/train1024.json').read().splitlines()[-1]); print('B=1024 cap 20000', round(d['env_steps_per_s']), 'env-steps/s', round(d['updates_per_s'],1), 'upd/s', round(d['conv_tflops_per_s'],1), 'conv TF/s', d['learner_updates'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- \
  python3 $R/examples/train_vec.py --amp --steps 60 > $O/train_prof.log 2>&1 || { tail -20 $O/train_prof.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/r05xg/trace/**/run_kernel_stats.csv", recursive=True))[-1]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
U = 63
print(f"total kernel time {tot/1e6:.1f} ms, {tot/1e6/U:.2f} ms per loop step ({U} incl. warm-up)")
print(" share  ms/step  calls/step  mean_us  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:30]:
    t = float(r["TotalDurationNs"])
    print(f"{100*t/tot:5.1f} {t/1e6/U:8.3f} {int(r['Calls'])/U:10.1f} {float(r['AverageNs'])/1e3:8.1f}  {r['Name'][:110]}")
PY
