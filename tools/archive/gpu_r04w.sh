#!/bin/bash
# round 4: conv LDS layout — lane groups on consecutive positions + XOR chunk swizzle (a probe build,
# FFMP_CONV_SWZ=1, not kept: profiles/r04w_conv_swizzle.txt) against the padded layout (=0): conv + learner parity with the new layout,
# the conv2 kernels at B = 256 for both, SQ counters (MFMA busy, LDS bank conflicts) of the new one,
# and the train loop
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04w
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_conv_mfma.py $R/tests/test_gpu_learner.py $R/tests/test_gpu_bev_series.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "conv + learner parity (swizzled layout): $(tail -1 $O/pytest.log)"
for rep in 0 1; do
  for v in sw0 sw1; do
    echo "== $v"
    FFMP_LIB=$R/tools/_build/libffmp_$v.so timeout -k 10 300 python $R/tools/conv_probe.py 256 --mfma-only 2>&1 | grep mfma || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE \
  --kernel-include-regex 'conv_' --kernel-trace --output-format csv -d $O/run -o run -- \
  python3 $R/tools/conv_probe.py 256 --mfma-only > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
cd $R && python3 - <<'PY'
import csv, glob, collections
f = sorted(glob.glob("gpurun_out/r04w/run/**/run_counter_collection.csv", recursive=True))[-1]
by = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    by[(int(r["Dispatch_Id"]), r["Kernel_Name"])][r["Counter_Name"]] += float(r["Counter_Value"])
kinds = collections.defaultdict(list)
for (d, name), c in sorted(by.items()):
    kinds[name].append(c)
print("kernel | MFMA busy of the cycles run | parked / issue-stall / issuing | LDS bank-conflict / LDS-active")
for name, lst in kinds.items():
    a = collections.Counter()
    for c in lst[1:] or lst:
        a.update(c)
    n = max(len(lst) - 1, 1)
    a = {k: v / n for k, v in a.items()}
    cyc = a.get("GRBM_GUI_ACTIVE", 0) / 8
    wc = a.get("SQ_WAVE_CYCLES", 1)
    print(f"{name[:70]} | {a.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (cyc * 1024):.3f} | {a.get('SQ_WAIT_ANY',0)/wc:.2f} / {a.get('SQ_WAIT_INST_ANY',0)/wc:.2f} / {a.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} | {a.get('SQ_LDS_BANK_CONFLICT',0)/max(a.get('SQ_LDS_IDX_ACTIVE',1),1):.3f}")
PY
for rep in 0 1; do
  timeout -k 10 300 python $R/examples/train_vec.py --amp --steps 100 2>/dev/null | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('train_vec --amp', round(d['env_steps_per_s']), 'env-steps/s,', d['learner_updates'], 'updates')" || exit 1
done
