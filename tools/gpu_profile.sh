#!/bin/bash
# rocprofv3 evidence for bench.py's default workload (C3):
#   pass 1: --kernel-trace --stats (per-kernel durations)
#   pass 2: --pmc WRITE_SIZE, pass 3: --pmc FETCH_SIZE (separate passes: TCC slot limits)
# then tools/summarize_profiles.py writes profiles/<tag>_*.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-r01}
CFG=${2:-C3}
FMT=${3:-f32}  # obs format: f32 (the bench metric) or u8f16 (compact); outputs are labelled <cfg>[_u8f16]
LBL=$CFG; [ "$FMT" = f32 ] || LBL=${CFG}_$FMT
FUSED=${4:-auto}  # one-launch step: auto (the autotune decides), on or off; "on" labels <cfg>[_fmt]_fused
[ "$FUSED" = on ] && LBL=${LBL}_fused
mkdir -p $R/gpurun_out/prof
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python3 -c "import sys; sys.path.insert(0,'$R'); import __graft_entry__ as g; g.build()" || exit 1
# 48 timed steps = 6 whole ring cycles (W = 8): 6 replays of the step graph (bench.py's default), so the
# trace and PMC passes average the same launches
# the launch choices come from one plain run first, so that the profiled runs contain no
# autotune launches: the trace's per-kernel average is then the timed launches' (plus warm-up)
echo "== tuning run"
timeout -k 10 300 python3 $R/bench.py --config $CFG --obs-format $FMT --fused $FUSED --steps 8 --warmup 2 --cpu-seconds 0 --save-tuning $R/gpurun_out/prof/tuning_$LBL.json > $R/gpurun_out/prof/bench_tuning_$LBL.log 2>&1 || exit 1
cat $R/gpurun_out/prof/tuning_$LBL.json; echo
# the graph form the tuning run's skew trial kept (skewed or two-launch), forced in the profiled runs so that
# every pass times the same kernels
SKEW=$(python3 -c "
import json
ls = [l for l in open('$R/gpurun_out/prof/bench_tuning_$LBL.log') if l.startswith('{')]
d = json.loads(ls[-1])
print('on' if (d['config'].get('graph') or {}).get('skewed') else 'off')" 2>/dev/null || echo off)
echo "graph skew: $SKEW"
BENCH="$R/bench.py --config $CFG --obs-format $FMT --fused $FUSED --graph-skew $SKEW --steps 48 --warmup 10 --cpu-seconds 0 --tuning $R/gpurun_out/prof/tuning_$LBL.json"
echo "== trace"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof/trace_$LBL -o run -- python3 $BENCH > $R/gpurun_out/prof/bench_trace_$LBL.log 2>&1 || exit 1
echo "== pmc write"
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'raster_kernel|env_kernel|skew_kernel' --output-format csv -d $R/gpurun_out/prof/pmcw_$LBL -o run -- python3 $R/bench.py --config $CFG --obs-format $FMT --fused $FUSED --graph-skew $SKEW --steps 48 --warmup 2 --cpu-seconds 0 --tuning $R/gpurun_out/prof/tuning_$LBL.json > $R/gpurun_out/prof/bench_pmcw_$LBL.log 2>&1 || exit 1
echo "== pmc fetch"
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'raster_kernel|env_kernel|skew_kernel' --output-format csv -d $R/gpurun_out/prof/pmcf_$LBL -o run -- python3 $R/bench.py --config $CFG --obs-format $FMT --fused $FUSED --graph-skew $SKEW --steps 48 --warmup 2 --cpu-seconds 0 --tuning $R/gpurun_out/prof/tuning_$LBL.json > $R/gpurun_out/prof/bench_pmcf_$LBL.log 2>&1 || exit 1
cd $R && python3 tools/summarize_profiles.py $TAG $LBL
