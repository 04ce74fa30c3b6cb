#!/bin/bash
# Round 3 (second session) GPU command lines, one task per evidence file: bash tools/gpu_r03b.sh <task>
# (run through gpurun from the repo root).  Tasks:
#   series            round 3 (second session): k-frame temporal maps (env, replay, Brain, 3-channel conv1 fold), then the
#   learner-prof      round 3 (second session): kernel split of the train.py-style loop on the current MFMA kernels, then
#   spec              round 3 (second session): the one-launch step rastering from the speculative record (the env wave
#   conv              round 3 (second session): the learner's MFMA convolutions (tools/conv_variants.py) + their parity tests
#   learner           round 3 (second session): learner tests + the train.py-style loop on the current MFMA kernels
#   ct8               round 3 (second session): compact raster with 8 cells per lane (FFMP_RASTER_MID8): launch shapes at
#   ct8-check         round 3 (second session): the 8-cells-per-lane compact raster: parity, then the default bench twice
#   compact-fresh     round 3 (second session): the compact layout as the only workload of a fresh process (no float32
#   bench             round 3 (second session): the default bench as the driver runs it (compact leg in a child process)
#   launches          round 3 (second session): per-launch raster times of the driver's command line (20 timed steps after
#   benchloop         round 3 (second session): the driver's bench command with the launch shape fixed to 4096-cell blocks
#   transient         round 3 (second session): the slow start of the timed loop (tools/transient_probe.py), two-launch step,
#   transient-shapes  round 3 (second session): the post-idle slow start by raster launch shape (tools/transient_shapes.py)
#   transient-reset   round 3 (second session): slow start after reset(): episodes or GPU state (tools/transient_reset.py)
#   full              round 3 (second session): the whole GPU suite as the driver runs it, then smoke()
#   shape-sweep       steady-state raster time of launch shapes beyond the autotune's (tools/shape_sweep.py)
#   configs           the other BASELINE configs' bench lines (C2, the C5 per-GPU share)
#   pipeline          the two-launch step with its env kernel in slices beside the raster (tools/pipeline_probe.py)
#   two-rank          bench.py --gpus 2 over gloo with both ranks on the one GPU (the N > 1 code path)
#   final-bench       round 3 (second session): the driver's bench command line on the final code, two fresh processes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out $R/gpurun_out/ab
export TMPDIR=/tmp

task_series() {
  timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_temporal_maps.py tests/test_gpu_replay.py tests/test_gpu_learner.py "tests/test_gpu_conv_mfma.py::test_folded_conv1_against_float64" > gpurun_out/r03b_series_tests.log 2>&1 || { tail -5 gpurun_out/r03b_series_tests.log; grep -E "^E " gpurun_out/r03b_series_tests.log | head -20; exit 1; }
  tail -2 gpurun_out/r03b_series_tests.log
  task_learner_prof
}

task_learner_prof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_train2 -o train -- python3 examples/train_vec.py --envs 256 --steps 60 --amp > gpurun_out/r03b_train_prof.log 2>&1 || { tail -20 gpurun_out/r03b_train_prof.log; exit 1; }
  tail -1 gpurun_out/r03b_train_prof.log
  timeout -k 10 400 python -u bench.py > gpurun_out/r03b_bench_default.log 2>&1 || { tail -20 gpurun_out/r03b_bench_default.log; exit 1; }
  tail -1 gpurun_out/r03b_bench_default.log | cut -c1-600
}

task_spec() {
  mkdir -p $R/gpurun_out/ab
  timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_timed_path.py tests/test_gpu_parity.py tests/test_gpu_compact.py tests/test_gpu_oracle_c.py > gpurun_out/r03b_spec_tests.log 2>&1 || { tail -5 gpurun_out/r03b_spec_tests.log; grep -E "^E " gpurun_out/r03b_spec_tests.log | head -20; exit 1; }
  tail -2 gpurun_out/r03b_spec_tests.log
  for rep in 1 2; do
    for v in base new; do
      if [ $v = base ]; then L=$R/tools/_build/libffmp_base.so; else L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; fi
      FFMP_LIB=$L timeout -k 10 300 python3 $R/bench.py --steps 50 --warmup 10 --cpu-seconds 0 > $R/gpurun_out/ab/s_${v}_$rep.log 2>&1 || exit 1
      grep '^{' $R/gpurun_out/ab/s_${v}_$rep.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; c=d.get('compact_layout') or {}; f=d['raster_autotune'].get('fused', {})
print('$v', 'f32', round(d['value']/1e6,3), 'M', r['kernel'], round(r['kernel_ms'],4), 'fused', f.get('chosen'), f.get('recheck'), 'slots', d['raster_autotune'].get('ring', {}).get('repair', [{}])[-1].get('slot_ms'), '| compact', round(c.get('value', 0)/1e6,2), 'M', c.get('kernel'), round(c.get('kernel_ms', 0),4), c.get('fused'))" || exit 1
    done
  done
}

task_conv() {
  timeout -k 10 120 python3 tools/conv_variants.py 256 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03b_conv_variants.txt || exit 1
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_conv_mfma.py > gpurun_out/r03b_conv_tests.log 2>&1 || { tail -5 gpurun_out/r03b_conv_tests.log; grep -E "^E " gpurun_out/r03b_conv_tests.log | head; exit 1; }
  tail -1 gpurun_out/r03b_conv_tests.log
}

task_learner() {
  timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_learner.py tests/test_gpu_conv_mfma.py > gpurun_out/r03b_learner_tests.log 2>&1 || { tail -5 gpurun_out/r03b_learner_tests.log; grep -E "^E " gpurun_out/r03b_learner_tests.log | head; exit 1; }
  tail -1 gpurun_out/r03b_learner_tests.log
  for i in 1 2; do
    timeout -k 10 300 python -u examples/train_vec.py --envs 256 --steps 100 --amp > gpurun_out/r03b_train_vec_amp_$i.log 2>&1 || { tail -20 gpurun_out/r03b_train_vec_amp_$i.log; exit 1; }
    tail -1 gpurun_out/r03b_train_vec_amp_$i.log | cut -c1-200
  done
  timeout -k 10 300 python -u examples/train_vec.py --envs 256 --steps 100 --amp --temporal-maps --input-channels 3 > gpurun_out/r03b_train_vec_tm3.log 2>&1 || { tail -20 gpurun_out/r03b_train_vec_tm3.log; exit 1; }
  tail -1 gpurun_out/r03b_train_vec_tm3.log | cut -c1-300
}

task_ct8() {
  for v in intree w7 w8; do
    if [ $v = intree ]; then L=$R/flow_field_based_motion_planner_amd/lib/libffmp.so; else L=$R/tools/_build/libffmp_ct8$v.so; fi
    echo "== $v"
    FFMP_LIB=$L timeout -k 10 300 python3 tools/compact_shapes.py C3 u8f16 2>&1 | grep -v amdgpu.ids || exit 1
  done | tee gpurun_out/r03b_ct8_shapes2.txt
}

task_ct8_check() {
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_timed_path.py tests/test_gpu_compact.py tests/test_gpu_oracle_c.py > gpurun_out/r03b_ct8_tests.log 2>&1 || { tail -5 gpurun_out/r03b_ct8_tests.log; grep -E "^E " gpurun_out/r03b_ct8_tests.log | head -20; exit 1; }
  tail -1 gpurun_out/r03b_ct8_tests.log
  for i in 1 2; do
    timeout -k 10 400 python -u bench.py > gpurun_out/r03b_ct8_bench_$i.log 2>&1 || { tail -20 gpurun_out/r03b_ct8_bench_$i.log; exit 1; }
    tail -1 gpurun_out/r03b_ct8_bench_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['compact_layout']; r=d['roofline']
print('f32', round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), '| compact', round(c['value']/1e6,2), c['kernel'], round(c['kernel_ms'],4), round(c['frac'],3), c['shape'], c['fused'])"
  done
}

task_compact_fresh() {
  for i in 1 2 3; do
    timeout -k 10 300 python -u bench.py --obs-format u8f16 --strong-config none --cpu-seconds 0 --steps 100 --warmup 10 > gpurun_out/r03b_compact_fresh_$i.log 2>&1 || { tail -20 gpurun_out/r03b_compact_fresh_$i.log; exit 1; }
    tail -1 gpurun_out/r03b_compact_fresh_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; a=d['raster_autotune']
print('u8f16', round(d['value']/1e6,2), 'M', r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), a.get('shape_newest'), a.get('fused', {}).get('chosen'), a.get('fused', {}).get('flags'), a.get('fused', {}).get('recheck'), {k: a.get('ring', {}).get(k) for k in ('pair_probes','pair_gbs_min','pair_gbs_max','partner_tries')})"
  done
}

task_bench() {
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b_bench_child.log 2>&1 || { tail -20 gpurun_out/r03b_bench_child.log; exit 1; }
  tail -1 gpurun_out/r03b_bench_child.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['compact_layout']; r=d['roofline']; s=d.get('strong') or {}
print('f32', round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), '| strong', round(s.get('value',0)/1e6,3), '| compact', round(c['value']/1e6,2), c['kernel'], round(c['kernel_ms'],4), round(c['frac'],3), c['shape'], c['fused'], c.get('process'))"
}

task_launches() {
  for i in 1 2 3; do
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --dump-launches --compact-steps 0 --strong-config none --cpu-seconds 0 > gpurun_out/r03b_launches_$i.log 2> gpurun_out/r03b_launches_$i.err || { tail -20 gpurun_out/r03b_launches_$i.err; exit 1; }
    tail -1 gpurun_out/r03b_launches_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; a=d['raster_autotune']
print(round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), 'fused', a['fused'].get('chosen'), a['fused'].get('recheck'), 'slots', a['ring']['repair'][-1]['slot_ms'])"
    grep -v amdgpu.ids gpurun_out/r03b_launches_$i.err | tail -25 | tr '\n' ' '; echo
  done
}

task_benchloop() {
  for i in 1 2 3; do
    timeout -k 10 400 python -u bench.py --steps 20 --warmup ${WARM:-5} --dump-launches --compact-steps 0 --strong-config none --cpu-seconds 0 --tuning tools/tuning_c3_4096x37.json > gpurun_out/r03b_loop_$i.log 2> gpurun_out/r03b_loop_$i.err || { tail -20 gpurun_out/r03b_loop_$i.err; exit 1; }
    tail -1 gpurun_out/r03b_loop_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4))"
    grep "raster ms" gpurun_out/r03b_loop_$i.err
  done
}

task_transient() {
  for s in 0 1; do echo "== SETTLE=$s"; SETTLE=$s FUSED=off timeout -k 10 300 python3 tools/transient_probe.py 2>&1 | grep -v amdgpu.ids || exit 1; done | tee gpurun_out/r03b_transient3.txt
  for i in 1 2; do
    timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --dump-launches --compact-steps 0 --strong-config none --cpu-seconds 0 > gpurun_out/r03b_settle_$i.log 2> gpurun_out/r03b_settle_$i.err || { tail -20 gpurun_out/r03b_settle_$i.err; exit 1; }
    tail -1 gpurun_out/r03b_settle_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; a=d['raster_autotune']
print(round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), 'fused', a['fused'].get('chosen'), a['fused'].get('recheck'), 'construct', d['construct_s'])"
    grep "raster ms" gpurun_out/r03b_settle_$i.err
  done
}

task_transient_shapes() {
  timeout -k 10 300 python3 tools/transient_shapes.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03b_transient_shapes.txt
}

task_transient_reset() {
  timeout -k 10 300 python3 tools/transient_reset.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03b_transient_reset.txt
}

task_full() {
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r03b_pytest_gpu.log 2>&1 || { tail -5 gpurun_out/r03b_pytest_gpu.log; grep -E "^E " gpurun_out/r03b_pytest_gpu.log | head -20; exit 1; }
  tail -3 gpurun_out/r03b_pytest_gpu.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
}

task_final_bench() {
  for i in 1 2; do
    timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r03b_final_bench_$i.log 2>&1 || { tail -20 gpurun_out/r03b_final_bench_$i.log; exit 1; }
    tail -1 gpurun_out/r03b_final_bench_$i.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); c=d['compact_layout']; r=d['roofline']; s=d.get('strong') or {}; b=d['cpu_baseline']
print('f32', round(d['value']/1e6,3), r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), d['raster_autotune']['shape_newest'], '| strong', round(s.get('value',0)/1e6,3), '| compact', round(c['value']/1e6,2), round(c['kernel_ms'],4), round(c['frac'],3), c['shape'], '| cpu', round(b['value']/1e3,1), 'K')"
  done
}

task_shape_sweep() {
  timeout -k 10 300 python3 tools/shape_sweep.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03b_shape_sweep.txt
}

task_configs() {
  for c in C2 C5; do
    timeout -k 10 600 python -u bench.py --config $c --steps 50 --warmup 10 --compact-steps 0 --strong-config none --cpu-seconds 0 > gpurun_out/r03b_config_$c.log 2>&1 || { tail -20 gpurun_out/r03b_config_$c.log; exit 1; }
    tail -1 gpurun_out/r03b_config_$c.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; a=d['raster_autotune']
print('$c', round(d['value']/1e6,3), 'M', r['kernel'], round(r['kernel_ms'],4), round(r['frac'],3), a.get('shape_newest'), a.get('fused', {}).get('chosen'), round(d['ms_per_step'],4))"
  done
}

task_pipeline() {
  timeout -k 10 300 python3 tools/pipeline_probe.py 2>&1 | grep -v amdgpu.ids | tee gpurun_out/r03b_pipeline.txt
}

task_two_rank() {
  timeout -k 10 900 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --steps 20 --warmup 5 --dist-backend gloo --cpu-seconds 0 > gpurun_out/r03b_two_rank.log 2>&1 || { tail -30 gpurun_out/r03b_two_rank.log; exit 1; }
  grep '^{' gpurun_out/r03b_two_rank.log | tail -1 | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); s=d.get('strong') or {}
print('n_gpus', d['n_gpus'], 'world_size_backend', d['config']['world_size_backend'], 'weak', round(d['value']/1e6,3), 'per-rank ms', d['per_rank_ms_per_step'], '| strong', round(s.get('value',0)/1e6,3), s.get('per_rank_ms_per_step'), '| compact', d.get('compact_layout'))"
}

case "$1" in
  series) task_series ;;
  learner-prof) task_learner_prof ;;
  spec) task_spec ;;
  conv) task_conv ;;
  learner) task_learner ;;
  ct8) task_ct8 ;;
  ct8-check) task_ct8_check ;;
  compact-fresh) task_compact_fresh ;;
  bench) task_bench ;;
  launches) task_launches ;;
  benchloop) task_benchloop ;;
  transient) task_transient ;;
  transient-shapes) task_transient_shapes ;;
  transient-reset) task_transient_reset ;;
  full) task_full ;;
  final-bench) task_final_bench ;;
  shape-sweep) task_shape_sweep ;;
  configs) task_configs ;;
  pipeline) task_pipeline ;;
  two-rank) task_two_rank ;;
  *) echo "usage: $0 {series|learner-prof|spec|conv|learner|ct8|ct8-check|compact-fresh|bench|launches|benchloop|transient|transient-shapes|transient-reset|full|final-bench|shape-sweep|configs|pipeline|two-rank}"; exit 2 ;;
esac
