#!/bin/bash
# round 4, evidence on the final env kernel: the full GPU suite (+ smoke), rocprofv3 trace + PMC of the
# C3 bench (tools/gpu_profile.sh r04 C3), the driver's bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04g
mkdir -p $O
export FFMP_TIMED_PATH_OUT=$O
timeout -k 10 900 python -u -m pytest -x -v --timeout 900 --timeout-method thread $R/tests -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash $R/tools/gpu_profile.sh r04 C3 > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
tail -5 $O/profile.log
timeout -k 10 400 python $R/bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit 1
# (the cost of the per-launch event markers was measured here once with a --event-every k option:
#  every launch 14.008 / 14.001 M, every 8th 14.034 / 13.995 M — none; profiles/r04g_event_markers.txt)
