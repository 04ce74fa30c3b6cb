#!/bin/bash
# round 6 (k): rocprofv3 evidence for the final bench (C3: trace + WRITE/FETCH passes) and the CPU baseline per config
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 1000 bash tools/gpu_profile.sh r06final C3 > gpurun_out/r06final_profile.log 2>&1 || { tail -30 gpurun_out/r06final_profile.log; exit 1; }
tail -12 gpurun_out/r06final_profile.log
