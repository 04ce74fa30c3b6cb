#!/bin/bash
# round 6 (f): PMC pass over the learner's MFMA convolutions (MFMA busy, wave states) at B = 256 with the
# final tile choice, then the rocprofv3 evidence for bench.py's default workload (C3: trace + WRITE/FETCH)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 bash tools/gpu_conv_pmc.sh r06f_conv > gpurun_out/r06f_conv_pmc.txt 2>&1 || { tail -20 gpurun_out/r06f_conv_pmc.txt; exit 1; }
cat gpurun_out/r06f_conv_pmc.txt
timeout -k 10 1000 bash tools/gpu_profile.sh r06f C3 > gpurun_out/r06f_profile.log 2>&1 || { tail -30 gpurun_out/r06f_profile.log; exit 1; }
tail -30 gpurun_out/r06f_profile.log
