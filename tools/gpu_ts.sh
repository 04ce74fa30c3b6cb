#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
D=$(ls -d /sys/class/drm/card*/device 2>/dev/null | head -1)
echo "sysfs: $D"; ls $D | grep -E 'pp_dpm|power_dpm' | tr '\n' ' '; echo
( for i in $(seq 1 400); do echo "$(date +%s.%N) fclk=$(grep '\*' $D/pp_dpm_fclk 2>/dev/null | tr -d '\n') mclk=$(grep '\*' $D/pp_dpm_mclk 2>/dev/null | tr -d '\n') socclk=$(grep '\*' $D/pp_dpm_socclk 2>/dev/null| tr -d '\n')"; sleep 0.05; done ) > gpurun_out/dpm.log 2>&1 &
SP=$!
timeout -k 10 300 python tools/time_series.py 0.0 150 > gpurun_out/ts1.log 2>&1
timeout -k 10 300 python tools/time_series.py 0.05 60 > gpurun_out/ts2.log 2>&1
kill $SP 2>/dev/null
awk '{print $2}' gpurun_out/ts1.log | grep -v amdgpu | tr '\n' ' ' ; echo
awk '{print $2}' gpurun_out/ts2.log | grep -v amdgpu | tr '\n' ' ' ; echo
sort gpurun_out/dpm.log | awk '{print $2, $3, $4}' | uniq -c | head -20
cat $D/pp_dpm_fclk $D/pp_dpm_mclk 2>/dev/null
