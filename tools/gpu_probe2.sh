#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
hipcc --offload-arch=gfx950 -O3 -o /tmp/placement_probe tools/placement_probe.hip > /dev/null 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 300 /tmp/placement_probe 256 32768 > gpurun_out/placement_$r.log 2>&1 || exit 1
  cat gpurun_out/placement_$r.log
done
