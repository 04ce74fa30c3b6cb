#!/bin/bash
set -o pipefail
hipcc --offload-arch=gfx950 -O3 -o /tmp/order_probe tools/order_probe.hip > /dev/null 2>&1 || exit 1
timeout -k 10 300 /tmp/order_probe 256 32768 10 4096 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 /tmp/order_probe 512 16384 3 4096 2>&1 | grep -v amdgpu.ids
