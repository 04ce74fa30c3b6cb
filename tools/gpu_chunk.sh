#!/bin/bash
set -o pipefail
hipcc --offload-arch=gfx950 -O3 -o /tmp/chunk_probe tools/chunk_probe.hip > /dev/null 2>&1 || exit 1
timeout -k 10 300 /tmp/chunk_probe 64 4 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 300 /tmp/chunk_probe 64 4 2>&1 | grep -v amdgpu.ids
