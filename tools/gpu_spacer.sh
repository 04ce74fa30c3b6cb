#!/bin/bash
set -o pipefail
hipcc --offload-arch=gfx950 -O3 -o /tmp/spacer_probe tools/spacer_probe.hip > /dev/null 2>&1 || exit 1
timeout -k 10 300 /tmp/spacer_probe 512 40 2>&1 | grep -v amdgpu.ids | tr '\n' ';' ; echo
timeout -k 10 300 /tmp/spacer_probe 2 40 2>&1 | grep -v amdgpu.ids | tr '\n' ';'; echo
