#!/bin/bash
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
for w in 1 4 1 4; do
  FFMP_ENV_WAVES=$w timeout -k 10 300 python tools/env_kernel_bench.py C3 32768 2>&1 | grep env_waves || exit 1
done
for w in 1 4; do
  FFMP_ENV_WAVES=$w timeout -k 10 300 python tools/env_kernel_bench.py C5 16384 2>&1 | grep env_waves || exit 1
  FFMP_ENV_WAVES=$w timeout -k 10 300 python tools/env_kernel_bench.py C2 4096 2>&1 | grep env_waves || exit 1
done
