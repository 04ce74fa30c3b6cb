#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
for r in 1 2 3; do
  echo "== process $r"
  timeout -k 10 300 python tools/alloc_ab.py 4 2>&1 | grep -v amdgpu.ids || exit 1
done
