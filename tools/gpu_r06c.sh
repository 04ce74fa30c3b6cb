#!/bin/bash
# round 6 (c): the whole GPU suite + smoke on the current HEAD; weight-gradient prefetch A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06c
mkdir -p $O
cd $R
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
timeout -k 10 300 python -u tools/conv_ab.py 256 9 0:0:0:0 0:0:0:1 > $O/conv_ab.txt 2>&1 || { tail -20 $O/conv_ab.txt; exit 1; }
cat $O/conv_ab.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 500 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log; grep -E "^FAILED|^ERROR" $O/pytest_gpu.log | head -20; ok $rc || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
