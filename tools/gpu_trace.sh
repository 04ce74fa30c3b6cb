#!/bin/bash
# Probe build with in-kernel wall-clock stamps (-DFFMP_TRACE) and tools/trace_probe.py on it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
test -f $R/tools/_build/libffmp_trace.so || exit 1
for a in "C2 4096" "C3 32768"; do
  FFMP_LIB=$R/tools/_build/libffmp_trace.so timeout -k 10 200 python3 $R/tools/archive/trace_probe.py $a || exit 1
done
