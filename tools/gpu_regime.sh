#!/bin/bash
set -o pipefail
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > /dev/null 2>&1 || exit 1
for r in 1 2; do timeout -k 10 300 python tools/regime_probe.py C3 2>&1 | grep shape || exit 1; done
timeout -k 10 300 python tools/regime_probe.py C2 2>&1 | grep shape
