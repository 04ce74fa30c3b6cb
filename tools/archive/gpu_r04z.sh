#!/bin/bash
# round 4, closing check of the final tree: the full GPU suite, smoke and the driver's bench line
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04z
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 900 --timeout-method thread $R/tests -m gpu > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import sys; sys.path.insert(0, '$R'); import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python $R/bench.py > $O/bench.json 2> $O/bench.err || exit 1
python -c "import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('bench', round(d['value']/1e6,3), round(d['roofline']['kernel_ms'],4), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2))"
