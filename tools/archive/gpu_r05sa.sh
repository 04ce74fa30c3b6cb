#!/bin/bash
# Round 5: the single-env surface with ffmp_reward_done_packed's kernel-argument form (flag 8): legacy API
# parity (incl. the form against the copies), then tools/single_env_probe.py with it and without it.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r05sa
mkdir -p $O
cd $R && timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_legacy_api.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
echo "legacy tests: $(tail -1 $O/pytest.log)"
cd /tmp && export TMPDIR=/tmp
for k in 1 2; do
  echo "== kernel arguments"; timeout -k 10 200 python3 $R/tools/single_env_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
  echo "== copies"; FFMP_SINGLE_ARGS=0 timeout -k 10 200 python3 $R/tools/single_env_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
done
