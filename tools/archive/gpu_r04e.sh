#!/bin/bash
# round 4: the data gradient on 4 x 8 patches (conv_dgrad_kernel): float64 parity of every conv
# kernel, conv2 fwd / dgrad / wgrad timing (patch kernel vs the row kernel, FFMP_CONV_DGRAD=0), the
# learner loop (examples/train_vec.py --amp) with and without
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04e
mkdir -p $O
timeout -k 10 400 python -u -m pytest $R/tests/test_gpu_conv_mfma.py $R/tests/test_gpu_learner.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in 1 0; do
  FFMP_CONV_DGRAD=$v timeout -k 10 300 python $R/tools/conv_probe.py 256 2>&1 | grep "mfma" | sed "s/^/dgrad_patches=$v /" || exit 1
done
for v in 1 0; do
  FFMP_CONV_DGRAD=$v timeout -k 10 300 python $R/examples/train_vec.py --amp --steps 60 2>&1 | tail -2 | sed "s/^/dgrad_patches=$v /" || exit 1
done
