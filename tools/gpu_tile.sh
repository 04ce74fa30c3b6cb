set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "shapes" > gpurun_out/tile_tests.log 2>&1; rc=$?; tail -3 gpurun_out/tile_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python tools/raster_compute_probe.py
