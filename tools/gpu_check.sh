set -o pipefail
mkdir -p gpurun_out
echo "== build"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 &&
echo "== parity report" && timeout -k 10 600 python tests/parity_report.py > gpurun_out/parity.log 2>&1 &&
echo "== bench" && timeout -k 10 300 python bench.py --steps 50 --warmup 10 --cpu-seconds 5 > gpurun_out/bench1.log 2>&1 &&
echo "== pytest gpu" && timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "rc=$rc"
tail -5 gpurun_out/*.log
exit $rc
