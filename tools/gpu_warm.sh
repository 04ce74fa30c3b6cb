set -o pipefail
mkdir -p gpurun_out
echo "== gpu tests"; timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu > gpurun_out/ring_tests.log 2>&1; rc=$?
tail -4 gpurun_out/ring_tests.log; [ $rc -eq 0 ] || exit $rc
for r in 0 1; do
timeout -k 10 300 python bench.py --steps 64 --warmup 0 --cpu-seconds 0 --dump-launches > gpurun_out/warm$r.log 2>&1 || exit 1
grep -E "raster ms" gpurun_out/warm$r.log | tr ' ' '\n' | tail -n +5 | paste -sd' ' | fold -w 96
python -c "import json;d=json.loads([l for l in open('gpurun_out/warm$r.log') if l.startswith('{')][0]);a=d['raster_autotune'];print(d['value'], a.get('placement_tries'), a['shape_newest'], a['gbs'], a.get('ring'))"
done
