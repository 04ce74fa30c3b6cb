set -o pipefail
mkdir -p gpurun_out
for cfg in C3 C2 C5; do
timeout -k 10 300 python bench.py --config $cfg --steps 64 --warmup 5 --cpu-seconds 0 --dump-launches > gpurun_out/warm_$cfg.log 2>&1 || exit 1
grep -E "raster ms" gpurun_out/warm_$cfg.log | tr ' ' '\n' | tail -n +5 | head -24 | paste -sd' ' | fold -w 120
python -c "import json;d=json.loads([l for l in open('gpurun_out/warm_$cfg.log') if l.startswith('{')][0]);a=d['raster_autotune'];print('$cfg', d['value'], d['roofline']['kernel'], round(d['roofline']['achieved']), a['gbs'], a.get('fused'))"
done
