set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
timeout -k 10 300 python3 bench.py --config C2 --cpu-seconds 0 --compact-steps 0 > gpurun_out/c2ab.log 2>&1 || { tail -20 gpurun_out/c2ab.log; exit 1; }
python3 -c "
import json;d=json.loads([l for l in open('gpurun_out/c2ab.log') if l.startswith('{')][0]);a=d['raster_autotune']
print('%.3f M' % (d['value']/1e6), 'step %.4f' % d['ms_per_step'], a['shape'], sorted(a['candidates'], key=lambda c:-c[-1])[:4])"
done
