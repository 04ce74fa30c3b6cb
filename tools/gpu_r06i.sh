#!/bin/bash
# round 6 (i): the other configs on the final bench (episodes restarted after the graph trials): the C5 share,
# the C4 8,192-env shard as rank 0 and rank 7 (the driver's step counts), C2 at 200 steps
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r06i
mkdir -p $O
cd $R
show() { python -c "import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', round(d['value']/1e6,3), round(d['roofline']['frac'],4), round(d['hbm_roofline_pct_whole_step'],2), d['roofline']['timed_resets'], d['config']['graph'].get('skewed'), {k: round(v['value']/1e6,3) for k, v in (d.get('closed_loop') or {}).items() if isinstance(v, dict)})"; }
timeout -k 10 500 python bench.py --config C5 --steps 40 --warmup 10 --cpu-seconds 0 --compact-steps 0 --strong-config none --closed-loop 0 > $O/bench_c5.json 2> $O/bench_c5.err || { tail -20 $O/bench_c5.err; exit 1; }
show $O/bench_c5.json C5
for off in 0 57344; do
  timeout -k 10 400 python bench.py --config C4 --envs 8192 --env-offset $off --steps 20 --warmup 5 --cpu-seconds 0 --compact-steps 0 --strong-config none --closed-loop 0 > $O/bench_c4_8192_$off.json 2> $O/bench_c4_8192_$off.err || { tail -20 $O/bench_c4_8192_$off.err; exit 1; }
  show $O/bench_c4_8192_$off.json C4s_$off
done
timeout -k 10 500 python bench.py --config C2 --steps 200 --warmup 20 --cpu-seconds 0 --compact-steps 0 --strong-config none > $O/bench_c2.json 2> $O/bench_c2.err || { tail -20 $O/bench_c2.err; exit 1; }
show $O/bench_c2.json C2
