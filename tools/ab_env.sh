#!/bin/bash
# Same-box A/B of environment settings: ab_env.sh "NAME=V ..." "-" ...
# ("-" = no extra setting); two alternating rounds of short bench runs (no
# CPU baseline, no demo line), printing value, CG-iteration time and the
# per-kernel durations of each run.
mkdir -p gpurun_out
for i in 1 2; do
  n=0
  for cfg in "$@"; do
    n=$((n+1))
    tag=e$n.$i
    if [ "$cfg" = "-" ]; then envs=(); else read -r -a envs <<< "$cfg"; fi
    env "${envs[@]}" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-demo --steps 5 > gpurun_out/ab_$tag.json 2> gpurun_out/ab_$tag.err || exit $?
    python3 -c "
import json
d=json.loads(open('gpurun_out/ab_$tag.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$tag [$cfg]', d['value'], r['avg_launch_us'], r['frac'], ' '.join('%s=%.1f' % (k, v['avg_us']) for k, v in d.get('kernels', {}).items()))
"
  done
done
