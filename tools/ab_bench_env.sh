#!/bin/bash
# Same-box A/B of an environment knob on the bench's samples/s:
# ab_bench_env.sh VAR "v1 v2" [bench args...] -- two alternating rounds of
# short bench runs (no CPU baseline, no demo line)
var=$1; vals=$2; shift 2
mkdir -p gpurun_out
for i in ${ROUNDS:-1 2}; do
  for v in $vals; do
    env $var=$v timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-demo "$@" > gpurun_out/abb_$v.$i.json 2> gpurun_out/abb_$v.$i.err || exit $?
    python3 -c "
import json
d=json.loads(open('gpurun_out/abb_$v.$i.json').read().strip().splitlines()[-1])
print('$var=$v', d['value'], d['ms_per_step'], d.get('cg_iter_per_s'), (d.get('cg_iteration') or {}).get('us_per_iteration'))
"
  done
done
