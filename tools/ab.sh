#!/bin/bash
# A/B of two builds of the library on one box: ab.sh PREV_SO [bench args]
# alternates prev / new bench runs (no CPU baseline, no demo line) and
# prints each run's value and CG-iteration time.
prev=$1; shift
mkdir -p gpurun_out
for i in 1 2; do
  for v in prev new; do
    if [ $v = prev ]; then lib=$PWD/$prev; else lib=$PWD/joss-nifty_amd/libnifty_amd.so; fi
    NFT_LIB=$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-demo --steps 5 "$@" > gpurun_out/ab_$v$i.json 2> gpurun_out/ab_$v$i.err || exit $?
    python3 -c "
import json,sys
d=json.loads(open('gpurun_out/ab_$v$i.json').read().strip().splitlines()[-1])
r=d['roofline']; print('$v$i', d['value'], r['avg_launch_us'], r['frac'], ' '.join('%s=%.1f' % (k, v['avg_us']) for k, v in d.get('kernels', {}).items()))
"
  done
done
