#!/bin/bash
# A/B of the fused prologue + R2C pass variants (NFT_PRO_R2C modes) on the
# bench configs' CG iteration (tools/iter_probe.py), same box:
#   tools/ab_pror2c.sh "C3 C5 C2" "0 2"
mkdir -p gpurun_out
L=gpurun_out/ab_pror2c.log
: > $L
for cfg in ${1:-C3 C5 C2}; do
  for m in ${2:-0 2}; do
    echo "== $cfg mode $m" >> $L
    PROBE_CONFIG=$cfg NFT_PRO_R2C=$m timeout -k 10 200 python -u tools/iter_probe.py 2>&1 | grep -v amdgpu.ids >> $L || exit 1
  done
done
