#!/bin/bash
# Same-box A/B over library builds x values of one environment knob:
# ab_grid.sh VAR "v1 v2" LIB1 LIB2 ... ("-" = in-tree), two alternating rounds
# of tools/iter_probe.py (PROBE_CONFIG=C2/C4/C5 for the other configs)
var=$1; vals=$2; shift 2
mkdir -p gpurun_out
for i in 1 2; do
  for lib in "$@"; do
    for v in $vals; do
      echo "lib=$lib $var=$v"
      if [ "$lib" = "-" ]; then
        env $var=$v timeout -k 10 240 python -u tools/iter_probe.py || exit $?
      else
        [ -d "$lib" ] && lib=$lib/libnifty_amd.so
        env $var=$v NFT_LIB=$PWD/$lib timeout -k 10 240 python -u tools/iter_probe.py || exit $?
      fi
    done
  done
done
