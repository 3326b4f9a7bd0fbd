#!/bin/bash
# Same-box A/B of library builds on the bench's C3 CG iteration:
# ab_libs.sh build_ab/A/libnifty_amd.so ... ("-" = the in-tree library);
# two alternating rounds of tools/iter_probe.py (graph-replayed iteration
# + per-kernel table).  PROBE_CONFIG=C2/C4/C5 for the other configs.
mkdir -p gpurun_out
for i in 1 2; do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then
      timeout -k 10 240 python -u tools/iter_probe.py || exit $?
    else
      [ -d "$lib" ] && lib=$lib/libnifty_amd.so
      NFT_LIB=$PWD/$lib timeout -k 10 240 python -u tools/iter_probe.py || exit $?
    fi
  done
done
