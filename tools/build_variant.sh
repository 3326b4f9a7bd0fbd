#!/bin/bash
# A/B build of libnifty_amd.so with extra compile definitions, in
# build_ab/NAME/ (on the CPU, before a GPU call):
#   build_variant.sh NAME "-DKNOB=V ..." [SOURCES]
# SOURCES (e.g. "nft_pro_r2c nft_amp2"): recompile only these with the knobs,
# the other objects are copied from the in-tree build (run make first);
# default: every source compiles with the knobs.
set -e
name=$1; defs=$2; only=$3
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/joss-nifty_amd/csrc
out=$R/build_ab/$name
mkdir -p $out
pids=()
for s in nft_fft nft_pro_r2c nft_blas nft_cf nft_spmv nft_amp nft_amp2 nft_los nft_prof; do
  if [ -n "$only" ] && [[ " $only " != *" $s "* ]]; then
    cp $C/$s.o $out/$s.o
    continue
  fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -I$R/include -Wall -Wno-unused-result $defs \
    -c $C/$s.hip -o $out/$s.o &
  pids+=($!)
done
for p in "${pids[@]}"; do wait $p; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $out/libnifty_amd.so $out/*.o
echo "built $out/libnifty_amd.so"
