# A/B of library builds on one box: graph-replayed CG iteration per build
# (interleaved, twice), then rocprofv3 kernel stats per build.
#   bash tools/ab_libs.sh base new ...   (build_ab/<name>.so)
R=$PWD
mkdir -p gpurun_out
for rep in 1 2; do
  for b in "$@"; do
    echo "== $b rep $rep" >> gpurun_out/ab.log
    NFT_LIB=$R/build_ab/$b.so timeout -k 10 240 python3 -u tools/amp2_probe.py >> gpurun_out/ab.log 2>&1 || exit $?
  done
done
cd /tmp && export TMPDIR=/tmp
for b in "$@"; do
  NFT_LIB=$R/build_ab/$b.so PROBE_REPS=20 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/ab_prof_$b -o run -- python3 -u $R/tools/amp2_probe.py >> $R/gpurun_out/ab.log 2>&1 || exit $?
done
