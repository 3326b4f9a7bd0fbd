export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in 1 2; do for b in base cgch2 prog4 prog1; do
  [ $b = base ] && L=$PWD/joss-nifty_amd/libnifty_amd.so || L=$PWD/build_ab/knob_$b.so
  echo "== $b rep $rep" >> gpurun_out/knob_ab.log
  NFT_LIB=$L timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/knob_ab.log 2>&1 || exit $?
done; done
