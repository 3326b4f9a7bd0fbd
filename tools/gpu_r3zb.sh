export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "fold or scatter" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_fold2.log 2>&1
echo "fold tests rc=$?"
for rep in 1 2; do for b in base foldv2 pair; do
  [ $b = foldv2 ] && L=$PWD/joss-nifty_amd/libnifty_amd.so || L=$PWD/build_ab/$b.so
  [ $b = pair ] && L=$PWD/build_ab/knob_pair.so
  echo "== $b rep $rep" >> gpurun_out/pair_ab.log
  NFT_LIB=$L timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/pair_ab.log 2>&1 || exit $?
done; done
