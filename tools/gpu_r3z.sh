export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "per_box" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_box.log 2>&1
echo "box test rc=$?"
for rep in 1 2; do for b in e4 e2 e8; do
  [ $b = e4 ] && L=$PWD/joss-nifty_amd/libnifty_amd.so || L=$PWD/build_ab/amp_$b.so
  echo "== $b rep $rep" >> gpurun_out/ampe_ab.log
  NFT_LIB=$L timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/ampe_ab.log 2>&1 || exit $?
done; done
