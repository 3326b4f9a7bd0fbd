export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
NFT_LIB=$PWD/build_ab/sil4k.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "fold or scatter" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_sil.log 2>&1
echo "sil tests rc=$?"
for rep in 1 2; do for b in base sil4k; do
  [ $b = base ] && L=$PWD/joss-nifty_amd/libnifty_amd.so || L=$PWD/build_ab/$b.so
  echo "== $b rep $rep" >> gpurun_out/sil_ab.log
  NFT_LIB=$L timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/sil_ab.log 2>&1 || exit $?
done; done
