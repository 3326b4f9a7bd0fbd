export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu --maxfail=6 -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests2.log 2>&1
echo "gpu tests rc=$?"
for rep in 1 2; do for b in base cge adj_w8; do
  [ $b = cge ] && L=$PWD/joss-nifty_amd/libnifty_amd.so || L=$PWD/build_ab/$b.so
  echo "== $b rep $rep" >> gpurun_out/occ_ab.log
  NFT_LIB=$L timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/occ_ab.log 2>&1 || exit $?
done; done
