export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu --maxfail=6 -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests4.log 2>&1
echo "gpu tests rc=$?"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke2.log 2>&1
echo "smoke rc=$?"
NFT_LIB=$PWD/build_ab/los_vload.so timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_transforms_gpu.py -k "los or LOS" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_vload.log 2>&1
echo "vload los tests rc=$?"
for rep in 1 2; do for b in base vload; do
  [ $b = base ] && L=$PWD/joss-nifty_amd/libnifty_amd.so || L=$PWD/build_ab/los_vload.so
  echo "== $b rep $rep" >> gpurun_out/vload_ab.log
  NFT_LIB=$L timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/vload_ab.log 2>&1 || exit $?
done; done
timeout -k 10 500 python3 -u bench.py > gpurun_out/bench_r03v5.json 2> gpurun_out/bench_r03v5.err
echo "bench rc=$?"
