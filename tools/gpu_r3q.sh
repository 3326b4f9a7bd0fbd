export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py -k "los or LOS" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_los.log 2>&1
echo "los tests rc=$?"
for v in ut0 ut1 ut2; do [ $v = ut0 ] && L=$PWD/joss-nifty_amd/libnifty_amd.so || L=$PWD/build_ab/los_$v.so;
  echo "== $v" >> gpurun_out/los_ut.log
  NFT_LIB=$L timeout -k 10 200 python -u tools/los_probe.py >> gpurun_out/los_ut.log 2>&1 || exit $?
done
for rep in 1 2; do
NFT_LOS_BOX_WG=0 timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/box_ab.log 2>&1 || exit $?
NFT_LOS_BOX_WG=1 timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/box_ab.log 2>&1 || exit $?
done
