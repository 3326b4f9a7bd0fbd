export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
LOS_DBGS=0,16,1,17 timeout -k 10 200 python -u tools/los_probe.py > gpurun_out/los_probe4.log 2>&1 || exit $?
for v in 1 0; do
  NFT_PRO_FOLD_PI=$v timeout -k 10 200 python -u tools/newton_probe.py 4 > gpurun_out/newton4_pi$v.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest tests/test_geovi_batch_gpu.py tests/test_compact_gpu.py tests/test_geovi_trace_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_geovi.log 2>&1
echo "tests rc=$?"
