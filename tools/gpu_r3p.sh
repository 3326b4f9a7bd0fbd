export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "fold or scatter or metric" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_fold.log 2>&1
echo "fold tests rc=$?"
for rep in 1 2; do
NFT_BIN_SORTED=0 timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/fold_ab.log 2>&1 || exit $?
NFT_BIN_SORTED=1 timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/fold_ab.log 2>&1 || exit $?
done
LOS_DBGS=0,1,2,4,8,16,6,10 timeout -k 10 200 python -u tools/los_probe.py > gpurun_out/los_dbg.log 2>&1
