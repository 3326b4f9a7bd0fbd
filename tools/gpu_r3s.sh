export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_transforms_gpu.py -k "los or LOS or fold or scatter" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_los2.log 2>&1
echo "los/fold tests rc=$?"
timeout -k 10 300 python -u tools/los_probe.py > gpurun_out/los_tiles.log 2>&1 || exit $?
for rep in 1 2; do for tl in 1 2 4; do
NFT_LOS_TILE=$tl timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/tile_ab.log 2>&1 || exit $?
done; NFT_BIN_IL=0 timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/tile_ab.log 2>&1 || exit $?
done
