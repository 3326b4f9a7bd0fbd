export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_configs_gpu.py tests/test_transforms_gpu.py -k "los or LOS" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_los5.log 2>&1
echo "los tests rc=$?"
timeout -k 10 300 python -u tools/los_probe.py > gpurun_out/los_vec.log 2>&1 || exit $?
for rep in 1 2; do for s in 0 1; do
NFT_LOS_ADJ_VEC=$s timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/vec_ab.log 2>&1 || exit $?
done; done
