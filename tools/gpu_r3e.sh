export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py -k "los or batched" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_los.log 2>&1
echo "los tests rc=$?"
timeout -k 10 200 python -u tools/los_probe.py > gpurun_out/los_probe2.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-demo --steps 5 > gpurun_out/b1.json 2> gpurun_out/b1.err
echo "bench rc=$?"
