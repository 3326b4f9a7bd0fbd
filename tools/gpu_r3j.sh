export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_geovi_trace_gpu.py tests/test_parity_gpu.py -q --timeout 300 --timeout-method thread -rA > gpurun_out/t_trace.log 2>&1
echo "tests rc=$?"
