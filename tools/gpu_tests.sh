# the whole GPU suite (one process), log in gpurun_out/gpu_tests.log
timeout -k 10 1100 python -u -m pytest tests -m gpu --maxfail=6 -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "gpu tests rc=$?"
