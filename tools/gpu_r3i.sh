export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u tools/demo_profile.py --steps 1 > gpurun_out/demo_profile3.log 2>&1 || exit $?
