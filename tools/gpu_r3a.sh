export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u tools/demo_profile.py --steps 1 > gpurun_out/demo_profile.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/los_probe.py > gpurun_out/los_probe.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 5 > gpurun_out/b0.json 2> gpurun_out/b0.err
echo "bench rc=$?"
