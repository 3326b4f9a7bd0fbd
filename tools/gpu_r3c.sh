export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_compact_gpu.py -x -v --timeout 200 --timeout-method thread > gpurun_out/t_compact.log 2>&1
echo "compact tests rc=$?"
timeout -k 10 300 python -u tools/demo_profile.py --steps 1 > gpurun_out/demo_profile2.log 2>&1 || exit $?
