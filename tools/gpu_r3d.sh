export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_compact_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_compact.log 2>&1
echo "compact tests rc=$?"
timeout -k 10 300 python -u tools/demo_profile.py --steps 1 > gpurun_out/demo_defer1.log 2>&1 || exit $?
NFT_GEOVI_DEFER_DIR=0 timeout -k 10 300 python -u tools/demo_profile.py --steps 1 > gpurun_out/demo_defer0.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/step_phases.py --demo > gpurun_out/phases_demo.log 2>&1 || exit $?
