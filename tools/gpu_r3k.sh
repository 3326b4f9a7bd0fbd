export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/debug_demo64.py 1 > gpurun_out/dbg_demo64_1.log 2>&1
timeout -k 10 200 python -u tools/debug_demo64.py 0 > gpurun_out/dbg_demo64_0.log 2>&1
