export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/newton_probe.py 4 > gpurun_out/newton4.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/newton_probe.py 1 > gpurun_out/newton1.log 2>&1 || exit $?
