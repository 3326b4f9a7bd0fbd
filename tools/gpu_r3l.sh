export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
LOS_DBGS=0,16,1,17 timeout -k 10 200 python -u tools/los_probe.py > gpurun_out/los_probe4.log 2>&1 || exit $?
