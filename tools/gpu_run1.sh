export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_amp2_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/t_amp2.log 2>&1
rc=$?
echo "tests rc=$rc"
if [ $rc -le 1 ]; then
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-demo --steps 5 > gpurun_out/b_amp2.json 2> gpurun_out/b_amp2.err
  echo "bench rc=$?"
fi
