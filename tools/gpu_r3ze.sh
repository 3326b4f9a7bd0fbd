export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu --maxfail=6 -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests4.log 2>&1
echo "gpu tests rc=$?"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke2.log 2>&1
echo "smoke rc=$?"
timeout -k 10 500 python3 -u bench.py > gpurun_out/bench_r03v5.json 2> gpurun_out/bench_r03v5.err
echo "bench rc=$?"
