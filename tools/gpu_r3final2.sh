export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu --maxfail=6 -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests5.log 2>&1
echo "gpu tests rc=$?"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke3.log 2>&1
echo "smoke rc=$?"
bash tools/profile_r03.sh r03v6
