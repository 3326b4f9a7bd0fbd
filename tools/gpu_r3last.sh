export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_transforms_gpu.py -k "fold or scatter or los or LOS" -x -q --timeout 200 --timeout-method thread > gpurun_out/t_last.log 2>&1
echo "tests rc=$?"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke4.log 2>&1
echo "smoke rc=$?"
