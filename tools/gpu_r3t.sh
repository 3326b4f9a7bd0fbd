export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu --maxfail=6 -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
echo "gpu tests rc=$?"
for rep in 1 2; do
NFT_BIN_IL=0 timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/il_ab.log 2>&1 || exit $?
NFT_BIN_IL=1 timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/il_ab.log 2>&1 || exit $?
done
bash tools/profile_r03.sh r03v2
