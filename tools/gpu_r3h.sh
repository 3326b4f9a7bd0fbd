export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in 1 2; do for v in base amp_e2 amp_e1; do
  NFT_LIB=$PWD/build_ab/$v.so timeout -k 10 200 python -u tools/iter_probe.py >> gpurun_out/amp_ab.log 2>&1 || exit $?
done; done
NFT_LIB=$PWD/build_ab/amp_e2.so timeout -k 10 300 python -u -m pytest tests/test_amp2_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_amp_e2.log 2>&1
echo "amp e2 tests rc=$?"
