# rocprofv3 kernel stats of the batched CG iteration, two-phase amplitude
# kernels on / off (tools/amp2_probe.py); then the amp2 GPU tests
R=$PWD
cd /tmp && export TMPDIR=/tmp
for m in 1 0; do
  NFT_CG_AMP2=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_amp2_$m -o run -- python3 -u $R/tools/amp2_probe.py >> $R/gpurun_out/probe.log 2>&1 || exit $?
done
cd $R
timeout -k 10 600 python -u -m pytest tests/test_amp2_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_amp2.log 2>&1
echo "tests rc=$?"
