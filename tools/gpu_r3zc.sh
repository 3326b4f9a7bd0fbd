export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
NFT_LIB=$PWD/build_ab/adjdbg.so timeout -k 10 300 python -u tools/los_adj_probe.py > gpurun_out/adj_dbg.log 2>&1
echo "rc=$?"
