export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in 1 2; do for v in 00 10 01 11; do
  echo "== $v rep $rep" >> gpurun_out/los_ab.log
  NFT_LIB=$PWD/build_ab/los$v.so LOS_DBGS=0,2 timeout -k 10 200 python -u tools/los_probe.py >> gpurun_out/los_ab.log 2>&1 || exit $?
done; done
