export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for rep in 1 2; do for v in ut0 ut2; do
  echo "== $v rep $rep" >> gpurun_out/los_ut.log
  NFT_LIB=$PWD/build_ab/los_$v.so LOS_DBGS=0,1 timeout -k 10 200 python -u tools/los_probe.py >> gpurun_out/los_ut.log 2>&1 || exit $?
done; done
