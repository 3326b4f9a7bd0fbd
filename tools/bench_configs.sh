# bench lines of the non-headline configs (one GPU), then their rocprofv3
# kernel stats (no CPU baseline under the profiler)
R=$PWD
mkdir -p gpurun_out
for c in "$@"; do
  timeout -k 10 600 python3 -u bench.py --config $c --steps 2 --warmup 1 > gpurun_out/bench_$c.json 2> gpurun_out/bench_$c.err || exit $?
done
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$c -o run -- python3 -u $R/bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline > $R/gpurun_out/bench_${c}_under_rocprof.json 2>> $R/gpurun_out/bench_$c.err || exit $?
done
