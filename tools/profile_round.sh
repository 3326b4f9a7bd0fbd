#!/bin/bash
# One round's evidence in one GPU call: PMC traffic passes (profiles/pmc_traffic.json
# on the box, copied to gpurun_out/), the default bench line, the graph-replayed
# CG iteration under rocprofv3 --kernel-trace (per-label summary by
# tools/trace_labels.py) and the bench under rocprofv3 --kernel-trace --stats.
# Usage (repo root, on the GPU box): tools/profile_round.sh TAG
tag=${1:-cur}
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/tools/pmc_probe.py > $R/gpurun_out/pmc1.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/tools/pmc_probe.py > $R/gpurun_out/pmc2.log 2>&1 || exit $?
cd $R
python3 tools/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.log || exit $?
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/replay_$tag -o run -- python3 $R/tools/replay_probe.py > $R/gpurun_out/replay_$tag.log 2>&1 || exit $?
cd $R
python3 tools/trace_labels.py gpurun_out/replay_$tag/run_kernel_trace.csv 20 > gpurun_out/trace_labels_$tag.json || exit $?
# the count-only chunk with the deferred iterate (19 replays, then the flush)
cd /tmp
LAZY_CHUNK=1 REPLAYS=19 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/replayl_$tag -o run -- python3 $R/tools/replay_probe.py > $R/gpurun_out/replayl_$tag.log 2>&1 || exit $?
cd $R
python3 tools/trace_labels.py gpurun_out/replayl_$tag/run_kernel_trace.csv 19 > gpurun_out/trace_labels_lazy_$tag.json || exit $?
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$tag -o run -- python3 $R/bench.py --no-cpu-baseline > $R/gpurun_out/bench_${tag}_under_rocprof.json 2> $R/gpurun_out/prof_$tag.err
echo "done rc=$?"
