#!/bin/bash
# One GPU call's worth of round-end evidence: PMC traffic passes (written to
# profiles/pmc_traffic.json, which bench.py reads for roofline.traffic), the
# default bench line, and the same bench under rocprofv3 --kernel-trace
# --stats.  Usage (repo root, on the GPU box): tools/profile_round.sh TAG
set -e
tag=${1:-cur}
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/tools/pmc_probe.py > $R/gpurun_out/pmc1.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/tools/pmc_probe.py > $R/gpurun_out/pmc2.log 2>&1
cd $R
python3 tools/pmc_summary.py gpurun_out > gpurun_out/pmc_summary.log
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
timeout -k 10 400 python3 -u bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err
cd /tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$tag -o run -- python3 $R/bench.py > $R/gpurun_out/bench_${tag}_under_rocprof.json 2> $R/gpurun_out/prof_$tag.err
