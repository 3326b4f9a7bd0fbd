#!/bin/bash
# The two rocprofv3 PMC passes of tools/pmc_probe.py (FETCH_SIZE, WRITE_SIZE,
# separate runs) and their summary, for config $1 (default C3); the summary
# is printed to gpurun_out/pmc_summary_$1$2.log ($2: a tag).
cfg=${1:-C3}; tag=$2
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
rm -rf $R/gpurun_out/pmc_fetch $R/gpurun_out/pmc_write
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python3 $R/tools/pmc_probe.py $cfg > $R/gpurun_out/pmc1.log 2>&1 || exit $?
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python3 $R/tools/pmc_probe.py $cfg > $R/gpurun_out/pmc2.log 2>&1 || exit $?
cd $R
python3 tools/pmc_summary.py gpurun_out > gpurun_out/pmc_summary_$cfg$tag.log
