#!/bin/bash
# SQ counter passes of tools/pmc_probe.py for config $1 (default C3), one
# rocprofv3 run per pass (at most 8 SQ counters each), summary to
# gpurun_out/pmc_sq_$1.json
cfg=${1:-C3}
R=$PWD
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD"
P2="SQ_WAVES SQ_INSTS_SALU SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES"
n=0
for P in "$P1" "$P2"; do
  n=$((n + 1))
  rm -rf $R/gpurun_out/pmc_sq$n
  timeout -s KILL 150 rocprofv3 --pmc $P --output-format csv -d $R/gpurun_out/pmc_sq$n -o run -- python3 $R/tools/pmc_probe.py $cfg > $R/gpurun_out/pmc_sq$n.log 2>&1 || exit $?
done
cd $R
python3 tools/pmc_sq.py gpurun_out pmc_sq1 pmc_sq2 > gpurun_out/pmc_sq_$cfg.json
