#!/bin/bash
# Counter passes over the check_sign probe (cell check and point count kernels), each pass its
# own run and time limit (development aid).
set -e
R=$(pwd)
OUT=${OUT:-gpurun_out/pmc_cs}
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'cs_' --output-format csv \
    -d $R/$OUT/p$n -o run -- python3 $R/scripts/dev/cs_probe.py 2 > $R/$OUT/p$n.log 2>&1 || echo "pass $n failed" >> $R/$OUT/status.txt
done
