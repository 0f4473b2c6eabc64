#!/bin/bash
# mesh_to_spc level-kernel counters: FP64 instruction mix, VALU issue and
# busy cycles of m2s_level_kernel over a few cfg4 mesh_to_spc calls (scripts/dev/cfg4_probe.py).
set -e
R=$(pwd)
OUT=${OUT:-gpurun_out/m2spmc}
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'm2s_level' --output-format csv \
    -d $R/$OUT/p$n -o run -- python3 $R/scripts/dev/cfg4_probe.py 2 > $R/$OUT/p$n.log 2>&1
done
