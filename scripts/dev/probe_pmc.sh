#!/bin/bash
# SQ counters of the compact soft-mask kernels on the bench workload (one rocprofv3 pass each).
set -e
R=$GRAFT_REPO_ROOT
cd /tmp; export TMPDIR=/tmp
n=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY" \
           "SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_ANY"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'soft_tile' --output-format csv -d $R/gpurun_out/pmcprobe$n -o run -- python3 $R/scripts/dev/softfwd_probe.py "bench K=30" > $R/gpurun_out/pmcprobe$n.log 2>&1
done
