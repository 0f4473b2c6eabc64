#!/bin/bash
# p2m counters: the probe (executed vs skipped (wave, face) pairs), then SQ counter passes on
# the bench's p2m leg (p2m_fwd_kernel / p2m_bwd_kernel)
set -e
R=$(pwd)
mkdir -p gpurun_out
timeout -k 10 120 scripts/dev/_bin/p2m_probe > gpurun_out/p2m_probe.log 2>&1
cd /tmp; export TMPDIR=/tmp
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'p2m_' --output-format csv \
    -d $R/gpurun_out/p2mpmc$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --steps 2 --warmup 1 > $R/gpurun_out/p2mpmc$n.log 2>&1
done
