#!/bin/bash
# r02 counter passes over a short bench (kaolin kernels only), each pass its own run and time
# limit: SQ occupancy / issue / wait groups, and the L2-side atomic count.
set -e
R=$(pwd)
OUT=${OUT:-gpurun_out/pmc_r02}
mkdir -p $OUT
cd /tmp; export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $R/$OUT/avail.txt 2>&1 || true
n=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VMEM_WR" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD" \
           "TCC_EA0_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum"; do
  n=$((n + 1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'kl::' --output-format csv \
    -d $R/$OUT/p$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 5 --warmup 2 > $R/$OUT/p$n.log 2>&1 || echo "pass $n failed" >> $R/$OUT/status.txt
done
