#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes (separate runs) over a short bench, kaolin kernels only
set -e
R=$(pwd)
mkdir -p gpurun_out
cd /tmp; export TMPDIR=/tmp
n=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  n=$((n + 1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex 'kl::' --output-format csv \
    -d $R/gpurun_out/pmcf$n -o run -- python3 $R/bench.py --no-cpu-baseline --no-extra --no-p2m --steps 5 --warmup 2 > $R/gpurun_out/pmcf$n.log 2>&1
done
