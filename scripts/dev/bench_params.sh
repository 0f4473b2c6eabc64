#!/bin/bash
# headline bench under dev parameter sets: BENCH_PARAMS="4=5 4=4 4=4,5=1 ..." ("-" = none)
set -e
OUT=${OUT:-gpurun_out/bench_params}
mkdir -p $OUT
k=0
for p in ${BENCH_PARAMS:--}; do
  k=$((k + 1))
  if [ "$p" = "-" ]; then unset KAOLIN_DEV_PARAMS; else export KAOLIN_DEV_PARAMS=$p; fi
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > "$OUT/bench_${k}_$p.json" 2> "$OUT/bench_${k}_$p.err"
done
