#!/bin/bash
# headline bench under dev flag sets (A/B): BENCH_FLAGS="0 0x400000 ..." (one short run each)
set -e
OUT=${OUT:-gpurun_out/bench_ab}
mkdir -p $OUT
for f in ${BENCH_FLAGS:-0}; do
  KAOLIN_DEV_FLAGS=$f timeout -k 10 200 python bench.py --no-cpu-baseline --no-extra --no-p2m --steps 30 > $OUT/bench_$f.json 2> $OUT/bench_$f.err
done
