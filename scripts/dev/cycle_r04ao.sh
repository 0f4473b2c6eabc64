#!/bin/bash
# backward halves on two streams (dev param 14 = 1): bit-equality, op timing, headline bench A/B
set -e
OUT=gpurun_out/r04ao; mkdir -p $OUT
timeout -k 10 120 python scripts/dev/bwd2s_check.py 14=1 > $OUT/check.txt 2>&1
export OUT
export BENCH_PARAMS="- 14=1 - 14=1"
OUT=$OUT/b bash scripts/dev/bench_params.sh
