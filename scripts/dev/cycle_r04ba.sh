#!/bin/bash
# soft forward evaluation: hits in flight per lane (KL_ST_EVAL_U builds in scripts/dev/vlib_u6 / vlib_u8)
set -e
OUT=gpurun_out/r04ba; mkdir -p $OUT; R=$(pwd)
for k in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 0 0 > $OUT/u4_$k.txt 2>&1
  for u in 6 8; do
    KAOLIN_HIP_LIB=$R/scripts/dev/vlib_u$u/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 > $OUT/u${u}_$k.txt 2>&1
  done
done
