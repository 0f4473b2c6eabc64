#!/bin/bash
# gather batch size A/B (KL_GATHER_BATCH builds in scripts/dev/vlib_gb*): dibr op timings, twice each
set -e
OUT=gpurun_out/r04av; mkdir -p $OUT; R=$(pwd)
for k in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 0 0 > $OUT/gb4_$k.txt 2>&1
  for b in 2 6 8; do
    KAOLIN_HIP_LIB=$R/scripts/dev/vlib_gb$b/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 > $OUT/gb${b}_$k.txt 2>&1
  done
done
