#!/bin/bash
# gather batch 2 as the default: dibr tests, then A/B against batch 1 and 3 builds
set -e
OUT=gpurun_out/r04aw; mkdir -p $OUT; R=$(pwd)
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dibr or rasteriz or soft or gather or fused or tutorial" > $OUT/tests.log 2>&1
for k in 1 2; do
  timeout -k 10 120 python scripts/dev/param_ab.py 0 0 > $OUT/gb2_$k.txt 2>&1
  for b in 1 3; do
    KAOLIN_HIP_LIB=$R/scripts/dev/vlib_gb$b/libkaolin_hip.so timeout -k 10 120 python scripts/dev/param_ab.py 0 0 > $OUT/gb${b}_$k.txt 2>&1
  done
done
